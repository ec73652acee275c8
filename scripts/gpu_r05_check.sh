#!/bin/bash
# Round-5 check: decrypt determinism probe, the -m gpu suite, the driver bench, then A/Bs
# (ring-fill lane pairs on the headline; edge-tile chunk trimming on the K = 16 and u8 multiplies)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 120 python3 scripts/probe/dec_diag.py > gpurun_out/dec_diag4.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_full.log 2>&1 || exit 1
bash scripts/ab_bench_only.sh ringh > gpurun_out/ab_ring.log 2>&1 || exit 1
KS=16 N=1024 bash scripts/ab_mulrate.sh k16edge edge0 edge2 > gpurun_out/ab_k16edge.log 2>&1 || exit 1
KS=8 N=16384 bash scripts/ab_mulrate.sh u8edge edge0 edge2 > gpurun_out/ab_u8edge.log 2>&1 || exit 1
echo ALLDONE
