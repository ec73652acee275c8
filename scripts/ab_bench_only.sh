#!/bin/bash
# Steady-state headline bench alternating between the in-tree library and variants (no parity
# tests: for diagnostic variants that drop work).  usage: scripts/ab_bench_only.sh v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_bench; mkdir -p $OUT
for r in 1 2; do
  for v in main "$@"; do
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so
    [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    HOMOMORPH_GPU_LIB=$L timeout -k 10 120 python3 -u bench.py --no-secondary --no-cpu > $OUT/b_${v}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))"
  done
done
