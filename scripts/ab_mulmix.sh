#!/bin/bash
# Multiplier A/B in one GPU call: the in-tree library's multiply/configs[4] parity tests, then
# scripts/ab_mixed.sh over the variants (their mul tests, configs[4] alternating with the in-tree
# library), then the K = 16 rate of each (scripts/mul_rate.py).  usage: scripts/ab_mulmix.sh v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_mulmix; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "mul or config4 or rem" > $OUT/pytest_main.log 2>&1 || { tail -20 $OUT/pytest_main.log; exit 1; }
tail -1 $OUT/pytest_main.log
bash scripts/ab_mixed.sh "$@" || exit 1
for v in main "$@"; do
  L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so; [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
  HOMOMORPH_GPU_LIB=$L KS=16 OPTS=256:256 timeout -k 10 200 python3 -u scripts/mul_rate.py > $OUT/k16_$v.log 2>&1 || exit 1
  echo $v $(tail -1 $OUT/k16_$v.log)
done
