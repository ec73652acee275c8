#!/bin/bash
# A/B of engine library builds on the multiplier: mul parity tests against each candidate
# (HOMOMORPH_GPU_LIB), then the K = 16 rate (scripts/mul_rate.py), alternating with the in-tree
# library.  usage: scripts/ab_mul.sh v1 v2 ...   (homomorph-rust_amd/lib/variants/libhm_<v>.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_mul; mkdir -p $OUT
for v in "$@"; do
  HOMOMORPH_GPU_LIB=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "mul or golden" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "[pytest $v] rc=$rc $(tail -n 1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in main "$@"; do
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so
    [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    echo "$v: $(HOMOMORPH_GPU_LIB=$L KS=16 OPTS=256:256 timeout -k 10 200 python3 -u scripts/mul_rate.py 2>/dev/null | tail -1)" || exit 1
  done
done
