#!/bin/bash
# A/B of engine library builds on the GPU: the harness checks of the candidate chain kernels, the
# -m gpu suite against each candidate library (HOMOMORPH_GPU_LIB), then the default bench line
# alternating between the in-tree library and the candidates.
# usage: scripts/ab_libs.sh tag v4 v5 ...   (libraries: homomorph-rust_amd/lib/variants/libhm_<v>.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  b=./tools/chain_check_$v
  [ -x $b ] || continue
  timeout -k 5 60 $b sweep | tail -1 | tee -a $OUT/check.log
  for args in "3 24 16 0" "3 24 16 1 767 0" "3 24 16 1 700 300" "3 25 17 0" "32 24 16 0" "32 13 9 0"; do
    timeout -k 5 30 $b $args | tail -1 | tee -a $OUT/check.log
  done
done
if grep -E "[1-9][0-9]* (mismatching|failing)" $OUT/check.log; then echo "harness mismatch"; exit 1; fi
for v in "$@"; do
  HOMOMORPH_GPU_LIB=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "[pytest $v] rc=$rc"; tail -n 2 $OUT/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in main "$@"; do
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so
    [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    HOMOMORPH_GPU_LIB=$L timeout -k 10 120 python3 -u bench.py --no-secondary --no-cpu > $OUT/bench_${v}_$r.log 2>&1 || exit 1
    python3 - $OUT/bench_${v}_$r.log $v <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[2]:6s} {d['value']:.4e} adds/s  {d['ms_per_step']:.4f} ms/step  chain {d['roofline']['kernel_ms']*1e3:.1f} us  frac {d['roofline']['frac']:.3f}")
PY
  done
done
echo ALLDONE
