#!/bin/bash
# configs[4] mixed-workload A/B of library variants (lib/variants/libhm_<v>.so): mul parity tests
# on each, then the mixed bench line alternating with the in-tree library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_mixed; mkdir -p $OUT
for v in "$@"; do
  HOMOMORPH_GPU_LIB=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "${KEXPR:-mul}" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "[pytest $v] rc=$rc $(tail -n 1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in main "$@"; do
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so
    [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    HOMOMORPH_GPU_LIB=$L timeout -k 10 200 python3 -u bench.py --workload mixed --steps 2 --warmup 1 > $OUT/b_${v}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],1), d['value'])"
  done
done
