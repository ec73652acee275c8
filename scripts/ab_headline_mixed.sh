#!/bin/bash
# Headline (steady state) and configs[4] A/B of the in-tree library against variants, alternating:
# add parity tests on each variant first.  usage: scripts/ab_headline_mixed.sh v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_hm; mkdir -p $OUT
for v in main "$@"; do
  L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so; [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
  HOMOMORPH_GPU_LIB=$L timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "add or golden" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "[pytest $v] rc=$rc $(tail -n 1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in main "$@"; do
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so; [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    HOMOMORPH_GPU_LIB=$L timeout -k 10 120 python3 -u bench.py --no-secondary --no-cpu > $OUT/h_${v}_$r.json 2>/dev/null || exit 1
    HOMOMORPH_GPU_LIB=$L timeout -k 10 120 python3 -u bench.py --no-secondary --no-cpu --steps 20 --warmup 5 > $OUT/d_${v}_$r.json 2>/dev/null || exit 1
    HOMOMORPH_GPU_LIB=$L timeout -k 10 200 python3 -u bench.py --workload mixed --steps 2 --warmup 1 --no-cpu > $OUT/m_${v}_$r.json 2>/dev/null || exit 1
    python3 -c "
import json
h=json.loads(open('$OUT/h_${v}_$r.json').read().strip().splitlines()[-1]); d=json.loads(open('$OUT/d_${v}_$r.json').read().strip().splitlines()[-1]); m=json.loads(open('$OUT/m_${v}_$r.json').read().strip().splitlines()[-1])
print('$v', 'steady %.4f chain %.4f' % (h['ms_per_step'], h['roofline']['kernel_ms']), '| 20/5 %.4f chain %.4f' % (d['ms_per_step'], d['roofline']['kernel_ms']), '| mixed %.1f ms' % m['ms_per_step'])"
  done
done
