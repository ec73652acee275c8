#!/bin/bash
# Headline bench at the driver's step counts (20 timed / 5 warm-up, no secondary/CPU legs): the
# in-tree library against variants under lib/variants, alternating, two rounds; an optional -m gpu
# -k subset first.  usage: scripts/ab_main.sh tag "pytest -k expr | none" v1[:chain] v2[:chain] ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
if [ "$K" != none ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/pytest.log 2>&1
  rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -20; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for vc in main "$@"; do
    v=${vc%%:*}; C=auto; [ "$vc" != "$v" ] && C=${vc#*:}
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so
    [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    HOMOMORPH_GPU_LIB=$L timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --no-secondary --no-cpu --add-chain $C > $OUT/b_${v}_${C}_$r.json 2> $OUT/b_${v}_${C}_$r.err || { tail -3 $OUT/b_${v}_${C}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_${v}_${C}_$r.json').read().strip().splitlines()[-1]); print('$vc', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['verified']['correct_sums'])"
  done
done
