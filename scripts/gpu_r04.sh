#!/bin/bash
# Round-4 GPU iteration: the -m gpu suite (or a -k subset; "none" skips it), then the default
# headline bench at the driver's 20 timed / 5 warm-up steps, twice.
# usage: scripts/gpu_r04.sh tag [pytest -k expr | all | none]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r04}; K=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$K" != none ]; then
  if [ "$K" = all ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
  else
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/pytest.log 2>&1
  fi
  rc=$?
  grep -E "FAILED|ERROR|passed|failed|Error" $OUT/pytest.log | tail -30
  [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --no-secondary --no-cpu > $OUT/b_$r.json 2> $OUT/b_$r.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/b_$r.json').read().strip().splitlines()[-1]); print('bench', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['verified']['correct_sums'])"
done
echo ALLDONE
