#!/bin/bash
# Round-3 GPU iteration: MFMA chain harness (both chunk configurations), then the -m gpu suite
# (optionally -k filtered).  usage: scripts/gpu_check.sh tag [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-check}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 bash scripts/cc_wide.sh > $OUT/harness.log 2>&1; rc=$?
cat $OUT/harness.log
[ $rc -eq 0 ] || exit $rc
if grep -E "[1-9][0-9]* (mismatching|failing)" $OUT/harness.log; then echo "harness mismatch"; exit 1; fi
if [ -n "$K" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/pytest.log 2>&1
else
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
fi
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" $OUT/pytest.log | tail -40
exit $rc
