#!/bin/bash
# Karatsuba multiplier: parity tests, then timing of strategies
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ka; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "karatsuba or mul or golden" > $OUT/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" $OUT/pytest.log | tail -30
[ $rc -eq 0 ] || exit $rc
N=${N:-1024} KS=${KS:-12,16} OPTS=${OPTS:-0:256,1024:256,1024:128,2048:384} timeout -k 10 400 python -u scripts/mul_rate.py > $OUT/rate.log 2>&1; rc=$?
cat $OUT/rate.log | tail -20
exit $rc
