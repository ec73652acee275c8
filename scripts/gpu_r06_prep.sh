#!/bin/bash
# Round 6: the prep kernel's one-round-trip operand staging -- the add parity tests (bad-input
# detection included), then alternating add steps against the previous staging (lib/variants).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-prep}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "add or bad or golden or config1 or noise" > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash scripts/ab_adds.sh 3 ${2:-prevstage} > $OUT/ab.log 2>&1; rc=$?; cat $OUT/ab.log; exit $rc
