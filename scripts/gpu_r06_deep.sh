#!/bin/bash
# Round 6: split Karatsuba plans (hm_ctx_set_mul_scratch) -- their tests, the multiplier's golden and
# Karatsuba tests on the default plans, then the deep-prefix probe (K = 22, 24 on one value).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-deep}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "split or low22 or low20 or mullow or karatsuba" > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u scripts/probe/mul_deep.py 22 24 > $OUT/deep.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/deep.log | tail -5; exit $rc
