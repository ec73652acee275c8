#!/bin/bash
# GPU parity tests only (optionally a -k filter); output under gpurun_out/<tag>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-tests}; K=${2:-}
mkdir -p gpurun_out/$TAG
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/$TAG/pytest.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/pytest.log 2>&1
fi
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/$TAG/pytest.log | tail -30
exit $rc
