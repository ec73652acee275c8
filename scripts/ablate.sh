#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for s in 0 1 2 3; do
  echo "skip=$s"; HM_DEBUG_SKIP=$s timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-secondary 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'], d['verified'])" || exit 1
done
