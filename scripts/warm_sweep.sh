#!/bin/bash
# Headline step time against warm-up / timed-step counts (clock ramp under sustained MFMA load).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for wk in "10 20" "50 50" "200 100" "10 20" "400 200"; do
  set -- $wk
  timeout -k 10 200 python3 -u bench.py --no-secondary --no-cpu --warmup $1 --steps $2 > gpurun_out/ws.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ws.json').read().strip().splitlines()[-1]); print('W=$1 K=$2', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))"
done
