#!/bin/bash
# Round-5 closing kernel-trace summary of the driver's headline command (committed tree)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_closing -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-secondary --no-cpu > gpurun_out/prof_closing.log 2>&1 || exit 1
echo ALLDONE
