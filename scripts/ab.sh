#!/bin/bash
# A/B timing of engine builds: scripts/ab.sh lib1.so lib2.so ...  (bench add only, no CPU leg)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in "$@"; do
  for rep in 1 2; do
    out=$(HOMOMORPH_GPU_LIB=$(realpath "$lib") timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-secondary 2>gpurun_out/ab_err.log) || { echo "$lib failed"; tail gpurun_out/ab_err.log; exit 1; }
    echo "$lib rep$rep $(echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['kernel_ms'], d['ms_per_step'], d['verified'])")"
  done
done
