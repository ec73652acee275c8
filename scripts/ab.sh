#!/bin/bash
# A/B timing of engine builds / settings (bench add only, no CPU leg).  Each argument is
# "lib.so" or "lib.so@VAR=VALUE,VAR2=VALUE" (environment for that run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  lib=${spec%%@*}; envs=""; [[ "$spec" == *@* ]] && envs=${spec#*@}
  for rep in 1 2; do
    out=$(env ${envs//,/ } HOMOMORPH_GPU_LIB=$(realpath "$lib") timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-secondary 2>gpurun_out/ab_err.log) || { echo "$spec failed"; tail gpurun_out/ab_err.log; exit 1; }
    echo "$spec rep$rep $(echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_ms'],4), d['verified'])")"
  done
done
