#!/bin/bash
# Round 3 session 2 PMC evidence of the multiplier kernels: configs[4] mixed (1 step) and the K = 16
# multiply, each as a kernel trace plus one PMC pass per counter group (scripts/pmc_cmd.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export N=1024 KS=16 OPTS=256:256
bash scripts/pmc_cmd.sh gpurun_out/pmc_k16 mul_ -- python3 scripts/mul_rate.py > gpurun_out/pmc_k16.log 2>&1 || { tail -5 gpurun_out/pmc_k16.log; exit 1; }
echo "[k16] done"
bash scripts/pmc_cmd.sh gpurun_out/pmc_mixed "" -- python3 bench.py --workload mixed --steps 1 --warmup 1 > gpurun_out/pmc_mixed.log 2>&1 || { tail -5 gpurun_out/pmc_mixed.log; exit 1; }
echo "[mixed] done"
