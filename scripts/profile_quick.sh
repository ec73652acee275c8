#!/bin/bash
# Counter passes for the add kernels of the current build (ENV may be passed in the caller).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pq/${1:-cur}; mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-secondary"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- $B > $OUT/t.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS -d $OUT/p1 -o run --output-format csv -- $B > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- $B > $OUT/p2.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $OUT add_
