#!/bin/bash
# PMC passes for the add kernel under HM_DEBUG_SKIP settings (timing-structure experiments).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-secondary"
for s in ${SKIPS:-2 3 0}; do
  OUT=gpurun_out/pa/skip$s; mkdir -p $OUT
  HM_DEBUG_SKIP=$s timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- $B > $OUT/t.log 2>&1 || exit 1
  HM_DEBUG_SKIP=$s timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/p1 -o run --output-format csv -- $B > $OUT/p1.log 2>&1 || exit 1
  HM_DEBUG_SKIP=$s timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- $B > $OUT/p2.log 2>&1 || exit 1
  echo "== skip=$s"; python3 scripts/pmc_summary.py $OUT add_kernel | grep -E "add_kernel|SQ_|GRBM"
done
