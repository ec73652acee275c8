#!/bin/bash
# PMC passes on the add-only bench (MFMA carry chain): instruction mix, MFMA busy, LDS waits.
# usage: scripts/profile_mfma.sh <tag>    (outputs under gpurun_out/<tag>/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc}
mkdir -p $OUT
B="python3 bench.py --steps 20 --warmup 3 --no-cpu --no-secondary"
run() { local name=$1; shift; timeout -k 10 300 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; tail -n 2 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
timeout -k 5 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
run trace rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B
run sqa rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/sqa -o run --output-format csv -- $B
run sqb rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d $OUT/sqb -o run --output-format csv -- $B
python3 scripts/pmc_summary.py $OUT add_ > $OUT/summary.txt
cat $OUT/summary.txt
