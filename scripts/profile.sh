#!/bin/bash
# rocprofv3 evidence for the bench line: kernel trace + stats of the default bench command, then
# PMC passes one by one (HBM bytes; SQ instruction mix, MFMA busy, LDS waits) on the add-only command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python3 bench.py --no-cpu --no-secondary"
run() { local name=$1; shift; timeout -k 10 400 "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; tail -n 2 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run trace rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py
run fetch rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B
run write rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B
run sq rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/sq -o run --output-format csv -- $B
run sq2 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- $B
python3 scripts/pmc_summary.py $OUT add_ > $OUT/summary.txt
cat $OUT/summary.txt
