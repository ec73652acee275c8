#!/bin/bash
# rocprofv3 evidence for one command: kernel trace + stats, then PMC passes one by one (SQ
# instruction mix / MFMA busy / LDS waits and conflicts; HBM bytes), each pass its own run.
# usage: scripts/pmc_cmd.sh OUTDIR KERNEL_FILTER -- python3 script.py args...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; FILT=$2; shift 3
mkdir -p $OUT
run() { local name=$1 lim=$2; shift 2; timeout -k 10 -s KILL $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; tail -n 2 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
run trace 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- "$@"
run sq 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES -d $OUT/sq -o run --output-format csv -- "$@"
run sq2 200 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE -d $OUT/sq2 -o run --output-format csv -- "$@"
run fetch 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- "$@"
run write 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- "$@"
python3 scripts/pmc_summary.py $OUT "$FILT" > $OUT/summary.txt
cat $OUT/summary.txt
