#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/kaprof; mkdir -p $OUT
export TMPDIR=/tmp
N=${N:-1024} KS=16 OPTS=${OPTS:-1024:256} timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 scripts/mul_rate.py > $OUT/log.txt 2>&1; rc=$?
tail -3 $OUT/log.txt
head -12 $OUT/run_kernel_stats.csv | cut -c1-160
exit $rc
