#!/bin/bash
# configs[4] mixed workload: bench line + per-kernel rocprofv3 stats (1 GPU, 2^20 values)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mixed; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --workload mixed --steps 2 --warmup 1 > $OUT/bench.log 2>&1; rc=$?
grep '^{' $OUT/bench.log | tail -1 | cut -c1-1500
head -14 $OUT/prof/run_kernel_stats.csv | cut -c1-150
exit $rc
