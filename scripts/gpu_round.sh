#!/bin/bash
# One GPU call: parity tests, default bench line, rocprofv3 kernel trace of the bench.
# usage: scripts/gpu_round.sh <tag>     (outputs under gpurun_out/<tag>/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; tail -n 3 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
step bench 400 python3 -u bench.py
step prof 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu
echo ALLDONE
