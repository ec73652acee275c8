#!/bin/bash
# One GPU iteration on a kernel change: chain harness (correctness + timing of the harness
# builds), then the -m gpu parity suite and the default bench line.  usage: scripts/gpu_iter.sh tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; tail -n ${TAILN:-3} $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
TAILN=40 step harness 200 bash scripts/cc_time.sh
grep -q "mismatching words, status 0" $OUT/harness.log || exit 1
! grep -E "^== check ./tools/chain_check(_v[0-9]+)?$" -A9 $OUT/harness.log | grep -E "[1-9][0-9]* mismatching|[1-9][0-9]* failing" || { echo "new kernel mismatches"; exit 1; }
step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench 400 python3 -u bench.py --no-secondary
echo ALLDONE
