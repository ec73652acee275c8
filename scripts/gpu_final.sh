#!/bin/bash
# Round-end style GPU check of the tree as committed: -m gpu suite, smoke(), default bench line
# (with the secondary configs and the CPU baseline).  usage: scripts/gpu_final.sh tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; tail -n 3 $OUT/$name.log; [ $rc -eq 0 ] || exit $rc; }
step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python3 -u bench.py
echo ALLDONE
