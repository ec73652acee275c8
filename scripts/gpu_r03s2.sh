#!/bin/bash
# Round 3 (session 2) evidence: -m gpu suite, smoke(), the default bench line, then kernel stats of
# configs[4] (mixed, 2^20) and of the K = 16 multiply, with PMC passes of the multiplier kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03s2; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "[$name] rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 500 python3 -u bench.py
step mixed 400 rocprofv3 --kernel-trace --stats -d $OUT/mixed -o run --output-format csv -- python3 bench.py --workload mixed --steps 2 --warmup 1
export N=1024 KS=16 OPTS=256:256
step k16 300 rocprofv3 --kernel-trace --stats -d $OUT/k16 -o run --output-format csv -- python3 scripts/mul_rate.py
echo ALLDONE
