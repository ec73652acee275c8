#!/bin/bash
# Multiplier iteration: mul parity tests, configs[4] mixed bench + kernel stats, K=16 rate + stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/muliter; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "${KEXPR:-mul or golden or mixed}" > $OUT/pytest.log 2>&1; rc=$?
echo "[pytest] rc=$rc $(tail -n 1 $OUT/pytest.log)"; [ $rc -eq 0 ] || { tail -30 $OUT/pytest.log; exit $rc; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/mixed -o run --output-format csv -- python3 bench.py --workload mixed --steps 2 --warmup 1 > $OUT/mixed.log 2>&1; rc=$?
echo "[mixed] rc=$rc"; grep '^{' $OUT/mixed.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
head -12 $OUT/mixed/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
[ $rc -eq 0 ] || exit $rc
N=1024 KS=16 OPTS=256:256 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/k16 -o run --output-format csv -- python3 scripts/mul_rate.py > $OUT/k16.log 2>&1; rc=$?
echo "[k16] rc=$rc"; tail -3 $OUT/k16.log
head -10 $OUT/k16/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
exit $rc
