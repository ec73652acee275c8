#!/bin/bash
# The round-end checks in one GPU call: the whole -m gpu suite, smoke(), and the driver's default
# bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5) with its secondary lines.
# usage: scripts/gpu_full.sh tag
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 - <<PY
import json
d = json.loads(open("$OUT/bench.json").read().strip().splitlines()[-1])
print("headline", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"])
for k, v in d.get("secondary", {}).items():
    if isinstance(v, dict):
        print(k, "%.4g" % v.get("value", 0), "roof" if "roofline" in v else "-", "cpu" if "cpu_baseline" in v else "-")
    else:
        print(k, v)
PY
echo ALLDONE
