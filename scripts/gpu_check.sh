#!/bin/bash
# One GPU session: parity tests, smoke, a short bench.  Every GPU step has its own time limit;
# a fault/abort/timeout (anything but pass/fail) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { # name limit cmd...
    local name=$1 lim=$2; shift 2
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step pytest_gpu 600 python -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5
