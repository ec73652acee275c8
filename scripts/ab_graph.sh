#!/bin/bash
# The headline at the driver's step counts with the step as one HIP graph (default) and as direct
# launches, alternating, three rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_graph; mkdir -p $OUT
for r in 1 2 3; do
  for g in 1 0; do
    timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --no-secondary --no-cpu --graph $g > $OUT/b_${g}_$r.json 2> $OUT/b_${g}_$r.err || { tail -3 $OUT/b_${g}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_${g}_$r.json').read().strip().splitlines()[-1]); print('graph=$g', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))"
  done
done
