#!/bin/bash
# A/B of the pipelined add (hm_ctx_set_add_pipeline) on the headline bench: alternating runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-abpipe}; mkdir -p $OUT
for r in 1 2 3; do for p in 1 0; do
  timeout -k 10 120 python3 -u bench.py --no-secondary --no-cpu --add-pipeline $p > $OUT/b_${p}_$r.log 2>&1 || exit 1
  python3 - $OUT/b_${p}_$r.log $p <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"pipe={sys.argv[2]} {d['value']:.4e} adds/s {d['ms_per_step']:.4f} ms/step ok={d['verified']['correct_sums']}")
PY
done; done
