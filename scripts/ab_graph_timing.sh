#!/bin/bash
# Headline step timing: direct launches with the chain's events inside the timed region
# (--graph 0) vs one graph replay per step (--graph 1), alternating on one box.  usage: scripts/ab_graph_timing.sh [ROUNDS]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${1:-3}
for i in $(seq $R); do
  for gm in 0 1; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-secondary --graph $gm > /tmp/ab_g.json || exit 1
    python3 -c "
import json; j=json.loads(open('/tmp/ab_g.json').read().strip().splitlines()[-1]); r=j['roofline']
print('graph=$gm', 'ms/step %.4f' % j['ms_per_step'], 'chain_ms %.4f' % r['kernel_ms'], 'frac %.3f' % r['frac'], 'n', r['kernel_ms_source'][:60], j['verified']['correct_sums'])"
  done
done
