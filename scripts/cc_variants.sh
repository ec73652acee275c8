#!/bin/bash
# Time MFMA chain harness variants (tools/chain_check_v*): correctness sweep, then time (NC = 13,
# 4096 values) and time25 (NC = 25, 131072 values), twice each, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for b in ./tools/chain_check_v*; do
  [ -x $b ] || continue
  echo "== $b"; timeout -k 5 60 $b sweep | tail -1; timeout -k 5 120 $b sweep25 | tail -1
done
for r in 1 2; do for b in ./tools/chain_check_v*; do
  echo "== $b $(timeout -k 5 60 $b time 4096) | $(timeout -k 5 120 $b time25 131072)"
done; done
