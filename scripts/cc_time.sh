#!/bin/bash
# MFMA chain harness on the GPU: correctness (sweep of single-bit products, random words, degrees,
# every output word) of the harness builds, then launch timing after a clock warm-up.
# tools/chain_check = the kernel with phase timers; tools/chain_check_{base,v*} = builds without
# them (-DHM_NO_PROFILE) of earlier / candidate kernels, when present.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$(ls ./tools/chain_check_base ./tools/chain_check_v* 2>/dev/null | grep -v '\.hip$')
for b in $V ./tools/chain_check; do
  echo "== check $b"
  timeout -k 5 60 $b sweep | tail -1 || exit 1
  for args in "3 24 16 0" "3 24 16 1 767 0" "3 24 16 1 700 300" "3 25 17 0" "5 24 16 0" "32 24 16 0" "32 13 9 0"; do
    timeout -k 5 30 $b $args | tail -1
  done
done
for r in 1 2; do for b in $V ./tools/chain_check; do
  echo "== $b"; timeout -k 5 60 $b time 4096 || exit 1
done; done
