#!/bin/bash
# MFMA chain harness on the GPU: correctness (sweep of single-bit products, random words) of
# tools/chain_check, then launch timing + per-phase s_memtime sums; other builds of the harness
# (tools/chain_check_base, tools/chain_check_v*: earlier kernels) timed alongside when present.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for b in ./tools/chain_check_base ./tools/chain_check_v1 ./tools/chain_check; do
  [ -x $b ] || continue
  echo "== check $b"
  timeout -k 5 60 $b sweep | tail -1 || exit 1
  for args in "3 24 16 0" "3 24 16 1 767 0" "3 24 16 1 700 300" "3 25 17 0" "5 24 16 0" "32 24 16 0"; do
    timeout -k 5 30 $b $args | tail -1
  done
done
for b in ./tools/chain_check_base ./tools/chain_check_v1 ./tools/chain_check ./tools/chain_check_base ./tools/chain_check_v1 ./tools/chain_check; do
  [ -x $b ] || continue
  echo "== $b"; timeout -k 5 30 $b time 4096 || exit 1
done
