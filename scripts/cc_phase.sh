#!/bin/bash
# MFMA chain phase split (tools/chain_check with HM_MFMA_PROFILE timers) and plain launch timing of
# every harness build present (tools/chain_check_base, tools/chain_check_v*), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$(ls ./tools/chain_check_base ./tools/chain_check_v* 2>/dev/null | grep -v '\.hip$')
for b in $V; do echo "== check $b"; timeout -k 5 60 $b sweep | tail -1 || exit 1; done
for r in 1 2; do
  echo "== phases"; timeout -k 5 60 ./tools/chain_check time 4096 || exit 1
  for b in $V; do echo "== $b"; timeout -k 5 60 $b time 4096 || exit 1; done
done
echo "== phases wide"; timeout -k 5 120 ./tools/chain_check time25 131072 || exit 1
