#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for b in ./tools/chain_check ./tools/chain_check_v*; do echo "== $b"; timeout -k 5 60 $b time 4096 || exit 1; done
