#!/bin/bash
# chain harness timing with a cold vs an L2-hot workspace (HM_CC_HOT: rewritten before each launch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  timeout -k 5 60 ./tools/chain_check time 4096 || exit 1
  HM_CC_HOT=1 timeout -k 5 60 ./tools/chain_check time 4096 || exit 1
  HM_CC_HOT=1 timeout -k 5 60 ./tools/chain_check_base time 4096 || exit 1
done
HM_CC_HOT=1 timeout -k 5 120 ./tools/chain_check time25 131072 || exit 1
