#!/bin/bash
# MFMA carry-chain checks (tools/chain_check.hip, GPU): a sweep of single-bit products, then
# random words and single set bits at several P / ab sizes
timeout -k 5 60 ./tools/chain_check sweep || exit 1
for args in "3 24 16 0" "3 24 16 1 0 0" "3 24 16 1 767 0" "3 24 16 1 0 511" "3 24 16 1 700 300" "3 24 16 1 40 0" "3 24 16 1 0 40" "3 25 17 0" "5 24 16 0"; do
  timeout -k 5 30 ./tools/chain_check $args | tail -4
done
