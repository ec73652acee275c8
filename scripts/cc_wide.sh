#!/bin/bash
# MFMA chain harness, both chunk configurations: NC = 13 (d + d' <= 256) and NC = 25 (P_i up to
# 49 words, d + d' <= 512): single-bit sweeps, random words, then launch timing of each shape.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
b=./tools/chain_check
timeout -k 5 60 $b sweep | tail -1 || exit 1
timeout -k 5 120 $b sweep25 | tail -1 || exit 1
for args in "3 24 16 0" "3 24 16 1 767 0" "32 24 16 0" "32 13 9 0" "3 26 17 0" "3 49 33 0" "3 49 33 1 1567 511" "5 40 30 0" "32 49 33 0" "32 30 20 0"; do
  timeout -k 5 30 $b $args | tail -1 || exit 1
done
timeout -k 5 60 $b time 4096 || exit 1
timeout -k 5 120 $b time25 131072 || exit 1
