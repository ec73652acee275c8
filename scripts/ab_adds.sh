#!/bin/bash
# A/B of adder builds on one box: scripts/probe/add_rates.py for the in-tree library and each
# variant under lib/variants, alternating, `rounds` rounds.  usage: scripts/ab_adds.sh rounds v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$1; shift
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in main "$@"; do
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so
    [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    HOMOMORPH_GPU_LIB=$L timeout -k 10 120 python3 -u scripts/probe/add_rates.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
