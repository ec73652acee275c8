#!/bin/bash
# K = 16 multiply rate (scripts/mul_rate.py, 1024 values) of the in-tree library and variants,
# alternating, three rounds.  usage: scripts/ab_k16.sh v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_k16; mkdir -p $OUT
for r in 1 2 3; do
  for v in main "$@"; do
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so; [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    HOMOMORPH_GPU_LIB=$L KS=16 OPTS=256:256 timeout -k 10 200 python3 -u scripts/mul_rate.py > $OUT/k16_${v}_$r.log 2>&1 || exit 1
    echo $v $(tail -1 $OUT/k16_${v}_$r.log)
  done
done
