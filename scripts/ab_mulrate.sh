#!/bin/bash
# Multiply-rate A/B (scripts/mul_rate.py) of the in-tree library against lib/variants/libhm_<v>.so,
# alternating, three rounds.  env: KS (default 8), N (default 16384: the bench's u8 batch), OPTS.
# usage: scripts/ab_mulrate.sh tag v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/ab_$TAG; mkdir -p $OUT
for r in 1 2 3; do
  for v in main "$@"; do
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so; [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    HOMOMORPH_GPU_LIB=$L KS=${KS:-8} N=${N:-16384} OPTS=${OPTS:-256:256} timeout -k 10 200 python3 -u scripts/mul_rate.py > $OUT/${v}_$r.log 2>&1 || { tail -3 $OUT/${v}_$r.log; exit 1; }
    echo $v $(tail -1 $OUT/${v}_$r.log)
  done
done
