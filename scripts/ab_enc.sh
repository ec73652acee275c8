#!/bin/bash
# Encrypt A/B (scripts/enc_rate.py) of the in-tree library against lib/variants/libhm_<v>.so,
# alternating, two rounds.  usage: scripts/ab_enc.sh v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_enc; mkdir -p $OUT
for r in 1 2; do
  for v in main "$@"; do
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so
    [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    HOMOMORPH_GPU_LIB=$L timeout -k 10 120 python3 -u scripts/enc_rate.py > $OUT/${v}_$r.log 2>&1 || { tail -3 $OUT/${v}_$r.log; exit 1; }
    echo "== $v round $r"; cat $OUT/${v}_$r.log
  done
done
