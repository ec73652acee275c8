#!/bin/bash
# Headline bench (driver step counts, no secondary/CPU legs) of the in-tree library and diagnostic
# variants under lib/variants (results may be wrong in a diagnostic variant; only timing is read).
# usage: scripts/ab_diag.sh tag v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in 1 2; do
  for v in main fused "$@"; do
    # main: the default (split) chain; fused and the variants: the fused chain (hm_ctx_set_add_options MFMA_FUSED)
    L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so; C=mfma_fused
    [ $v = main ] && C=auto
    [ $v = main ] || [ $v = fused ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
    HOMOMORPH_GPU_LIB=$L timeout -k 10 120 python3 -u bench.py --steps 20 --warmup 5 --no-secondary --no-cpu --add-chain $C > $OUT/b_${v}_$r.json 2> $OUT/b_${v}_$r.err || { tail -3 $OUT/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/b_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['verified']['correct_sums'])"
  done
done
