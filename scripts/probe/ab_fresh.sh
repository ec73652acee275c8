set -u
for v in main st64; do
  L=homomorph-rust_amd/lib/libhomomorph_gpu.so; [ $v = main ] || L=homomorph-rust_amd/lib/variants/libhm_$v.so
  echo "== $v"; HOMOMORPH_GPU_LIB=$PWD/$L timeout -k 10 200 python3 -u scripts/probe/fresh_rep.py 25 || exit 1
done
