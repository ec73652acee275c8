set -u
bash scripts/probe/ab_fresh.sh || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "encrypt or golden or config2 or csprng or mask" > gpurun_out/t_encst.log 2>&1; echo "pytest rc=$? $(tail -1 gpurun_out/t_encst.log)"
for v in main st64 main st64 main st64; do L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so; [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so; echo "== $v"; HOMOMORPH_GPU_LIB=$L timeout -k 10 200 python3 scripts/probe/kt_overhead.py 2>&1 | grep encrypt || exit 1; done
