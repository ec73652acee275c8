# decrypt_bits A/B (kt_overhead.py's graph steps), then configs[4] with the tiny ppg at 5 waves/SIMD
set -u
for v in main decbold main decbold; do L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so; [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so; echo "== $v"; HOMOMORPH_GPU_LIB=$L timeout -k 10 200 python3 scripts/probe/kt_overhead.py 2>&1 | grep -v amdgpu || exit 1; done
HOMOMORPH_GPU_LIB=$PWD/homomorph-rust_amd/lib/variants/libhm_decbold.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "encrypt or decrypt" 2>&1 | tail -1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_properties.py -k "encrypt or decrypt or config2" 2>&1 | tail -1
bash scripts/ab_mixed.sh ppgt5
