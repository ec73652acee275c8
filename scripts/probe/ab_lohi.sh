set -u
HOMOMORPH_GPU_LIB=$PWD/homomorph-rust_amd/lib/variants/libhm_lohi.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests -k "add or golden" > gpurun_out/t_lohi.log 2>&1; echo "pytest(lohi) rc=$? $(tail -1 gpurun_out/t_lohi.log)"
bash scripts/ab_bench_only.sh lohi || exit 1
bash scripts/ab_bench_only.sh lohi || exit 1
