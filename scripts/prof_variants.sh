#!/bin/bash
# kernel stats of the default bench under library variants (lib/variants/libhm_<v>.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pv
for v in main "$@"; do
  L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so
  [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
  HOMOMORPH_GPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pv/$v -o run --output-format csv -- python3 bench.py --no-secondary --no-cpu --steps 20 --warmup 20 > gpurun_out/pv/$v.log 2>&1 || exit 1
  echo "== $v"; head -4 gpurun_out/pv/$v/run_kernel_stats.csv | cut -d, -f1-4
done
