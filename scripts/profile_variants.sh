#!/bin/bash
# PMC comparison of engine builds (scripts/profile_variants.sh lib1.so lib2.so ...): kernel trace
# plus two counter passes per build, summarised for the add kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-secondary"
for lib in "$@"; do
  name=$(basename "$lib" .so); OUT=gpurun_out/pv/$name; mkdir -p $OUT
  export HOMOMORPH_GPU_LIB=$(realpath "$lib")
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t -o run --output-format csv -- $B > $OUT/t.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_IFETCH -d $OUT/p1 -o run --output-format csv -- $B > $OUT/p1.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_IFETCH_LEVEL SQ_INST_CYCLES_SALU -d $OUT/p2 -o run --output-format csv -- $B > $OUT/p2.log 2>&1 || exit 1
  echo "== $name"; python3 scripts/pmc_summary.py $OUT add_ | grep -E "add_|SQ_|GRBM"
done
