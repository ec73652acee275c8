#!/bin/bash
# SQ counter passes (scripts/pmc_cmd.sh's first two) of the headline add for the in-tree library
# and library variants under lib/variants: usage scripts/pmc_ab.sh tag chain v1 v2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; CH=$2; shift 2
for v in main "$@"; do
  L=$PWD/homomorph-rust_amd/lib/libhomomorph_gpu.so
  [ $v = main ] || L=$PWD/homomorph-rust_amd/lib/variants/libhm_$v.so
  O=gpurun_out/$TAG/$v; mkdir -p $O
  for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES" "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
    n=$(echo $pass | cut -c1-12 | tr -d ' ')
    HOMOMORPH_GPU_LIB=$L timeout -k 10 -s KILL 120 rocprofv3 --pmc $pass -d $O/$n -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-secondary --no-cpu --add-chain $CH > $O/$n.log 2>&1 || { echo "[$v $n] failed"; tail -3 $O/$n.log; exit 1; }
  done
  echo "== $v"; python3 scripts/pmc_summary.py $O add_chain | grep -v "calls="
done
