#!/bin/bash
# Round-6 profile evidence (each rocprofv3 run its own process and time limit; scripts/pmc_cmd.sh):
#   enc      configs[2]'s encrypt / decrypt kernels (scripts/enc_rate.py, 65,536 u32)
#   u8mul    the u8 multiply of benches/u8.rs at batch 16,384 (scripts/mul_rate.py KS=8)
#   k16      configs[3]: the u32 multiply's low 16 bits at batch 1024
#   headline configs[1]: the bench's add step (20 timed + 5 warm-up)
#   mixed    configs[4] (bench.py --workload mixed, 1 + 1 steps of 2^20 values)
#   driver   the driver's bench command under --kernel-trace --stats
# usage: scripts/gpu_prof_r06.sh OUTDIR parts...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
for p in "$@"; do
  case $p in
    enc) REPS=30 bash scripts/pmc_cmd.sh $OUT/enc hm:: -- python3 scripts/enc_rate.py || exit 1;;
    u8mul) KS=8 N=16384 OPTS=256:256 bash scripts/pmc_cmd.sh $OUT/u8mul hm:: -- python3 scripts/mul_rate.py || exit 1
           python3 scripts/pmc_classes.py $OUT/u8mul > $OUT/u8mul/mfma_classes.txt;;
    k16) KS=16 N=1024 OPTS=256:256 bash scripts/pmc_cmd.sh $OUT/k16 hm:: -- python3 scripts/mul_rate.py || exit 1
         python3 scripts/pmc_classes.py $OUT/k16 > $OUT/k16/mfma_classes.txt;;
    headline) bash scripts/pmc_cmd.sh $OUT/headline add_ -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-secondary || exit 1
              python3 scripts/pmc_classes.py $OUT/headline > $OUT/headline/mfma_classes.txt;;
    mixed) bash scripts/pmc_cmd.sh $OUT/mixed hm:: -- python3 bench.py --workload mixed --steps 1 --warmup 1 --no-cpu || exit 1
           python3 scripts/pmc_classes.py $OUT/mixed > $OUT/mixed/mfma_classes.txt;;
    driver) timeout -k 10 -s KILL 500 rocprofv3 --kernel-trace --stats -d $OUT/driver -o run --output-format csv \
              -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver.log 2>&1 || { tail -5 $OUT/driver.log; exit 1; }
            grep '^{' $OUT/driver.log | tail -1 > $OUT/driver_line.json;;
  esac
  echo "[$p] done"
done
echo ALLDONE
