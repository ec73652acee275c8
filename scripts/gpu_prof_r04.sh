#!/bin/bash
# Round-4 profile evidence in one GPU call (each rocprofv3 run its own process and time limit):
#  1. the driver's bench command under --kernel-trace --stats (headline + every secondary line);
#  2. the headline add alone: trace + SQ/SQ2/FETCH/WRITE passes (scripts/pmc_cmd.sh);
#  3. configs[4] (bench.py --workload mixed, 1 warm-up + 1 timed step of 2^20 values);
#  4. the K = 16 u32 multiply prefix (scripts/mul_rate.py, 1024 values, thresholds 256/256).
# usage: scripts/gpu_prof_r04.sh [parts...]   parts: driver headline mixed k16 (default: all)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/p4
mkdir -p $OUT
PARTS=${*:-driver headline mixed k16}
for p in $PARTS; do
  case $p in
    driver)
      timeout -k 10 -s KILL 500 rocprofv3 --kernel-trace --stats -d $OUT/driver -o run --output-format csv \
        -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver.log 2>&1 || { tail -5 $OUT/driver.log; exit 1; }
      grep '^{' $OUT/driver.log | tail -1 > $OUT/driver_line.json
      echo "[driver] ok";;
    headline)
      bash scripts/pmc_cmd.sh $OUT/headline add_ -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-secondary || exit 1;;
    mixed)
      bash scripts/pmc_cmd.sh $OUT/mixed hm:: -- python3 bench.py --workload mixed --steps 1 --warmup 1 --no-cpu || exit 1;;
    k16)
      KS=16 OPTS=256:256 bash scripts/pmc_cmd.sh $OUT/k16 hm:: -- python3 scripts/mul_rate.py || exit 1;;
  esac
done
echo ALLDONE
