#!/bin/bash
# Copy the rocprofv3 outputs of scripts/profile.sh (gpurun_out/prof, merged back from the GPU box)
# into the tracked profiles/<tag>/ directory and refresh profiles/add_traffic.json.
# usage: scripts/save_profiles.sh <tag>   e.g. r01
set -eu
cd "$(dirname "$0")/.."
TAG=${1:?tag}
SRC=gpurun_out/prof
DST=profiles/$TAG
mkdir -p "$DST"
cp $SRC/trace/run_kernel_stats.csv "$DST/kernel_stats.csv"
cp $SRC/trace/run_kernel_trace.csv "$DST/kernel_trace.csv"
for p in fetch write sq sq2; do cp $SRC/$p/run_counter_collection.csv "$DST/pmc_$p.csv"; done
cp $SRC/summary.txt "$DST/summary.txt"
grep '^{' $SRC/trace.log | tail -1 > "$DST/bench_line.json"
python3 scripts/traffic_json.py $SRC profiles/add_traffic.json > /dev/null
echo "saved to $DST"
