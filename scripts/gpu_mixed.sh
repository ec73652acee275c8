#!/bin/bash
# configs[4] runs on one GPU: the mixed workload at a reduced and at the full global batch, and a
# two-rank gloo rehearsal of its gather path (ranks share the card; not a measured configuration).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() { # name limit cmd...
    local name=$1 lim=$2; shift 2
    timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 4
    [ $rc -eq 0 ] || exit $rc
}
step add 200 python3 bench.py --steps 5 --warmup 1 --no-cpu --no-secondary
step mixed_256k 300 python3 bench.py --workload mixed --batch 262144 --steps 2 --warmup 1
step mixed_full 400 python3 bench.py --workload mixed --steps 2 --warmup 1
HM_BENCH_BACKEND=gloo step mixed_gloo2 300 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
    --workload mixed --batch 262144 --steps 2 --warmup 1
