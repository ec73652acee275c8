"""World-size-2 CPU (gloo) coverage of bench.py's multi-rank path.

The GPU bench runs one process per GPU over RCCL; the distributed pieces are backend-agnostic
and are exercised here with gloo on the CPU: rank 0's keys reach every rank bit for bit, each
rank's shard is distinct (the batch partitions into independent values), and the reduction
gives the summed correct count and the max wall time that `value` is computed from.
"""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    for p in (ROOT, os.path.join(ROOT, "homomorph-rust_amd"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    import bench
    from oracle import oracle_py as oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cpu")
        sk = pk = None
        if rank == 0:
            sk, pk, _ = oracle.keygen(*bench.PARAMS, 0xB0B)
        sk, pk = bench.broadcast_keys(world, rank, dev, sk, pk)
        a, b = bench.shard_inputs(rank, 64)
        correct, wall = bench.reduce_over_ranks(world, dev, 60 + rank, 1.5 + rank)
        q.put((rank, sk.copy(), pk.copy(), a.copy(), correct, wall))
    finally:
        dist.destroy_process_group()


def test_two_rank_keys_shards_and_reduction():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, sk, pk, a, correct, wall = q.get(timeout=240)
        res[r] = (sk, pk, a, correct, wall)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from oracle import oracle_py as oracle
    import bench
    sk0, pk0, _ = oracle.keygen(*bench.PARAMS, 0xB0B)
    for r in range(world):
        sk, pk, a, correct, wall = res[r]
        assert np.array_equal(sk[: len(sk0)], sk0) and not sk[len(sk0):].any()
        assert np.array_equal(pk[:, : pk0.shape[1]], pk0)
        assert correct == 60 + 61          # summed over ranks
        assert wall == 2.5                 # max over ranks
    assert not np.array_equal(res[0][2], res[1][2])  # distinct shards

