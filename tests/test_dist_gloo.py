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
        # the mixed workload's d = dp = tau = 256 keys travel the same way
        sk2 = pk2 = None
        if rank == 0:
            sk2, pk2, _ = oracle.keygen(*bench.MIXED_PARAMS, 0xB0C)
        sk2, pk2 = bench.broadcast_keys(world, rank, dev, sk2, pk2, bench.MIXED_PARAMS)
        a, b = bench.shard_inputs(rank, 64)
        res = torch.from_numpy((a + b).astype(np.uint32).view(np.uint8).reshape(-1, 4).copy())
        got, wall = bench.gather_results(world, dev, res, 1.5 + rank)
        q.put((rank, sk.copy(), pk.copy(), a.copy(), got.copy(), wall, pk2.copy()))
    finally:
        dist.destroy_process_group()


def test_two_rank_keys_shards_and_gather():
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
        r, sk, pk, a, got, wall, pk2 = q.get(timeout=240)
        res[r] = (sk, pk, a, got, wall, pk2)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sys.path.insert(0, ROOT)
    from oracle import oracle_py as oracle
    import bench
    sk0, pk0, _ = oracle.keygen(*bench.PARAMS, 0xB0B)
    _, pk20, _ = oracle.keygen(*bench.MIXED_PARAMS, 0xB0C)
    want = np.concatenate([sum(bench.shard_inputs(r, 64)).astype(np.uint32) for r in range(world)])
    for r in range(world):
        sk, pk, a, got, wall, pk2 = res[r]
        assert np.array_equal(pk2[:, : pk20.shape[1]], pk20)
        assert np.array_equal(sk[: len(sk0)], sk0) and not sk[len(sk0):].any()
        assert np.array_equal(pk[:, : pk0.shape[1]], pk0)
        assert np.array_equal(got.view("<u4").reshape(-1), want)  # every rank's results, rank order
        assert wall == 2.5                 # max over ranks
    assert not np.array_equal(res[0][2], res[1][2])  # distinct shards

