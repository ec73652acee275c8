#!/usr/bin/env python3
"""Headline benchmark: homomorphic u32 additions per second at d = d' = tau = 128, delta = 1.

One step = one batched launch of the ripple-carry adder (src/impls/numbers/common.rs:37-56) over
`--batch` u32 ciphertext pairs per GPU (BASELINE.json configs[1]: batch 4096), inputs already
resident in HBM.  Multi-GPU: one process per GPU (torchrun), each rank adds its own shard (weak
scaling, no data-path collective); keys are broadcast once over RCCL at setup, and after the timed
region the decrypted results are gathered over RCCL (all_gather) and checked on rank 0.

`--workload mixed` runs configs[4] instead: one u32 add plus one u32 multiply (low 8 result bits)
per value at d = dp = tau = 256, global batch 2^20 split over the ranks (strong scaling).

`--gpus N` with N > 1 and no torchrun environment starts N rank processes itself (one per GPU,
before this process touches the GPU) and exits with their status; under torchrun it checks that
WORLD_SIZE equals N.  `--workload distcheck` runs only the multi-rank plumbing (spawn, key
broadcast, shards, result gather, max-over-ranks time) on the CPU with gloo, for the CPU tests.

Prints ONE JSON line (rank 0).  Besides the contract fields it carries
  roofline      MFMA roofline of the dominant kernel (the carry chain on fp4 matrix cores):
                algorithmic bit-pair ops per launch / its HIP-event duration, vs the dense fp4 peak
  cpu_baseline  the CPU oracle (operation-for-operation restatement of the reference) timed on a
                bounded sample on this host: one thread (the reference is single-threaded) and
                all host cores (values split over OpenMP threads), CPU model stated
  secondary     u32 encrypt+decrypt throughput (configs[2]) and multiply throughput (u8, and the
                low result bits of the u32 circuit; a full u32 mul is infeasible)
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "homomorph-rust_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import homomorph as H  # noqa: E402

PARAMS = (128, 128, 1, 128)
MUL_LOW_BENCH = 16  # configs[3]: result bits of the u32 multiply that are run
BENCH_SEED = 0xB0B  # rank 0's keys and the mask stream (hm_ctx_seed_rng, the test contract)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
FP4_MFMA_PEAK_TFLOPS = 10000.0  # MI355X dense FP4 MFMA peak (MI355X_MICROARCH.md; not the sparse 20 PF)
PCIE_PEAK_GBS = 63.0  # host link, PCIe Gen5 x16 one direction (MI355X_MICROARCH.md "Host link")
MUL_BATCH = 1024  # configs[3]: "u32 homomorphic mul, batch=1024"


def chain_bit_pairs(ba, bb):
    """Schoolbook bit pairs of the adder chain's carry products (common.rs:37-56 as carry' =
    ab_i ^ P_i * carry_i): sum over bits i = 1 .. L-2 of (deg P_i + 1) * (deg carry_i + 1) at the
    static degree bounds, deg P_i <= max(a_i, b_i) + a_i + b_i and deg carry_{i+1} <= deg P_i +
    deg carry_i with carry_1 = a_0 b_0.  Bit 0 multiplies a null carry, bit L-1 has no carry out."""
    ba, bb = [int(x) for x in ba], [int(x) for x in bb]
    total, carry = 0, ba[0] + bb[0]
    for i in range(1, len(ba) - 1):
        p = max(ba[i], bb[i]) + ba[i] + bb[i]
        total += (p + 1) * (carry + 1)
        carry = max(ba[i] + bb[i], p + carry)
    return total


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def spawn_ranks(args):
    """`bench.py --gpus N` outside torchrun: start N rank processes of this same script (one per
    GPU; RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their environment) and return their exit status.
    Runs before anything here touches the GPU; a rank that fails takes the others down."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:  # the exact child PIDs this process started
                    q.terminate()
        time.sleep(0.2)
    return rc


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.workload == "distcheck":  # CPU plumbing only: gloo, no GPU
        if world > 1:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        return world, rank, local, torch.device("cpu")
    # one rank per GPU; HM_BENCH_BACKEND=gloo with more ranks than GPUs is a rehearsal mode for
    # a one-GPU box (ranks share the card), never the measured configuration
    backend = os.environ.get("HM_BENCH_BACKEND", "nccl")
    dev = local % torch.cuda.device_count() if backend == "gloo" else local
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: {dist.get_world_size()} ranks joined, --gpus {args.gpus}")
    return world, rank, local, torch.device("cuda", dev)


def barrier(world):
    if world > 1:
        dist.barrier()


def coll_device(device):
    """Where a collective's tensors live: the rank's GPU under RCCL; the host under gloo (the CPU
    tests, and the one-GPU rehearsal mode of setup_dist)."""
    return torch.device("cpu") if dist.get_backend() == "gloo" else device


def broadcast_keys(world, rank, device, sk=None, pk=None, params=PARAMS):
    """Rank 0's (sk, pk) limbs -> every rank (setup, untimed; RCCL on GPUs, gloo in the CPU
    tests).  Returns host uint64 arrays (sk: d/64+1 limbs, pk: tau x (d+dp)/64+1 limbs)."""
    if world == 1:
        return sk, pk
    device = coll_device(device)
    d, dp, delta, tau = params
    skt = torch.zeros(d // 64 + 1, dtype=torch.int64, device=device)
    pkt = torch.zeros((tau, (d + dp) // 64 + 1), dtype=torch.int64, device=device)
    if rank == 0:
        skt[: len(sk)].copy_(torch.from_numpy(np.ascontiguousarray(sk, np.uint64).view(np.int64)))
        pk = np.ascontiguousarray(pk, np.uint64)
        pkt[:, : pk.shape[1]].copy_(torch.from_numpy(pk.view(np.int64)))
    dist.broadcast(skt, 0)
    dist.broadcast(pkt, 0)
    return skt.cpu().numpy().view(np.uint64), pkt.cpu().numpy().view(np.uint64)


def make_context(world, rank, device, params=PARAMS):
    """Keys are generated on rank 0 and broadcast to every rank (setup, untimed)."""
    ctx = H.Context(H.Parameters(*params), device=device)
    sk = pk = None
    if rank == 0:
        ctx.seed_rng(BENCH_SEED)  # reproducible keys and masks (the test contract)
        ctx.generate_secret_key()
        ctx.generate_public_key()
        sk, pk = ctx.get_secret_key().limbs, ctx.get_public_key().limbs
    if world > 1:
        sk, pk = broadcast_keys(world, rank, device, sk, pk, params)
        if rank != 0:
            ctx.set_secret_key(H.SecretKey(sk))
            ctx.set_public_key(H.PublicKey(pk))
    return ctx


def shard_inputs(rank, n):
    """This rank's shard of the synthetic batch: n seeded u32 pairs, distinct per rank (the batch
    is partitioned into independent values, no exchange between ranks)."""
    rng = np.random.default_rng(1000 + rank)
    a = rng.integers(0, 2**32, size=n, dtype=np.uint32)
    b = rng.integers(0, 2**32, size=n, dtype=np.uint32)
    return a, b


def gather_results(world, device, res, wall):
    """The final result gather (RCCL all_gather on GPUs, gloo in the CPU tests): every rank's
    decrypted plaintext bytes (n x k uint8, equal n per rank) and wall time reach every rank.
    Returns (world*n x k numpy array in rank order, max wall time).  Identity at world 1."""
    if world == 1:
        return res.cpu().numpy(), float(wall)
    device = coll_device(device)
    res = res.to(device)
    parts = [torch.empty_like(res) for _ in range(world)]
    dist.all_gather(parts, res.contiguous())
    w = torch.tensor([float(wall)], dtype=torch.float64, device=device)
    walls = [torch.empty_like(w) for _ in range(world)]
    dist.all_gather(walls, w)
    return torch.cat(parts).cpu().numpy(), max(float(x.item()) for x in walls)


def time_loop(fn, steps, warmup, world, stream=None):
    """Warmup, then time exactly `steps` calls between barrier+synchronize brackets.  HIP events
    are recorded on the stream the kernels run on (the engine's stream)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        fn()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    return wall, ev0.elapsed_time(ev1) / 1e3


def sustained_chain(ctx, fn, reps, n, pairs, replays=6):
    """The headline's chain kernel at sustained clocks, AFTER the timed region and outside it
    (never part of `value`): the K-step graph replayed `replays` times back to back; the last
    replay's chain stamps and HIP events are reported.  With the driver's --warmup 5 the timed
    region starts on a GPU that has been busy for ~3 ms and its clocks are still ramping
    (DESIGN.md s4.1); this line shows what the same kernel does once they have settled."""
    ctx.set_kernel_timing(True, "add_chain")

    def steps():
        for _ in range(reps):
            fn()

    gk = ctx.graph(steps, warmup=0)
    for _ in range(replays - 1):
        gk.replay()
    ctx.clear_kernel_timing()  # (synchronizes; the slots stay, the earlier replays' stamps go)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(ctx.stream)
    gk.replay()
    ev1.record(ctx.stream)
    torch.cuda.synchronize()
    kms, kn = ctx.kernel_timing()
    ctx.set_kernel_timing(False)
    ctx.synchronize()
    chain_s = kms / 1e3 / max(1, kn)
    step_s = ev0.elapsed_time(ev1) / 1e3 / reps
    achieved = 2.0 * pairs * n / chain_s / 1e12
    return {"replays_before": replays - 1, "steps": reps, "kernel_ms": 1e3 * chain_s,
            "ms_per_step": 1e3 * step_s, "adds_per_s": n / step_s, "achieved": achieved,
            "frac": achieved / FP4_MFMA_PEAK_TFLOPS,
            "note": "not the headline: the same K-step graph replayed after the timed region; "
                    "the last replay's chain stamps and HIP events"}


def timed_graph(ctx, fn, reps, warmup, world=1, kernel=None):
    """The timed region as ONE replay of a HIP graph holding `reps` steps of `fn` (the warm-up:
    `warmup` replays of a one-step graph).  With `kernel` ("add_chain", "encrypt", "decrypt")
    every launch of that kernel in the timed steps is timed by the engine's device wall-clock
    stamps (hm_ctx_set_kernel_timing: one record slot per captured launch, filled by the timed
    replay).  Returns (wall s, step s by HIP events, kernel s per launch or None, launches)."""
    g1 = ctx.graph(fn, warmup=2)
    for _ in range(warmup):
        g1.replay()
    torch.cuda.synchronize()
    if kernel:
        ctx.set_kernel_timing(True, kernel)

    def steps():
        for _ in range(reps):
            fn()

    gk = ctx.graph(steps, warmup=0)
    wall, ev_s = time_loop(gk.replay, 1, 0, world, ctx.stream)  # (replays on the engine stream)
    ks, kn = None, 0
    if kernel:
        kms, kn = ctx.kernel_timing()
        ctx.set_kernel_timing(False)
        ks = kms / 1e3 / max(1, kn)
    ctx.synchronize()
    return wall, ev_s / reps, ks, kn


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores():
    """CPUs this process may use (the GPU box's share; os.cpu_count() shows the whole host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n))))


def cpu_baseline_add(seconds):
    """Oracle (C restatement of the reference's add path) on a bounded sample of the configs[1]
    workload: one thread (comparable with the single-threaded reference) and all host cores
    (values split over OpenMP threads)."""
    from oracle import oracle_py as oracle
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import as_bytes, fresh_bound, keys, masks
    d, dp, delta, tau = PARAMS
    sk, pk, _ = keys(d, dp, delta, tau, 77)
    cores = host_cores()
    n = max(4, cores)
    rng = np.random.default_rng(5)
    a = rng.integers(0, 2**32, size=n, dtype=np.uint32)
    b = rng.integers(0, 2**32, size=n, dtype=np.uint32)
    bound = fresh_bound(d, dp, 32)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), masks(n, 32, tau, 1), bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), masks(n, 32, tau, 2), bound)
    ob = H.add_out_bounds(bound, bound)

    def leg(threads, secs, per_call):
        oracle.set_threads(threads)
        done, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < secs:
            oracle.add_batch(la[: per_call * len(la) // n], da[: per_call * 32], bound,
                             lb[: per_call * len(lb) // n], db[: per_call * 32], bound, 32,
                             per_call, ob)
            done += per_call
        el = time.perf_counter() - t0
        oracle.set_threads(1)
        return done, el

    d1, e1 = leg(1, seconds * 0.6, 4)
    dn, en = leg(cores, seconds * 0.4, n)
    return {"value": d1 / e1, "unit": "adds/s", "cores": 1, "kind": "port",
            "cpu": cpu_model(), "host_cores_available": cores,
            "sample": f"{d1} u32 homomorphic adds (4 seeded pairs, repeated) in {e1:.1f} s on 1 "
                      f"thread; C oracle restating src/polynomial.rs + common.rs, -O3",
            "all_cores": {"value": dn / en, "unit": "adds/s", "cores": cores,
                          "sample": f"{dn} adds ({n} seeded pairs per call, values split over "
                                    f"{cores} OpenMP threads) in {en:.1f} s"}}


def confirm_noise(ctx, a, b, ca, cb, out, got):
    """Checker for the sums that decrypt wrongly (part of the CPU-oracle leg, after the timed
    region): the oracle, fed the same keys and the seeded engine masks (draws 0 and 1 of the
    context, tests/helpers.py), must produce bit-identical sum ciphertexts and decrypt them to the
    same wrong values -- the reference's path would fail on them identically (scheme noise)."""
    from oracle import oracle_py as oracle
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import as_bytes, seeded_value_masks
    want = (a + b).astype(np.uint32)
    wrong = np.nonzero(got != want)[0]
    res = {"wrong_sums": wrong.tolist()}
    if len(wrong) == 0 or len(wrong) > 64:
        res["noise_confirmed_bit_exact"] = len(wrong) == 0
        return res
    sk, pk = ctx.get_secret_key().limbs, ctx.get_public_key().limbs
    mb = ctx.mask_bytes()
    ma = seeded_value_masks(BENCH_SEED, 0, wrong, 32, mb)
    mbb = seeded_value_masks(BENCH_SEED, 1, wrong, 32, mb)
    la, da = oracle.encrypt_batch(pk, as_bytes(a[wrong]), ma, ca.bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b[wrong]), mbb, cb.bound)
    rl, rd = oracle.add_batch(la, da, ca.bound, lb, db, cb.bound, 32, len(wrong), out.bound)
    rows = [H.value_slice(out, int(e), int(e) + 1).to_host() for e in wrong]
    gl, gd = np.concatenate([r[0] for r in rows]), np.concatenate([r[1] for r in rows])
    rdec = oracle.decrypt_batch(sk, rl, rd, out.bound, 32, len(wrong)).view(np.uint32).reshape(-1)
    res["noise_confirmed_bit_exact"] = bool(np.array_equal(gl, rl) and np.array_equal(gd, rd) and
                                            np.array_equal(rdec, got[wrong]))
    return res


def oracle_leg(fn, per_call, seconds, what):
    """The oracle (C restatement of the reference's path) on ONE host thread, as the reference
    runs: fn() repeated for about `seconds`, per_call units each.  A baseline, not a target."""
    from oracle import oracle_py as oracle
    oracle.set_threads(1)
    done, t0 = 0, time.perf_counter()
    while True:
        fn()
        done += per_call
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": done / el, "cores": 1, "kind": "port", "cpu": cpu_model(),
            "sample": f"{done} {what} in {el:.2f} s on 1 thread (C oracle, -O3)"}


def hbm_roofline(alg_bytes, seconds, kernel, note):
    achieved = alg_bytes / seconds / 1e9
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "kernel": kernel, "note": note}


def mfma_roofline(ops, seconds, kernel, note):
    achieved = ops / seconds / 1e12
    return {"bound": "mfma", "achieved": achieved, "peak": FP4_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP4_MFMA_PEAK_TFLOPS, "kernel": kernel, "note": note}


def mul_roofline(ctx, a_bound, b_bound, k, n, seconds, what):
    """MFMA roofline of a multiply (all of its launches): the carry products' bit pairs as the
    context's plan issues them (hm_mul_plan_work: schoolbook products at their static bounds,
    Karatsuba products by their leaves; word pairs x 1024), 2 ops per pair, over the multiply's
    HIP-event time, vs the dense fp4 peak.  The schoolbook count of the same circuit
    (hm_mul_cost, the reference's own algorithm) rides beside it."""
    issued = ctx.mul_plan_work(a_bound, b_bound, k)
    school = H.mul_cost(a_bound, b_bound, k)["word_pairs"]
    r = mfma_roofline(2.0 * 1024.0 * issued * n, seconds,
                      "mul_mfma_kernel + scan / partial-product / Karatsuba launches (whole multiply)",
                      f"{what}: {issued:.4g} issued carry-product word pairs (32x32 bit) per value "
                      "(hm_mul_plan_work), 2 ops per bit pair, over the multiply's HIP-event time on "
                      "the engine stream (every launch of the multiply, not one kernel; the partial "
                      "products, scans and Karatsuba sums are not counted as work)")
    r["schoolbook_word_pairs"] = school
    r["schoolbook_equivalent_tflops"] = 2.0 * 1024.0 * school * n / seconds / 1e12
    return r


def s0_zero_context(device, params=PARAMS):
    """A seeded context whose secret key has S(0) = 0: (C mod S)(0) = C(0) and evaluation at 0 is a
    ring homomorphism, so every circuit output decrypts whatever its noise degree;
    the multiply lines use it so that their decrypt check covers every product."""
    for seed in range(BENCH_SEED, BENCH_SEED + 64):
        ctx = H.Context(H.Parameters(*params), device=device)
        ctx.seed_rng(seed)
        ctx.generate_secret_key()
        if not int(ctx.get_secret_key().limbs[0]) & 1:
            ctx.generate_public_key()
            return ctx, seed
    raise RuntimeError("no S(0) = 0 seed")


def config0_lines(device, leg_s):
    """BASELINE.json configs[0]: the reference's `cargo bench --bench u8` plumbing (u8 encrypt,
    decrypt and add at d = dp = tau = 64, delta = 1) -- on the GPU over a batch of 65536 u8 values
    (the reference benches one value: the batch is a throughput choice; 4096 left these
    microsecond kernels launch-bound), each op one HIP graph replay per step, with the oracle's
    1-thread rate of the same op beside it."""
    import ctypes
    from oracle import oracle_py as oracle
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import as_bytes, keys, masks
    params = (64, 64, 1, 64)
    L = H.lib()
    c0 = H.Context(H.Parameters(*params), device=device)
    c0.seed_rng(BENCH_SEED)
    c0.generate_secret_key()
    c0.generate_public_key()
    n = 65536
    a_np = np.random.default_rng(31).integers(0, 256, size=n, dtype=np.uint8)
    b_np = np.random.default_rng(32).integers(0, 256, size=n, dtype=np.uint8)
    da = torch.from_numpy(a_np).to(device).reshape(n, 1)
    bound = np.full(8, c0.fresh_bound(), dtype=np.uint32)
    ca = H.Ciphered.empty(n, bound, device)
    cb = c0.encrypt(b_np)
    dec = torch.empty((n, 1), dtype=torch.uint8, device=device)
    cac = ca._c()
    ob = H.add_out_bounds(bound, cb.bound)
    co = H.Ciphered.empty(n, ob, device, np.dtype(np.uint8))
    reps = 100

    def timed(fn, kernel):
        wall, step_s, ks, _ = timed_graph(c0, fn, reps, 5, 1, kernel)
        return n * reps / wall, step_s, ks

    enc_r, enc_s, enc_ks = timed(lambda: c0._launch(lambda: L.hm_encrypt_batch(
        c0._h, da.data_ptr(), 1, None, ctypes.byref(cac)), "encrypt"), "encrypt")
    dec_r, dec_s, dec_ks = timed(lambda: c0._launch(lambda: L.hm_decrypt_batch(
        c0._h, ctypes.byref(cac), dec.data_ptr()), "decrypt"), "decrypt")
    dec_ok = bool(np.array_equal(dec.cpu().numpy().reshape(-1), a_np))
    add_r, add_s, add_ks = timed(lambda: H.add_into(c0, ca, cb, co), "add_chain")
    got = c0.decrypt(co, np.uint8)
    add_ok = int(np.sum(got == (a_np.astype(np.uint16) + b_np).astype(np.uint8)))
    # the oracle on the same ops (its own seeded keys of the same parameters)
    sk, pk, _ = keys(*params, 33)
    ns = 64
    ms = masks(ns, 8, params[3], 34)
    la, lda = oracle.encrypt_batch(pk, as_bytes(a_np[:ns]), ms, bound)
    lb, ldb = oracle.encrypt_batch(pk, as_bytes(b_np[:ns]), masks(ns, 8, params[3], 35), bound)
    cpu_enc = oracle_leg(lambda: oracle.encrypt_batch(pk, as_bytes(a_np[:ns]), ms, bound), ns, leg_s,
                         "u8 encryptions (64 per call)")
    cpu_dec = oracle_leg(lambda: oracle.decrypt_batch(sk, la, lda, bound, 8, ns), ns, leg_s,
                         "u8 decryptions of fresh ciphertexts (64 per call)")
    cpu_add = oracle_leg(lambda: oracle.add_batch(la, lda, bound, lb, ldb, bound, 8, ns, ob), ns,
                         leg_s, "u8 homomorphic adds (64 per call)")
    cap = int(bound[0]) // 64 + 1
    enc_b, dec_b = 8 * (8 * cap) + 8 * ((params[3] + 7) // 8), 8 * (8 * cap) + 1
    add_b = 2 * 8 * (8 * cap) + 8 * co.stride
    pairs = chain_bit_pairs(bound, cb.bound)
    add_roof = mfma_roofline(2.0 * pairs * n, add_ks, "add_chain_mfma_kernel",
                             f"{pairs} carry-product bit pairs per u8 add (static bounds), 2 ops "
                             "per pair, over the chain kernel's duration (device stamps of the "
                             "timed replays)")
    add_roof["hbm_frac"] = add_b * n / add_ks / 1e9 / HBM_PEAK_GBS
    out = {
        "config0_u8_encrypt": {
            "value": enc_r, "unit": "u8 encryptions/s", "batch": n, "params": params,
            "kernel_us_per_step": 1e6 * enc_s, "masks": "drawn per step (engine CSPRNG)",
            "encrypt_kernel_us": 1e6 * enc_ks,
            "roofline": hbm_roofline(enc_b * n, enc_ks, "encrypt_table_kernel",
                                     f"{enc_b} algorithmic B per u8: ciphertext written, masks "
                                     "read; the encryption kernel's duration (device stamps of "
                                     "the timed replays; the mask draw is not in it)"),
            "cpu_baseline": cpu_enc},
        "config0_u8_decrypt": {
            "value": dec_r, "unit": "u8 decryptions/s", "batch": n, "params": params,
            "verified": dec_ok, "kernel_us_per_step": 1e6 * dec_s,
            "roofline": hbm_roofline(dec_b * n, dec_ks, "decrypt_bits_kernel",
                                     f"{dec_b} algorithmic B per u8: ciphertext read, 1 B "
                                     "written; the kernel's duration (device stamps)"),
            "cpu_baseline": cpu_dec},
        "config0_u8_add": {
            "value": add_r, "unit": "u8 homomorphic adds/s", "batch": n, "params": params,
            "verified": {"correct_sums": add_ok, "of": n}, "kernel_us_per_step": 1e6 * add_s,
            "roofline": add_roof, "cpu_baseline": cpu_add}}
    del ca, cb, co, c0
    return out

def secondary_metrics(ctx, device, steps, add_out, cpu_seconds, cpu_add=None):
    """The other BASELINE configs and the README's other published timings (README.md:73-77,
    benches/u32.rs:17-23, 47-49), each with the oracle's single-thread CPU rate beside it."""
    import ctypes
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    out = {}
    L = H.lib()
    leg_s = max(1.0, cpu_seconds / 6)
    # configs[2]: u32 encrypt + decrypt, batch 65536.  Like the reference (whose encryption
    # draws its subset masks from getrandom), each step draws fresh masks from the engine's
    # CSPRNG (device ChaCha20) inside the timed step; the same pair over pre-drawn masks is
    # reported beside it.  Encryption and decryption alone are timed the same way.
    n = 65536
    vals_np = np.random.default_rng(7).integers(0, 2**32, size=n, dtype=np.uint32)
    vals = torch.from_numpy(vals_np.view(np.int32)).to(device)
    data = vals.view(torch.uint8).reshape(n, 4)
    m = ctx.random_bytes(n * 32 * ctx.mask_bytes())
    bound = np.full(32, ctx.fresh_bound(), dtype=np.uint32)
    c = H.Ciphered.empty(n, bound, device)
    dec = torch.empty((n, 4), dtype=torch.uint8, device=device)
    cb = c._c()

    def enc(masks_ptr):
        ctx._launch(lambda: L.hm_encrypt_batch(ctx._h, data.data_ptr(), 4, masks_ptr,
                                               ctypes.byref(cb)), "encrypt")

    def decr():
        ctx._launch(lambda: L.hm_decrypt_batch(ctx._h, ctypes.byref(cb), dec.data_ptr()), "decrypt")

    reps = max(20, 5 * steps)

    def timed(fn, kernel=None):
        # launch-bound (tens of us of kernels): replayed as one captured HIP graph per step
        wall, step_s, ks, _ = timed_graph(ctx, fn, reps, 2, 1, kernel)
        return n * reps / wall, step_s, ks

    res = {}
    for key, mp in (("csprng", None), ("predrawn", m.data_ptr())):
        dec.zero_()
        r, ks, _ = timed(lambda: (enc(mp), decr()))
        res[key] = (r, bool(torch.equal(dec, data)), 1e6 * ks)
    enc_r, enc_k, enc_ks = timed(lambda: enc(m.data_ptr()), "encrypt")
    encc_r, encc_k, _ = timed(lambda: enc(None))
    enc(m.data_ptr())
    dec.zero_()
    dec_r, dec_k, dec_ks = timed(decr, "decrypt")
    dec_ok = bool(torch.equal(dec, data))
    ctx.synchronize()

    from helpers import as_bytes, masks as hmasks
    from oracle import oracle_py as oracle
    sk, pk = ctx.get_secret_key().limbs, ctx.get_public_key().limbs
    ns = 64
    xs = vals_np[:ns]
    ms = hmasks(ns, 32, PARAMS[3], 3)
    cl, cd = oracle.encrypt_batch(pk, as_bytes(xs), ms, bound)
    cpu_enc = oracle_leg(lambda: oracle.encrypt_batch(pk, as_bytes(xs), ms, bound), ns, leg_s,
                         "u32 encryptions (64 values per call)")
    cpu_dec = oracle_leg(lambda: oracle.decrypt_batch(sk, cl, cd, bound, 32, ns), ns, leg_s,
                         "u32 decryptions of fresh ciphertexts (64 per call)")
    cpu_pair = {"value": 1.0 / (1.0 / cpu_enc["value"] + 1.0 / cpu_dec["value"]), "cores": 1,
                "kind": "port", "cpu": cpu_model(),
                "sample": "from the encrypt and decrypt legs below (1 thread each)"}
    # algorithmic bytes per u32: encrypt writes 32 x 40 B, reads 32 x 16 B of
    # masks; decrypt reads the 1280 B and writes 4 B
    out["u32_encrypt_decrypt"] = {
        "value": res["csprng"][0], "unit": "u32 enc+dec/s", "batch": n,
        "verified": res["csprng"][1] and res["predrawn"][1], "steps": reps,
        "kernel_us_per_step": res["csprng"][2],
        "masks": "drawn per step from the engine CSPRNG (ChaCha20 on device), as the "
                 "reference's getrandom draw is part of its encryption",
        "predrawn_masks": {"value": res["predrawn"][0], "kernel_us_per_step": res["predrawn"][2]},
        "launch": "one HIP graph replay per step (mask draw + encrypt + decrypt)",
        "roofline": hbm_roofline(2564 * n, enc_ks + dec_ks,
                                 "encrypt_table_kernel + decrypt_bits_kernel (pre-drawn masks)",
                                 "2564 algorithmic B per u32 (SURVEY.md s8(d)): 1280 B written by "
                                 "encrypt, 1280 B read + 4 B written by decrypt; over the sum of "
                                 "the two kernels' durations (device stamps in the u32_encrypt "
                                 "and u32_decrypt_fresh legs' timed replays)"),
        "cpu_baseline": cpu_pair}
    out["u32_encrypt"] = {
        "value": encc_r, "unit": "u32 encryptions/s", "batch": n, "kernel_us_per_step": 1e6 * encc_k,
        "masks": "drawn per step (engine CSPRNG)",
        "predrawn_masks": {"value": enc_r, "kernel_us_per_step": 1e6 * enc_k,
                           "encrypt_kernel_us": 1e6 * enc_ks},
        "readme_reference": "76.0 us per u32 on a Ryzen 7 7800X3D, 1 thread (README.md:73)",
        "roofline": hbm_roofline(1792 * n, enc_ks, "encrypt_table_kernel (pre-drawn masks)",
                                 "1792 algorithmic B per u32: 1280 B of ciphertext written, 512 B "
                                 "of masks read; over the kernel's duration (device stamps of "
                                 "the timed replays)"),
        "cpu_baseline": cpu_enc}
    out["u32_decrypt_fresh"] = {
        "value": dec_r, "unit": "u32 decryptions/s", "batch": n, "verified": dec_ok,
        "kernel_us_per_step": 1e6 * dec_k,
        "readme_reference": "12.5 us per u32 on a Ryzen 7 7800X3D, 1 thread (README.md:74)",
        "roofline": hbm_roofline(1284 * n, dec_ks, "decrypt_bits_kernel",
                                 "1284 algorithmic B per u32: 1280 B read, 4 B written; over the "
                                 "kernel's duration (device stamps of the timed replays)"),
        "cpu_baseline": cpu_dec}
    del c, dec, m

    # README.md:76 "Dec. after add" (benches/u32.rs:47-49): decrypting the 4096 add outputs of
    # the headline step (46.9 KB of 369-limb polynomials per u32: the rem-heavy case)
    na = add_out.n
    dbuf = torch.empty((na, 4), dtype=torch.uint8, device=device)
    ab = add_out._c()
    wall, step_s, dks, _ = timed_graph(
        ctx, lambda: ctx._launch(lambda: L.hm_decrypt_batch(ctx._h, ctypes.byref(ab),
                                                            dbuf.data_ptr()), "decrypt"),
        reps, 2, 1, "decrypt")
    per_u32 = 8 * add_out.stride + 4
    ol, od = H.value_slice(add_out, 0, 4).to_host()
    cpu_dadd = oracle_leg(lambda: oracle.decrypt_batch(sk, ol, od, add_out.bound, 32, 4), 4, leg_s,
                          "u32 decryptions of add outputs (4 per call; long division, "
                          "polynomial.rs:316-365)")
    out["u32_decrypt_after_add"] = {
        "value": na * reps / wall, "unit": "u32 decryptions/s", "batch": na,
        "kernel_us_per_step": 1e6 * step_s,
        "readme_reference": "1.03 ms per u32 on a Ryzen 7 7800X3D, 1 thread (README.md:76)",
        "roofline": hbm_roofline(per_u32 * na, dks, "decrypt_kernel (wave per value)",
                                 f"{per_u32} algorithmic B per u32: the add output at its static "
                                 f"capacity read once, 4 B written; over the kernel's duration "
                                 "(device stamps of the timed replays)"),
        "cpu_baseline": cpu_dadd}
    del dbuf

    # PCIe-inclusive add rate: the same 4096-value add with its inputs copied host->device and
    # its outputs device->host (pinned buffers) inside every step -- what a caller handing host
    # Ciphered<u32> values across the C ABI would see; never the headline value
    n4 = 4096
    a4 = np.random.default_rng(8).integers(0, 2**32, size=n4, dtype=np.uint32)
    b4 = np.random.default_rng(9).integers(0, 2**32, size=n4, dtype=np.uint32)
    c4a, c4b = ctx.encrypt(a4), ctx.encrypt(b4)
    o4 = H.Ciphered.empty(n4, H.add_out_bounds(c4a.bound, c4b.bound), device, np.dtype(np.uint32))
    host = {k: torch.empty_like(v, device="cpu").pin_memory() for k, v in
            (("al", c4a.limbs), ("ad", c4a.degree), ("bl", c4b.limbs), ("bd", c4b.degree),
             ("ol", o4.limbs), ("od", o4.degree))}
    for k, v in (("al", c4a.limbs), ("ad", c4a.degree), ("bl", c4b.limbs), ("bd", c4b.degree)):
        host[k].copy_(v)

    def pcie_step():
        for k, v in (("al", c4a.limbs), ("ad", c4a.degree), ("bl", c4b.limbs), ("bd", c4b.degree)):
            v.copy_(host[k], non_blocking=True)
        H.add_into(ctx, c4a, c4b, o4)
        host["ol"].copy_(o4.limbs, non_blocking=True)
        host["od"].copy_(o4.degree, non_blocking=True)

    preps = max(4, steps // 2)
    wall, _ = time_loop(pcie_step, preps, 1, 1)
    moved = sum(v.numel() * v.element_size() for v in host.values())
    out["u32_add_pcie_inclusive"] = {
        "value": n4 * preps / wall, "unit": "adds/s", "batch": n4, "bytes_moved_per_step": moved,
        "note": "H2D inputs + add + D2H outputs per step",
        "roofline": {"bound": "pcie", "achieved": moved * preps / wall / 1e9, "peak": PCIE_PEAK_GBS,
                     "unit": "GB/s", "frac": moved * preps / wall / 1e9 / PCIE_PEAK_GBS,
                     "kernel": "H2D copies + add + D2H copies (wall time of the step)",
                     "note": "the bytes crossing the host link per step (inputs in, outputs and "
                             "degrees out, one direction at a time on one stream) over the step's "
                             "wall time vs PCIe Gen5 x16's 63 GB/s per direction"},
        "cpu_baseline": cpu_add if cpu_add is not None else {"value": None, "note": "--no-cpu"}}
    del c4a, c4b, o4, host

    # Multiplies under an S(0) = 0 key, so that every product's decryption is checked: the u8
    # multiply (benches/u8.rs, batch n8 = 16384: the reference benches one value, so the batch is a
    # throughput choice; 1024 values are one wave per SIMD), and the low K result bits of the u32
    # circuit at configs[3]'s own batch, MUL_BATCH = 1024 (plus a labelled batch-16384 aside at
    # K = 16).
    mctx, mseed = s0_zero_context(device)
    n8 = 16384
    a8 = np.random.default_rng(1).integers(0, 256, size=n8, dtype=np.uint8)
    b8 = np.random.default_rng(2).integers(0, 256, size=n8, dtype=np.uint8)
    ca, cbb = mctx.encrypt(a8), mctx.encrypt(b8)
    co = H.Ciphered.empty(n8, H.mul_out_bounds(ca.bound, cbb.bound), device)
    H.mul_into(mctx, ca, cbb, co)  # sizes the workspace outside the timed loop
    mctx.synchronize()
    mreps = max(1, steps // 4)
    # the timed region as one replay of an mreps-step HIP graph, like the other legs (the
    # multiply's ~dozens of launches per batch without host launch gaps; scripts/probe/mul_graph.py:
    # bit-identical to direct launches)
    wall, step_s, _, _ = timed_graph(mctx, lambda: H.mul_into(mctx, ca, cbb, co), mreps, 1, 1)
    ev_s = step_s * mreps
    got = mctx.decrypt(co, np.uint8)
    # the oracle (1 thread) on the same workload: benches/u8.rs:9, 21-29 multiply u8 values at
    # (128, 128, 1, 128); two values per call, the engine context's keys, seeded masks
    msk, mpk = mctx.get_secret_key().limbs, mctx.get_public_key().limbs
    b8b = ca.bound
    o8a, o8ad = oracle.encrypt_batch(mpk, as_bytes(a8[:2]), hmasks(2, 8, PARAMS[3], 11), b8b)
    o8b, o8bd = oracle.encrypt_batch(mpk, as_bytes(b8[:2]), hmasks(2, 8, PARAMS[3], 12), b8b)
    ol8, od8 = oracle.mul_batch(o8a, o8ad, b8b, o8b, o8bd, b8b, 8, 2, co.bound)
    cpu_m8 = oracle_leg(lambda: oracle.mul_batch(o8a, o8ad, b8b, o8b, o8bd, b8b, 8, 2, co.bound), 2,
                        leg_s, "u8 homomorphic multiplies (2 per call; common.rs:66-105)")
    out["u8_mul"] = {"value": n8 * mreps / wall, "unit": "u8 muls/s", "batch": n8,
                     "verified": bool(np.array_equal(got, (a8.astype(int) * b8).astype(np.uint8))),
                     "key_seed": mseed, "kernel_ms_per_batch": 1e3 * ev_s / mreps,
                     "reference_bench": "benches/u8.rs:21-29 (mul at d=dp=tau=128, delta=1)",
                     "roofline": mul_roofline(mctx, ca.bound, cbb.bound, 8, n8, ev_s / mreps,
                                              "u8 multiply"),
                     "cpu_baseline": cpu_m8}
    # benches/u8.rs:31-37 "decipher after mul": decrypting the u8 products (the rem-heavy
    # case of the multiply's wide outputs), one HIP graph replay per step
    d8 = torch.empty((n8, 1), dtype=torch.uint8, device=device)
    coc = co._c()
    dreps = max(20, 5 * steps)
    wall, step_s, dks, _ = timed_graph(
        mctx, lambda: mctx._launch(lambda: L.hm_decrypt_batch(mctx._h, ctypes.byref(coc),
                                                              d8.data_ptr()), "decrypt"),
        dreps, 2, 1, "decrypt")
    per_u8 = 8 * co.stride + 1
    cpu_d8 = oracle_leg(lambda: oracle.decrypt_batch(msk, ol8, od8, co.bound, 8, 2), 2, leg_s,
                        "u8 decryptions of multiply outputs (2 per call; long division, "
                        "polynomial.rs:316-365)")
    out["u8_decrypt_after_mul"] = {
        "value": n8 * dreps / wall, "unit": "u8 decryptions/s", "batch": n8,
        "verified": bool(np.array_equal(d8.cpu().numpy().reshape(-1), got)),
        "kernel_us_per_step": 1e6 * step_s,
        "reference_bench": "benches/u8.rs:31-37 (decipher after mul)",
        "roofline": hbm_roofline(per_u8 * n8, dks, "decrypt_kernel (wave per value)",
                                 f"{per_u8} algorithmic B per u8: the product at its static "
                                 f"capacity read once, 1 B written; over the kernel's duration "
                                 "(device stamps of the timed replays)"),
        "cpu_baseline": cpu_d8}
    del ca, cbb, co, d8

    # SURVEY.md s8 row A14, configs[3] (u32 mul, batch 1024): the first K result bits of the u32
    # carry-save circuit, bit-exact (tests: oracle fixture at K = 16, residue checks of the full
    # batch at K = 16 and of K = 20); the full u32 circuit is infeasible for any engine and is
    # priced, not run: the planner's own cost model (hm_mul_cost) scales the measured rate up
    n32 = 16384  # encrypted values: configs[3]'s 1024 are the first MUL_BATCH of them
    a32 = np.random.default_rng(3).integers(0, 2**32, size=n32, dtype=np.uint32)
    b32 = np.random.default_rng(4).integers(0, 2**32, size=n32, dtype=np.uint32)
    c32a, c32b = mctx.encrypt(a32), mctx.encrypt(b32)
    # the oracle's K = 12 circuit on one value (the low 12 bits of u32 ciphertexts, as the engine
    # reads them); K >= 16 takes the oracle minutes to hours per value, so their CPU rates are this
    # leg's word-pair rate applied to their word pairs (labelled extrapolated)
    from helpers import low_bits
    b32b = c32a.bound
    o32a, o32ad = oracle.encrypt_batch(mpk, as_bytes(a32[:1]), hmasks(1, 32, PARAMS[3], 13), b32b)
    o32b, o32bd = oracle.encrypt_batch(mpk, as_bytes(b32[:1]), hmasks(1, 32, PARAMS[3], 14), b32b)
    l12a, d12a, bk12 = low_bits(o32a, o32ad, b32b, 1, 12)
    l12b, d12b, _ = low_bits(o32b, o32bd, b32b, 1, 12)
    ob12 = H.mul_out_bounds(bk12, bk12)
    cpu_k12 = oracle_leg(lambda: oracle.mul_batch(l12a, d12a, bk12, l12b, d12b, bk12, 12, 1, ob12),
                         1, leg_s, "u32 multiplies, result bits 0..11 (1 value per call; the "
                                   "12-bit circuit over the low 12 input bits)")
    k12_pairs_s = cpu_k12["value"] * H.mul_cost(b32b, b32b, 12)["word_pairs"]

    def cpu_mul_low(k):
        if k == 12:
            return cpu_k12
        wp = H.mul_cost(b32b, b32b, k)["word_pairs"]
        return {"value": k12_pairs_s / wp, "cores": 1, "kind": "port", "cpu": cpu_model(),
                "extrapolated": True,
                "sample": f"EXTRAPOLATED: the K = 12 oracle leg's {k12_pairs_s:.3g} word pairs/s "
                          f"(1 thread) applied to K = {k}'s {wp:.4g} word pairs (hm_mul_cost)"}
    for name, k, nk in (("u32_mul_low12", 12, MUL_BATCH),
                        (f"u32_mul_low{MUL_LOW_BENCH}", MUL_LOW_BENCH, MUL_BATCH),
                        (f"u32_mul_low{MUL_LOW_BENCH}_batch{n32}", MUL_LOW_BENCH, n32),
                        ("u32_mul_low20", 20, MUL_BATCH),
                        ("u32_mul_low20_batch16", 20, 16),
                        # result bits 20..23: products planned one subtree at a time
                        # (hm_ctx_set_mul_scratch), 2.3 GB of arena and 57e6 leaf products per value
                        ("u32_mul_low24_batch2", 24, 2)):
        ob = H.mul_out_bounds(c32a.bound[:k], c32b.bound[:k])
        va, vb = H.value_slice(c32a, 0, nk), H.value_slice(c32b, 0, nk)
        cp = H.Ciphered.empty(nk, ob, device)
        H.mul_low_into(mctx, va, vb, k, cp)  # plan + workspace outside the timed loop
        mctx.synchronize()
        reps = 1 if k >= 20 or nk > MUL_BATCH else 2 if k >= 16 else max(2, steps // 4)
        step = lambda: H.mul_low_into(mctx, va, vb, k, cp)  # noqa: E731
        if k == 12:  # milliseconds per batch: one K-step graph replay, like the u8 leg
            wall, step_s, _, _ = timed_graph(mctx, step, reps, 1, 1)
            ev_s = step_s * reps
        else:        # tenths of a second and up per batch: launch gaps are noise, direct launches
            wall, ev_s = time_loop(step, reps, 0, 1, mctx.stream)
        mctx.synchronize()
        # decrypt through a 24-bit view: output bits >= k are null polynomials
        raw = mctx.decrypt_bytes(H.pad_bits(cp, 24)).cpu().numpy().astype(np.uint64)
        lo = raw[:, 0] | (raw[:, 1] << np.uint64(8)) | (raw[:, 2] << np.uint64(16))
        want = (a32[:nk].astype(np.uint64) * b32[:nk]) & np.uint64((1 << k) - 1)
        cost = H.mul_cost(c32a.bound, c32b.bound, k)
        rate = nk * reps / wall
        out[name] = {
            "value": rate, "unit": f"u32 muls/s (result bits 0..{k - 1})", "batch": nk,
            "config": "configs[3] (batch 1024)" if nk == MUL_BATCH else
                      f"aside: configs[3]'s circuit at batch {nk} (not configs[3]'s batch; a "
                      "labelled aside)",
            "ms_per_batch": 1e3 * wall / reps, "kernel_ms_per_batch": 1e3 * ev_s / reps,
            "decrypt_correct": int(np.sum(lo == want)), "of": nk, "key_seed": mseed,
            "secret_key_s0": int(mctx.get_secret_key().limbs[0] & 1),
            "word_pairs_per_mul": cost["word_pairs"],
            "word_pairs_per_s": cost["word_pairs"] * rate,
            "bit_exact": "tests/test_golden.py (oracle fixtures: K=16, 8 values; K=20, 4 "
                         "values), test_gpu_properties.py (residue check of all 1024 K=16 "
                         "products; K=20 at batch 1024 under an S(0)=0 key: all decrypt, 64 "
                         "by residue; K=20 Karatsuba = schoolbook; K=22 split plans: decrypt + "
                         "residues; split = whole plans at K=16), test_gpu_parity.py",
            "roofline": mul_roofline(mctx, c32a.bound, c32b.bound, k, nk, ev_s / reps,
                                     f"u32 multiply, low {k} bits"),
            "cpu_baseline": cpu_mul_low(k)}
        del cp
    full = H.mul_cost(c32a.bound, c32b.bound)
    kx = out["u32_mul_low24_batch2"]
    est = kx["word_pairs_per_s"] / full["word_pairs"]
    out["u32_mul_full_extrapolated"] = {
        "value": est * 1.0, "unit": "u32 muls/s (EXTRAPOLATED, not measured)",
        "basis": "the low-24 rate (the deepest prefix run) in schoolbook word pairs/s (hm_mul_cost) "
                 "applied to the full circuit's word pairs; the full circuit also needs its "
                 "outputs and carries resident (8.4 GiB of output per value) and per-leaf task "
                 "tables that grow 7.4x per 2 result bits (2.3 GB at K = 24)",
        "word_pairs_per_mul": full["word_pairs"], "out_bytes_per_mul": full["out_bytes"],
        "max_degree": full["max_degree"], "seconds_per_mul_one_gpu": 1.0 / est,
        "roofline": dict(kx["roofline"], note="EXTRAPOLATED: the low-24 multiply's measured "
                         "roofline (the rate above is that word-pair rate)"),
        "cpu_baseline": dict(cpu_mul_low(24), value=k12_pairs_s / full["word_pairs"],
                             sample=f"EXTRAPOLATED: the K = 12 oracle leg's {k12_pairs_s:.3g} word "
                                    f"pairs/s (1 thread) applied to the full circuit's "
                                    f"{full['word_pairs']:.4g} word pairs")}
    del c32a, c32b, mctx
    torch.cuda.empty_cache()

    # configs[4]: the mixed workload at its global batch, 2^20 values on this one GPU (the N = 1
    # point of the strong-scaling configuration), bench.py --workload mixed's own step
    w = MixedWorkload(1, 0, device, 1 << 20)
    msteps = 2
    wall, ev_s = time_loop(w.step, msteps, 1, 1, w.ctx.stream)
    w.ctx.synchronize()
    ok_s, ok_p, wall = w.verify(device, wall)
    add_pairs = chain_bit_pairs(w.ca.bound, w.cb.bound)
    mul_wp = w.ctx.mul_plan_work(w.ca.bound, w.cb.bound, MUL_LOW_K)
    out["mixed_config4"] = {
        "value": w.glob * msteps / wall,
        "unit": f"u32 values/s (one add + one mul, low {MUL_LOW_K} result bits, per value)",
        "global_batch": w.glob, "n_gpus": 1, "steps": msteps, "ms_per_step": 1e3 * wall / msteps,
        "kernel_ms_per_step": 1e3 * ev_s / msteps,
        "config": {"d": MIXED_PARAMS[0], "dp": MIXED_PARAMS[1], "delta": MIXED_PARAMS[2],
                   "tau": MIXED_PARAMS[3], "launch_chunk": MIXED_CHUNK},
        "verified": {"correct_sums": ok_s, "correct_products": ok_p, "of": w.glob},
        "roofline": mfma_roofline(
            2.0 * (add_pairs + 1024.0 * mul_wp) * w.glob, ev_s / msteps,
            "add_chain_mfma_kernel<25> + the multiply's launches (whole step)",
            f"per value: the add chain's {add_pairs:.4g} carry-product bit pairs (static bounds, "
            f"DESIGN.md s4.1) + the low-{MUL_LOW_K} multiply's {mul_wp:.4g} issued carry-product "
            "word pairs x 1024 (hm_mul_plan_work), 2 ops per bit pair, over the step's HIP-event "
            "time"),
        "cpu_baseline": mixed_cpu_leg(leg_s)}
    del w
    torch.cuda.empty_cache()
    out.update(config0_lines(device, leg_s))
    return out


def mixed_cpu_leg(seconds):
    """configs[4] on the oracle (1 thread): one u32 add and one u32 multiply (low MUL_LOW_K bits)
    of one value per call at d = dp = tau = 256, timed on a sample and reported per value: the
    2^20-value batch is extrapolated linearly (BASELINE.md:50)."""
    from oracle import oracle_py as oracle
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import as_bytes, fresh_bound, keys, low_bits, masks
    d, dp, delta, tau = MIXED_PARAMS
    _, pk, _ = keys(d, dp, delta, tau, 78)
    bound = fresh_bound(d, dp, 32)
    a = np.array([0x9E3779B9], dtype=np.uint32)
    b = np.array([0x7F4A7C15], dtype=np.uint32)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), masks(1, 32, tau, 21), bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), masks(1, 32, tau, 22), bound)
    ob = H.add_out_bounds(bound, bound)
    lka, dka, bk = low_bits(la, da, bound, 1, MUL_LOW_K)
    lkb, dkb, _ = low_bits(lb, db, bound, 1, MUL_LOW_K)
    obk = H.mul_out_bounds(bk, bk)

    def one():
        oracle.add_batch(la, da, bound, lb, db, bound, 32, 1, ob)
        oracle.mul_batch(lka, dka, bk, lkb, dkb, bk, MUL_LOW_K, 1, obk)

    leg = oracle_leg(one, 1, seconds, f"values (one u32 add + one u32 multiply, low {MUL_LOW_K} "
                                      "bits, at d = dp = tau = 256; 1 value per call)")
    leg["extrapolated"] = "per-value rate of the sample; the 2^20 batch scales linearly (BASELINE.md:50)"
    return leg


MIXED_PARAMS = (256, 256, 1, 256)  # BASELINE.json configs[4]: d = dp = tau = 256, delta = 1
MIXED_CHUNK = 131072                # values per launch (the 8-GPU shard of 2^20)
MUL_LOW_K = 8                       # result bits of the multiply half
MIXED_KARATSUBA = (224, 224)        # hm_ctx_set_mul_options for the multiply half (scripts/sweep_mixed_ka.sh)


def run_add(args, world, rank, device):
    """configs[1]: u32 homomorphic add, batch 4096 per GPU (weak scaling)."""
    ctx = make_context(world, rank, device)
    ctx.set_add_pipeline(bool(args.add_pipeline))
    ctx.set_add_options(args.add_chain)
    n = args.batch or 4096
    a, b = shard_inputs(rank, n)
    ca, cb = ctx.encrypt(a), ctx.encrypt(b)  # masks from the (seeded) engine CSPRNG
    ob = H.add_out_bounds(ca.bound, cb.bound)
    out = H.Ciphered.empty(n, ob, device, np.dtype(np.uint32))
    ctx.synchronize()

    if args.graph:  # the K timed steps (prep + chain each) as one captured HIP graph
        wall, step_s, chain_s, chain_n = timed_graph(
            ctx, lambda: H.add_into(ctx, ca, cb, out), args.steps, args.warmup, world, "add_chain")
        ev_s = step_s * args.steps
        chain_src = (f"device wall-clock stamps of each of the timed region's {chain_n} chain "
                     "launches (one replay of the K-step graph; hm_ctx_set_kernel_timing)")
    else:
        for _ in range(args.warmup):
            H.add_into(ctx, ca, cb, out)
        ctx.set_kernel_timing(True)  # stamps of every chain launch of the timed region
        wall, ev_s = time_loop(lambda: H.add_into(ctx, ca, cb, out), args.steps, 0, world,
                               ctx.stream)
        chain_ms, chain_n = ctx.kernel_timing()
        ctx.set_kernel_timing(False)
        chain_s = chain_ms / 1e3 / max(1, chain_n)
        chain_src = (f"device wall-clock stamps of each of the timed region's {chain_n} chain "
                     "launches (direct launches; hm_ctx_set_kernel_timing)")
    ctx.synchronize()  # raises on any device-side error flag
    sustained = sustained_chain(ctx, lambda: H.add_into(ctx, ca, cb, out), args.steps, n,
                                chain_bit_pairs(ca.bound, cb.bound)) if args.graph else None
    # verification (untimed): decrypt on device, gather the plaintexts over RCCL, check on rank 0
    got, wall = gather_results(world, device, ctx.decrypt_bytes(out), wall)
    want = np.concatenate([sum(shard_inputs(r, n)).astype(np.uint32) for r in range(world)])
    got = got.view("<u4").reshape(-1)
    correct = int(np.sum(got == want))
    total = n * world * args.steps

    in_bytes = 8 * (ca.stride + cb.stride)
    out_bytes = 8 * out.stride
    per_add = in_bytes + out_bytes
    kernel_s = ev_s / args.steps
    pairs = chain_bit_pairs(ca.bound, cb.bound)
    achieved = 2.0 * pairs * n / chain_s / 1e12  # TFLOP/s: one bit-pair AND+XOR = one MAC = 2 ops
    traffic, issue = None, {}
    try:
        with open(args.traffic) as f:
            tj = json.load(f)
        traffic = tj.get("hbm_bytes_per_launch_per_4096")
        if traffic is not None:
            traffic = traffic * n / 4096
        ck = tj.get("kernels", {}).get("hm::add_chain_mfma_kernel", {})
        issue = {key: ck[key] for key in ("mfma_busy_frac", "valu_active_frac") if key in ck}
    except (OSError, ValueError):
        traffic = None

    result = {
        "metric": "homomorphic u32 ops/sec (add, mul) at d=dp=tau=128; 1/2/4/8 MI355X",
        "value": total / wall,
        "unit": "u32 homomorphic adds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * wall / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: seeded u32 plaintexts, seeded keys, subset masks from the seeded engine CSPRNG",
        "config": {"workload": "u32 homomorphic add (configs[1])", "global_batch": n * world,
                   "add_pipeline": bool(args.add_pipeline),
                   "add_chain": args.add_chain,
                   "batch_per_gpu": n, "d": PARAMS[0], "dp": PARAMS[1], "delta": PARAMS[2],
                   "tau": PARAMS[3], "parallelism": f"batch-sharded x{world}"},
        "verified": {"correct_sums": correct, "of": n * world},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP4_MFMA_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / FP4_MFMA_PEAK_TFLOPS, "traffic": traffic,
                     "kernel": "add_chain_mfma_kernel (carry products as {0,1} Toeplitz GEMMs on "
                               "fp4 MFMA)",
                     "kernel_ms": 1e3 * chain_s, "kernel_ms_source": chain_src,
                     "alg_bit_pairs_per_add": pairs, "step_kernels_ms": 1e3 * kernel_s,
                     # PMC issue shares of the chain kernel (profiles/add_traffic.json, same passes
                     # as traffic): matrix-core busy cycles and VALU-active cycles over SIMD-cycles
                     **issue,
                     "hbm_gbs_step": n * per_add / kernel_s / 1e9, "alg_bytes_per_add": per_add,
                     # the north star's HBM view of the same kernel: algorithmic bytes of the add
                     # (SURVEY.md s8(d), 49,472 B at d + d' = 256) over the chain's duration
                     "hbm_achieved_gbs": n * per_add / chain_s / 1e9,
                     "hbm_frac": n * per_add / chain_s / 1e9 / HBM_PEAK_GBS,
                     "note": "frac: algorithmic work = schoolbook bit pairs of the chain's carry "
                             "products P_i * carry_i over the static degree bounds (DESIGN.md "
                             "s4.1), 2 ops per pair, vs the dense fp4 MFMA peak; hbm_frac: "
                             "algorithmic bytes per add over the same kernel time vs 8 TB/s; "
                             "traffic (PMC HBM bytes of one add step, prep + chain), "
                             "mfma_busy_frac and valu_active_frac are read from "
                             "profiles/add_traffic.json (rocprofv3 --pmc passes of this bench "
                             "command), not measured in this run"},
    }
    if sustained:
        result["roofline"]["sustained"] = sustained
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline_add(args.cpu_seconds)
        result["verified"].update(confirm_noise(ctx, a, b, ca, cb, out, got[:n]))
    if rank == 0 and world == 1 and not args.no_secondary:
        try:
            # (the secondary lines' own repetition counts, independent of the headline's)
            result["secondary"] = secondary_metrics(ctx, device, 10, out, args.cpu_seconds,
                                                    result.get("cpu_baseline"))
        except Exception as e:  # reported, never fatal to the headline line
            result["secondary"] = {"error": repr(e)}
    return result


class MixedWorkload:
    """configs[4]'s per-rank state: keys (rank 0's, broadcast), this rank's shard of the global
    batch encrypted, the output batches, and the launch chunks.  `step()` is one pass of the
    workload: per chunk of MIXED_CHUNK values one u32 add and one u32 multiply reduced to its low
    MUL_LOW_K result bits.  Shared by run_mixed, the default bench's `secondary` line and the
    full-batch test (tests/test_gpu_properties.py)."""

    def __init__(self, world, rank, device, glob):
        if glob % world:
            raise SystemExit("--batch must divide by the number of ranks")
        self.world, self.rank, self.glob = world, rank, glob
        self.ctx = ctx = make_context(world, rank, device, MIXED_PARAMS)
        # Karatsuba leaves of at most 192 words for products from 192 words up: the fastest
        # strategy for this workload's multiply (scripts/mul_rate.py sweep);
        # every strategy gives identical bits
        ctx.set_mul_options(*MIXED_KARATSUBA)
        self.n = n = glob // world
        self.a, self.b = shard_inputs(rank, n)
        self.ca, self.cb = ctx.encrypt(self.a), ctx.encrypt(self.b)  # seeded engine CSPRNG masks
        self.sums = H.Ciphered.empty(n, H.add_out_bounds(self.ca.bound, self.cb.bound),
                                     ctx.device, np.dtype(np.uint32))
        kb = H.mul_out_bounds(self.ca.bound[:MUL_LOW_K], self.cb.bound[:MUL_LOW_K])
        self.prods = H.Ciphered.empty(n, kb, ctx.device, np.dtype(np.uint8))
        self.chunks = [(lo, min(n, lo + MIXED_CHUNK)) for lo in range(0, n, MIXED_CHUNK)]
        self.views = [tuple(H.value_slice(c, lo, hi) for c in (self.ca, self.cb, self.sums,
                                                                  self.prods))
                      for lo, hi in self.chunks]
        ctx.synchronize()

    def step(self):
        for va, vb, vs, vp in self.views:
            H.add_into(self.ctx, va, vb, vs)
            H.mul_low_into(self.ctx, va, vb, MUL_LOW_K, vp)

    def verify(self, device, wall):
        """Decrypt on device, gather every rank's plaintexts (RCCL all_gather), count the
        correct sums and products on every rank; returns (ok_sums, ok_products, max wall)."""
        ctx, n, world = self.ctx, self.n, self.world
        res = torch.cat([ctx.decrypt_bytes(self.sums), ctx.decrypt_bytes(self.prods)], dim=1)
        got, wall = gather_results(world, device, res, wall)
        want_s, want_p = [], []
        for r in range(world):
            ra, rb = shard_inputs(r, n)
            want_s.append((ra + rb).astype(np.uint32))
            want_p.append((ra.astype(np.uint64) * rb % (1 << MUL_LOW_K)).astype(np.uint8))
        ok_s = int(np.sum(np.ascontiguousarray(got[:, :4]).view("<u4").reshape(-1) ==
                          np.concatenate(want_s)))
        ok_p = int(np.sum(got[:, 4] == np.concatenate(want_p)))
        return ok_s, ok_p, wall


def run_mixed(args, world, rank, device):
    """configs[4]: u32 mixed add + mul at d = dp = tau = 256, global batch 2^20 sharded over the
    ranks (strong scaling), RCCL gather of the decrypted results.  Per value: one u32 add and one
    u32 multiply reduced to its low MUL_LOW_K result bits (the full u32 multiply circuit is
    infeasible; its low bits are bit-exact, row A14).  Each rank processes its
    shard in launches of MIXED_CHUNK values."""
    glob = args.batch or (1 << 20)
    w = MixedWorkload(world, rank, device, glob)
    wall, ev_s = time_loop(w.step, args.steps, args.warmup, world, w.ctx.stream)
    w.ctx.synchronize()
    ok_s, ok_p, wall = w.verify(device, wall)
    total = glob * args.steps
    return {
        "metric": "homomorphic u32 ops/sec (add, mul) at d=dp=tau=256; 1/2/4/8 MI355X",
        "value": total / wall,
        "unit": f"u32 values/s (one add + one mul, low {MUL_LOW_K} result bits, per value)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * wall / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: seeded u32 plaintexts, seeded keys, subset masks from the seeded engine CSPRNG",
        "config": {"workload": "u32 mixed add+mul (configs[4])", "global_batch": glob,
                   "batch_per_gpu": w.n, "launch_chunk": MIXED_CHUNK, "d": MIXED_PARAMS[0],
                   "dp": MIXED_PARAMS[1], "delta": MIXED_PARAMS[2], "tau": MIXED_PARAMS[3],
                   "mul_result_bits": MUL_LOW_K, "parallelism": f"batch-sharded x{world}",
                   "collective": "RCCL all_gather of decrypted results (5 B per value)"},
        "verified": {"correct_sums": ok_s, "correct_products": ok_p, "of": glob},
        "kernel_ms_per_step": 1e3 * ev_s / args.steps,
    }


def run_distcheck(args, world, rank, device):
    """The multi-rank plumbing alone, on the CPU (gloo): rank 0's keys reach every rank, each
    rank owns a distinct shard, results are gathered in rank order and the time is the max over
    ranks.  No engine call: the CPU tests drive `bench.py --gpus 2 --workload distcheck`."""
    n = args.batch or 64
    sk = pk = None
    if rank == 0:
        rng = np.random.default_rng(0xB0B)
        sk = rng.integers(0, 2**63, size=3, dtype=np.uint64)
        pk = rng.integers(0, 2**63, size=(PARAMS[3], 5), dtype=np.uint64)
    t0 = time.perf_counter()
    sk, pk = broadcast_keys(world, rank, device, sk, pk)
    a, b = shard_inputs(rank, n)
    res = torch.from_numpy((a + b).astype(np.uint32).view(np.uint8).reshape(n, 4).copy())
    got, wall = gather_results(world, device, res, time.perf_counter() - t0 + rank)
    want = np.concatenate([sum(shard_inputs(r, n)).astype(np.uint32) for r in range(world)])
    digest = int(np.bitwise_xor.reduce(pk.reshape(-1))) ^ int(np.bitwise_xor.reduce(sk))
    return {"metric": "distcheck", "value": float(n * world), "unit": "values gathered",
            "n_gpus": world, "world_size_seen": dist.get_world_size() if world > 1 else 1,
            "gathered_ok": bool(np.array_equal(got.view("<u4").reshape(-1), want)),
            "max_wall_s": wall, "key_digest": digest}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # Defaults per workload (add: 100 / 100, mixed: 2 / 5).  The add's first ~30-50 steps after
    # idle run 10-15 % slower while the clock settles under the sustained MFMA load (kernel trace:
    # 505 -> 590 -> 476 us per chain launch); the warm-up runs past that and the
    # timed steps measure the sustained rate (100 steps of the add are 0.05 s).
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--workload", choices=["add", "mixed", "distcheck"], default="add",
                    help="add: configs[1] (headline); mixed: configs[4]; distcheck: CPU plumbing")
    ap.add_argument("--batch", type=int, default=0,
                    help="add: u32 pairs per GPU (default 4096); mixed: global batch (2^20)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--add-chain", choices=["auto", "mfma", "valu"], default="auto",
                    help="hm_ctx_set_add_options (auto = the MFMA chain where it applies)")
    ap.add_argument("--add-pipeline", type=int, default=0,
                    help="1: big adds run as two pipelined halves; 0: one pass (engine default)")
    ap.add_argument("--graph", type=int, default=1,
                    help="1: the K timed add steps as one captured HIP graph (default); 0: direct "
                         "launches")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "add_traffic.json"),
                    help="PMC-derived HBM bytes per add launch (scripts/traffic_json.py)")
    args = ap.parse_args()
    dw, ds = {"add": (100, 100), "mixed": (2, 5)}.get(args.workload, (10, 20))
    args.warmup = dw if args.warmup is None else args.warmup
    args.steps = ds if args.steps is None else args.steps
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))

    world, rank, local, device = setup_dist(args)
    run = {"add": run_add, "mixed": run_mixed, "distcheck": run_distcheck}[args.workload]
    result = run(args, world, rank, device)
    if rank == 0:
        result.setdefault("world_size_seen", dist.get_world_size() if world > 1 else 1)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
