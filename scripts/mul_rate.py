"""Multiply throughput probe: u8 mul and the low-K u32 prefix at d = dp = tau = 128, batch n."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "homomorph-rust_amd")]
import numpy as np
import torch
import homomorph as H

n = int(os.environ.get("N", "1024"))
ks = [int(k) for k in os.environ.get("KS", "8,12,14").split(",")]
ctx = H.Context(H.Parameters(128, 128, 1, 128), device="cuda:0")
ctx.seed_rng(5)
ctx.generate_secret_key(); ctx.generate_public_key()
a8 = np.random.default_rng(1).integers(0, 256, size=n, dtype=np.uint8)
b8 = np.random.default_rng(2).integers(0, 256, size=n, dtype=np.uint8)
ca, cb = ctx.encrypt(a8), ctx.encrypt(b8)
co = H.Ciphered.empty(n, H.mul_out_bounds(ca.bound, cb.bound), ctx.device)
H.mul_into(ctx, ca, cb, co); ctx.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    H.mul_into(ctx, ca, cb, co)
ctx.synchronize()
dt = (time.perf_counter() - t0) / 5
ok = np.array_equal(ctx.decrypt(co, np.uint8), (a8.astype(int) * b8).astype(np.uint8))
print(f"u8 mul n={n}: {dt*1e3:.2f} ms  {n/dt:.3g}/s  verified={ok}", flush=True)
a = np.random.default_rng(3).integers(0, 2**32, size=n, dtype=np.uint32)
b = np.random.default_rng(4).integers(0, 2**32, size=n, dtype=np.uint32)
c32a, c32b = ctx.encrypt(a), ctx.encrypt(b)
for k in ks:
    o = ctx.mul_low(c32a, c32b, k); ctx.synchronize()
    reps = 3 if k <= 12 else 1
    t0 = time.perf_counter()
    for _ in range(reps):
        o = ctx.mul_low(c32a, c32b, k)
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / reps
    got = ctx.decrypt_bytes(o).cpu().numpy() if k % 8 == 0 else None
    msg = ""
    if got is not None:
        want = (a.astype(np.uint64) * b) % (1 << k)
        gv = np.zeros(n, dtype=np.uint64)
        for byte in range(k // 8):
            gv |= got[:, byte].astype(np.uint64) << (8 * byte)
        msg = f" decrypt-correct {int(np.sum(gv == want))}/{n}"
    print(f"u32 mul low{k} n={n}: {dt*1e3:.1f} ms  {n/dt:.4g}/s{msg}", flush=True)
