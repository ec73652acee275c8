"""Timing probe for BASELINE configs[4] (d = dp = tau = 256): u32 add and u32 mul low-8 per batch."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "homomorph-rust_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import homomorph as H  # noqa: E402


def t(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


dev = torch.device("cuda", 0)
ctx = H.Context(H.Parameters(256, 256, 1, 256), device=dev)
ctx.seed_rng(5)
ctx.generate_secret_key()
ctx.generate_public_key()
for n in [int(x) for x in os.environ.get("NS", "4096,32768").split(",")]:
    rng = np.random.default_rng(n)
    a = rng.integers(0, 2**32, size=n, dtype=np.uint32)
    b = rng.integers(0, 2**32, size=n, dtype=np.uint32)
    ca, cb = ctx.encrypt(a), ctx.encrypt(b)
    out = H.Ciphered.empty(n, H.add_out_bounds(ca.bound, cb.bound), dev, np.dtype(np.uint32))
    s = t(lambda: H.add_into(ctx, ca, cb, out), 3)
    ctx.synchronize()
    ok = np.mean(ctx.decrypt(out) == (a + b).astype(np.uint32))
    print(f"add  n={n}: {s*1e3:.2f} ms  {n/s:.3g} adds/s  correct={ok:.4f}", flush=True)
    k = int(os.environ.get("K", "8"))
    nm = min(n, 4096)
    cam = H.Ciphered(ca.limbs[: nm * ca.stride], ca.degree[:nm], ca.bound, 32, nm)
    cbm = H.Ciphered(cb.limbs[: nm * cb.stride], cb.degree[:nm], cb.bound, 32, nm)
    holder = {}
    s = t(lambda: holder.__setitem__("o", ctx.mul_low(cam, cbm, k)), 2)
    ctx.synchronize()
    got = ctx.decrypt(holder["o"], np.uint8)
    ok = np.mean(got == ((a[:nm].astype(np.uint64) * b[:nm]) % 256).astype(np.uint8))
    print(f"mul_low{k} n={nm}: {s*1e3:.2f} ms  {nm/s:.3g} muls/s  correct={ok:.4f}", flush=True)
    del ca, cb, out, holder
    torch.cuda.empty_cache()
