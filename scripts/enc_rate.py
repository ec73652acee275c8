"""Encrypt/decrypt probe for profiling (configs[2] shape): u32 encrypt of a 65,536-value batch at
d = dp = tau = 128 with pre-drawn masks (hm_encrypt_batch), then with masks drawn per call (the
engine's ChaCha20), then decrypt_bits of the result; REPS launches each, direct (no graph).
env: N (batch), REPS."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "homomorph-rust_amd")]
import numpy as np
import torch
import homomorph as H

n = int(os.environ.get("N", "65536"))
reps = int(os.environ.get("REPS", "50"))
ctx = H.Context(H.Parameters(128, 128, 1, 128), device="cuda:0")
ctx.seed_rng(5)
ctx.generate_secret_key(); ctx.generate_public_key()
vals = np.random.default_rng(3).integers(0, 2**32, size=n, dtype=np.uint32)
m = ctx.random_bytes(n * 32 * ctx.mask_bytes())
for name, kw in (("predrawn", {"masks": m}), ("csprng", {})):
    c = ctx.encrypt(vals, **kw)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        c = ctx.encrypt(vals, **kw)
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ok = bool(np.array_equal(ctx.decrypt(c), vals))
    print(f"encrypt {name} n={n}: {dt * 1e6:.1f} us per call (host loop), {n / dt:.4g}/s, "
          f"decrypts {ok}", flush=True)
t0 = time.perf_counter()
for _ in range(reps):
    d = ctx.decrypt_bytes(c)
ctx.synchronize()
print(f"decrypt n={n}: {(time.perf_counter() - t0) / reps * 1e6:.1f} us per call", flush=True)
