"""Multiplier timing probe: u8 mul at d = dp = tau = 128 and u32 mul low-8 at d = dp = tau = 256
(BASELINE configs[3] / configs[4] forms), REPS launches each, for rocprofv3 passes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "homomorph-rust_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import homomorph as H  # noqa: E402

dev = torch.device("cuda", 0)
reps = int(os.environ.get("REPS", "3"))
for params, dtype, k, n in [((128, 128, 1, 128), np.uint8, 8, int(os.environ.get("N8", "1024"))),
                            ((256, 256, 1, 256), np.uint32, 8, int(os.environ.get("N32", "4096")))]:
    ctx = H.Context(H.Parameters(*params), device=dev)
    ctx.seed_rng(3)
    ctx.generate_secret_key()
    ctx.generate_public_key()
    rng = np.random.default_rng(1)
    a = rng.integers(0, np.iinfo(dtype).max, size=n, dtype=dtype, endpoint=True)
    b = rng.integers(0, np.iinfo(dtype).max, size=n, dtype=dtype, endpoint=True)
    ca, cb = ctx.encrypt(a), ctx.encrypt(b)
    kb = H.mul_out_bounds(ca.bound[:k], cb.bound[:k])
    out = H.Ciphered.empty(n, kb, dev, np.dtype(np.uint8))
    H.mul_low_into(ctx, ca, cb, k, out)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        H.mul_low_into(ctx, ca, cb, k, out)
    ctx.synchronize()
    s = (time.perf_counter() - t0) / reps
    ok = np.mean(ctx.decrypt(out, np.uint8) == (a.astype(np.uint64) * b % 256).astype(np.uint8))
    print(f"{params} {np.dtype(dtype).name} low{k} n={n}: {s*1e3:.2f} ms  {n/s:.3g}/s  ok={ok:.4f}",
          flush=True)
