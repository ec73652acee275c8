"""Time the u32-multiply low-k kernel at d=dp=tau=128 for a few k, batch."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "homomorph-rust_amd")]
import numpy as np, torch
import homomorph as H
ctx = H.Context(H.Parameters(128, 128, 1, 128), device="cuda:0")
ctx.seed_rng(3); ctx.generate_secret_key(); ctx.generate_public_key()
for k, n in [(int(a.split(":")[0]), int(a.split(":")[1])) for a in sys.argv[1:]]:
    a = np.random.default_rng(1).integers(0, 2**32, n, dtype=np.uint32)
    b = np.random.default_rng(2).integers(0, 2**32, n, dtype=np.uint32)
    ca, cb = ctx.encrypt(a), ctx.encrypt(b)
    out = ctx.mul_low(ca, cb, k); ctx.synchronize()
    t0 = time.perf_counter(); out = ctx.mul_low(ca, cb, k); ctx.synchronize(); el = time.perf_counter() - t0
    ok = ""
    if k % 8 == 0:
        got = ctx.decrypt_bytes(out).cpu().numpy().astype(np.uint64) @ (256 ** np.arange(k // 8, dtype=np.uint64))
        ok = int(np.sum(got == ((a.astype(np.uint64) * b) & ((1 << k) - 1))))
    print(f"k={k} n={n}: {el*1e3:.1f} ms -> {n/el:.1f} low-k u32 muls/s; stride {out.stride} limbs; correct {ok}", flush=True)
