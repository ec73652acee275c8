"""Multiply throughput probe: the low-K u32 prefix at d = dp = tau = 128, batch n, under several
multiplier strategies (hm_ctx_set_mul_options: "min:leaf", min 0 = schoolbook only).
env: N (batch), KS (comma list of K), OPTS (comma list of min:leaf[:scratch words]), PARAMS
(d,dp,delta,tau)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "homomorph-rust_amd")]
import numpy as np
import torch
import homomorph as H

n = int(os.environ.get("N", "1024"))
ks = [int(k) for k in os.environ.get("KS", "12,16").split(",")]
opts = [tuple(int(x) for x in o.split(":")) for o in os.environ.get("OPTS", "0:256,1024:256").split(",")]
opts = [o if len(o) == 3 else o + (200_000_000,) for o in opts]
params = tuple(int(x) for x in os.environ.get("PARAMS", "128,128,1,128").split(","))
ctx = H.Context(H.Parameters(*params), device="cuda:0")
ctx.seed_rng(5)
ctx.generate_secret_key(); ctx.generate_public_key()
a = np.random.default_rng(3).integers(0, 2**32, size=n, dtype=np.uint32)
b = np.random.default_rng(4).integers(0, 2**32, size=n, dtype=np.uint32)
c32a, c32b = ctx.encrypt(a), ctx.encrypt(b)
ref = {}
for k in ks:
    for mn, leaf, scr in opts:
        ctx.set_mul_options(mn, leaf)
        ctx.set_mul_scratch(scr)
        o = ctx.mul_low(c32a, c32b, k); ctx.synchronize()
        reps = 3 if k <= 12 else 1
        t0 = time.perf_counter()
        for _ in range(reps):
            o = ctx.mul_low(c32a, c32b, k)
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / reps
        l, d = o.to_host()
        same = ""
        if k in ref:
            same = " same-as-first=" + str(bool(np.array_equal(l, ref[k][0]) and np.array_equal(d, ref[k][1])))
        else:
            ref[k] = (l, d)
        print(f"u32 mul low{k} n={n} params={params} opts={mn}:{leaf}:{scr}: {dt*1e3:.1f} ms  {n/dt:.4g}/s{same}", flush=True)
        del o
