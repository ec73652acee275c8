"""A/B probe: the headline u32 add (d = dp = tau = 128, batch 4096) and configs[0]'s u8 add
(d = dp = tau = 64, batch 65536), each as one replay of a K-step graph after warm-up replays;
prints the step time and the carry chain's time per launch (device stamps), so step - chain is
the prep.  Library: HOMOMORPH_GPU_LIB (an A/B variant) or the in-tree build."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import homomorph as H  # noqa: E402


def leg(params, n, dtype, reps, warm, chain="auto"):
    ctx = H.Context(H.Parameters(*params), device="cuda:0")
    ctx.set_add_options(chain)
    ctx.seed_rng(bench.BENCH_SEED)
    ctx.generate_secret_key()
    ctx.generate_public_key()
    rng = np.random.default_rng(7)
    a = rng.integers(0, np.iinfo(dtype).max, size=n, dtype=dtype)
    b = rng.integers(0, np.iinfo(dtype).max, size=n, dtype=dtype)
    ca, cb = ctx.encrypt(a), ctx.encrypt(b)
    out = H.Ciphered.empty(n, H.add_out_bounds(ca.bound, cb.bound), "cuda:0", np.dtype(dtype))
    wall, step_s, ks, _ = bench.timed_graph(ctx, lambda: H.add_into(ctx, ca, cb, out), reps, warm, 1,
                                            "add_chain")
    got = ctx.decrypt(out, dtype)
    ok = int(np.sum(got == (a.astype(np.uint64) + b).astype(dtype)))
    return 1e6 * step_s, 1e6 * ks, ok


tag = os.path.basename(os.environ.get("HOMOMORPH_GPU_LIB", "main"))
s, k, ok = leg((128, 128, 1, 128), 4096, np.uint32, 20, 5)
s0, k0, ok0 = leg((64, 64, 1, 64), 65536, np.uint8, 100, 5)
print(f"{tag} u32: step {s:.1f} us chain {k:.1f} prep~{s - k:.1f} ok {ok} | u8: step {s0:.1f} "
      f"chain {k0:.1f} prep~{s0 - k0:.1f} ok {ok0}", flush=True)
if os.environ.get("MIXED_ADD"):  # configs[4]'s add (d = dp = tau = 256), one 131,072-value chunk
    s2, k2, ok2 = leg((256, 256, 1, 256), 131072, np.uint32, 3, 1)
    print(f"{tag} configs[4] add chunk: step {s2:.1f} us chain {k2:.1f} prep~{s2 - k2:.1f} ok {ok2}", flush=True)
if os.environ.get("VALU_U8"):  # configs[0] on the VALU chain (hm_ctx_set_add_options), for comparison
    s1, k1, ok1 = leg((64, 64, 1, 64), 65536, np.uint8, 100, 5, "valu")
    print(f"{tag} u8 valu chain: step {s1:.1f} us chain {k1:.1f} ok {ok1}", flush=True)
