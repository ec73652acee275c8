"""Diagnostic: the same add with the MFMA carry chain and with the VALU chain; report which output
bits' degrees differ (used to debug an MFMA form of the prep products)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "homomorph-rust_amd"))
import homomorph as H  # noqa: E402

for params, dt, n in (((64, 64, 1, 64), np.uint8, 128), ((128, 128, 1, 128), np.uint32, 64)):
    ctx = H.Context(H.Parameters(*params), device="cuda:0")
    ctx.seed_rng(5)
    ctx.generate_secret_key()
    ctx.generate_public_key()
    rng = np.random.default_rng(1)
    a = rng.integers(0, np.iinfo(dt).max, size=n, dtype=dt)
    b = rng.integers(0, np.iinfo(dt).max, size=n, dtype=dt)
    ca, cb = ctx.encrypt(a), ctx.encrypt(b)
    outs = {}
    for chain in ("mfma", "valu"):
        ctx.set_add_options(chain)
        c = ctx.apply2(H.HomomorphicAddition, ca, cb)
        try:
            ctx.synchronize()
        except Exception as exc:
            print(params, chain, "raised", exc)
        outs[chain] = c.to_host()
    (lm, dm), (lv, dv) = outs["mfma"], outs["valu"]
    nb = dm.size // n
    dm, dv = dm.reshape(n, nb), dv.reshape(n, nb)
    diff = np.nonzero((dm != dv).any(axis=0))[0]
    print(params, "bits whose degrees differ:", diff.tolist(), "values:", int((dm != dv).any(axis=1).sum()))
    if len(diff):
        i = diff[0]
        e = int(np.nonzero(dm[:, i] != dv[:, i])[0][0])
        print("  first: value", e, "bit", i, "deg mfma", dm[e, i], "valu", dv[e, i])
