"""Probe: the u32 multiply's low K result bits past the bench's K = 20 (split Karatsuba plans,
hm_ctx_set_mul_scratch) on a few values under an S(0) = 0 key: plan + run time, decryption =
a*b mod 2^K, residue check of every output polynomial.
usage: python3 scripts/probe/mul_deep.py K [K ...]   (values: env N, default 1)"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "homomorph-rust_amd"), os.path.join(ROOT, "tests")]
import homomorph as H  # noqa: E402
import helpers  # noqa: E402
from helpers import keys, plain  # noqa: E402

PARAMS = (128, 128, 1, 128)


def main():
    n = int(os.environ.get("N", "1"))
    seed = next(s for s in range(1, 1000) if not int(keys(*PARAMS, s)[0][0]) & 1)  # S(0) = 0
    ctx = H.Context(H.Parameters(*PARAMS))
    ctx.seed_rng(seed)
    ctx.generate_secret_key()
    ctx.generate_public_key()
    a, b = plain(n, np.uint32, 236), plain(n, np.uint32, 237)
    ca, cb = ctx.encrypt(a), ctx.encrypt(b)
    for k in [int(x) for x in sys.argv[1:]]:
        t0 = time.perf_counter()
        work = ctx.mul_plan_work(ca.bound, cb.bound, k)  # builds (and caches) the plan
        t1 = time.perf_counter()
        cp = ctx.mul_low(ca, cb, k)
        ctx.synchronize()
        t2 = time.perf_counter()
        cp = ctx.mul_low(ca, cb, k)  # the plan and workspace exist now
        ctx.synchronize()
        t3 = time.perf_counter()
        raw = ctx.decrypt_bytes(H.pad_bits(cp, 32)).cpu().numpy().astype(np.uint64)
        got = sum(raw[:, i] << np.uint64(8 * i) for i in range(4))
        want = (a.astype(np.uint64) * b) & np.uint64((1 << k) - 1)
        res = helpers.check_residues(H, "mul", cp, ca, cb, k=k, seed=238)
        print(f"K={k} n={n}: plan {t1 - t0:.1f} s, first call {t2 - t1:.2f} s, second {t3 - t2:.2f} s "
              f"({n / (t3 - t2):.3g} muls/s), issued word pairs {work:.3g} per value, "
              f"decrypt ok {int(np.sum(got == want))}/{n}, residues ok {res}/{n}", flush=True)
        del cp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
