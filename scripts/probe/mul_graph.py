"""Is the u8 multiply capturable as a HIP graph, bit-identical to direct launches, and does a
K-step graph replay shorten it (inter-launch gaps)?  bench.py's u8_mul leg workload."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402
import homomorph as H  # noqa: E402

mctx, _ = bench.s0_zero_context("cuda:0")
n8 = 16384
a8 = np.random.default_rng(1).integers(0, 256, size=n8, dtype=np.uint8)
b8 = np.random.default_rng(2).integers(0, 256, size=n8, dtype=np.uint8)
ca, cb = mctx.encrypt(a8), mctx.encrypt(b8)
co = H.Ciphered.empty(n8, H.mul_out_bounds(ca.bound, cb.bound), "cuda:0")
H.mul_into(mctx, ca, cb, co)
mctx.synchronize()
ref_l, ref_d = co.limbs.clone(), co.degree.clone()
fn = lambda: H.mul_into(mctx, ca, cb, co)  # noqa: E731
for rnd in range(3):
    wall, ev = bench.time_loop(fn, 5, 1, 1, mctx.stream)
    co.limbs.zero_()
    wg, sg, _, _ = bench.timed_graph(mctx, fn, 5, 2, 1, None)
    same = bool(torch.equal(co.limbs, ref_l) and torch.equal(co.degree, ref_d))
    print(f"direct {1e3 * ev / 5:.3f} ms (wall {1e3 * wall / 5:.3f})  graph {1e3 * sg:.3f} ms (wall {1e3 * wg / 5:.3f})  same={same}", flush=True)
got = mctx.decrypt(co, np.uint8)
print("decrypt ok", bool(np.array_equal(got, (a8.astype(int) * b8).astype(np.uint8))))
