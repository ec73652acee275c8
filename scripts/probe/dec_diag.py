"""Diagnostic: decrypt a 4096-value add output (decrypt_kernel, wave per value) and report which
values come out wrong (compare libraries via HOMOMORPH_GPU_LIB)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402
import homomorph as H  # noqa: E402

ctx = bench.make_context(1, 0, None, bench.PARAMS)
n = 4096
a, b = bench.shard_inputs(0, n)
ca, cb = ctx.encrypt(a), ctx.encrypt(b)
cs = ctx.apply2(H.HomomorphicAddition, ca, cb)
dec = ctx.decrypt(cs)
ctx.synchronize()
want = (a + b).astype(np.uint32)
wrong = np.nonzero(dec != want)[0]
print(os.environ.get("HOMOMORPH_GPU_LIB", "default"), "wrong", len(wrong), "first", wrong[:6].tolist(),
      "zeros among wrong", int(np.sum(dec[wrong] == 0)))
ctx.synchronize()
dec2 = ctx.decrypt(cs)
dec3 = ctx.decrypt(cs)
print("  after sync: wrong", int(np.sum(dec2 != want)), "dec2 vs dec3 differ", int(np.sum(dec2 != dec3)),
      "dec vs dec2 differ", int(np.sum(dec != dec2)))
