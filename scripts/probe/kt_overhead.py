"""Cost of the device kernel timer: graph replays of the same step captured with and without
hm_ctx_set_kernel_timing (headline add, u32 encrypt over pre-drawn masks, fresh decrypt)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import bench  # noqa: E402
import homomorph as H  # noqa: E402

ctx = bench.make_context(1, 0, None, bench.PARAMS)
L = H.lib()
n = 4096
a, b = bench.shard_inputs(0, n)
ca, cb = ctx.encrypt(a), ctx.encrypt(b)
out = H.Ciphered.empty(n, H.add_out_bounds(ca.bound, cb.bound), "cuda:0", np.dtype(np.uint32))
ne = 65536
data = torch.randint(0, 256, (ne, 4), dtype=torch.uint8, device="cuda:0")
m = ctx.random_bytes(ne * 32 * ctx.mask_bytes())
c = H.Ciphered.empty(ne, np.full(32, ctx.fresh_bound(), dtype=np.uint32), "cuda:0")
cc = c._c()
dec = torch.empty((ne, 4), dtype=torch.uint8, device="cuda:0")
steps = {
    "add_chain": lambda: H.add_into(ctx, ca, cb, out),
    "encrypt": lambda: ctx._launch(lambda: L.hm_encrypt_batch(ctx._h, data.data_ptr(), 4, m.data_ptr(),
                                                             ctypes.byref(cc)), "encrypt"),
    "decrypt": lambda: ctx._launch(lambda: L.hm_decrypt_batch(ctx._h, ctypes.byref(cc), dec.data_ptr()),
                                   "decrypt"),
}
for kernel, fn in steps.items():
    res = {}
    for rnd in range(2):
        for mode in ("off", "on"):
            wall, step_s, ks, kn = bench.timed_graph(ctx, fn, 50, 20, 1, kernel if mode == "on" else None)
            res.setdefault(mode, []).append(1e6 * step_s)
            if ks is not None:
                res.setdefault("kernel", []).append(1e6 * ks)
    print(kernel, {k: [round(x, 1) for x in v] for k, v in res.items()}, flush=True)
