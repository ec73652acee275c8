"""A/B probe: configs[2]'s fresh u32 decryption (65,536 values, d = dp = tau = 128) as the bench times
it -- one replay of a 50-step graph after warm-up, the decrypt kernel's duration by the engine's
device stamps (bench.timed_graph) -- and the encrypt kernel the same way (pre-drawn masks).
Library: HOMOMORPH_GPU_LIB (an A/B variant) or the in-tree build."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import homomorph as H  # noqa: E402


def main():
    ctx = bench.make_context(1, 0, None, bench.PARAMS)
    L = H.lib()
    n = 65536
    vals = torch.from_numpy(np.random.default_rng(7).integers(0, 2**32, size=n, dtype=np.uint32)
                            .view(np.int32)).to("cuda:0")
    data = vals.view(torch.uint8).reshape(n, 4)
    m = ctx.random_bytes(n * 32 * ctx.mask_bytes())
    c = H.Ciphered.empty(n, np.full(32, ctx.fresh_bound(), dtype=np.uint32), "cuda:0")
    dec = torch.empty((n, 4), dtype=torch.uint8, device="cuda:0")
    cb = c._c()
    enc = lambda: ctx._launch(lambda: L.hm_encrypt_batch(ctx._h, data.data_ptr(), 4, m.data_ptr(),  # noqa: E731
                                                         ctypes.byref(cb)), "encrypt")
    decr = lambda: ctx._launch(lambda: L.hm_decrypt_batch(ctx._h, ctypes.byref(cb), dec.data_ptr()),  # noqa: E731
                               "decrypt")
    enc()
    _, _, eks, _ = bench.timed_graph(ctx, enc, 50, 2, 1, "encrypt")
    _, dstep, dks, _ = bench.timed_graph(ctx, decr, 50, 2, 1, "decrypt")
    ok = bool(torch.equal(dec, data))
    print(f"encrypt kernel {1e6 * eks:.2f} us | decrypt kernel {1e6 * dks:.2f} us (step {1e6 * dstep:.2f} us,"
          f" {1284 * n / dks / 1e12:.2f} TB/s) ok={ok}", flush=True)


if __name__ == "__main__":
    main()
