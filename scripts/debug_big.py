import sys, os, ctypes
sys.path[:0] = ['.', 'tests', 'homomorph-rust_amd']
import numpy as np, torch
import homomorph as H
from helpers import *
params = (128, 128, 1, 128)
ctx = H.Context(H.Parameters(*params)); ctx.seed_rng(7); ctx.generate_secret_key(); ctx.generate_public_key()
n = 4096
vals = plain(n, np.uint32, 8)
m = masks(n, 32, 128, 9)
c = ctx.encrypt(vals, masks=m)
ctx.synchronize()
torch.cuda.synchronize()
for r in range(3):
    out = torch.full((n, 4), 0xAB, dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    cb = c._c()
    st = H.lib().hm_decrypt_batch(ctx._h, ctypes.byref(cb), out.data_ptr())
    st2 = H.lib().hm_ctx_synchronize(ctx._h)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    dec = o.view(np.uint32).reshape(-1)
    bad = np.nonzero(dec != vals)[0]
    sentinel = np.nonzero((o == 0xAB).all(axis=1))[0]
    print("st", st, st2, "bad", len(bad), "all-sentinel rows", len(sentinel), "bad&sentinel", len(np.intersect1d(bad, sentinel)), bad[:6])
