"""Encrypt/decrypt probe (configs[2] shape, for A/B runs and profiles): u32 encryption of a 65,536-
value batch at d = dp = tau = 128 through the C ABI on device-resident data, with pre-drawn masks
and with masks drawn by the engine's ChaCha20 (fused into the tau = 128 kernel), then decrypt_bits
of the result; REPS launches each, timed by HIP events on the engine stream, both as direct
launches and as one captured HIP graph per call.  env: N (batch), REPS."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "homomorph-rust_amd")]
import numpy as np
import torch
import homomorph as H
from homomorph._lib import lib

n = int(os.environ.get("N", "65536"))
reps = int(os.environ.get("REPS", "50"))
L = lib()
ctx = H.Context(H.Parameters(128, 128, 1, 128), device="cuda:0")
ctx.seed_rng(5)
ctx.generate_secret_key(); ctx.generate_public_key()
vals = torch.from_numpy(np.random.default_rng(3).integers(0, 2**32, size=n, dtype=np.uint32).view(np.int32)).to("cuda:0")
data = vals.view(torch.uint8).reshape(n, 4)
m = ctx.random_bytes(n * 32 * ctx.mask_bytes())
c = H.Ciphered.empty(n, np.full(32, ctx.fresh_bound(), dtype=np.uint32), "cuda:0")
cb = c._c()
dec = torch.empty((n, 4), dtype=torch.uint8, device="cuda:0")


def enc(mp):
    ctx._launch(lambda: L.hm_encrypt_batch(ctx._h, data.data_ptr(), 4, mp, ctypes.byref(cb)), "encrypt")


def decr():
    ctx._launch(lambda: L.hm_decrypt_batch(ctx._h, ctypes.byref(cb), dec.data_ptr()), "decrypt")


def timed(fn, graph):
    f = ctx.graph(fn, warmup=2).replay if graph else fn
    for _ in range(3):
        f()
    ctx.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    ctx.synchronize()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for graph in (False, True):
    for name, fn in (("encrypt predrawn", lambda: enc(m.data_ptr())), ("encrypt csprng", lambda: enc(None)),
                     ("decrypt", decr), ("encrypt csprng + decrypt", lambda: (enc(None), decr()))):
        us = timed(fn, graph)
        print(f"{name:26s} {'graph ' if graph else 'direct'} n={n}: {us:7.1f} us per call, {n / us * 1e6:.4g}/s",
              flush=True)
enc(None); decr(); ctx.synchronize()
print("round trip ok:", bool(torch.equal(dec, data)))
