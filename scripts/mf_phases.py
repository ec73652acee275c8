"""Phase split of the multiplier's MFMA product kernels (a -DHM_MF_PROFILE build under
lib/variants, e.g. scripts/mk_variant.sh mfprof "-DHM_MF_PROFILE" mul_mfma): one multiply of the
u8 bench workload (or KS/N from the env), then the per-class wave-summed s_memtime deltas of
hm_debug_mf_prof.  env: HOMOMORPH_GPU_LIB (the profiling build), KS, N."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "homomorph-rust_amd")]
import numpy as np
import homomorph as H
from homomorph._lib import lib

k, n = int(os.environ.get("KS", "8")), int(os.environ.get("N", "16384"))
ctx = H.Context(H.Parameters(128, 128, 1, 128), device="cuda:0")
ctx.seed_rng(5)
ctx.generate_secret_key(); ctx.generate_public_key()
a = np.random.default_rng(3).integers(0, 2**32, size=n, dtype=np.uint32)
b = np.random.default_rng(4).integers(0, 2**32, size=n, dtype=np.uint32)
ca, cb = ctx.encrypt(a), ctx.encrypt(b)
o = ctx.mul_low(ca, cb, k); ctx.synchronize()
buf = (ctypes.c_ulonglong * 64)()
f = lib().hm_debug_mf_prof
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
f(buf, 1)
o = ctx.mul_low(ca, cb, k); ctx.synchronize()
f(buf, 0)
names = ["leaf", "lean leaf", "tiny", "narrow", "wide (win)", "wide"]
print(f"K={k} n={n}: per class, s_memtime ticks per wave (share of the wave's life)")
for c, nm in enumerate(names):
    w = buf[8 * c]
    if not w:
        continue
    ph = [buf[8 * c + i] / w for i in range(1, 5)]
    tot = sum(ph)
    print(f"{nm:11s} waves {w:8d}  records {ph[0]:8.0f} ({ph[0]/tot:4.0%})  images {ph[1]:8.0f} ({ph[1]/tot:4.0%})"
          f"  groups {ph[2]:8.0f} ({ph[2]/tot:4.0%})  copy-out {ph[3]:8.0f} ({ph[3]/tot:4.0%})")
