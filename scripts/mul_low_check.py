"""One-off parity probe for the low-k multiply at large k: GPU vs the C oracle on n values."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "homomorph-rust_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import homomorph as H
from helpers import as_bytes, fresh_bound, keys, low_bits, masks, plain
from oracle import oracle_py as oracle
k, n = int(sys.argv[1]), int(sys.argv[2])
params = (128, 128, 1, 128)
ctx = H.Context(H.Parameters(*params), device="cuda:0")
ctx.seed_rng(81); ctx.generate_secret_key(); ctx.generate_public_key()
sk, pk, _ = keys(*params, 81)
a, b = plain(n, np.uint32, 5), plain(n, np.uint32, 6)
ma, mb = masks(n, 32, 128, 7), masks(n, 32, 128, 8)
cp = ctx.mul_low(ctx.encrypt(a, masks=ma), ctx.encrypt(b, masks=mb), k)
gl, gd = cp.to_host()
bound = fresh_bound(128, 128, 32)
la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, bound)
lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bound)
lak, dak, bk = low_bits(la, da, bound, n, k)
lbk, dbk, _ = low_bits(lb, db, bound, n, k)
t0 = time.perf_counter()
rl, rd = oracle.mul_batch(lak, dak, bk, lbk, dbk, bk, k, n, cp.bound)
print(f"oracle {time.perf_counter()-t0:.1f} s", flush=True)
print("degrees equal", np.array_equal(gd, rd), "limbs equal", np.array_equal(gl, rl))
dec = oracle.decrypt_batch(sk, rl, rd, cp.bound, k, n).reshape(n, -1)
got = dec.astype(np.uint64) @ (256 ** np.arange(k // 8, dtype=np.uint64))
print("oracle decrypt", got, "want", (a.astype(np.uint64) * b) & ((1 << k) - 1))
print("top degrees", rd.reshape(n, k)[:, -3:])
