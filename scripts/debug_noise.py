"""For the bench's own inputs: find sums that decrypt wrong and check them against the oracle
(bit-exact ciphertext + oracle decryption) to separate engine bugs from scheme noise."""
import sys
sys.path[:0] = ['.', 'tests', 'homomorph-rust_amd']
import numpy as np, torch
import homomorph as H
from helpers import as_bytes, assert_batches_equal, fresh_bound
from oracle import oracle_py as oracle
ctx = H.Context(H.Parameters(128, 128, 1, 128))
ctx.seed_rng(0xB0B); ctx.generate_secret_key(); ctx.generate_public_key()
sk, pk = ctx.get_secret_key().limbs, ctx.get_public_key().limbs
n = 4096
rng = np.random.default_rng(1000)
a = rng.integers(0, 2**32, size=n, dtype=np.uint32)
b = rng.integers(0, 2**32, size=n, dtype=np.uint32)
gen = torch.Generator(device='cuda'); gen.manual_seed(31)
ca, cb = ctx.encrypt(a, generator=gen), ctx.encrypt(b, generator=gen)
s = ctx.apply2(H.HomomorphicAddition, ca, cb)
dec = ctx.decrypt(s); ctx.synchronize()
bad = np.nonzero(dec != (a + b).astype(np.uint32))[0]
print("wrong sums:", bad.tolist())
ma = ca._keep[1].cpu().numpy(); mb = cb._keep[1].cpu().numpy()
bound = fresh_bound(128, 128, 32)
idx = np.concatenate([bad, np.arange(4)])
la, da = oracle.encrypt_batch(pk, as_bytes(a[idx]), ma[idx], bound)
lb, db = oracle.encrypt_batch(pk, as_bytes(b[idx]), mb[idx], bound)
rl, rd = oracle.add_batch(la, da, bound, lb, db, bound, 32, len(idx), s.bound)
gl, gd = s.to_host()
st = H.batch_stride(s.bound)
g_sel = np.concatenate([gl[e*st:(e+1)*st] for e in idx]); d_sel = np.concatenate([gd[e*32:(e+1)*32] for e in idx])
assert_batches_equal(g_sel, d_sel, rl, rd, s.bound, len(idx), "bench inputs")
odec = oracle.decrypt_batch(sk, rl, rd, s.bound, 32, len(idx)).view(np.uint32).reshape(-1)
print("ciphertexts bit-exact vs oracle for", len(idx), "values; oracle decrypt:", odec[:len(bad)].tolist(), "gpu:", dec[bad].tolist(), "true:", (a[bad]+b[bad]).astype(np.uint32).tolist())
