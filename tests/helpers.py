"""Shared seeded-input helpers for the parity tests (keys, masks, plaintexts, layout views)."""
from __future__ import annotations

import numpy as np

from oracle import gf2_model as model
from oracle import oracle_py as oracle


def keys(d, dp, delta, tau, seed):
    return oracle.keygen(d, dp, delta, tau, seed)


def masks(n, nbits, tau, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(n, nbits, (tau + 7) // 8), dtype=np.uint8)


def plain(n, dtype, seed, lo=None, hi=None):
    rng = np.random.default_rng(seed)
    info = np.iinfo(dtype)
    lo = info.min if lo is None else lo
    hi = info.max if hi is None else hi
    return rng.integers(lo, hi, size=n, dtype=dtype, endpoint=True)


def as_bytes(values: np.ndarray) -> np.ndarray:
    """bincode fixint little-endian image of each value (src/cipher.rs:6-13)."""
    v = np.ascontiguousarray(values.astype(values.dtype.newbyteorder("<")))
    return v.view(np.uint8).reshape(len(values), values.dtype.itemsize)


def offsets(bound):
    c = oracle.caps(bound)
    return np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.int64), c, int(c.sum())


def bit_ints(limbs, deg, bound, e):
    """The nbits polynomials of value e as Python ints (model form)."""
    off, cap, stride = offsets(bound)
    out = []
    for i in range(len(bound)):
        seg = limbs[e * stride + off[i]: e * stride + off[i] + cap[i]]
        out.append(model.limbs_to_int(seg))
    return out


def assert_batches_equal(l1, d1, l2, d2, bound, n, what=""):
    """Bit-exact: same degrees and same limbs (limbs above the degree are zero on both sides)."""
    d1 = np.asarray(d1, dtype=np.uint32).reshape(-1)
    d2 = np.asarray(d2, dtype=np.uint32).reshape(-1)
    if not np.array_equal(d1, d2):
        bad = np.nonzero(d1 != d2)[0][:5]
        raise AssertionError(f"{what}: degree mismatch at {bad.tolist()}: {d1[bad]} vs {d2[bad]}")
    l1 = np.asarray(l1, dtype=np.uint64).reshape(-1)
    l2 = np.asarray(l2, dtype=np.uint64).reshape(-1)
    if not np.array_equal(l1, l2):
        bad = np.nonzero(l1 != l2)[0][:5]
        _, _, stride = offsets(bound)
        raise AssertionError(f"{what}: limb mismatch at {bad.tolist()} (value {bad // stride})")


def pad_bits_host(limbs, deg, bound, n, nbits):
    """A host batch widened to nbits ciphertext bits per value, the new bits null polynomials
    (bound 0, one zero limb): a k-bit product decrypted as whole bytes (k % 8 != 0)."""
    _, _, stride = offsets(bound)
    extra = int(nbits) - len(bound)
    l = np.concatenate([np.asarray(limbs, dtype=np.uint64).reshape(n, stride),
                        np.zeros((n, extra), dtype=np.uint64)], axis=1).reshape(-1)
    d = np.concatenate([np.asarray(deg, dtype=np.uint32).reshape(n, len(bound)),
                        np.zeros((n, extra), dtype=np.uint32)], axis=1).reshape(-1)
    return l, d, np.concatenate([np.asarray(bound, dtype=np.uint32), np.zeros(extra, dtype=np.uint32)])


def digest(limbs, bound, n):
    """Per-value SHA-256 (hex) of a batch's limbs (the batch layout, capacity limbs per bit)."""
    import hashlib
    _, _, stride = offsets(bound)
    l = np.ascontiguousarray(np.asarray(limbs, dtype=np.uint64).reshape(n, stride))
    return [hashlib.sha256(l[e].astype("<u8").tobytes()).hexdigest() for e in range(n)]


def fresh_bound(d, dp, nbits):
    return np.full(nbits, d + dp, dtype=np.uint32)


def low_bits(limbs, deg, bound, n, k):
    """The low k bit-polynomials of every value of a batch, as a k-bit batch (host copy)."""
    _, cap, stride = offsets(bound)
    sk = int(cap[:k].sum())
    l = np.asarray(limbs, dtype=np.uint64).reshape(n, stride)[:, :sk].reshape(-1).copy()
    d = np.asarray(deg, dtype=np.uint32).reshape(n, len(bound))[:, :k].reshape(-1).copy()
    return l, d, np.ascontiguousarray(np.asarray(bound, dtype=np.uint32)[:k])


# ------------------------------------------------------------------ mask CSPRNG contract
def _splitmix64(state):
    state = (state + 0x9E3779B97F4A7C15) & (2**64 - 1)
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
    return state, z ^ (z >> 31)


def chacha20_block(key_words, counter, nonce):
    """One 64-byte ChaCha20 block (Bernstein's layout: 64-bit counter, 64-bit nonce), pure
    Python: the test-side restatement of the engine's mask generator (kernels.hip)."""
    M = 0xFFFFFFFF

    def rotl(x, r):
        return ((x << r) | (x >> (32 - r))) & M

    def qr(x, a, b, c, d):
        x[a] = (x[a] + x[b]) & M; x[d] = rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & M; x[b] = rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & M; x[d] = rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & M; x[b] = rotl(x[b] ^ x[c], 7)

    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(key_words) + [
        counter & M, counter >> 32, nonce & M, (nonce >> 32) & M]
    x = list(s)
    for _ in range(10):
        qr(x, 0, 4, 8, 12); qr(x, 1, 5, 9, 13); qr(x, 2, 6, 10, 14); qr(x, 3, 7, 11, 15)
        qr(x, 0, 5, 10, 15); qr(x, 1, 6, 11, 12); qr(x, 2, 7, 8, 13); qr(x, 3, 4, 9, 14)
    return b"".join(((x[i] + s[i]) & M).to_bytes(4, "little") for i in range(16))


def seeded_chacha(seed):
    """(key words, first nonce) of a context after hm_ctx_seed_rng(seed) (capi.cpp)."""
    st = seed ^ 0x6D61736B73636861
    key = []
    for _ in range(4):
        st, w = _splitmix64(st)
        key += [w & 0xFFFFFFFF, w >> 32]
    st, nonce = _splitmix64(st)
    return key, nonce


def seeded_random_bytes(seed, draw, n, start=0):
    """Bytes [start, start+n) of the `draw`-th (0-based) hm_random_bytes call after seeding."""
    key, nonce = seeded_chacha(seed)
    nonce = (nonce + draw) & (2**64 - 1)
    c0, c1 = start // 64, (start + n + 63) // 64
    blocks = b"".join(chacha20_block(key, c, nonce) for c in range(c0, c1))
    return np.frombuffer(blocks[start - 64 * c0: start - 64 * c0 + n], dtype=np.uint8)


def seeded_value_masks(seed, draw, idx, nbits, mask_bytes):
    """Masks the engine drew for values idx in its `draw`-th CSPRNG draw of an encrypt call
    (masks=None): value e's nbits*mask_bytes bytes start at e*nbits*mask_bytes.  Returns
    (len(idx), nbits, mask_bytes) uint8 -- only the ChaCha20 blocks of those values are made."""
    per = nbits * mask_bytes
    return np.stack([seeded_random_bytes(seed, draw, per, int(e) * per).reshape(nbits, mask_bytes)
                     for e in idx])


# ------------------------------------------------------------------ residue checksum
def residue_modulus(seed):
    """A random f = X^64 + g for the residue checksum (oracle/residue_check.c)."""
    return int(np.random.default_rng(seed).integers(0, 2**63, dtype=np.uint64)) * 2 + 1


def check_residues(H, op, out, a, b=None, k=None, signed=False, seed=0, chunk=32768):
    """Every output polynomial of the device batch `out` against the reference circuit `op`
    ("add", "mul", "and", "or", "xor", "not") run on the residues of the device inputs: P mod f
    is a ring homomorphism, so residue(out) must equal circuit(residue(a), residue(b)) for every
    (value, bit), and every degree word must be the exact top bit of its limbs.  Values are
    copied to the host in chunks.  k: the mul_low result bits (out has k bits).  Returns the
    number of values checked."""
    g = residue_modulus(seed)
    n = out.n
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        al, ad = H.value_slice(a, lo, hi).to_host()
        ra, bad = oracle.residues(al, ad, a.bound, a.nbits, hi - lo, g)
        assert bad == 0, f"{op}: {bad} input degree words disagree with their limbs"
        rb = None
        if b is not None:
            bl, bd = H.value_slice(b, lo, hi).to_host()
            rb, bad = oracle.residues(bl, bd, b.bound, b.nbits, hi - lo, g)
            assert bad == 0
        ol, od = H.value_slice(out, lo, hi).to_host()
        ro, bad = oracle.residues(ol, od, out.bound, out.nbits, hi - lo, g)
        assert bad == 0, f"{op}: {bad} output degree words disagree with their limbs"
        if op == "add":
            want = oracle.residue_add(ra, rb, g)
        elif op == "mul":
            want = oracle.residue_mul(ra, rb, k or a.nbits, g, signed=signed)
        else:
            want = oracle.residue_gate(op, ra, rb, g)
        if not np.array_equal(ro, want):
            e, i = np.argwhere(ro != want)[0]
            raise AssertionError(f"{op}: residue mismatch at value {lo + e}, bit {i} "
                                 f"({int((ro != want).sum())} polynomials differ)")
    return n
