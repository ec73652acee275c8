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


def fresh_bound(d, dp, nbits):
    return np.full(nbits, d + dp, dtype=np.uint32)


def low_bits(limbs, deg, bound, n, k):
    """The low k bit-polynomials of every value of a batch, as a k-bit batch (host copy)."""
    _, cap, stride = offsets(bound)
    sk = int(cap[:k].sum())
    l = np.asarray(limbs, dtype=np.uint64).reshape(n, stride)[:, :sk].reshape(-1).copy()
    d = np.asarray(deg, dtype=np.uint32).reshape(n, len(bound))[:, :k].reshape(-1).copy()
    return l, d, np.ascontiguousarray(np.asarray(bound, dtype=np.uint32)[:k])
