"""ctypes binding of the C oracle (oracle/_build/liboracle.so) — test infrastructure only.

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product.
All arrays are numpy; the batch layout is the one documented in oracle/homomorph_oracle.h and
shared with the GPU engine (include/homomorph_gpu.h, "Batch layout").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

u64p = ctypes.POINTER(ctypes.c_uint64)
u32p = ctypes.POINTER(ctypes.c_uint32)
u8p = ctypes.POINTER(ctypes.c_uint8)
szp = ctypes.POINTER(ctypes.c_size_t)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        L.oracle_compute_degree.restype = ctypes.c_size_t
        L.oracle_compute_degree.argtypes = [u64p, ctypes.c_size_t]
        for f in (L.oracle_poly_add, L.oracle_poly_mul, L.oracle_poly_rem):
            f.restype = ctypes.c_int
            f.argtypes = [u64p, ctypes.c_size_t, u64p, ctypes.c_size_t, u64p, ctypes.c_size_t,
                          szp, szp]
        L.oracle_poly_evaluate.restype = ctypes.c_int
        L.oracle_poly_evaluate.argtypes = [u64p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_poly_eq.restype = ctypes.c_int
        L.oracle_poly_eq.argtypes = [u64p, ctypes.c_size_t, u64p, ctypes.c_size_t]
        L.oracle_splitmix64.restype = ctypes.c_uint64
        L.oracle_splitmix64.argtypes = [u64p]
        L.oracle_keygen.restype = ctypes.c_int
        L.oracle_keygen.argtypes = [ctypes.c_uint16] * 4 + [ctypes.c_uint64, u64p, u64p, u32p]
        L.oracle_encrypt_batch.restype = ctypes.c_int
        L.oracle_encrypt_batch.argtypes = [u64p, ctypes.c_uint32, ctypes.c_uint32, u8p,
                                           ctypes.c_uint32, ctypes.c_size_t, u8p, u64p, u32p, u32p]
        L.oracle_decrypt_batch.restype = ctypes.c_int
        L.oracle_decrypt_batch.argtypes = [u64p, ctypes.c_uint32, u64p, u32p, u32p,
                                           ctypes.c_uint32, ctypes.c_size_t, u8p]
        binargs = [u64p, u32p, u32p, u64p, u32p, u32p, ctypes.c_uint32, ctypes.c_size_t]
        L.oracle_add_batch.restype = ctypes.c_int
        L.oracle_add_batch.argtypes = binargs + [u64p, u32p, u32p]
        L.oracle_mul_batch.restype = ctypes.c_int
        L.oracle_mul_batch.argtypes = binargs + [ctypes.c_int, u64p, u32p, u32p]
        L.oracle_gate_batch.restype = ctypes.c_int
        L.oracle_gate_batch.argtypes = [ctypes.c_int] + binargs + [u64p, u32p, u32p]
        L.oracle_set_threads.restype = None
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_limb_products.restype = ctypes.c_uint64
        L.oracle_reset_counters.restype = None
        # residue_check.c: the ring-homomorphism checksum (residues mod X^64 + g)
        L.oracle_residue_threads.restype = None
        L.oracle_residue_threads.argtypes = [ctypes.c_int]
        L.oracle_residues.restype = ctypes.c_int
        L.oracle_residues.argtypes = [u64p, u32p, u32p, ctypes.c_uint32, ctypes.c_size_t,
                                      ctypes.c_uint64, u64p, szp]
        L.oracle_residue_add.restype = ctypes.c_int
        L.oracle_residue_add.argtypes = [u64p, u64p, ctypes.c_uint32, ctypes.c_size_t,
                                         ctypes.c_uint64, u64p]
        L.oracle_residue_mul.restype = ctypes.c_int
        L.oracle_residue_mul.argtypes = [u64p, u64p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                         ctypes.c_size_t, ctypes.c_uint64, u64p]
        L.oracle_residue_gate.restype = ctypes.c_int
        L.oracle_residue_gate.argtypes = [ctypes.c_int, u64p, u64p, ctypes.c_size_t,
                                          ctypes.c_uint64, u64p]
        L.oracle_residue_of.restype = ctypes.c_uint64
        L.oracle_residue_of.argtypes = [u64p, ctypes.c_size_t, ctypes.c_uint64]
        L.oracle_residue_mulmod.restype = ctypes.c_uint64
        L.oracle_residue_mulmod.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


class OracleError(RuntimeError):
    pass


def _check(st: int, what: str):
    if st != 0:
        raise OracleError(f"{what}: oracle status {st}")


# ---------------- single polynomials ----------------
def _arr(limbs) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(limbs, dtype=np.uint64))


def compute_degree(limbs) -> int:
    a = _arr(limbs)
    return int(lib().oracle_compute_degree(_p(a, u64p), a.size))


def _binop(fn, a, b, cap):
    a, b = _arr(a), _arr(b)
    out = np.zeros(max(cap, 1), dtype=np.uint64)
    deg, olen = ctypes.c_size_t(), ctypes.c_size_t()
    st = fn(_p(a, u64p), a.size, _p(b, u64p), b.size, _p(out, u64p), out.size,
            ctypes.byref(deg), ctypes.byref(olen))
    _check(st, fn.__name__)
    return out[: olen.value], deg.value


def poly_add(a, b):
    return _binop(lib().oracle_poly_add, a, b, max(len(a), len(b)))


def poly_mul(a, b):
    return _binop(lib().oracle_poly_mul, a, b, len(a) + len(b))


def poly_rem(a, b):
    return _binop(lib().oracle_poly_rem, a, b, len(a))


def poly_evaluate(a, x: bool) -> bool:
    a = _arr(a)
    return bool(lib().oracle_poly_evaluate(_p(a, u64p), a.size, int(bool(x))))


def poly_eq(a, b) -> bool:
    a, b = _arr(a), _arr(b)
    return bool(lib().oracle_poly_eq(_p(a, u64p), a.size, _p(b, u64p), b.size))


# ---------------- keys / batches ----------------
def keygen(d, dp, delta, tau, seed):
    sk = np.zeros(d // 64 + 1, dtype=np.uint64)
    cap = (d + dp) // 64 + 1
    pk = np.zeros((tau, cap), dtype=np.uint64)
    pkdeg = np.zeros(tau, dtype=np.uint32)
    _check(lib().oracle_keygen(d, dp, delta, tau, seed & (2**64 - 1), _p(sk, u64p),
                               _p(pk, u64p), _p(pkdeg, u32p)), "keygen")
    return sk, pk, pkdeg


def caps(bound) -> np.ndarray:
    return np.asarray(bound, dtype=np.uint32) // 64 + 1


def stride(bound) -> int:
    return int(caps(bound).sum())


def encrypt_batch(pk, data: np.ndarray, masks: np.ndarray, bound):
    """data: (n, nbytes) uint8; masks: (n, 8*nbytes, ceil(tau/8)) uint8."""
    pk = np.ascontiguousarray(pk, dtype=np.uint64)
    data = np.ascontiguousarray(data, dtype=np.uint8)
    masks = np.ascontiguousarray(masks, dtype=np.uint8)
    n, nbytes = data.shape
    bound = np.ascontiguousarray(bound, dtype=np.uint32)
    out = np.zeros(n * stride(bound), dtype=np.uint64)
    deg = np.zeros(n * 8 * nbytes, dtype=np.uint32)
    _check(lib().oracle_encrypt_batch(_p(pk, u64p), pk.shape[0], pk.shape[1], _p(data, u8p),
                                      nbytes, n, _p(masks, u8p), _p(out, u64p), _p(deg, u32p),
                                      _p(bound, u32p)), "encrypt_batch")
    return out, deg


def decrypt_batch(sk, limbs, deg, bound, nbits, n):
    sk = np.ascontiguousarray(sk, dtype=np.uint64)
    limbs = np.ascontiguousarray(limbs, dtype=np.uint64)
    deg = np.ascontiguousarray(deg, dtype=np.uint32)
    bound = np.ascontiguousarray(bound, dtype=np.uint32)
    out = np.zeros(n * (nbits // 8), dtype=np.uint8)
    _check(lib().oracle_decrypt_batch(_p(sk, u64p), sk.size, _p(limbs, u64p), _p(deg, u32p),
                                      _p(bound, u32p), nbits, n, _p(out, u8p)), "decrypt_batch")
    return out.reshape(n, nbits // 8)


def _binary(kind, a, adeg, abound, b, bdeg, bbound, nbits, n, obound, extra=None):
    arrs = [np.ascontiguousarray(x, dtype=t) for x, t in
            ((a, np.uint64), (adeg, np.uint32), (abound, np.uint32),
             (b, np.uint64), (bdeg, np.uint32), (bbound, np.uint32))]
    obound = np.ascontiguousarray(obound, dtype=np.uint32)
    out = np.zeros(n * stride(obound), dtype=np.uint64)
    odeg = np.zeros(n * nbits, dtype=np.uint32)
    ptrs = [_p(arrs[0], u64p), _p(arrs[1], u32p), _p(arrs[2], u32p),
            _p(arrs[3], u64p), _p(arrs[4], u32p), _p(arrs[5], u32p), nbits, n]
    L = lib()
    if kind == "add":
        st = L.oracle_add_batch(*ptrs, _p(out, u64p), _p(odeg, u32p), _p(obound, u32p))
    elif kind in ("mul", "muls"):
        st = L.oracle_mul_batch(*ptrs, int(kind == "muls"), _p(out, u64p), _p(odeg, u32p),
                                _p(obound, u32p))
    else:
        st = L.oracle_gate_batch(extra, *ptrs, _p(out, u64p), _p(odeg, u32p), _p(obound, u32p))
    _check(st, kind)
    return out, odeg


def add_batch(a, adeg, abound, b, bdeg, bbound, nbits, n, obound):
    return _binary("add", a, adeg, abound, b, bdeg, bbound, nbits, n, obound)


def mul_batch(a, adeg, abound, b, bdeg, bbound, nbits, n, obound, signed=False):
    return _binary("muls" if signed else "mul", a, adeg, abound, b, bdeg, bbound, nbits, n,
                   obound)


GATES = {"and": 0, "or": 1, "xor": 2, "not": 3}


def gate_batch(op, a, adeg, abound, b, bdeg, bbound, nbits, n, obound):
    return _binary("gate", a, adeg, abound, b, bdeg, bbound, nbits, n, obound, GATES[op])


def set_threads(n: int):
    """Threads for the batch entry points (values split over threads); 1 = the reference's
    single-threaded execution."""
    lib().oracle_set_threads(int(n))


def limb_products() -> int:
    return int(lib().oracle_limb_products())


def reset_counters():
    lib().oracle_reset_counters()


# ---------------- residue checksum (residue_check.c) ----------------
# P -> P mod (X^64 + g) is a ring homomorphism, so every circuit output's residue equals the
# circuit evaluated on the input residues: a size-independent check of whole batches.
def residues(limbs, deg, bound, nbits, n, g):
    """(n, nbits) uint64 residues of a batch and the count of degree words that disagree with
    their limbs (deg may be None: not checked)."""
    limbs = np.ascontiguousarray(limbs, dtype=np.uint64)
    bound = np.ascontiguousarray(bound, dtype=np.uint32)
    dp = None
    if deg is not None:
        deg = np.ascontiguousarray(deg, dtype=np.uint32)
        dp = _p(deg, u32p)
    out = np.zeros(n * nbits, dtype=np.uint64)
    bad = ctypes.c_size_t()
    _check(lib().oracle_residues(_p(limbs, u64p), dp, _p(bound, u32p), nbits, n, g & (2**64 - 1),
                                 _p(out, u64p), ctypes.byref(bad)), "residues")
    return out.reshape(n, nbits), int(bad.value)


def residue_add(ra, rb, g):
    ra, rb = np.ascontiguousarray(ra, np.uint64), np.ascontiguousarray(rb, np.uint64)
    n, nbits = ra.shape
    out = np.zeros_like(ra)
    _check(lib().oracle_residue_add(_p(ra, u64p), _p(rb, u64p), nbits, n, g & (2**64 - 1),
                                    _p(out, u64p)), "residue_add")
    return out


def residue_mul(ra, rb, k, g, signed=False):
    ra, rb = np.ascontiguousarray(ra, np.uint64), np.ascontiguousarray(rb, np.uint64)
    n, nbits = ra.shape
    out = np.zeros((n, k), dtype=np.uint64)
    _check(lib().oracle_residue_mul(_p(ra, u64p), _p(rb, u64p), nbits, k, int(signed), n,
                                    g & (2**64 - 1), _p(out, u64p)), "residue_mul")
    return out


def residue_gate(op, ra, rb, g):
    ra = np.ascontiguousarray(ra, np.uint64)
    rb = ra if rb is None else np.ascontiguousarray(rb, np.uint64)
    out = np.zeros_like(ra)
    _check(lib().oracle_residue_gate(GATES[op], _p(ra, u64p), _p(rb, u64p), ra.size,
                                     g & (2**64 - 1), _p(out, u64p)), "residue_gate")
    return out


def residue_of(limbs, g) -> int:
    a = _arr(limbs)
    return int(lib().oracle_residue_of(_p(a, u64p), a.size, g & (2**64 - 1)))


def residue_mulmod(a: int, b: int, g: int) -> int:
    return int(lib().oracle_residue_mulmod(a, b, g & (2**64 - 1)))
