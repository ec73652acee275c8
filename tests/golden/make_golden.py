"""Generate the circuit-level golden fixtures under tests/golden/ (run here, on the CPU).

The reference has no circuit-level vectors: its circuits are pinned only by
decrypt round trips (src/impls/numbers/uint.rs:176-293, src/cipher.rs:275-304).  These fixtures
are made by the C oracle (oracle/homomorph_oracle.c, the reference's call sequence) from seeded
keys, masks and plaintexts, and every output polynomial is cross-checked against the independent
big-int model (oracle/gf2_model.py) before it is written.  The reference itself cannot run here
(Rust crate, no toolchain), so these pin the GPU path to the oracle, not to the reference binary.

Each case is one .npz (numpy arrays only, no pickles): params, seed, keys, input ciphertexts in
the batch layout of include/homomorph_gpu.h, the masks that made them, the operation's output,
and the oracle's decryption of it.

    python tests/golden/make_golden.py      # rewrites tests/golden/*.npz
    python tests/golden/make_golden.py --model-check-saved mullow20_u32_d128   # see model_check_saved
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "homomorph-rust_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

from helpers import (as_bytes, bit_ints, fresh_bound, low_bits, masks, offsets, pad_bits_host,  # noqa: E402
                     plain, digest)
from oracle import gf2_model as model  # noqa: E402
from oracle import oracle_py as oracle  # noqa: E402

# name: (op, params (d, dp, delta, tau), plaintext dtype, n, key seed)
CASES = {
    "add_u8_d64": ("add", (64, 64, 1, 64), np.uint8, 4, 101),
    "add_u32_d64": ("add", (64, 64, 1, 64), np.uint32, 2, 102),
    "add_u32_d128": ("add", (128, 128, 1, 128), np.uint32, 4, 103),  # the bench configuration
    "mul_u8_d128": ("mul", (128, 128, 1, 128), np.uint8, 2, 104),    # benches/u8.rs:9
    "mul_i8_d512": ("smul", (512, 64, 1, 64), np.int8, 2, 105),      # int.rs:247-268 params
    "encdec_u32_d128": ("encdec", (128, 128, 1, 128), np.uint32, 8, 106),
    "and_u8_d32": ("and", (32, 8, 8, 8), np.uint8, 2, 107),          # uint.rs:108-174 params
    "or_u8_d32": ("or", (32, 8, 8, 8), np.uint8, 2, 108),
    "xor_u8_d32": ("xor", (32, 16, 16, 16), np.uint8, 2, 109),
    "not_u8_d32": ("not", (32, 16, 16, 16), np.uint8, 2, 110),
    # SURVEY §8(d) configs[3] / row A14: the low 16 result bits of the u32 multiply (the circuit's
    # columns 0..15), stored as degrees + a SHA-256 per value (the outputs are ~200 KB a value)
    "mullow16_u32_d128": ("mullow16", (128, 128, 1, 128), np.uint32, 8, 111),
    # result bits 16..19 too (columns 0..19): ~30 CPU-minutes per value on the oracle, one value
    # per OpenMP thread; test_golden regenerates it only with HM_SLOW_GOLDEN=1
    "mullow20_u32_d128": ("mullow20", (128, 128, 1, 128), np.uint32, 4, 112),
}


def _plain_result(op, a, b, dtype):
    a64, b64 = a.astype(np.int64), b.astype(np.int64)
    r = {"add": a64 + b64, "mul": a64 * b64, "smul": a64 * b64, "encdec": a64,
         "and": a64 & b64, "or": a64 | b64, "xor": a64 ^ b64, "not": ~a64}[op]
    return r.astype(dtype)


def _check_model(op, la, da, lb, db, bound, lo, do, obound, n):
    for e in range(n):
        A, B = bit_ints(la, da, bound, e), bit_ints(lb, db, bound, e)
        if op == "add":
            ref = model.add_circuit(A, B)
        elif op in ("mul", "smul"):
            ref = model.mul_circuit(A, B, signed=op == "smul")
        elif op == "and":
            ref = [model.clmul(x, y) for x, y in zip(A, B)]
        elif op == "xor":
            ref = [x ^ y for x, y in zip(A, B)]
        elif op == "or":
            ref = [x ^ y ^ model.clmul(x, y) for x, y in zip(A, B)]
        elif op == "not":
            ref = [x ^ 1 for x in A]
        else:
            raise ValueError(op)
        got = bit_ints(lo, do, obound, e)
        assert got == ref, f"{op}: oracle != model at value {e}"
        degs = np.asarray(do, dtype=np.int64).reshape(n, -1)[e]
        assert [model.degree(x) for x in ref] == degs.tolist()


MODEL_RESIDUE_SEED = 0x6D6F64656C  # the model's residue modulus f = X^64 + g, g from SplitMix64


def model_check_mullow(z, lo=None, values=(0,)):
    """Cross-check a low-k multiply fixture against the big-int model (oracle/gf2_model.py).

    - k <= 16: the model's own carry-save circuit (mul_circuit over clmul_fast) on `values`, whose
      output degrees and per-value SHA-256 must equal the fixture's;
    - with the product limbs `lo` (at generation; K = 20 takes the model hours per value): every
      value's output residues mod f = X^64 + g (the model's residue_int) against the circuit run on
      the inputs' residues (a ring homomorphism), and the product's digests against the fixture's.
    Returns a description of what was checked (stored in the fixture as `model_check`)."""
    k, bound, ob = int(z["k"]), z["in_bound"], z["out_bound"]
    n = len(z["a_plain"])
    la, da, b1 = low_bits(z["a_limbs"], z["a_degree"], bound, n, k)
    lb, db, b2 = low_bits(z["b_limbs"], z["b_degree"], bound, n, k)
    _, cap, _ = offsets(ob)
    done = []
    if k <= 16:
        for e in values:
            ref = model.mul_circuit(bit_ints(la, da, b1, e), bit_ints(lb, db, b2, e), mul=model.clmul_fast)
            degs = np.asarray(z["out_degree"]).reshape(n, k)[e]
            assert [model.degree(x) for x in ref] == degs.tolist(), f"model degrees, value {e}"
            limbs = np.concatenate([np.array(model.int_to_limbs(x, int(c)), dtype=np.uint64)
                                    for x, c in zip(ref, cap)])
            assert digest(limbs, ob, 1)[0] == str(z["out_sha256"][e]), f"model SHA-256, value {e}"
        done.append(f"model circuit (gf2_model.mul_circuit, clmul_fast) = fixture on values "
                    f"{list(values)}")
    if lo is not None:
        assert digest(lo, ob, n) == [str(x) for x in z["out_sha256"]], "product != fixture"
        g = model.splitmix64([MODEL_RESIDUE_SEED])
        mul = model.residue_mul(g)
        off, _, stride = offsets(ob)
        lo2 = np.asarray(lo, dtype=np.uint64).reshape(n, stride)
        for e in range(n):
            ra = [model.residue_int(x, g) for x in bit_ints(la, da, b1, e)]
            rb = [model.residue_int(x, g) for x in bit_ints(lb, db, b2, e)]
            want = model.mul_circuit(ra, rb, mul=mul)
            got = [model.residue_limbs(lo2[e, off[i]:off[i] + cap[i]], g) for i in range(k)]
            assert got == want, f"model residues, value {e}"
        done.append(f"model residues mod X^64 + g of all {n} values = the circuit on the inputs' "
                    "residues (gf2_model.residue_int)")
    return "; ".join(done)


def make(name):
    import homomorph as H
    op, params, dtype, n, seed = CASES[name]
    d, dp, delta, tau = params
    sk, pk, pkdeg = oracle.keygen(d, dp, delta, tau, seed)
    s, T = model.keygen(d, dp, delta, tau, seed)
    assert model.limbs_to_int(sk) == s and [model.limbs_to_int(r) for r in pk] == T
    nbits = 8 * np.dtype(dtype).itemsize
    a, b = plain(n, dtype, seed + 1), plain(n, dtype, seed + 2)
    ma, mb = masks(n, nbits, tau, seed + 3), masks(n, nbits, tau, seed + 4)
    bound = fresh_bound(d, dp, nbits)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bound)
    ab = as_bytes(a)
    for e in range(n):  # encryption vs the model, bit by bit (bit k = bit k%8 of byte k/8)
        A = bit_ints(la, da, bound, e)
        for k in range(nbits):
            x = (int(ab[e, k // 8]) >> (k % 8)) & 1
            assert A[k] == model.cipher_bit(x, T, bytes(ma[e, k]))
    out = dict(params=np.array(params, dtype=np.uint32), seed=np.array(seed), sk=sk, pk=pk,
               pk_degree=np.asarray(pkdeg, dtype=np.uint32), a_plain=a, b_plain=b,
               a_masks=ma, b_masks=mb, in_bound=bound, a_limbs=la, a_degree=da,
               b_limbs=lb, b_degree=db, op=np.array(op))
    if op.startswith("mullow"):
        k = int(op[len("mullow"):])
        l1, d1, b1 = low_bits(la, da, bound, n, k)
        l2, d2, b2 = low_bits(lb, db, bound, n, k)
        ob = H.mul_out_bounds(b1, b2)
        oracle.set_threads(n)
        lo, do = oracle.mul_batch(l1, d1, b1, l2, d2, b2, k, n, ob)
        oracle.set_threads(1)
        # (K = 20 takes the oracle hours: keep the product before anything else can fail)
        np.savez(os.path.join(HERE, f".{name}_product.npz"), lo=lo, do=do, ob=ob)
        kb = (k + 7) // 8  # decrypted as whole bytes: bits k .. 8 kb - 1 are null polynomials
        pl, pd, pb = pad_bits_host(lo, do, ob, n, 8 * kb)
        dec = oracle.decrypt_batch(sk, pl, pd, pb, 8 * kb, n).reshape(n, kb)
        val = np.zeros(n, dtype=np.uint64)
        for byte in range(kb):
            val |= dec[:, byte].astype(np.uint64) << np.uint64(8 * byte)
        out.update(k=np.array(k), out_bound=ob, out_degree=do,
                   out_sha256=np.array(digest(lo, ob, n)), out_plain=val,
                   expected_plain=(a.astype(np.uint64) * b.astype(np.uint64)) % (1 << k))
        out["model_check"] = np.array(model_check_mullow(out, lo))
    elif op == "encdec":
        dec = oracle.decrypt_batch(sk, la, da, bound, nbits, n).view(dtype).reshape(-1)
        out.update(out_bound=bound, out_limbs=la, out_degree=da, out_plain=dec,
                   expected_plain=a)
    else:
        if op == "add":
            ob = H.add_out_bounds(bound, bound)
            lo, do = oracle.add_batch(la, da, bound, lb, db, bound, nbits, n, ob)
        elif op in ("mul", "smul"):
            ob = H.mul_out_bounds(bound, bound, signed=op == "smul")
            lo, do = oracle.mul_batch(la, da, bound, lb, db, bound, nbits, n, ob,
                                      signed=op == "smul")
        else:
            opcls = {"and": H.HomomorphicAndGate, "or": H.HomomorphicOrGate,
                     "xor": H.HomomorphicXorGate, "not": H.HomomorphicNotGate}[op]
            ob = H.gate_out_bounds(opcls, bound, bound)
            lo, do = oracle.gate_batch(op, la, da, bound, lb, db, bound, nbits, n, ob)
        _check_model(op, la, da, lb, db, bound, lo, do, ob, n)
        dec = oracle.decrypt_batch(sk, lo, do, ob, nbits, n).view(dtype).reshape(-1)
        out.update(out_bound=ob, out_limbs=lo, out_degree=do, out_plain=dec,
                   expected_plain=_plain_result(op, a, b, dtype))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    ok = int(np.sum(out["out_plain"] == out["expected_plain"]))
    print(f"{name}: {os.path.getsize(path)} B, decrypts correctly for {ok}/{n}")


def model_check_saved(name):
    """Model-check an existing low-k multiply fixture against the product its generation saved
    (.NAME_product.npz, not committed: 20 MB at K = 20), without re-running the oracle, and record
    the check in the fixture (`model_check`)."""
    path = os.path.join(HERE, f"{name}.npz")
    z = dict(np.load(path, allow_pickle=False))
    prod = os.path.join(HERE, f".{name}_product.npz")
    lo = np.load(prod, allow_pickle=False)["lo"] if os.path.exists(prod) else None
    z["model_check"] = np.array(model_check_mullow(z, lo))
    np.savez(path, **z)
    print(name, str(z["model_check"]))


if __name__ == "__main__":
    if sys.argv[1:2] == ["--model-check-saved"]:
        for name in sys.argv[2:]:
            model_check_saved(name)
        sys.exit(0)
    oracle.build()
    for name in (sys.argv[1:] or CASES):
        make(name)
