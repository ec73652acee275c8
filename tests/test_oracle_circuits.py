"""CPU-only checks of the oracle's cipher and circuits.

1. The C oracle (reference call sequence) equals the independent big-int model bit for bit on
   seeded keys / masks / plaintexts (keygen, encrypt, add, carry-save mul, gates).
2. The reference's own round-trip tests hold (src/cipher.rs:275-304,
   src/impls/numbers/uint.rs:108-293, int.rs:247-268): decrypt(op(encrypt(x))) == op(x).
"""
import numpy as np
import pytest

from helpers import as_bytes, bit_ints, fresh_bound, keys, masks, plain
from oracle import gf2_model as model

P_SMALL = (64, 32, 8, 32)   # cipher.rs:277
P_ADD8 = (64, 16, 1, 16)    # uint.rs:179 (u8 add)
P_MUL8 = (128, 64, 1, 64)   # uint.rs:157 (u8 mul)


def _enc(oracle, params, values, seed):
    d, dp, delta, tau = params
    sk, pk, _ = keys(d, dp, delta, tau, seed)
    data = as_bytes(values)
    nbits = data.shape[1] * 8
    m = masks(len(values), nbits, tau, seed + 1)
    bound = fresh_bound(d, dp, nbits)
    limbs, deg = oracle.encrypt_batch(pk, data, m, bound)
    return sk, pk, m, bound, limbs, deg


def test_keygen_matches_model(oracle):
    for params, seed in ((P_SMALL, 1), ((128, 128, 1, 128), 2), ((256, 256, 1, 8), 3)):
        sk, pk, pkdeg = oracle.keygen(*params, seed)
        s, T = model.keygen(*params, seed)
        assert model.limbs_to_int(sk) == s
        assert model.degree(s) == params[0]
        for i, t in enumerate(T):
            assert model.limbs_to_int(pk[i]) == t
            assert pkdeg[i] == model.degree(t) == params[0] + params[1]


@pytest.mark.parametrize("dtype", [np.uint8, np.uint32])
def test_encrypt_matches_model(oracle, dtype):
    vals = plain(16, dtype, 5)
    sk, pk, m, bound, limbs, deg = _enc(oracle, P_SMALL, vals, 11)
    s, T = model.keygen(*P_SMALL, 11)
    nbits = 8 * np.dtype(dtype).itemsize
    for e in range(len(vals)):
        got = bit_ints(limbs, deg, bound, e)
        for k in range(nbits):
            x = (int(vals[e]) >> k) & 1
            assert got[k] == model.cipher_bit(x, T, bytes(m[e, k]))
            assert deg[e * nbits + k] == model.degree(got[k])


def test_cipher_roundtrip(oracle):  # cipher.rs:275-294
    for dtype, v in ((np.uint8, [2]), (np.uint64, [2**64 - 1])):
        vals = np.array(v, dtype=dtype)
        sk, pk, m, bound, limbs, deg = _enc(oracle, P_SMALL, vals, 21)
        assert len(bound) == 8 * np.dtype(dtype).itemsize
        out = oracle.decrypt_batch(sk, limbs, deg, bound, len(bound), 1)
        assert out.view(dtype)[0] == vals[0]


def test_add_matches_model_and_roundtrip(oracle):  # uint.rs:176-208
    vals_a = np.array([22, 255, 0, 127, 1, 200], dtype=np.uint8)
    vals_b = np.array([20, 240, 0, 128, 255, 100], dtype=np.uint8)
    sk, pk, ma, bound, la, da = _enc(oracle, P_ADD8, vals_a, 31)
    _, _, mb, _, lb, db = _enc(oracle, P_ADD8, vals_b, 31)  # same keys (same seed)
    mb2 = masks(len(vals_b), 8, P_ADD8[3], 77)
    lb, db = oracle.encrypt_batch(pk, as_bytes(vals_b), mb2, bound)
    from homomorph import add_out_bounds
    ob = add_out_bounds(bound, bound)
    lo, do = oracle.add_batch(la, da, bound, lb, db, bound, 8, len(vals_a), ob)
    dec = oracle.decrypt_batch(sk, lo, do, ob, 8, len(vals_a)).view(np.uint8).reshape(-1)
    assert np.array_equal(dec, (vals_a.astype(int) + vals_b.astype(int)) % 256)
    for e in range(len(vals_a)):
        ref = model.add_circuit(bit_ints(la, da, bound, e), bit_ints(lb, db, bound, e))
        assert bit_ints(lo, do, ob, e) == ref


def test_mul_matches_model_and_roundtrip(oracle):  # uint.rs:254-293
    vals_a = np.array([6, 0, 255, 13], dtype=np.uint8)
    vals_b = np.array([7, 151, 240, 11], dtype=np.uint8)
    d, dp, delta, tau = P_MUL8
    sk, pk, _ = keys(d, dp, delta, tau, 41)
    bound = fresh_bound(d, dp, 8)
    la, da = oracle.encrypt_batch(pk, as_bytes(vals_a), masks(4, 8, tau, 1), bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(vals_b), masks(4, 8, tau, 2), bound)
    from homomorph import mul_out_bounds
    ob = mul_out_bounds(bound, bound)
    lo, do = oracle.mul_batch(la, da, bound, lb, db, bound, 8, 4, ob)
    dec = oracle.decrypt_batch(sk, lo, do, ob, 8, 4).view(np.uint8).reshape(-1)
    assert np.array_equal(dec, (vals_a.astype(int) * vals_b.astype(int)) % 256)
    for e in range(2):
        ref = model.mul_circuit(bit_ints(la, da, bound, e), bit_ints(lb, db, bound, e))
        assert bit_ints(lo, do, ob, e) == ref


def test_signed_mul_roundtrip(oracle):  # int.rs:247-268 (6 * -7 = -42 at (512,64,1,64))
    d, dp, delta, tau = 512, 64, 1, 64
    sk, pk, _ = keys(d, dp, delta, tau, 51)
    bound = fresh_bound(d, dp, 8)
    a = np.array([6, 0], dtype=np.int8)
    b = np.array([-7, -100], dtype=np.int8)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), masks(2, 8, tau, 1), bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), masks(2, 8, tau, 2), bound)
    from homomorph import mul_out_bounds
    ob = mul_out_bounds(bound, bound, signed=True)
    lo, do = oracle.mul_batch(la, da, bound, lb, db, bound, 8, 2, ob, signed=True)
    dec = oracle.decrypt_batch(sk, lo, do, ob, 8, 2).view(np.int8).reshape(-1)
    assert dec.tolist() == [-42, 0]
    ref = model.mul_circuit(bit_ints(la, da, bound, 0), bit_ints(lb, db, bound, 0), signed=True)
    assert bit_ints(lo, do, ob, 0) == ref


@pytest.mark.parametrize("op,f", [("and", lambda x, y: x & y), ("or", lambda x, y: x | y),
                                  ("xor", lambda x, y: x ^ y), ("not", lambda x, y: ~x & 0xFF)])
def test_gates_roundtrip(oracle, op, f):  # uint.rs:108-174 at (32, 8, 8, 8) / (32,16,16,16)
    params = (32, 8, 8, 8) if op in ("and", "or") else (32, 16, 16, 16)
    d, dp, delta, tau = params
    sk, pk, _ = keys(d, dp, delta, tau, 61)
    bound = fresh_bound(d, dp, 8)
    a = np.array([0b1010, 0b1100], dtype=np.uint8)
    b = np.array([0b1100, 0b1010], dtype=np.uint8)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), masks(2, 8, tau, 1), bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), masks(2, 8, tau, 2), bound)
    import homomorph as H
    opcls = {"and": H.HomomorphicAndGate, "or": H.HomomorphicOrGate,
             "xor": H.HomomorphicXorGate, "not": H.HomomorphicNotGate}[op]
    ob = H.gate_out_bounds(opcls, bound, bound)
    lo, do = oracle.gate_batch(op, la, da, bound, lb, db, bound, 8, 2, ob)
    dec = oracle.decrypt_batch(sk, lo, do, ob, 8, 2).reshape(-1)
    assert dec.tolist() == [f(int(x), int(y)) for x, y in zip(a, b)]


@pytest.mark.parametrize("signed", [False, True])
def test_mul_low_bits_identity(oracle, signed):
    """output bits 0..k-1 of the L-bit carry-save multiplier equal the
    k-bit unsigned circuit on the low k input bits (common.rs:66-155: column i reads only input
    bits <= i; the signed flips live in column L-1)."""
    from helpers import low_bits
    d, dp, delta, tau = 32, 8, 1, 8
    sk, pk, _ = keys(d, dp, delta, tau, 71)
    n, L, k = 2, 16, 8
    bound = fresh_bound(d, dp, L)
    a, b = plain(n, np.uint16, 1), plain(n, np.uint16, 2)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), masks(n, L, tau, 3), bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), masks(n, L, tau, 4), bound)
    from homomorph import mul_out_bounds
    ob = mul_out_bounds(bound, bound, signed)
    lo, do = oracle.mul_batch(la, da, bound, lb, db, bound, L, n, ob, signed=signed)
    la8, da8, b8 = low_bits(la, da, bound, n, k)
    lb8, db8, _ = low_bits(lb, db, bound, n, k)
    ob8 = mul_out_bounds(b8, b8)
    assert np.array_equal(ob8, ob[:k])
    l8, d8 = oracle.mul_batch(la8, da8, b8, lb8, db8, b8, k, n, ob8)
    got_l, got_d, _ = low_bits(lo, do, ob, n, k)
    assert np.array_equal(got_d, d8) and np.array_equal(got_l, l8)


def test_model_fast_product_and_residues():
    """The model's big-operand tools used by the golden multiply prefixes (make_golden.py):
    clmul_fast (window + Karatsuba) equals clmul, residue_int equals long division by X^64 + g,
    and residue_mul is the product of the residue ring."""
    rng = np.random.default_rng(71)
    for la, lb in ((1, 1), (63, 200), (1000, 1000), (40000, 70000), (100000, 30)):
        a = int.from_bytes(rng.bytes(la // 8 + 1), "little") >> (7 - la % 8)
        b = int.from_bytes(rng.bytes(lb // 8 + 1), "little") >> (7 - lb % 8)
        assert model.clmul_fast(a, b) == model.clmul(a, b), (la, lb)
    g = int(rng.integers(0, 2**63)) | 1
    f = (1 << 64) ^ g
    for n in (5, 64, 65, 129, 3000):
        p = int.from_bytes(rng.bytes(n // 8 + 1), "little")
        assert model.residue_int(p, g) == model.gf2_mod(p, f), n
    x, y = int.from_bytes(rng.bytes(300), "little"), int.from_bytes(rng.bytes(200), "little")
    mul = model.residue_mul(g)
    assert mul(model.gf2_mod(x, f), model.gf2_mod(y, f)) == model.gf2_mod(model.clmul(x, y), f)
