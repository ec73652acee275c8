"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle regenerates every fixture bit for bit from its seed (keygen RNG contract,
encryption with the stored masks, the circuit, the decryption).
GPU: the HIP engine, fed the fixture's keys and input ciphertexts through the C ABI, reproduces
the stored outputs bit for bit (and encrypts the stored masks to the stored ciphertexts).
"""
import glob
import os

import numpy as np
import pytest

from helpers import as_bytes, assert_batches_equal, digest, low_bits, pad_bits_host

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = sorted(os.path.splitext(os.path.basename(p))[0]
                  for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def nbits_n(g):
    return int(g["in_bound"].size), int(g["a_plain"].size)


def test_fixtures_present():
    assert len(FIXTURES) >= 10, FIXTURES


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_reproduces_golden(oracle, name):
    g = load(name)
    d, dp, delta, tau = (int(x) for x in g["params"])
    sk, pk, pkdeg = oracle.keygen(d, dp, delta, tau, int(g["seed"]))
    assert np.array_equal(sk, g["sk"]) and np.array_equal(pk, g["pk"])
    assert np.array_equal(np.asarray(pkdeg, dtype=np.uint32), g["pk_degree"])
    nbits, n = nbits_n(g)
    bound = g["in_bound"]
    la, da = oracle.encrypt_batch(pk, as_bytes(g["a_plain"]), g["a_masks"], bound)
    assert_batches_equal(la, da, g["a_limbs"], g["a_degree"], bound, n, name + " encrypt a")
    lb, db = oracle.encrypt_batch(pk, as_bytes(g["b_plain"]), g["b_masks"], bound)
    assert_batches_equal(lb, db, g["b_limbs"], g["b_degree"], bound, n, name + " encrypt b")
    op, ob = str(g["op"]), g["out_bound"]
    if op.startswith("mullow"):  # low k bits of the u32 multiply: degrees + per-value SHA-256
        k = int(g["k"])
        if k >= 20 and os.environ.get("HM_SLOW_GOLDEN") != "1":
            # ~30 CPU-minutes per value: the inputs were re-checked above; the product is
            # regenerated only on request (make_golden.py made it with this oracle)
            pytest.skip("K >= 20 oracle regeneration takes ~30 min per value (HM_SLOW_GOLDEN=1)")
        l1, d1, b1 = low_bits(la, da, bound, n, k)
        l2, d2, b2 = low_bits(lb, db, bound, n, k)
        oracle.set_threads(n)
        try:
            lo, do = oracle.mul_batch(l1, d1, b1, l2, d2, b2, k, n, ob)
        finally:
            oracle.set_threads(1)
        assert np.array_equal(do, g["out_degree"])
        assert digest(lo, ob, n) == [str(x) for x in g["out_sha256"]]
        kb = (k + 7) // 8
        _check_mullow_plain(g, oracle.decrypt_batch(sk, *pad_bits_host(lo, do, ob, n, 8 * kb), 8 * kb, n),
                            k, n)
        return
    if op == "add":
        lo, do = oracle.add_batch(la, da, bound, lb, db, bound, nbits, n, ob)
    elif op in ("mul", "smul"):
        lo, do = oracle.mul_batch(la, da, bound, lb, db, bound, nbits, n, ob, signed=op == "smul")
    elif op == "encdec":
        lo, do = la, da
    else:
        lo, do = oracle.gate_batch(op, la, da, bound, lb, db, bound, nbits, n, ob)
    assert_batches_equal(lo, do, g["out_limbs"], g["out_degree"], ob, n, name + " " + op)
    dec = oracle.decrypt_batch(sk, lo, do, ob, nbits, n).reshape(-1)
    assert np.array_equal(dec, g["out_plain"].view(np.uint8).reshape(-1))
    assert np.array_equal(g["out_plain"], g["expected_plain"])  # the scheme decrypts correctly


def _check_mullow_plain(g, dec, k, n):
    """The decryption matches the fixture's (oracle) decryption; at d = 128 the scheme's noise
    outgrows the key in the deep columns of the multiplier, so only the low result bits decrypt
    to a*b (the ciphertexts are bit-exact either way)."""
    kb = (k + 7) // 8  # (k % 8 != 0: decrypted through null pad bits)
    dec = np.asarray(dec).reshape(n, kb)
    val = np.zeros(n, dtype=np.uint64)
    for byte in range(kb):
        val |= dec[:, byte].astype(np.uint64) << np.uint64(8 * byte)
    assert np.array_equal(val, g["out_plain"])
    assert np.array_equal(val & 0xFF, g["expected_plain"] & 0xFF)


@pytest.mark.parametrize("name", [f for f in FIXTURES if f.startswith("mullow")])
def test_mullow_fixture_model_cross_check(name):
    """The low-k multiply fixtures rest on the oracle AND the independent big-int model: at
    generation every value's output residues were checked by the model (make_golden.py
    model_check_mullow, recorded as `model_check`), and for k <= 16 the model's own carry-save
    circuit reproduces value 0's degrees and SHA-256 here (~20 s)."""
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden
    g = load(name)
    rec = str(g.get("model_check", ""))
    assert "model residues" in rec and "all" in rec, rec
    if int(g["k"]) <= 16:
        assert "model circuit" in make_golden.model_check_mullow(g, values=(0,))


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_gpu_reproduces_golden(name):
    import homomorph as H
    g = load(name)
    d, dp, delta, tau = (int(x) for x in g["params"])
    nbits, n = nbits_n(g)
    ctx = H.Context(H.Parameters(d, dp, delta, tau), device="cuda:0")
    ctx.set_secret_key(H.SecretKey(g["sk"]))
    ctx.set_public_key(H.PublicKey(g["pk"]))
    dtype = g["a_plain"].dtype
    bound = g["in_bound"]
    enc = ctx.encrypt(g["a_plain"], masks=g["a_masks"])
    gl, gd = enc.to_host()
    assert_batches_equal(gl, gd, g["a_limbs"], g["a_degree"], bound, n, name + " gpu encrypt")
    a = H.Ciphered.from_host(g["a_limbs"], g["a_degree"], bound, n, "cuda:0", dtype)
    b = H.Ciphered.from_host(g["b_limbs"], g["b_degree"], bound, n, "cuda:0", dtype)
    op = str(g["op"])
    if op.startswith("mullow"):
        k = int(g["k"])
        out = ctx.mul_low(a, b, k)
        assert np.array_equal(out.bound, g["out_bound"])
        ol, od = out.to_host()
        assert np.array_equal(od, g["out_degree"]), name + " gpu degrees"
        assert digest(ol, out.bound, n) == [str(x) for x in g["out_sha256"]], name + " gpu limbs"
        _check_mullow_plain(g, ctx.decrypt_bytes(H.pad_bits(out, 8 * ((k + 7) // 8))).cpu().numpy(), k, n)
        return
    if op == "encdec":
        out = a
    elif op == "add":
        out = ctx.apply2(H.HomomorphicAddition, a, b)
    elif op in ("mul", "smul"):
        out = ctx.apply2(H.HomomorphicMultiplication, a, b, signed=op == "smul")
    elif op == "not":
        out = ctx.apply1(H.HomomorphicNotGate, a)
    else:
        opcls = {"and": H.HomomorphicAndGate, "or": H.HomomorphicOrGate,
                 "xor": H.HomomorphicXorGate}[op]
        out = ctx.apply2(opcls, a, b)
    assert np.array_equal(out.bound, g["out_bound"])
    ol, od = out.to_host()
    assert_batches_equal(ol, od, g["out_limbs"], g["out_degree"], out.bound, n, name + " gpu")
    dec = ctx.decrypt(out, dtype)
    assert np.array_equal(dec, g["out_plain"])
