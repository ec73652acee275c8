"""The residue checksum (oracle/residue_check.c) that the full-size GPU tests rely on.

P -> P mod f (f = X^64 + g) is a ring homomorphism GF(2)[X] -> GF(2)[X]/(f), so a circuit's
output residues equal the circuit run on the input residues.  These CPU tests pin the checker
itself: against the independent big-int model (oracle/gf2_model.py), against the oracle's
products, and on every golden fixture (whose outputs the oracle made); a corrupted output must
fail it.
"""
import glob
import os

import numpy as np
import pytest

from helpers import as_bytes, low_bits

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
G = [0x1B, 0x9E3779B97F4A7C15, (1 << 63) | 12345, 0xFFFFFFFFFFFFFFFF]


def _mod(model, p, g):
    return model.gf2_mod(p, (1 << 64) | g)


@pytest.mark.parametrize("g", G)
def test_residue_matches_model(oracle, model, g):
    rng = np.random.default_rng(g & 0xFFFF)
    for cap in (1, 2, 5, 40):
        limbs = rng.integers(0, 2**64, size=cap, dtype=np.uint64)
        assert oracle.residue_of(limbs, g) == _mod(model, model.limbs_to_int(limbs), g)
    for _ in range(50):
        a, b = (int(x) for x in rng.integers(0, 2**64, size=2, dtype=np.uint64))
        assert oracle.residue_mulmod(a, b, g) == _mod(model, model.clmul(a, b), g)


@pytest.mark.parametrize("g", G[:2])
def test_residue_is_a_ring_homomorphism(oracle, g):
    rng = np.random.default_rng(3)
    for ca, cb in ((1, 1), (3, 7), (20, 33)):
        A = rng.integers(0, 2**64, size=ca, dtype=np.uint64)
        B = rng.integers(0, 2**64, size=cb, dtype=np.uint64)
        prod, _ = oracle.poly_mul(A, B)
        assert oracle.residue_of(prod, g) == oracle.residue_mulmod(
            oracle.residue_of(A, g), oracle.residue_of(B, g), g)


def _load(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


FIXTURES = sorted(p for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(p).startswith(("mullow", "encdec")))


@pytest.mark.parametrize("path", FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_residue_circuits_on_golden(oracle, path):
    """Every golden output polynomial's residue = the residue circuit on the golden inputs, for
    three moduli; one flipped output bit is caught."""
    g_ = _load(path)
    op, bound, ob = str(g_["op"]), g_["in_bound"], g_["out_bound"]
    nbits, n = int(bound.size), int(g_["a_plain"].size)
    for g in G[:3]:
        ra, bad_a = oracle.residues(g_["a_limbs"], g_["a_degree"], bound, nbits, n, g)
        rb, bad_b = oracle.residues(g_["b_limbs"], g_["b_degree"], bound, nbits, n, g)
        ro, bad_o = oracle.residues(g_["out_limbs"], g_["out_degree"], ob, nbits, n, g)
        assert bad_a == bad_b == bad_o == 0
        if op == "add":
            want = oracle.residue_add(ra, rb, g)
        elif op in ("mul", "smul"):
            want = oracle.residue_mul(ra, rb, nbits, g, signed=op == "smul")
        else:
            want = oracle.residue_gate(op, ra, None if op == "not" else rb, g)
        assert np.array_equal(ro, want), op
    bad = g_["out_limbs"].copy()
    bad[len(bad) // 2] ^= np.uint64(1 << 17)
    rbad, _ = oracle.residues(bad, None, ob, nbits, n, G[0])
    ra, _ = oracle.residues(g_["a_limbs"], None, bound, nbits, n, G[0])
    rb, _ = oracle.residues(g_["b_limbs"], None, bound, nbits, n, G[0])
    if op == "add":
        want = oracle.residue_add(ra, rb, G[0])
    elif op in ("mul", "smul"):
        want = oracle.residue_mul(ra, rb, nbits, G[0], signed=op == "smul")
    else:
        want = oracle.residue_gate(op, ra, None if op == "not" else rb, G[0])
    assert not np.array_equal(rbad, want)


def test_residue_mul_low_bits(oracle):
    """The k-bit circuit on the low k input residues = the residues of the oracle's k-bit
    product on the low k input bits (the mul_low contract)."""
    from helpers import fresh_bound, keys, masks, plain
    params, n, k = (64, 64, 1, 64), 3, 6
    sk, pk, _ = keys(*params, 5)
    bound = fresh_bound(64, 64, 16)
    a, b = plain(n, np.uint16, 6), plain(n, np.uint16, 7)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), masks(n, 16, 64, 8), bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), masks(n, 16, 64, 9), bound)
    lak, dak, bk = low_bits(la, da, bound, n, k)
    lbk, dbk, _ = low_bits(lb, db, bound, n, k)
    import homomorph as H
    ob = H.mul_out_bounds(bk, bk)
    lo, do = oracle.mul_batch(lak, dak, bk, lbk, dbk, bk, k, n, ob)
    g = G[1]
    ra, _ = oracle.residues(la, da, bound, 16, n, g)
    rb, _ = oracle.residues(lb, db, bound, 16, n, g)
    ro, bad = oracle.residues(lo, do, ob, k, n, g)
    assert bad == 0
    assert np.array_equal(ro, oracle.residue_mul(ra, rb, k, g))
