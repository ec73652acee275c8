"""Pin the CPU oracle to every known-answer test the reference holds for the hot path.

Each case is the reference's own KAT (src/polynomial.rs:433-612), run through BOTH CPU
restatements: the C oracle (oracle/homomorph_oracle.c, operation-for-operation) and the
independent Python big-int model (oracle/gf2_model.py).
"""
import numpy as np
import pytest

U64MAX = (1 << 64) - 1


def test_compute_degree(oracle):  # polynomial.rs:439-449
    assert oracle.compute_degree([0b10010]) == 4
    assert oracle.compute_degree([0b10010, 0b1]) == 64
    assert oracle.compute_degree([0b10010, 0b0]) == 4
    assert oracle.compute_degree([0]) == 0


def test_eq(oracle):  # :451-472
    assert oracle.poly_eq([0b1001], [0b1001])
    p = [0b1001, 0b1000_0011_0101_1010, 0b0, 0b1, 0b0]
    assert oracle.poly_eq(p, list(p))
    assert oracle.poly_eq([0b1001], [0b1001, 0b0])
    assert not oracle.poly_eq([0b1001], [0b1000])
    assert not oracle.poly_eq([0b1000, 0b10, 0b0], [0b1000, 0b0, 0b0])


def test_monomial_layout(oracle, model):  # :474-487 — X^k is bit k%64 of limb k/64
    for k in (5, 63, 64):
        limbs = [0] * (k // 64 + 1)
        limbs[k // 64] = 1 << (k % 64)
        assert oracle.compute_degree(limbs) == k
        assert model.limbs_to_int(limbs) == 1 << k


def test_random(oracle):  # :489-496
    from oracle.oracle_py import lib
    import ctypes
    st = ctypes.c_uint64(7)
    for deg in (5, 64, 128, 255):
        out = np.zeros(deg // 64 + 1, dtype=np.uint64)
        lib().oracle_poly_random(deg, ctypes.byref(st), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)))
        assert oracle.compute_degree(out) == deg


def test_evaluate(oracle):  # :511-520
    assert not oracle.poly_evaluate([0b1001], True)
    assert oracle.poly_evaluate([0b1001], False)
    assert oracle.poly_evaluate([0b1111_00010, 0b1001], True)
    assert not oracle.poly_evaluate([0b1111_00010, 0b1001], False)


def test_add(oracle, model):  # :522-535
    out, _ = oracle.poly_add([0b1001], [0b0011])
    assert list(out) == [0b1010]
    out, deg = oracle.poly_add([0b1001, 0b1], [0b0101, 0b1])
    assert list(out) == [0b1100, 0b0]  # buffer keeps max_deg/64+1 limbs
    assert deg == 3
    assert model.limbs_to_int([0b1001, 1]) ^ model.limbs_to_int([0b0101, 1]) == 0b1100


def test_mul(oracle, model):  # :537-561
    assert list(oracle.poly_mul([0b1001], [0b11])[0]) == [0b11011]
    assert list(oracle.poly_mul([0b111], [0b11])[0]) == [0b1001]
    assert list(oracle.poly_mul([U64MAX], [0b11])[0]) == [0b1, 0b1]
    out, deg = oracle.poly_mul([0], [0b11])  # null short-circuit
    assert list(out) == [0] and deg == 0
    assert model.clmul(0b1001, 0b11) == 0b11011
    assert model.clmul(0b111, 0b11) == 0b1001
    assert model.clmul(U64MAX, 0b11) == (1 << 64) | 1


def test_rem(oracle, model):  # :563-582
    out, deg = oracle.poly_rem([0b1001], [0b11])
    assert list(out) == [0] and deg < 1
    out, deg = oracle.poly_rem([0b1], [0b10])
    assert list(out) == [1] and deg < 1
    out, deg = oracle.poly_rem([0b10_1010_1101], [0b11011])
    assert list(out) == [0b1010] and deg < 4
    assert model.gf2_mod(0b10_1010_1101, 0b11011) == 0b1010


def test_rem_zero(oracle):  # :584-590 "attempt to divide by zero"
    with pytest.raises(oracle.OracleError, match="status 4"):
        oracle.poly_rem([0b1001], [0])


def test_rem_by_one_guarded(oracle):  # the reference never terminates here (:330-343)
    with pytest.raises(oracle.OracleError, match="status 5"):
        oracle.poly_rem([0b1001], [1])


def test_new_empty(oracle):  # :433-437 "must not be empty"
    with pytest.raises(oracle.OracleError):
        oracle.poly_add([], [1])


def test_random_cross_model(oracle, model):
    """Random polynomials: C oracle (bit-serial mul, long division) == big-int model."""
    rng = np.random.default_rng(1234)
    for _ in range(200):
        na, nb = rng.integers(1, 9, size=2)
        a = rng.integers(0, 2**63, size=na, dtype=np.uint64) * 2 + rng.integers(0, 2, size=na, dtype=np.uint64)
        b = rng.integers(0, 2**63, size=nb, dtype=np.uint64) * 2 + rng.integers(0, 2, size=nb, dtype=np.uint64)
        ia, ib = model.limbs_to_int(a), model.limbs_to_int(b)
        prod, deg = oracle.poly_mul(a, b)
        assert model.limbs_to_int(prod) == model.clmul(ia, ib)
        assert deg == (model.degree(model.clmul(ia, ib)))
        s, _ = oracle.poly_add(a, b)
        assert model.limbs_to_int(s) == ia ^ ib
        if ib > 1:
            r, rdeg = oracle.poly_rem(a, b)
            assert model.limbs_to_int(r) == model.gf2_mod(ia, ib)
            assert rdeg == model.degree(model.gf2_mod(ia, ib))
