"""Independent GF(2)[X] big-integer model — CPU ORACLE, test infrastructure only.

A second restatement of the reference's mathematics (mathisbot/homomorph-rust) written in a
deliberately different form from oracle/homomorph_oracle.c: a polynomial is a Python int whose
bit k is the coefficient of X^k (the layout of src/polynomial.rs:142-150 / :168-173), products
use shift-and-xor over the smaller operand, remainders use int.bit_length long division, and the
circuits use the algebraic identities of the reference rather than its call sequence.  Used only
by tests/ to cross-check the C oracle on small cases and to make golden fixtures.

Citations (reference file:line):
  keygen            src/context.rs:160-162, :249-261  (S = random(d); T_i = S*Q_i + X*R_i)
  random            src/polynomial.rs:73-96           (fill, mask above degree, force top bit)
  cipher            src/cipher.rs:99-115              (subset sum of T_i, mask bit i = byte[i/8]>>(i%8))
  decipher          src/cipher.rs:119-122             ((C mod S)(0))
  add circuit       src/impls/numbers/common.rs:37-56
  mul circuit       src/impls/numbers/common.rs:66-105 (unsigned), :115-155 (signed)
"""
from __future__ import annotations

MASK64 = (1 << 64) - 1


def splitmix64(state: list[int]) -> int:
    """SplitMix64 — the deterministic stand-in for getrandom (polynomial.rs:87)."""
    state[0] = (state[0] + 0x9E3779B97F4A7C15) & MASK64
    z = state[0]
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
    return z ^ (z >> 31)


def random_poly(degree: int, state: list[int]) -> int:
    n = degree // 64 + 1
    v = 0
    for k in range(n):
        v |= splitmix64(state) << (64 * k)
    v &= (1 << degree) - 1
    return v | (1 << degree)


def clmul(a: int, b: int) -> int:
    if a.bit_count() > b.bit_count():
        a, b = b, a
    r = 0
    while a:
        low = a & -a
        r ^= b << (low.bit_length() - 1)
        a ^= low
    return r


def clmul_fast(a: int, b: int, leaf: int = 1 << 15) -> int:
    """The same product for operands of millions of bits (the golden multiply prefixes): an 8-bit
    window table over the shorter operand below `leaf` bits, Karatsuba above (z1 = (a0+a1)(b0+b1)
    - z0 - z2, exact over GF(2)[X]).  Checked against clmul in tests/test_oracle_circuits.py."""
    la, lb = a.bit_length(), b.bit_length()
    if la > lb:
        a, b, la, lb = b, a, lb, la
    if la <= 64:
        return clmul(a, b)
    if la <= leaf:
        t = [0] * 256
        for i in range(1, 256):
            low = i & -i
            t[i] = t[i ^ low] ^ (b << (low.bit_length() - 1))
        r, sh = 0, 0
        while a:
            r ^= t[a & 255] << sh
            a >>= 8
            sh += 8
        return r
    h = lb // 2
    m = (1 << h) - 1
    if la <= h:  # unbalanced: split the longer operand only
        return clmul_fast(a, b & m, leaf) ^ (clmul_fast(a, b >> h, leaf) << h)
    a0, a1, b0, b1 = a & m, a >> h, b & m, b >> h
    z0, z2 = clmul_fast(a0, b0, leaf), clmul_fast(a1, b1, leaf)
    z1 = clmul_fast(a0 ^ a1, b0 ^ b1, leaf) ^ z0 ^ z2
    return z0 ^ (z1 << h) ^ (z2 << (2 * h))


def residue_int(p: int, g: int) -> int:
    """P mod f, f = X^64 + g (deg g < 64): P = P_hi X^h + P_lo folds to P_hi (X^h mod f) + P_lo,
    halving P's length per fold (X^h mod f by square-and-multiply in the residue ring).  P -> P mod
    f is a ring homomorphism, so a circuit's output residues equal the circuit run on its inputs'
    residues (mul_circuit(..., mul=residue_mul(g))): the model's own form of
    oracle/residue_check.c, for products far too big for the model's circuit itself."""
    mul = residue_mul(g)

    def xpow(e):  # X^e mod f
        r, base = 1, 2
        while e:
            if e & 1:
                r = mul(r, base)
            base = mul(base, base)
            e >>= 1
        return r

    while p.bit_length() > 128:
        h = p.bit_length() // 2
        p = clmul(p >> h, xpow(h)) ^ (p & ((1 << h) - 1))
    return mul(p, 1) if p >> 64 else p


def residue_limbs(limbs, g: int) -> int:
    """residue_int of a polynomial given as little-endian u64 limbs"""
    return residue_int(limbs_to_int(limbs), g)


def residue_mul(g: int):
    """The product of the residue ring GF(2)[X]/(X^64 + g) on reduced operands."""
    def mul(a: int, b: int) -> int:
        t = clmul(a, b)
        while t >> 64:
            t = (t & MASK64) ^ clmul(t >> 64, g)
        return t
    return mul


def gf2_mod(a: int, s: int) -> int:
    if s == 0:
        raise ZeroDivisionError("attempt to divide by zero")
    ds = s.bit_length()
    while a.bit_length() >= ds:
        a ^= s << (a.bit_length() - ds)
    return a


def degree(p: int) -> int:
    """Exact degree; the null polynomial has degree 0 (polynomial.rs:126-137)."""
    return max(p.bit_length() - 1, 0)


def keygen(d: int, dp: int, delta: int, tau: int, seed: int) -> tuple[int, list[int]]:
    st = [seed & MASK64]
    s = random_poly(d, st)
    pk = []
    for _ in range(tau):
        q = random_poly(dp, st)
        r = random_poly(delta, st)
        pk.append(clmul(s, q) ^ (r << 1))
    return s, pk


def cipher_bit(x: int, pk: list[int], mask: bytes) -> int:
    c = 0
    for i, t in enumerate(pk):
        if (mask[i // 8] >> (i % 8)) & 1:
            c ^= t
    return c ^ (x & 1)


def decipher_bit(c: int, s: int) -> int:
    return gf2_mod(c, s) & 1


def add_circuit(a: list[int], b: list[int]) -> list[int]:
    """Ripple carry: s_i = a^b^c, c' = ab + (a^b)(1+ab) c (same polynomial as common.rs:51-52)."""
    out, c = [], 0
    n = min(len(a), len(b))
    for i in range(n):
        x = a[i] ^ b[i]
        out.append(x ^ c)
        if i + 1 < n:
            ab = clmul(a[i], b[i])
            c = ab ^ clmul(clmul(x, ab ^ 1), c)
    return out


def mul_circuit(a: list[int], b: list[int], signed: bool = False, mul=clmul) -> list[int]:
    """The carry-save array of common.rs:66-105 (:115-155 signed).  `mul`: the ring product
    (clmul; clmul_fast for big operands; a product mod f for the residue ring)."""
    clmul_ = mul
    L = len(a)
    pp = [[clmul_(a[j], b[k]) for k in range(L)] for j in range(L)]
    if signed:
        pp[0][L - 1] ^= 1
        pp[L - 1][0] ^= 1
    res = [0] * L
    prev: list[int] = []
    for i in range(L):
        nxt: list[int] = []
        for j in range(i + 1):
            p = pp[j][i - j]
            if i + 1 < L:
                nxt.append(clmul_(p, res[i]))
            res[i] ^= p
        for c in prev:
            if i + 1 < L:
                nxt.append(clmul_(res[i], c))
            res[i] ^= c
        prev = nxt
    return res


def limbs_to_int(limbs) -> int:
    return int.from_bytes(b"".join(int(w).to_bytes(8, "little") for w in limbs), "little")


def int_to_limbs(v: int, cap: int) -> list[int]:
    if v.bit_length() > 64 * cap:
        raise ValueError("capacity")
    return [(v >> (64 * k)) & MASK64 for k in range(cap)]
