"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle, bit-exact.

Every test feeds identical seeded keys, masks and plaintexts to both sides and compares exact
degrees and every limb (src/polynomial.rs:417-426 equality; limbs above the degree are zero on
both sides).  Sizes are those the oracle finishes in seconds; the full-size configurations are
covered by size-independent properties in test_gpu_properties.py.
"""
import numpy as np
import pytest

from helpers import as_bytes, assert_batches_equal, fresh_bound, keys, masks, plain

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import homomorph
    homomorph.lib()  # loud failure if the engine is not built
    return homomorph


def make_ctx(H, params, seed):
    ctx = H.Context(H.Parameters(*params))
    ctx.seed_rng(seed)
    ctx.generate_secret_key()
    ctx.generate_public_key()
    return ctx


# ------------------------------------------------------------------ polynomial primitives
def _rand_polys(rng, n, cap, maxdeg=None):
    out = np.zeros((n, cap), dtype=np.uint64)
    for i in range(n):
        deg = int(rng.integers(0, 64 * cap)) if maxdeg is None else int(rng.integers(0, maxdeg + 1))
        kind = rng.integers(0, 8)
        if kind == 0:
            continue  # null polynomial
        if kind == 1:
            out[i, 0] = 1  # the unit
            continue
        nl = deg // 64 + 1
        out[i, :nl] = rng.integers(0, 2**64, size=nl, dtype=np.uint64)
        out[i, nl - 1] &= np.uint64((1 << (deg % 64)) - 1) if deg % 64 else np.uint64(0)
        out[i, nl - 1] |= np.uint64(1 << (deg % 64))
    return out


@pytest.mark.parametrize("ca,cb", [(1, 1), (5, 5), (3, 17), (40, 2), (200, 9), (400, 400)])
def test_poly_mul_add(H, oracle, ca, cb):
    import torch
    rng = np.random.default_rng(ca * 1000 + cb)
    n = 64
    A, B = _rand_polys(rng, n, ca), _rand_polys(rng, n, cb)
    ctx = make_ctx(H, (64, 64, 1, 64), 1)
    dev = ctx.device
    pa, pb = H.Polys.from_host(A, dev), H.Polys.from_host(B, dev)
    pm = ctx.poly_mul(pa, pb)
    ps = ctx.poly_add(pa, pb)
    ctx.synchronize()
    ml, md = pm.to_host()
    sl, sd = ps.to_host()
    for i in range(n):
        ref, rdeg = oracle.poly_mul(A[i], B[i])
        assert md[i] == rdeg, (i, md[i], rdeg)
        w = min(len(ref), ml.shape[1])
        assert np.array_equal(ml[i, :w], ref[:w]) and not ml[i, w:].any()
        ref, rdeg = oracle.poly_add(A[i], B[i])
        assert sd[i] == rdeg
        w = min(len(ref), sl.shape[1])
        assert np.array_equal(sl[i, :w], ref[:w]) and not sl[i, w:].any()


@pytest.mark.parametrize("cap,sdeg", [(1, 1), (3, 128), (20, 128), (9, 63), (9, 64), (50, 700),
                                      (369, 128), (512, 256), (4, 300),
                                      # dividends past the 512 limbs held in registers: configs[4]'s
                                      # add outputs (737 limbs) and multiplier-sized ones
                                      (737, 256), (3000, 700),
                                      # divisor near / far above every dividend's degree (the
                                      # remainder is the dividend; no table is built)
                                      (20, 1279), (4, 5000)])
def test_poly_rem(H, oracle, cap, sdeg):
    rng = np.random.default_rng(cap + sdeg)
    A = _rand_polys(rng, 64, cap)
    S = _rand_polys(rng, 1, sdeg // 64 + 1, maxdeg=sdeg)[0]
    S[sdeg // 64] |= np.uint64(1 << (sdeg % 64))
    ctx = make_ctx(H, (64, 64, 1, 64), 2)
    pr = ctx.poly_rem(H.Polys.from_host(A, ctx.device), S)
    ctx.synchronize()
    rl, rd = pr.to_host()
    for i in range(len(A)):
        ref, rdeg = oracle.poly_rem(A[i], S)
        assert rd[i] == rdeg
        assert np.array_equal(rl[i, : len(ref)], ref) and not rl[i, len(ref):].any()


def test_poly_rem_table_cache(H, oracle):
    """The remainder table is cached per (divisor, dividend capacity): a second call with the same
    divisor reuses it, and a different divisor of the same length or a wider dividend rebuilds it."""
    rng = np.random.default_rng(404)
    ctx = make_ctx(H, (64, 64, 1, 64), 2)
    S1 = _rand_polys(rng, 1, 3, maxdeg=150)[0]
    S1[150 // 64] |= np.uint64(1 << (150 % 64))
    S2 = S1.copy()
    S2[0] ^= np.uint64(0b1010)
    for S, cap in ((S1, 9), (S1, 9), (S2, 9), (S2, 30), (S1, 9)):
        A = _rand_polys(rng, 32, cap)
        pr = ctx.poly_rem(H.Polys.from_host(A, ctx.device), S)
        ctx.synchronize()
        rl, rd = pr.to_host()
        for i in range(len(A)):
            ref, rdeg = oracle.poly_rem(A[i], S)
            assert rd[i] == rdeg
            assert np.array_equal(rl[i, : len(ref)], ref) and not rl[i, len(ref):].any()
    # a graph captured on S1's cached table refuses to replay once S2 rewrote the table in place
    # (the rewrite keeps the buffer, so the generation must advance)
    A = H.Polys.from_host(_rand_polys(rng, 32, 9), ctx.device)
    g = ctx.graph(lambda: ctx.poly_rem(A, S1))
    g.replay()
    ctx.synchronize()
    ctx.poly_rem(A, S2)
    ctx.synchronize()
    with pytest.raises(H.EngineError):
        g.replay()


def test_poly_rem_errors(H):
    ctx = make_ctx(H, (64, 64, 1, 64), 3)
    p = H.Polys.from_host(np.ones((2, 2), dtype=np.uint64), ctx.device)
    with pytest.raises(ZeroDivisionError):
        ctx.poly_rem(p, np.zeros(1, dtype=np.uint64))
    with pytest.raises(H.EngineError):
        ctx.poly_rem(p, np.ones(1, dtype=np.uint64))


# ------------------------------------------------------------------ keys and cipher
@pytest.mark.parametrize("params", [(64, 32, 8, 32), (128, 128, 1, 128), (256, 256, 1, 256),
                                    (64, 64, 1, 64), (100, 27, 3, 40)])
def test_keygen_parity(H, oracle, params):
    ctx = make_ctx(H, params, 99)
    sk, pk, _ = keys(*params, 99)
    assert np.array_equal(ctx.get_secret_key().limbs, sk)
    assert np.array_equal(ctx.get_public_key().limbs, pk)


@pytest.mark.parametrize("params,dtype", [((64, 32, 8, 32), np.uint8), ((128, 128, 1, 128), np.uint32),
                                          ((256, 256, 1, 256), np.uint32), ((64, 64, 1, 64), np.uint8),
                                          ((100, 27, 3, 40), np.uint16), ((128, 128, 64, 128), np.uint64)])
def test_encrypt_decrypt_parity(H, oracle, params, dtype):
    d, dp, delta, tau = params
    ctx = make_ctx(H, params, 7)
    sk, pk, _ = keys(*params, 7)
    n = 96
    vals = plain(n, dtype, 8)
    nbits = 8 * np.dtype(dtype).itemsize
    m = masks(n, nbits, tau, 9)
    c = ctx.encrypt(vals, masks=m)
    dec = ctx.decrypt(c)
    ctx.synchronize()
    gl, gd = c.to_host()
    bound = fresh_bound(d, dp, nbits)
    rl, rd = oracle.encrypt_batch(pk, as_bytes(vals), m, bound)
    assert_batches_equal(gl, gd, rl, rd, bound, n, "encrypt")
    assert np.array_equal(dec, vals)
    rdec = oracle.decrypt_batch(sk, rl, rd, bound, nbits, n).view(dtype).reshape(-1)
    assert np.array_equal(rdec, dec)


def test_decrypt_errors(H):
    ctx = H.Context(H.Parameters(64, 32, 8, 32))
    with pytest.raises(H.ContextCryptoError):
        ctx.encrypt(np.array([1], dtype=np.uint8))  # public key unset
    ctx.seed_rng(1)
    ctx.generate_secret_key()
    ctx.generate_public_key()
    c = ctx.encrypt(np.array([3], dtype=np.uint8))
    sk = ctx.get_secret_key()
    ctx.set_secret_key(sk)
    assert ctx.get_public_key() is None  # context.rs:656-667
    assert ctx.decrypt(c)[0] == 3


# ------------------------------------------------------------------ circuits
def _pair(H, ctx, params, dtype, n, seed, lo=None, hi=None):
    d, dp, delta, tau = params
    nbits = 8 * np.dtype(dtype).itemsize
    a = plain(n, dtype, seed, lo, hi)
    b = plain(n, dtype, seed + 1, lo, hi)
    ma, mb = masks(n, nbits, tau, seed + 2), masks(n, nbits, tau, seed + 3)
    return a, b, ma, mb, ctx.encrypt(a, masks=ma), ctx.encrypt(b, masks=mb)


@pytest.mark.parametrize("chain", ["auto", "mfma", "valu"])
@pytest.mark.parametrize("params,dtype,n", [((64, 64, 1, 64), np.uint8, 128),
                                            ((64, 64, 1, 64), np.uint32, 32),
                                            ((128, 128, 1, 128), np.uint32, 7),
                                            ((64, 16, 1, 16), np.uint8, 64),
                                            ((128, 128, 1, 128), np.uint32, 24),
                                            ((128, 128, 4, 128), np.uint16, 32),
                                            ((256, 256, 1, 256), np.uint32, 4),
                                            ((256, 128, 1, 128), np.uint64, 2)])
def test_add_parity(H, oracle, params, dtype, n, chain):
    """Both carry chains (fp4 MFMA Toeplitz products and VALU XORs) against the oracle.  "auto"
    and "mfma" run the MFMA chain: 13 chunks where P_i fits 25 words (d + dp <= 256), 25 chunks
    up to 49 words (d + dp = 512 here)."""
    d, dp, delta, tau = params
    ctx = make_ctx(H, params, 17)
    ctx.set_add_options(chain)
    sk, pk, _ = keys(*params, 17)
    a, b, ma, mb, ca, cb = _pair(H, ctx, params, dtype, n, 18)
    cs = ctx.apply2(H.HomomorphicAddition, ca, cb)
    dec = ctx.decrypt(cs)
    ctx.synchronize()
    nbits = 8 * np.dtype(dtype).itemsize
    bound = fresh_bound(d, dp, nbits)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bound)
    ob = H.add_out_bounds(bound, bound)
    assert np.array_equal(cs.bound, ob)
    rl, rd = oracle.add_batch(la, da, bound, lb, db, bound, nbits, n, ob)
    gl, gd = cs.to_host()
    assert_batches_equal(gl, gd, rl, rd, ob, n, "add")
    # decryption parity always; the plaintext sum only where the scheme's noise allows it
    # ((64,64,1,64) u32 and (128,128,4,128) u16 exceed the noise budget in the reference too)
    rdec = oracle.decrypt_batch(sk, rl, rd, ob, nbits, n).view(dtype).reshape(-1)
    assert np.array_equal(dec, rdec)
    if params in {(64, 16, 1, 16), (128, 128, 1, 128), (256, 256, 1, 256), (256, 128, 1, 128)}:
        assert np.array_equal(dec, (a + b).astype(dtype))


@pytest.mark.parametrize("chain", ["mfma", "valu"])
def test_add_edge_values(H, oracle, chain):
    """Wrap-around and extremes (uint.rs:202-208: 255 + 240 = 239), zero, all-ones; the zero
    operands give null P_i and null carries (the MFMA chain's copy-ab branch)."""
    params = (128, 128, 1, 128)
    ctx = make_ctx(H, params, 5)
    ctx.set_add_options(chain)
    sk, pk, _ = keys(*params, 5)
    a = np.array([0, 0xFFFFFFFF, 0xFFFFFFFF, 255, 1, 0x80000000], dtype=np.uint32)
    b = np.array([0, 1, 0xFFFFFFFF, 240, 0, 0x80000000], dtype=np.uint32)
    n = len(a)
    ma, mb = masks(n, 32, 128, 1), masks(n, 32, 128, 2)
    mb[0] = 0  # an all-zero subset: encryption of 0 is the null polynomial
    cs = ctx.apply2(H.HomomorphicAddition, ctx.encrypt(a, masks=ma), ctx.encrypt(b, masks=mb))
    dec = ctx.decrypt(cs)
    ctx.synchronize()
    bound = fresh_bound(128, 128, 32)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bound)
    ob = H.add_out_bounds(bound, bound)
    rl, rd = oracle.add_batch(la, da, bound, lb, db, bound, 32, n, ob)
    gl, gd = cs.to_host()
    assert_batches_equal(gl, gd, rl, rd, ob, n, "add edges")
    assert np.array_equal(dec, (a.astype(np.uint64) + b) .astype(np.uint32))


@pytest.mark.parametrize("chain", ["auto", "mfma", "valu"])
@pytest.mark.parametrize("skew", ["random", "last_bit_wide"])
def test_add_skewed_bounds(H, oracle, chain, skew):
    """Non-uniform per-bit input bounds (capacities above the fresh degree, different for every
    bit and operand).  "random" keeps P_i within 25 words, so the MFMA chain runs; "last_bit_wide"
    gives only the last bit a 1100-degree capacity (x_{L-1} of 35 words, past the 32 sum words
    the MFMA chain XORs x into): the engine must pick the VALU chain on "auto" and refuse a forced
    MFMA chain, never drop x's upper words."""
    params = (64, 64, 1, 64)
    d, dp, delta, tau = params
    ctx = make_ctx(H, params, 71)
    ctx.set_add_options(chain)
    sk, pk, _ = keys(*params, 71)
    n, nbits = 16, 8
    rng = np.random.default_rng(72 if skew == "random" else 73)
    if skew == "random":
        ba = rng.integers(d + dp, 2 * (d + dp) + 1, size=nbits).astype(np.uint32)
        bb = rng.integers(d + dp, 2 * (d + dp) + 1, size=nbits).astype(np.uint32)
    else:
        ba = np.full(nbits, d + dp, dtype=np.uint32)
        bb = ba.copy()
        ba[-1] = 1100
    a, b = plain(n, np.uint8, 74), plain(n, np.uint8, 75)
    ma, mb = masks(n, nbits, tau, 76), masks(n, nbits, tau, 77)
    ca, cb = ctx.encrypt(a, masks=ma, bound=ba), ctx.encrypt(b, masks=mb, bound=bb)
    if chain == "mfma" and skew == "last_bit_wide":
        with pytest.raises(H.EngineError):
            ctx.apply2(H.HomomorphicAddition, ca, cb)
            ctx.synchronize()
        return
    cs = ctx.apply2(H.HomomorphicAddition, ca, cb)
    dec = ctx.decrypt(cs)
    ctx.synchronize()
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, ba)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bb)
    ob = H.add_out_bounds(ba, bb)
    rl, rd = oracle.add_batch(la, da, ba, lb, db, bb, nbits, n, ob)
    gl, gd = cs.to_host()
    assert_batches_equal(gl, gd, rl, rd, ob, n, f"skewed add {skew}/{chain}")
    rdec = oracle.decrypt_batch(sk, rl, rd, ob, nbits, n).reshape(-1)
    assert np.array_equal(dec, rdec)


@pytest.mark.parametrize("skew", ["uniform", "per_bit"])
def test_add_prep_top_word_copies(H, oracle, skew):
    """The prep's top-word copies (AddArgs.top1): when the largest input bound is a multiple of 32
    and shorter rows save waves or row passes, the multiplier words that hold only that bit are
    added as shifted copies instead of product rows.  Uniform bounds of 256: a batch of 4096
    takes that path (4 waves per value, one pass) and a batch of 1024 does not (8 waves per
    value): the first 1024 sums must be identical bit for bit, and 16 values equal the oracle's.
    Per-bit bounds of 256, 288 or 320 check the same batch split where the host's choice
    differs (fresh ciphertexts never set those top words)."""
    params = (128, 128, 1, 128)
    ctx = make_ctx(H, params, 161)
    sk, pk, _ = keys(*params, 161)
    rng = np.random.default_rng(162)
    if skew == "uniform":
        ba = bb = np.full(32, 256, dtype=np.uint32)
    else:
        ba = rng.choice([256, 288, 320], size=32).astype(np.uint32)
        bb = rng.choice([256, 288, 320], size=32).astype(np.uint32)
    n, m = 4096, 1024
    a, b = plain(n, np.uint32, 163), plain(n, np.uint32, 164)
    ma, mb = masks(n, 32, 128, 165), masks(n, 32, 128, 166)
    ca, cb = ctx.encrypt(a, masks=ma, bound=ba), ctx.encrypt(b, masks=mb, bound=bb)
    big = ctx.apply2(H.HomomorphicAddition, ca, cb)
    small = ctx.apply2(H.HomomorphicAddition, H.value_slice(ca, 0, m), H.value_slice(cb, 0, m))
    ctx.synchronize()
    gl, gd = H.value_slice(big, 0, m).to_host()
    sl, sd = small.to_host()
    assert_batches_equal(gl, gd, sl, sd, big.bound, m, f"top-word copies ({skew}) vs product rows")
    k = 16
    la, da = oracle.encrypt_batch(pk, as_bytes(a[:k]), ma[:k], ba)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b[:k]), mb[:k], bb)
    rl, rd = oracle.add_batch(la, da, ba, lb, db, bb, 32, k, big.bound)
    gl, gd = H.value_slice(big, 0, k).to_host()
    assert_batches_equal(gl, gd, rl, rd, big.bound, k, f"top-word copies ({skew}) vs oracle")


@pytest.mark.parametrize("params", [(64, 64, 1, 64), (32, 32, 1, 32)])
def test_add_prep_values_per_wave(H, oracle, params):
    """The prep with several whole values per wave (AddArgs.vpw: u8 values, a batch of at least
    16,384; 2 values per wave at d = d' = 64, 4 at 32): the same adds at a batch of 1024 run one
    value per wave, and the first 1024 sums must be identical bit for bit; 16 values equal the
    oracle's, and a batch whose last wave holds fewer values (16,387) agrees too."""
    d, dp, delta, tau = params
    ctx = make_ctx(H, params, 171)
    sk, pk, _ = keys(*params, 171)
    n, m = 16387, 1024
    a, b = plain(n, np.uint8, 172), plain(n, np.uint8, 173)
    ma, mb = masks(n, 8, tau, 174), masks(n, 8, tau, 175)
    ca, cb = ctx.encrypt(a, masks=ma), ctx.encrypt(b, masks=mb)
    big = ctx.apply2(H.HomomorphicAddition, ca, cb)
    small = ctx.apply2(H.HomomorphicAddition, H.value_slice(ca, 0, m), H.value_slice(cb, 0, m))
    tail = ctx.apply2(H.HomomorphicAddition, H.value_slice(ca, n - 3, n), H.value_slice(cb, n - 3, n))
    dec = ctx.decrypt(big)
    ctx.synchronize()
    gl, gd = H.value_slice(big, 0, m).to_host()
    sl, sd = small.to_host()
    assert_batches_equal(gl, gd, sl, sd, big.bound, m, f"values per wave {params} vs one per wave")
    gl, gd = H.value_slice(big, n - 3, n).to_host()
    tl, td = tail.to_host()
    assert_batches_equal(gl, gd, tl, td, big.bound, 3, f"values per wave {params}: batch tail")
    k = 16
    bound = fresh_bound(d, dp, 8)
    la, da = oracle.encrypt_batch(pk, as_bytes(a[:k]), ma[:k], bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b[:k]), mb[:k], bound)
    rl, rd = oracle.add_batch(la, da, bound, lb, db, bound, 8, k, big.bound)
    gl, gd = H.value_slice(big, 0, k).to_host()
    assert_batches_equal(gl, gd, rl, rd, big.bound, k, f"values per wave {params} vs oracle")
    rdec = oracle.decrypt_batch(sk, rl, rd, big.bound, 8, k).reshape(-1)
    assert np.array_equal(dec[:k], rdec)


@pytest.mark.parametrize("n", [2048, 2051])
def test_add_pipeline_same_bits(H, n):
    """hm_ctx_set_add_pipeline: an add as two stream-pipelined halves writes the same ciphertexts
    as the one-pass add (the halves use disjoint workspace and outputs), also for a batch whose
    halves are not multiples of the block's 4 values, and for two pipelined adds in a row (the
    second reuses the stream and events the first created)."""
    params = (128, 128, 1, 128)
    ctx = make_ctx(H, params, 77)
    ca = ctx.encrypt(plain(n, np.uint32, 78))
    cb = ctx.encrypt(plain(n, np.uint32, 79))
    one = ctx.apply2(H.HomomorphicAddition, ca, cb)
    ctx.set_add_pipeline(True)
    two = ctx.apply2(H.HomomorphicAddition, ca, cb)
    three = ctx.apply2(H.HomomorphicAddition, cb, ca)
    ctx.synchronize()
    l1, d1 = one.to_host()
    for c in (two, three):
        l2, d2 = c.to_host()
        assert_batches_equal(l1, d1, l2, d2, one.bound, n, "pipelined add")


def test_add_chain_mfma_unsupported(H):
    """A forced MFMA chain on a plan whose P_i exceeds 49 words (d + dp = 1024: 97 words) is
    refused, not approximated."""
    params = (768, 256, 1, 64)
    ctx = make_ctx(H, params, 3)
    ctx.set_add_options("mfma")
    a = ctx.encrypt(np.array([1, 2], dtype=np.uint8), masks=masks(2, 8, 64, 1))
    with pytest.raises(H.EngineError):
        ctx.apply2(H.HomomorphicAddition, a, a)
        ctx.synchronize()


def test_no_fp4_mfma_fallback(H, oracle, monkeypatch):
    """A context on a device without the gfx950 fp4 MFMA (forced with the HM_TEST_NO_FP4_MFMA=1
    hook, read at context creation): the AUTO strategies take the VALU carry chain and the VALU
    products, bit-exact against the oracle, and an explicit MFMA request is HM_ERR_UNSUPPORTED
    (the products at the setter, the chain at the add)."""
    from homomorph import _lib
    monkeypatch.setenv("HM_TEST_NO_FP4_MFMA", "1")
    params = (128, 128, 1, 128)
    ctx = make_ctx(H, params, 61)
    monkeypatch.delenv("HM_TEST_NO_FP4_MFMA")
    sk, pk, _ = keys(*params, 61)
    with pytest.raises(H.EngineError) as e:
        ctx.set_mul_products("mfma")
    assert e.value.status == _lib.ERR_UNSUPPORTED
    n = 4
    a, b, ma, mb, ca, cb = _pair(H, ctx, params, np.uint8, n, 62)
    bound = fresh_bound(128, 128, 8)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bound)
    cs = ctx.apply2(H.HomomorphicAddition, ca, cb)
    cp = ctx.apply2(H.HomomorphicMultiplication, ca, cb)
    ctx.synchronize()
    ob = H.add_out_bounds(bound, bound)
    rl, rd = oracle.add_batch(la, da, bound, lb, db, bound, 8, n, ob)
    assert_batches_equal(*cs.to_host(), rl, rd, ob, n, "VALU-fallback add")
    ob = H.mul_out_bounds(bound, bound)
    rl, rd = oracle.mul_batch(la, da, bound, lb, db, bound, 8, n, ob)
    assert_batches_equal(*cp.to_host(), rl, rd, ob, n, "VALU-fallback mul")
    assert np.array_equal(ctx.decrypt(cs), (a.astype(int) + b).astype(np.uint8))
    ctx.set_add_options("mfma")
    with pytest.raises(H.EngineError) as e:
        ctx.apply2(H.HomomorphicAddition, ca, cb)
        ctx.synchronize()
    assert e.value.status == _lib.ERR_UNSUPPORTED
    # a context created without the hook on the same device uses the matrix cores again
    ctx2 = make_ctx(H, params, 61)
    ctx2.set_mul_products("mfma")


def test_successive_add(H, oracle):
    """uint.rs:225-252 — an add whose inputs are add outputs (non-fresh bounds)."""
    params = (256, 128, 1, 128)
    ctx = make_ctx(H, params, 23)
    sk, pk, _ = keys(*params, 23)
    n = 4
    a, b, ma, mb, ca, cb = _pair(H, ctx, params, np.uint8, n, 24, 0, 127)
    c = plain(n, np.uint8, 30, 0, 127)
    mc = masks(n, 8, 128, 31)
    cc = ctx.encrypt(c, masks=mc)
    d1 = ctx.apply2(H.HomomorphicAddition, ca, cb)
    d2 = ctx.apply2(H.HomomorphicAddition, d1, cc)
    dec = ctx.decrypt(d2)
    ctx.synchronize()
    assert np.array_equal(dec, (a.astype(int) + b + c).astype(np.uint8))
    bound = fresh_bound(256, 128, 8)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bound)
    lc, dc = oracle.encrypt_batch(pk, as_bytes(c), mc, bound)
    b1 = H.add_out_bounds(bound, bound)
    r1l, r1d = oracle.add_batch(la, da, bound, lb, db, bound, 8, n, b1)
    b2 = H.add_out_bounds(b1, bound)
    r2l, r2d = oracle.add_batch(r1l, r1d, b1, lc, dc, bound, 8, n, b2)
    gl, gd = d2.to_host()
    assert_batches_equal(gl, gd, r2l, r2d, b2, n, "successive add")


@pytest.mark.parametrize("params,dtype,n,signed", [((128, 64, 1, 64), np.uint8, 8, False),
                                                   ((128, 128, 1, 128), np.uint8, 4, False),
                                                   ((512, 64, 1, 64), np.int8, 4, True),
                                                   ((64, 32, 1, 32), np.uint16, 2, False)])
def test_mul_parity(H, oracle, params, dtype, n, signed):
    d, dp, delta, tau = params
    ctx = make_ctx(H, params, 41)
    sk, pk, _ = keys(*params, 41)
    a, b, ma, mb, ca, cb = _pair(H, ctx, params, dtype, n, 42)
    cp = ctx.apply2(H.HomomorphicMultiplication, ca, cb)
    dec = ctx.decrypt(cp)
    ctx.synchronize()
    nbits = 8 * np.dtype(dtype).itemsize
    bound = fresh_bound(d, dp, nbits)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bound)
    ob = H.mul_out_bounds(bound, bound, signed)
    rl, rd = oracle.mul_batch(la, da, bound, lb, db, bound, nbits, n, ob, signed=signed)
    gl, gd = cp.to_host()
    assert_batches_equal(gl, gd, rl, rd, ob, n, "mul")
    rdec = oracle.decrypt_batch(sk, rl, rd, ob, nbits, n).view(dtype).reshape(-1)
    assert np.array_equal(dec, rdec)
    if params != (64, 32, 1, 32):  # the reference's own mul parameters decrypt correctly
        assert np.array_equal(dec, (a.astype(np.int64) * b).astype(dtype))


@pytest.mark.parametrize("op", ["and", "or", "xor", "not"])
def test_gate_parity(H, oracle, op):
    params = (32, 8, 8, 8) if op in ("and", "or") else (32, 16, 16, 16)
    d, dp, delta, tau = params
    ctx = make_ctx(H, params, 61)
    sk, pk, _ = keys(*params, 61)
    n = 64
    a, b, ma, mb, ca, cb = _pair(H, ctx, params, np.uint16, n, 62)
    opcls = {"and": H.HomomorphicAndGate, "or": H.HomomorphicOrGate,
             "xor": H.HomomorphicXorGate, "not": H.HomomorphicNotGate}[op]
    co = ctx.apply1(opcls, ca) if op == "not" else ctx.apply2(opcls, ca, cb)
    dec = ctx.decrypt(co)
    ctx.synchronize()
    bound = fresh_bound(d, dp, 16)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bound)
    rl, rd = oracle.gate_batch(op, la, da, bound, lb, db, bound, 16, n, co.bound)
    gl, gd = co.to_host()
    assert_batches_equal(gl, gd, rl, rd, co.bound, n, op)
    f = {"and": np.bitwise_and, "or": np.bitwise_or, "xor": np.bitwise_xor}
    ref = ~a if op == "not" else f[op](a, b)
    assert np.array_equal(dec, ref)


def test_operation_requirements(H):
    """Context::apply2 validation (context.rs:310-323): add needs d >= 21 delta."""
    ctx = make_ctx(H, (64, 32, 8, 32), 3)
    c = ctx.encrypt(np.array([1, 2], dtype=np.uint8))
    with pytest.raises(H.OperationError) as ei:
        ctx.apply2(H.HomomorphicAddition, c, c)
    assert ei.value.required_min_d_over_delta == 21
    assert ei.value.actual_d == 64 and ei.value.actual_delta == 8
    with pytest.raises(H.OperationError):
        ctx.apply2(H.HomomorphicMultiplication, c, c)
    ctx.apply2(H.HomomorphicXorGate, c, c)  # d/delta = 8 >= 1


def test_bad_input_is_flagged(H):
    """A degree word that disagrees with the limbs is reported (device-side check)."""
    import torch
    ctx = make_ctx(H, (64, 64, 1, 64), 4)
    c = ctx.encrypt(np.array([5, 6], dtype=np.uint8), masks=masks(2, 8, 64, 1))
    ctx.synchronize()
    d0 = int(c.degree[0, 3])
    c.degree[0, 3] = d0 + 1 if d0 < 128 else d0 - 1  # wrong either way: top bit / stray bits
    ctx.apply2(H.HomomorphicAddition, c, c)
    with pytest.raises(H.EngineError):
        ctx.synchronize()


@pytest.mark.parametrize("k,n", [(8, 4), (12, 2)])
def test_mul_low_parity(H, oracle, k, n):
    """u32 multiply, low k result bits at the bench parameters: the GPU
    reads the low k bits of u32 ciphertexts in place; the oracle runs the k-bit circuit on them."""
    from helpers import low_bits
    params = (128, 128, 1, 128)
    ctx = make_ctx(H, params, 81)
    sk, pk, _ = keys(*params, 81)
    a, b, ma, mb, ca, cb = _pair(H, ctx, params, np.uint32, n, 82)
    cp = ctx.mul_low(ca, cb, k)
    dec_bytes = ctx.decrypt_bytes(cp).cpu().numpy() if k % 8 == 0 else None
    ctx.synchronize()
    bound = fresh_bound(128, 128, 32)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bound)
    lak, dak, bk = low_bits(la, da, bound, n, k)
    lbk, dbk, _ = low_bits(lb, db, bound, n, k)
    ob = H.mul_out_bounds(bk, bk)
    assert np.array_equal(cp.bound, ob)
    rl, rd = oracle.mul_batch(lak, dak, bk, lbk, dbk, bk, k, n, ob)
    gl, gd = cp.to_host()
    assert_batches_equal(gl, gd, rl, rd, ob, n, f"mul low {k}")
    if dec_bytes is not None:
        rdec = oracle.decrypt_batch(sk, rl, rd, ob, k, n).reshape(n, -1)
        assert np.array_equal(dec_bytes, rdec)
        want = ((a.astype(np.uint64) * b) & ((1 << k) - 1)).astype(np.uint64)
        got = dec_bytes.astype(np.uint64) @ (256 ** np.arange(k // 8, dtype=np.uint64))
        assert np.array_equal(got, want)


@pytest.mark.parametrize("products", ["mfma", "valu"])
@pytest.mark.parametrize("ka_min,leaf", [(32, 32), (64, 96), (128, 256), (256, 512)])
def test_mul_karatsuba_parity(H, oracle, ka_min, leaf, products):
    """The Karatsuba carry products (hm_ctx_set_mul_options) forced down
    to small sizes, their leaves on the fp4 matrix cores or as VALU XORs (hm_ctx_set_mul_products):
    u8 multiply and the u32 low-12 prefix, bit-exact vs the oracle's bit-serial products, and equal
    to the schoolbook-only engine (karatsuba_min_words = 0)."""
    from helpers import low_bits
    params = (128, 128, 1, 128)
    ctx = make_ctx(H, params, 91)
    ctx.set_mul_options(ka_min, leaf)
    ctx.set_mul_products(products)
    sk, pk, _ = keys(*params, 91)
    bound = fresh_bound(128, 128, 32)
    # u8: products up to ~450 words
    a, b, ma, mb, ca, cb = _pair(H, ctx, params, np.uint8, 4, 92)
    cp = ctx.apply2(H.HomomorphicMultiplication, ca, cb)
    ctx.synchronize()
    b8 = fresh_bound(128, 128, 8)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, b8)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, b8)
    rl, rd = oracle.mul_batch(la, da, b8, lb, db, b8, 8, 4, cp.bound)
    gl, gd = cp.to_host()
    assert_batches_equal(gl, gd, rl, rd, cp.bound, 4, f"u8 karatsuba {ka_min}/{leaf}")
    # u32, low 12 result bits: products up to ~2500 words, several recursion levels
    a, b, ma, mb, ca, cb = _pair(H, ctx, params, np.uint32, 2, 93)
    cp = ctx.mul_low(ca, cb, 12)
    ctx.synchronize()
    la, da = oracle.encrypt_batch(pk, as_bytes(a), ma, bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), mb, bound)
    lak, dak, bk = low_bits(la, da, bound, 2, 12)
    lbk, dbk, _ = low_bits(lb, db, bound, 2, 12)
    rl, rd = oracle.mul_batch(lak, dak, bk, lbk, dbk, bk, 12, 2, cp.bound)
    gl, gd = cp.to_host()
    assert_batches_equal(gl, gd, rl, rd, cp.bound, 2, f"u32 low-12 karatsuba {ka_min}/{leaf}")
    ctx.set_mul_options(0, 256)  # schoolbook only: the same bits
    cs = ctx.mul_low(ca, cb, 12)
    ctx.synchronize()
    sl, sd = cs.to_host()
    assert_batches_equal(sl, sd, gl, gd, cp.bound, 2, "schoolbook vs karatsuba")


def test_mul_karatsuba_low16_matches_schoolbook(H):
    """At the bench's K = 16 (products up to ~28k words, 6-7 recursion levels) the default
    Karatsuba path and the schoolbook-only path give identical ciphertexts (the K = 16 golden
    fixture pins the default path to the oracle, tests/test_golden.py)."""
    params = (128, 128, 1, 128)
    ctx = make_ctx(H, params, 95)
    x = plain(3, np.uint32, 96)
    ca, cb = ctx.encrypt(x), ctx.encrypt(x[::-1].copy())
    ka = ctx.mul_low(ca, cb, 16)
    ctx.synchronize()
    ctx.set_mul_products("valu")
    kv = ctx.mul_low(ca, cb, 16)
    ctx.synchronize()
    ctx.set_mul_options(0, 256)
    sb = ctx.mul_low(ca, cb, 16)
    ctx.synchronize()
    kl, kd = ka.to_host()
    vl, vd = kv.to_host()
    sl, sd = sb.to_host()
    assert_batches_equal(kl, kd, vl, vd, ka.bound, 3, "K=16 MFMA leaves vs VALU leaves")
    assert_batches_equal(kl, kd, sl, sd, ka.bound, 3, "K=16 karatsuba vs schoolbook")


@pytest.mark.parametrize("chain", ["mfma", "valu"])
def test_add_output_capacity_is_checked(H, chain):
    """An add into outputs whose static bounds are below the circuit's (sum bits of degree up to
    (3i-1)D) never truncates silently: the engine refuses the batch or flags HM_ERR_CAPACITY, on
    both carry chains (the MFMA chain stores sum words from its tiles and checks the degree once
    per bit)."""
    params = (64, 64, 1, 64)
    ctx = make_ctx(H, params, 41)
    ctx.set_add_options(chain)
    n = 4
    a, b = plain(n, np.uint8, 42), plain(n, np.uint8, 43)
    ca = ctx.encrypt(a, masks=masks(n, 8, 64, 44))
    cb = ctx.encrypt(b, masks=masks(n, 8, 64, 45))
    small = np.minimum(H.add_out_bounds(ca.bound, cb.bound), 200).astype(np.uint32)
    out = H.Ciphered.empty(n, small, ca.limbs.device, np.dtype(np.uint8))
    with pytest.raises(H.EngineError):
        H.add_into(ctx, ca, cb, out)
        ctx.synchronize()


def _u128(rng, n):
    """n random u128 plaintexts as Python ints and as their bincode fixint LE images (n, 16)."""
    vals = [int.from_bytes(rng.bytes(16), "little") for _ in range(n)]
    img = np.frombuffer(b"".join(v.to_bytes(16, "little") for v in vals), dtype=np.uint8)
    return vals, img.reshape(n, 16).copy()


@pytest.mark.parametrize("op", ["add", "and", "or", "xor", "not"])
def test_u128_parity(H, oracle, op):
    """u128, the widest type the reference implements (uint.rs:58, 77): add and the gates on
    128-bit ciphertexts, bit-exact vs the oracle, plaintexts as (n, 16) byte images."""
    params = (64, 16, 1, 16)
    d, dp, delta, tau = params
    # a key with S(0) = 0: every output decrypts to the plaintext result whatever its noise
    seed = next(s for s in range(128, 1000) if not int(keys(*params, s)[0][0]) & 1)
    ctx = make_ctx(H, params, seed)
    sk, pk, _ = keys(*params, seed)
    n = 4
    rng = np.random.default_rng(129)
    av, ai = _u128(rng, n)
    bv, bi = _u128(rng, n)
    ma, mb = masks(n, 128, tau, 130), masks(n, 128, tau, 131)
    ca, cb = ctx.encrypt(ai, masks=ma), ctx.encrypt(bi, masks=mb)
    opcls = {"add": H.HomomorphicAddition, "and": H.HomomorphicAndGate, "or": H.HomomorphicOrGate,
             "xor": H.HomomorphicXorGate, "not": H.HomomorphicNotGate}[op]
    co = ctx.apply1(opcls, ca) if op == "not" else ctx.apply2(opcls, ca, cb)
    dec = ctx.decrypt_bytes(co).cpu().numpy()
    ctx.synchronize()
    bound = fresh_bound(d, dp, 128)
    la, da = oracle.encrypt_batch(pk, ai, ma, bound)
    lb, db = oracle.encrypt_batch(pk, bi, mb, bound)
    if op == "add":
        rl, rd = oracle.add_batch(la, da, bound, lb, db, bound, 128, n, co.bound)
    else:
        rl, rd = oracle.gate_batch(op, la, da, bound, lb, db, bound, 128, n, co.bound)
    gl, gd = co.to_host()
    assert_batches_equal(gl, gd, rl, rd, co.bound, n, f"u128 {op}")
    rdec = oracle.decrypt_batch(sk, rl, rd, co.bound, 128, n)
    assert np.array_equal(dec, rdec)
    M = (1 << 128) - 1
    f = {"add": lambda x, y: (x + y) & M, "and": lambda x, y: x & y, "or": lambda x, y: x | y,
         "xor": lambda x, y: x ^ y, "not": lambda x, y: ~x & M}[op]
    want = [f(x, y) for x, y in zip(av, bv)]
    got = [int.from_bytes(bytes(r), "little") for r in dec]
    assert got == want
