"""The reference's own polynomial known-answer tests (src/polynomial.rs:522-590) run directly
through the C ABI's hm_poly_{add,mul,rem}_batch on the GPU, and the ciphertext batch wire format
(include/homomorph_gpu.h) round-tripped through the device."""
import numpy as np
import pytest

from helpers import assert_batches_equal, keys, masks, plain

pytestmark = pytest.mark.gpu
U64MAX = (1 << 64) - 1


@pytest.fixture(scope="module")
def H():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import homomorph
    homomorph.lib()
    return homomorph


@pytest.fixture(scope="module")
def ctx(H):
    c = H.Context(H.Parameters(64, 64, 1, 64))
    c.seed_rng(9)
    c.generate_secret_key()
    c.generate_public_key()
    return c


def _polys(H, ctx, rows, cap):
    a = np.zeros((len(rows), cap), dtype=np.uint64)
    for i, r in enumerate(rows):
        a[i, : len(r)] = np.array(r, dtype=np.uint64)
    return H.Polys.from_host(a, ctx.device)


def _got(p, i):
    l, d = p.to_host()
    return l[i], int(d[i])


def test_kat_add(H, ctx):  # polynomial.rs:522-535
    a = _polys(H, ctx, [[0b1001], [0b1001, 0b1]], 2)
    b = _polys(H, ctx, [[0b0011], [0b0101, 0b1]], 2)
    s = ctx.poly_add(a, b)
    ctx.synchronize()
    l, d = _got(s, 0)
    assert l.tolist() == [0b1010, 0] and d == 3
    l, d = _got(s, 1)
    assert l.tolist() == [0b1100, 0] and d == 3  # equal top limbs cancel; degree recomputed


def test_kat_mul(H, ctx):  # polynomial.rs:537-561
    a = _polys(H, ctx, [[0b1001], [0b111], [U64MAX], [0]], 1)
    b = _polys(H, ctx, [[0b11], [0b11], [0b11], [0b11]], 1)
    m = ctx.poly_mul(a, b)
    ctx.synchronize()
    want = [([0b11011, 0], 4), ([0b1001, 0], 3), ([1, 1], 64), ([0, 0], 0)]
    for i, (limbs, deg) in enumerate(want):
        l, d = _got(m, i)
        assert l.tolist() == limbs and d == deg, (i, l, d)


def test_kat_rem(H, ctx):  # polynomial.rs:563-582
    for num, den, rem in (([0b1001], [0b11], 0), ([0b1], [0b10], 1),
                          ([0b10_1010_1101], [0b11011], 0b1010)):
        r = ctx.poly_rem(_polys(H, ctx, [num], 1), np.array(den, dtype=np.uint64))
        ctx.synchronize()
        l, d = _got(r, 0)
        assert l.tolist() == [rem] and d == max(rem.bit_length() - 1, 0)


def test_kat_rem_zero(H, ctx):  # polynomial.rs:584-590 "attempt to divide by zero"
    with pytest.raises(ZeroDivisionError):
        ctx.poly_rem(_polys(H, ctx, [[0b1001]], 1), np.zeros(1, dtype=np.uint64))


def test_wire_round_trip(H, ctx, oracle):
    """Encrypt -> add -> wire image -> new device batch: bit-identical, decrypts, and the image
    matches the documented byte layout field by field."""
    x, y = plain(50, np.uint16, 1), plain(50, np.uint16, 2)
    s = ctx.apply2(H.HomomorphicAddition, ctx.encrypt(x, masks=masks(50, 16, 64, 3)),
                   ctx.encrypt(y, masks=masks(50, 16, 64, 4)))
    img = s.to_wire(ctx)
    info = H.wire_info(img)
    assert info["nbits"] == 16 and info["n"] == 50 and np.array_equal(info["bound"], s.bound)
    assert img[:4] == b"HMCB" and int.from_bytes(img[4:8], "little") == 1
    assert len(img) == H.lib().hm_wire_bytes(16, H._p32(s.bound), 50)
    back = H.Ciphered.from_wire(ctx, img, np.dtype(np.uint16))
    gl, gd = s.to_host()
    bl, bd = back.to_host()
    assert_batches_equal(bl, bd, gl, gd, s.bound, 50, "wire round trip")
    assert np.array_equal(ctx.decrypt(back), (x + y).astype(np.uint16))
    # the documented layout: degrees after the bounds, limbs 8-byte aligned after the degrees
    doff = 24 + 4 * 16
    assert np.array_equal(np.frombuffer(img, "<u4", 50 * 16, doff), gd)
    loff = (doff + 4 * 50 * 16 + 7) // 8 * 8
    assert np.array_equal(np.frombuffer(img, "<u8", offset=loff), gl)


def test_wire_rejects_corruption(H, ctx):
    c = ctx.encrypt(np.arange(4, dtype=np.uint8), masks=masks(4, 8, 64, 5))
    img = bytearray(c.to_wire(ctx))
    loff = (24 + 4 * 8 + 4 * 32 + 7) // 8 * 8
    bad = bytearray(img)
    bad[loff + 23] ^= 0x80  # coefficient 191 of value 0, bit 0: above any degree <= its bound 128
    with pytest.raises(H.EngineError):
        H.Ciphered.from_wire(ctx, bytes(bad))
    bad = bytearray(img)
    bad[24 + 32] = 0xFF  # degree word of value 0 bit 0 beyond its bound
    with pytest.raises(H.EngineError):
        H.Ciphered.from_wire(ctx, bytes(bad))
    with pytest.raises(H.EngineError):
        H.Ciphered.from_wire(ctx, bytes(img[:-8]))  # truncated
