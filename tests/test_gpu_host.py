"""GPU tests of the context's host contracts: CSPRNG keys and masks, loaded keys of unusual
shape (context.rs:555-595 examples), captured-graph validity across buffer changes."""
import numpy as np
import pytest

from helpers import as_bytes, assert_batches_equal, masks, plain, seeded_random_bytes, seeded_value_masks

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def H():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    import homomorph
    homomorph.lib()
    return homomorph


def test_random_bytes_match_chacha20_contract(H):
    """Seeded contexts draw masks from ChaCha20 keyed by SplitMix64(seed ^ K); each draw
    advances the device nonce (tests/helpers.py restates the generator)."""
    ctx = H.Context(H.Parameters(128, 128, 1, 128))
    ctx.seed_rng(1234)
    r0 = ctx.random_bytes(1000).cpu().numpy()
    r1 = ctx.random_bytes(1000).cpu().numpy()
    assert np.array_equal(r0, seeded_random_bytes(1234, 0, 1000))
    assert np.array_equal(r1, seeded_random_bytes(1234, 1, 1000))
    big = ctx.random_bytes(1 << 20).cpu().numpy()
    assert np.array_equal(big[:4096], seeded_random_bytes(1234, 2, 4096))
    # roughly uniform bytes
    counts = np.bincount(big, minlength=256)
    assert counts.min() > 3500 and counts.max() < 4700


def test_unseeded_keys_and_masks_are_fresh(H):
    """Without seed_rng, keys come from getrandom and masks from an OS-keyed stream: two
    contexts never agree, and two encryptions of one value differ (polynomial.rs:73-96,
    cipher.rs:92-97)."""
    p = H.Parameters(128, 128, 1, 128)
    c1, c2 = H.Context(p), H.Context(p)
    for c in (c1, c2):
        c.generate_secret_key()
        c.generate_public_key()
    assert not np.array_equal(c1.get_secret_key().limbs, c2.get_secret_key().limbs)
    assert not np.array_equal(c1.random_bytes(64).cpu().numpy(), c2.random_bytes(64).cpu().numpy())
    x = np.arange(64, dtype=np.uint32)
    e1, e2 = c1.encrypt(x), c1.encrypt(x)
    assert not np.array_equal(e1.limbs.cpu().numpy(), e2.limbs.cpu().numpy())
    assert np.array_equal(c1.decrypt(e1), x) and np.array_equal(c1.decrypt(e2), x)


@pytest.mark.parametrize("params,dtype,n", [((64, 64, 1, 64), np.uint16, 40),
                                            ((128, 128, 1, 128), np.uint32, 41),
                                            ((128, 128, 1, 128), np.uint32, 40000)])
def test_engine_masks_reproduce_with_seed(H, oracle, params, dtype, n):
    """Engine-drawn masks under a seed are the seeded ChaCha20 bytes: the oracle, fed those
    bytes, produces the identical ciphertexts.  At tau = 128 the masks are drawn inside the
    encryption kernel (encrypt_chacha_kernel: 256 bits per wave, a partial last slice at
    n = 41; n = 40000 takes several grid strides, checked on sampled values); the second
    encryption uses the next nonce."""
    ctx = H.Context(H.Parameters(*params))
    ctx.seed_rng(77)
    ctx.generate_secret_key()
    ctx.generate_public_key()
    nbits = 8 * np.dtype(dtype).itemsize
    pk = ctx.get_public_key().limbs
    for draw in range(2):
        x = plain(n, dtype, 3 + draw)
        c = ctx.encrypt(x)  # draw `draw` of this context
        ctx.synchronize()
        idx = np.arange(n) if n <= 64 else np.array([0, 1, 7, 8191, 8192, 12345, 32767, 32768, n - 1])
        m = seeded_value_masks(77, draw, idx, nbits, ctx.mask_bytes())
        rl, rd = oracle.encrypt_batch(pk, as_bytes(x[idx]), m, c.bound)
        gl, gd = c.to_host()
        gl = gl.reshape(n, -1)[idx].reshape(-1)
        gd = gd.reshape(n, -1)[idx].reshape(-1)
        assert_batches_equal(gl, gd, rl, rd, c.bound, len(idx), f"engine-mask encrypt, draw {draw}")
        assert np.array_equal(ctx.decrypt(c), x)


def test_loaded_secret_key_of_high_degree(H, oracle):
    """context.rs:555-571 example: SecretKey::from_bytes(&[5, 14, 8]) (degree 19) in a
    (6, 3, 2, 5) context.  Public-key rows widen to deg S + dp and the fresh bound follows, so
    encrypt -> decrypt round-trips (the scheme: C mod S = X*sum(R) + x for deg S > delta + 1)."""
    ctx = H.Context(H.Parameters(6, 3, 2, 5))
    ctx.seed_rng(5)
    ctx.set_secret_key(H.SecretKey.from_bytes(bytes([5, 14, 8])))
    assert ctx.get_public_key() is None          # setting sk clears pk (context.rs:568-571)
    ctx.generate_public_key()
    pk = ctx.get_public_key().limbs
    assert max(H._deg(r) for r in pk) == 19 + 3
    assert ctx.fresh_bound() == 22
    x = np.arange(200, dtype=np.uint8)
    m = masks(200, 8, 5, 9)
    c = ctx.encrypt(x, masks=m)
    assert np.array_equal(ctx.decrypt(c), x)
    rl, rd = oracle.encrypt_batch(pk, as_bytes(x), m, c.bound)
    gl, gd = c.to_host()
    assert_batches_equal(gl, gd, rl, rd, c.bound, 200, "encrypt under a loaded key")


def test_loaded_public_key_with_fewer_rows(H, oracle):
    """context.rs:580-595 example: a 3-row public key in a tau = 5 context.  Masks are
    ceil(3/8) = 1 byte per bit (CipheredBit::cipher takes tau = pk.len(), cipher.rs:101-103)."""
    ctx = H.Context(H.Parameters(6, 3, 2, 5))
    pk = H.PublicKey.from_bytes([bytes([4, 7, 5]), bytes([1, 2, 3]), bytes([5, 4, 6])])
    ctx.set_public_key(pk)
    assert ctx.mask_bytes() == 1
    x = np.arange(32, dtype=np.uint8)
    m = masks(32, 8, 3, 1)
    c = ctx.encrypt(x, masks=m)
    rl, rd = oracle.encrypt_batch(pk.limbs, as_bytes(x), m, c.bound)
    gl, gd = c.to_host()
    assert_batches_equal(gl, gd, rl, rd, c.bound, 32, "encrypt with a 3-row key")
    with pytest.raises(ValueError):
        ctx.encrypt(x, masks=masks(32, 8, 5 * 8, 1))  # sized for the wrong tau


def test_graph_refuses_replay_after_buffer_change(H):
    """A captured graph holds raw buffer pointers: after the context grows a workspace (a
    bigger batch) the old graph must not replay (hm_ctx_generation)."""
    ctx = H.Context(H.Parameters(128, 128, 1, 128))
    ctx.seed_rng(3)
    ctx.generate_secret_key()
    ctx.generate_public_key()
    a = ctx.encrypt(np.arange(8, dtype=np.uint32))
    out = H.Ciphered.empty(8, H.add_out_bounds(a.bound, a.bound), ctx.device, np.dtype(np.uint32))
    g = ctx.graph(lambda: H.add_into(ctx, a, a, out))
    g.replay()
    ctx.synchronize()
    assert np.array_equal(ctx.decrypt(out), 2 * np.arange(8, dtype=np.uint32))
    big = ctx.encrypt(np.arange(512, dtype=np.uint32))
    ctx.apply2(H.HomomorphicAddition, big, big)  # grows the adder workspace
    ctx.synchronize()
    with pytest.raises(H.EngineError):
        g.replay()
    g2 = ctx.graph(lambda: H.add_into(ctx, a, a, out))  # a fresh capture is fine
    g2.replay()
    ctx.synchronize()
    assert np.array_equal(ctx.decrypt(out), 2 * np.arange(8, dtype=np.uint32))


def test_apply1_is_in_place_and_apply_n_runs_user_ops(H, oracle):
    """Context::apply1 mutates its argument (src/context.rs:496-510: `a: &mut Ciphered<T>`):
    NOT runs with out == a and the result equals the oracle's.  Context::apply_n validates the
    user operation's requirement and calls it (operations.rs:204-213; the doc example's N-ary
    op on [&a, &b]), here a 3-ary sum composed of the batched additions."""
    params = (64, 64, 1, 64)
    ctx = H.Context(H.Parameters(*params))
    ctx.seed_rng(8)
    ctx.generate_secret_key()
    ctx.generate_public_key()
    x = plain(40, np.uint16, 1)
    m = masks(40, 16, 64, 2)
    c = ctx.encrypt(x, masks=m)
    ptr = c.limbs.data_ptr()
    assert ctx.apply1(H.HomomorphicNotGate, c) is c and c.limbs.data_ptr() == ptr
    pk = ctx.get_public_key().limbs
    la, da = oracle.encrypt_batch(pk, as_bytes(x), m, c.bound)
    rl, rd = oracle.gate_batch("not", la, da, c.bound, la, da, c.bound, 16, 40, c.bound)
    gl, gd = c.to_host()
    assert_batches_equal(gl, gd, rl, rd, c.bound, 40, "in-place not")
    assert np.array_equal(ctx.decrypt(c), ~x)

    class Sum3:  # a user HomomorphicOperation<3, u16> (+ OperationRequirement)
        MIN_D_OVER_DELTA = 21

        @staticmethod
        def apply(cx, args):
            a, b, d = args
            return cx.apply2(H.HomomorphicAddition, cx.apply2(H.HomomorphicAddition, a, b), d)

    y, z = plain(40, np.uint16, 3), plain(40, np.uint16, 4)
    s = ctx.apply_n(Sum3, [ctx.encrypt(x), ctx.encrypt(y), ctx.encrypt(z)])
    assert np.mean(ctx.decrypt(s) == (x + y + z).astype(np.uint16)) > 0.9

    class Needy(Sum3):
        MIN_D_OVER_DELTA = 1000

    with pytest.raises(H.OperationError):
        ctx.apply_n(Needy, [c, c, c])


def test_kernel_timing_counts_direct_and_graph_launches(H):
    """hm_ctx_set_kernel_timing: every launch of the selected kernel is stamped on the device,
    direct launches and launches captured into a graph alike (the bench times one replay of a
    K-step graph this way), and a launch's duration fits inside the event-timed steps around it."""
    import torch
    ctx = H.Context(H.Parameters(128, 128, 1, 128))
    ctx.seed_rng(77)
    ctx.generate_secret_key()
    ctx.generate_public_key()
    a = np.arange(256, dtype=np.uint32) * np.uint32(2654435761)  # wraps mod 2^32
    ca, cb = ctx.encrypt(a.astype(np.uint32)), ctx.encrypt((a ^ 0xFFFF).astype(np.uint32))
    out = H.Ciphered.empty(256, H.add_out_bounds(ca.bound, cb.bound), "cuda:0", np.dtype(np.uint32))
    H.add_into(ctx, ca, cb, out)
    ctx.set_kernel_timing(True, "add_chain")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(ctx.stream)
    for _ in range(3):
        H.add_into(ctx, ca, cb, out)
    ev1.record(ctx.stream)
    ms, n = ctx.kernel_timing()
    torch.cuda.synchronize()
    assert n == 3 and 0 < ms < ev0.elapsed_time(ev1)
    ctx.set_kernel_timing(True, "add_chain")  # reset
    # three launches captured into one graph: three record slots, valid for one replay
    g = ctx.graph(lambda: [H.add_into(ctx, ca, cb, out) for _ in range(3)], warmup=0)
    ev0.record(ctx.stream)
    g.replay()
    ev1.record(ctx.stream)
    ms1, n = ctx.kernel_timing()
    torch.cuda.synchronize()
    assert n == 3 and 0 < ms1 <= ev0.elapsed_time(ev1)
    # without a reset a second replay extends every slot (documented in the header): the stamps
    # then span both replays
    g.replay()
    ms2, n = ctx.kernel_timing()
    assert n == 3 and ms2 > ms1
    # hm_ctx_clear_kernel_timing: the slots stay, the stamps go; the next replay reads alone
    ctx.clear_kernel_timing()
    ev0.record(ctx.stream)
    g.replay()
    ev1.record(ctx.stream)
    ms3, n = ctx.kernel_timing()
    torch.cuda.synchronize()
    assert n == 3 and 0 < ms3 <= ev0.elapsed_time(ev1)
    got = ctx.decrypt(out, np.uint32)
    assert np.array_equal(got, (a + (a ^ 0xFFFF)).astype(np.uint32))
    ctx.set_kernel_timing(True, "encrypt")
    c = ctx.encrypt(a)
    assert ctx.kernel_timing()[1] == 1
    ctx.set_kernel_timing(True, "decrypt")
    assert np.array_equal(ctx.decrypt(c, np.uint32), a)
    assert ctx.kernel_timing()[1] == 1
    ctx.set_kernel_timing(False)
    H.add_into(ctx, ca, cb, out)
    assert ctx.kernel_timing() == (0.0, 0)
