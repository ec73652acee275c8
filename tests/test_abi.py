"""CPU checks of the C-ABI library (no GPU needed, no compute launched).

- libhomomorph_gpu.so loads and exports every function include/homomorph_gpu.h declares, and the
  ctypes binding covers exactly that set.
- The host-only entry points (status strings, output bounds, batch stride) match SURVEY.md
  Appendix A and the oracle's own layout.
"""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "homomorph_gpu.h")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    return sorted(set(re.findall(r"\b(hm_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def L():
    from homomorph import _lib
    return _lib.lib()


def test_header_declares_the_boundary():
    names = declared()
    for must in ("hm_ctx_create", "hm_encrypt_batch", "hm_decrypt_batch", "hm_add_batch",
                 "hm_mul_batch", "hm_gate_batch", "hm_poly_add_batch", "hm_poly_mul_batch",
                 "hm_poly_rem_batch", "hm_add_out_bounds", "hm_validate_operation"):
        assert must in names


def test_library_exports_every_declared_symbol(L):
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing


def test_binding_matches_header():
    from homomorph import _lib
    assert sorted(_lib.SIGNATURES) == declared()


def test_abi_version_and_status_strings(L):
    assert L.hm_abi_version() >= 1
    for s in range(12):
        msg = L.hm_status_string(s)
        assert msg and len(msg) >= 2
    assert L.hm_status_string(0).decode().lower().startswith("ok")


def test_add_bounds_match_survey():
    import homomorph as H
    D = 256
    ob = H.add_out_bounds(np.full(32, D, np.uint32), np.full(32, D, np.uint32))
    # s_0 <= D, s_i <= (3i-1) D ; cap_i = 12i-3 at D = 256, total 5864 limbs
    assert ob[0] == D and all(ob[i] == (3 * i - 1) * D for i in range(1, 32))
    caps = H.caps(ob)
    assert caps[0] == 5 and all(caps[i] == 12 * i - 3 for i in range(1, 32))
    assert H.batch_stride(ob) == 5864
    ob512 = H.add_out_bounds(np.full(32, 512, np.uint32), np.full(32, 512, np.uint32))
    assert H.batch_stride(ob512) == 11696


def test_bounds_agree_with_oracle_layout(oracle):
    import homomorph as H
    for bound in (np.full(8, 128, np.uint32), np.arange(1, 33, dtype=np.uint32) * 100):
        assert H.batch_stride(bound) == oracle.stride(bound)
        assert np.array_equal(H.caps(bound), oracle.caps(bound))


def test_mul_and_gate_bounds_cover_model(oracle):
    """Output bounds dominate the actual degrees the oracle produces (u8 mul, gates)."""
    import homomorph as H
    from helpers import as_bytes, fresh_bound, keys, masks, plain
    d, dp, delta, tau = 128, 64, 1, 64
    sk, pk, _ = keys(d, dp, delta, tau, 5)
    bound = fresh_bound(d, dp, 8)
    a, b = plain(3, np.uint8, 1), plain(3, np.uint8, 2)
    la, da = oracle.encrypt_batch(pk, as_bytes(a), masks(3, 8, tau, 3), bound)
    lb, db = oracle.encrypt_batch(pk, as_bytes(b), masks(3, 8, tau, 4), bound)
    ob = H.mul_out_bounds(bound, bound)
    lo, do = oracle.mul_batch(la, da, bound, lb, db, bound, 8, 3, ob)
    assert np.all(np.asarray(do).reshape(3, 8) <= ob[None, :])
    for opcls, name in ((H.HomomorphicAndGate, "and"), (H.HomomorphicOrGate, "or"),
                        (H.HomomorphicXorGate, "xor")):
        gb = H.gate_out_bounds(opcls, bound, bound)
        lo, do = oracle.gate_batch(name, la, da, bound, lb, db, bound, 8, 3, gb)
        assert np.all(np.asarray(do).reshape(3, 8) <= gb[None, :])


def test_mul_cost_matches_survey_appendix_a3():
    """hm_mul_cost prices the carry-save circuit from its static bounds (SURVEY.md Appendix A.3:
    top-bit degree per K; the full u32 circuit ~4.7e17 limb-clmuls = 1.9e18 word pairs and
    ~8.4 GiB of output bits), and agrees with hm_mul_out_bounds where both apply."""
    import homomorph as H
    b = np.full(32, 256, np.uint32)
    top = {8: 14336, 12: 146432, 16: 1.6e6, 20: 1.9e7, 32: 3.4e10}
    prev = 0
    for k, deg in top.items():
        c = H.mul_cost(b, b, k)
        assert abs(c["max_degree"] - deg) / deg < 0.05, (k, c)
        assert c["word_pairs"] > prev
        prev = c["word_pairs"]
    full = H.mul_cost(b, b)
    assert 1.8e18 < full["word_pairs"] < 2.0e18 and 8.0 * 2**30 < full["out_bytes"] < 8.8 * 2**30
    ob = H.mul_out_bounds(b[:8], b[:8])
    assert H.mul_cost(b[:8], b[:8])["out_bytes"] == 8 * H.batch_stride(ob)


def test_wire_header_host_only():
    """The wire format's header (include/homomorph_gpu.h): a hand-built image parses, and bad
    magic / version / flags / length are rejected -- host-only entry points, no GPU."""
    import homomorph as H
    bound = np.array([128, 300, 0], np.uint32)
    n = 2
    stride = int((bound // 64 + 1).sum())
    size = H.lib().hm_wire_bytes(3, H._p32(bound), n)
    doff = 24 + 4 * 3
    loff = (doff + 4 * n * 3 + 7) // 8 * 8
    assert size == loff + 8 * n * stride
    img = bytearray(size)
    img[:4] = b"HMCB"
    img[4:8] = (1).to_bytes(4, "little")
    img[8:12] = (3).to_bytes(4, "little")
    img[16:24] = n.to_bytes(8, "little")
    img[24:doff] = bound.astype("<u4").tobytes()
    info = H.wire_info(bytes(img))
    assert info["nbits"] == 3 and info["n"] == n and np.array_equal(info["bound"], bound)
    for off, val in ((0, b"XMCB"), (4, (2).to_bytes(4, "little")), (12, (1).to_bytes(4, "little"))):
        bad = bytearray(img)
        bad[off:off + len(val)] = val
        with pytest.raises(H.EngineError):
            H.wire_info(bytes(bad))
    with pytest.raises(H.EngineError):
        H.wire_info(bytes(img[:-1]))


def test_invalid_bounds_rejected(L):
    from homomorph import _lib
    a = np.full(4, 10, np.uint32)
    out = np.zeros(4, np.uint32)
    p = lambda x: x.ctypes.data_as(_lib.u32p)  # noqa: E731
    assert L.hm_add_out_bounds(0, p(a), p(a), p(out)) != 0      # empty value
    assert L.hm_gate_out_bounds(99, 4, p(a), p(a), p(out)) != 0  # unknown gate


def test_product_fails_loudly_without_library(monkeypatch, tmp_path):
    """No CPU fallback: a missing engine is an error, not a silent slow path."""
    from homomorph import _lib
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.LibraryMissing):
        _lib.lib()
