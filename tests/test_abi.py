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
