"""INTEGRATION.md's Rust patch, checked mechanically (no Rust toolchain exists here):

- every `hm_*` function its extern block declares is declared in include/homomorph_gpu.h with
  the same number of parameters, and every header function is bound;
- every crate item it calls or imports on the reference's own types (`Context::parameters`,
  `Polynomial::coefficients`, `SecretKey::get_polynomial`, `Ciphered::new_from_raw`, the
  operation markers, ...) is defined in the reference sources, or is defined by the patch itself;
- the remaining method names are standard-library ones (an explicit list).
The reference-source part needs /root/reference (this container); it is skipped elsewhere.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src"

STD = {
    # core / alloc / std methods and associated functions the patch uses
    "iter", "map", "collect", "max", "min", "unwrap_or", "unwrap_or_else", "len", "as_ptr",
    "as_mut_ptr", "cast", "enumerate", "take", "clone", "first", "map_or", "into_iter", "pop",
    "ok", "lock", "unwrap", "as_ref", "push", "with_capacity", "into_boxed_slice", "var_os", "var",
    "into", "null_mut", "null", "is_some", "new", "from", "fmt", "main", "borrow_mut", "get_mut",
    "into_inner", "is_null", "iter_mut",
}


def rust_blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return "\n".join(re.findall(r"```rust\n(.*?)```", text, flags=re.S))


def strip_comments(code):
    return re.sub(r"//[^\n]*", "", code)


def header_arity():
    text = open(os.path.join(ROOT, "include", "homomorph_gpu.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for name, args in re.findall(r"\b(hm_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", text):
        a = args.strip()
        out[name] = 0 if a in ("", "void") else a.count(",") + 1
    return out


def test_extern_block_matches_header():
    code = strip_comments(rust_blocks())
    decl = {}
    for name, args in re.findall(r"pub fn (hm_[a-z0-9_]+)\(([^)]*)\)", code, flags=re.S):
        a = args.strip().rstrip(",")
        decl[name] = 0 if not a else a.count(",") + 1
    hdr = header_arity()
    assert set(decl) == set(hdr), (set(hdr) - set(decl), set(decl) - set(hdr))
    for name, n in hdr.items():
        assert decl[name] == n, (name, decl[name], n)


def _defined_in_doc(code):
    names = set(re.findall(r"\b(?:fn|struct|enum|trait|static|mod|type)\s+([A-Za-z_][A-Za-z0-9_]*)",
                           code))
    return names | set(re.findall(r"\bconst\s+(?!fn\b)([A-Za-z_][A-Za-z0-9_]*)", code))


def _ref_sources():
    if not os.path.isdir(REF):
        pytest.skip("reference sources not present (only in the build container)")
    text = ""
    for dp, _, files in os.walk(REF):
        for f in files:
            if f.endswith(".rs"):
                text += open(os.path.join(dp, f)).read() + "\n"
    return text


def test_calls_resolve_to_reference_or_patch():
    code = strip_comments(rust_blocks())
    ref = _ref_sources()
    ref_fns = set(re.findall(r"\bfn\s+([a-z_][a-z0-9_]*)", ref))
    doc = _defined_in_doc(code)
    called = set(re.findall(r"\.([a-z_][a-z0-9_]*)\s*(?:::<[^>]*>)?\(", code))
    called |= set(re.findall(r"::([a-z_][a-z0-9_]*)\s*(?:::<[^>]*>)?\(", code))
    missing = sorted(n for n in called
                     if n not in doc and n not in STD and n not in ref_fns
                     and not n.startswith(("hm_", "hip")))
    assert not missing, f"calls defined nowhere: {missing}"
    # the reference items the patch relies on, with the receiver type they must live on
    for item in ("fn parameters", "fn d(", "fn dp(", "fn delta(", "fn tau(", "fn get_secret_key",
                 "fn get_public_key", "fn get_polynomial", "fn get_polynomials", "fn coefficients",
                 "fn degree", "fn new_from_raw", "fn validate_operation", "fn add<",
                 "fn gate_not", "fn cipher(", "fn generate_secret_key", "fn generate_public_key",
                 "fn apply2<"):
        assert item in ref, item


def test_imports_resolve_to_reference():
    code = strip_comments(rust_blocks())
    ref = _ref_sources()
    for path in re.findall(r"use (crate::[A-Za-z_:{}, \n]+);", code):
        for name in re.findall(r"\b([A-Z][A-Za-z0-9]+)\b", path):
            assert re.search(r"\b(?:struct|enum|trait)\s+%s\b" % name, ref), name
    reexported = set(re.findall(r"pub use bincode::\{([^}]*)\}", ref)[0].replace(" ", "").split(","))
    for name in re.findall(r"crate::(?!gpu::)(?:[a-z_]+::)*([A-Z][A-Za-z0-9]+)", code):
        if name not in _defined_in_doc(code) and name not in reexported:
            assert re.search(r"\b(?:struct|enum|trait)\s+%s\b" % name, ref), name
