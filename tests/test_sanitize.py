"""SURVEY.md s5 "race detection / sanitizers": ASan + UBSan builds of the CPU oracle and of the
engine library's host code, run on the CPU (GPU sanitizers are not available on this pool).

- tests/sanitize/oracle_san.c: the reference's polynomial KATs and an encrypt -> add / mul /
  gates -> decrypt round trip through oracle/homomorph_oracle.c;
- tests/sanitize/capi_san.cpp: every host-only C-ABI entry point (status strings, bounds, the
  multiplier cost model, strides, the wire-format parser under 20k corrupted headers, NULL
  contexts), with the device kernels linked in unsanitised;
- tests/sanitize/plan_split.cpp: the multiplier planner's split Karatsuba plans (host only): the
  same leaf products as the breadth-first plans at K = 16, K = 21 planned;
- tests/sanitize/capi_oom.cpp (not sanitised): every allocation inside the multiplier's plan
  builder failed in turn, each call returning HM_ERR_OUT_OF_MEMORY instead of throwing across
  the C ABI.
Any sanitizer report aborts the binary (-fno-sanitize-recover=all) and fails the test.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")


@pytest.fixture(scope="module")
def built():
    if shutil.which("gcc") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("needs gcc and hipcc")
    eng = os.path.join(ROOT, "homomorph-rust_amd")
    subprocess.run(["make", "-s", "-C", eng], check=True, timeout=1200)
    subprocess.run(["make", "-s", "-j4", "-C", SAN], check=True, timeout=1200)
    return os.path.join(SAN, "_build")


def _run(path):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([path], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return r.stdout


def test_oracle_under_asan_ubsan(built):
    assert "ok" in _run(os.path.join(built, "oracle_san"))


def test_engine_host_code_under_asan_ubsan(built):
    assert "ok" in _run(os.path.join(built, "capi_san"))


def test_engine_abi_returns_oom_instead_of_throwing(built):
    out = _run(os.path.join(built, "capi_oom"))
    assert "ok" in out and "allocation points" in out


def test_split_karatsuba_plans_under_asan_ubsan(built):
    assert "ok" in _run(os.path.join(built, "plan_split"))
