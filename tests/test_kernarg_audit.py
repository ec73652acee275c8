"""Code-object audit of the engine's kernels (CPU only; tools/kernarg_audit.py).

Round 5 lost hours to non-deterministic wrong decryptions: a kernel indexed its
by-value `Bounds` argument with a lane-varying index, which compiles to VECTOR loads from the
kernarg segment.  These tests read the device code of every object the library is linked from
and assert that
  - no kernel reads its argument block through the vector memory path (every argument read is an
    s_load with a wave-uniform address);
  - the kernels on the headline and cipher paths use no private (scratch) segment at all, and the
    MFMA carry chain's scratch holds register spills only (no stack arrays).
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import kernarg_audit  # noqa: E402

PKG = os.path.join(ROOT, "homomorph-rust_amd")


@pytest.fixture(scope="module")
def audit():
    subprocess.run(["make", "-C", PKG, "-j8", "-s"], check=True, capture_output=True)
    res = {}
    for obj in sorted(glob.glob(os.path.join(PKG, "build", "*.o"))):
        res.update(kernarg_audit.parse(obj))
    assert len(res) > 50, "device code objects not found"
    return res


def test_no_kernel_reads_its_arguments_per_lane(audit):
    bad = {k: v["findings"][:2] for k, v in audit.items() if v["findings"]}
    assert not bad, bad


def test_the_pinned_construct_is_detected():
    """The audit itself: round 5's failing decrypt_kernel form (a per-lane cursor over D.ib.b[])
    compiled here must be flagged, and its uniform rewrite must not."""
    src = r'''
#include <hip/hip_runtime.h>
struct Bnd { unsigned b[128]; };
struct Args { const unsigned long long *in; unsigned n; unsigned char *out; Bnd ib; };
__global__ void cursor(Args D) {
    unsigned lane = threadIdx.x & 63u, i = 0, hi = D.ib.b[0] / 64 + 1;
    unsigned long long acc = 0;
    for (unsigned g = lane; g < D.n; g += 64) {
        while (g >= hi) ++i, hi += D.ib.b[i] / 64 + 1;   // lane-varying i
        acc ^= D.in[g] << (i & 63);
    }
    D.out[threadIdx.x] = (unsigned char)acc;
}
__global__ void uniform(Args D) {
    unsigned long long acc = 0;
    for (unsigned i = 0, o = 0; i < 32; ++i) {           // wave-uniform i
        const unsigned cap = D.ib.b[i] / 64 + 1;
        for (unsigned k = threadIdx.x & 63u; k < cap; k += 64) acc ^= D.in[o + k];
        o += cap;
    }
    D.out[threadIdx.x] = (unsigned char)acc;
}
'''
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        hip, asm = os.path.join(tmp, "k.hip"), os.path.join(tmp, "k.s")
        open(hip, "w").write(src)
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", hip, "-o", asm], check=True, capture_output=True)
        res = kernarg_audit.parse(asm)
    cur = next(v for k, v in res.items() if "cursor" in k)
    uni = next(v for k, v in res.items() if "uniform" in k)
    assert cur["findings"], "the per-lane kernarg cursor was not detected"
    assert not uni["findings"], uni["findings"]


ZERO_SCRATCH = [
    "_ZN2hm15add_prep_kernelILi10ELi17ELb0ELb0EEEvNS_7AddArgsE",  # (fixed rows at d + d' = 256)
    "_ZN2hm15add_prep_kernelILi0ELi0ELb0ELb0EEEvNS_7AddArgsE",
    "_ZN2hm15add_prep_kernelILi0ELi0ELb1ELb0EEEvNS_7AddArgsE",  # (top-word copies: the bench's)
    "_ZN2hm15add_prep_kernelILi0ELi0ELb1ELb1EEEvNS_7AddArgsE",  # (values per wave: configs[0])
    "_ZN2hm14decrypt_kernelENS_7DecArgsE",
    "_ZN2hm19decrypt_bits_kernelENS_7DecArgsE",
    "_ZN2hm16mul_final_kernelENS_12MulFinalArgsE",
    "_ZN2hm16rand_fill_kernelENS_8RandArgsE",
    # the bench's encryption instances (d + d' = 256: 5 limbs; tau = 128, with and without TOP1)
    "_ZN2hm20encrypt_table_kernelILi5ELi32ELb1EEEvNS_7EncArgsE",
    "_ZN2hm20encrypt_table_kernelILi5ELi32ELb0EEEvNS_7EncArgsE",
]


@pytest.mark.parametrize("kernel", ZERO_SCRATCH)
def test_zero_private_segment(audit, kernel):
    assert kernel in audit, sorted(audit)[:8]
    assert audit[kernel]["private"] == 0


def test_chain_scratch_is_spills_only():
    """add_chain_mfma_kernel<13>: its private segment (if any) holds register spills only -- no
    stack array (checked on the compiler's annotated assembly of adder_mfma.hip)."""
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        asm = os.path.join(tmp, "a.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "-Wno-unused-result", "--cuda-device-only", "-S",
                        os.path.join(PKG, "csrc", "adder_mfma.hip"), "-o", asm],
                       check=True, capture_output=True)
        res = kernarg_audit.parse(asm)
    ch = res["_ZN2hm21add_chain_mfma_kernelILi13EEEvNS_7AddArgsE"]
    assert not ch["findings"]
    assert ch["scratch_nonspill"] == 0
    assert ch["private"] <= 32
