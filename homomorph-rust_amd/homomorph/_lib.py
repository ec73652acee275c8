"""ctypes binding of the engine's C ABI (include/homomorph_gpu.h -> lib/libhomomorph_gpu.so).

The product path: there is no CPU fallback.  If the shared library is missing or fails to load,
every entry point raises.  Build it with `make -C homomorph-rust_amd` (or __graft_entry__.build()).
"""
from __future__ import annotations

import ctypes
import os

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# HOMOMORPH_GPU_LIB: an alternative build of the same engine (A/B timing of kernel variants)
LIB_PATH = os.environ.get("HOMOMORPH_GPU_LIB") or os.path.join(_PKG, "lib", "libhomomorph_gpu.so")

HM_MAX_BITS = 128

# hm_status
OK = 0
ERR_INVALID_PARAMETERS = 1
ERR_SECRET_KEY_UNSET = 2
ERR_PUBLIC_KEY_UNSET = 3
ERR_DIVIDE_BY_ZERO = 4
ERR_DIVISOR_IS_ONE = 5
ERR_CAPACITY = 6
ERR_UNSUPPORTED = 7
ERR_HIP = 8
ERR_INVALID_ARGUMENT = 9
ERR_INVALID_CIPHERED_LENGTH = 10
ERR_BAD_INPUT = 11
ERR_RANDOMNESS = 12
ERR_OUT_OF_MEMORY = 13
ERR_INTERNAL = 14

# hm_op
OP_AND, OP_OR, OP_XOR, OP_NOT, OP_ADD, OP_MUL, OP_MUL_SIGNED = range(7)

u64p = ctypes.POINTER(ctypes.c_uint64)
u32p = ctypes.POINTER(ctypes.c_uint32)
u16p = ctypes.POINTER(ctypes.c_uint16)
u8p = ctypes.POINTER(ctypes.c_uint8)
vp = ctypes.c_void_p


class HmBatch(ctypes.Structure):
    _fields_ = [("limbs", vp), ("degree", vp), ("bound", u32p), ("nbits", ctypes.c_uint32),
                ("n", ctypes.c_uint64)]


class HmPolys(ctypes.Structure):
    _fields_ = [("limbs", vp), ("degree", vp), ("cap", ctypes.c_uint32), ("n", ctypes.c_uint64)]


# name -> (restype, argtypes); every symbol include/homomorph_gpu.h declares
SIGNATURES = {
    "hm_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "hm_abi_version": (ctypes.c_uint32, []),
    "hm_ctx_create": (ctypes.c_int, [ctypes.c_uint16] * 4 + [ctypes.c_int, ctypes.POINTER(vp)]),
    "hm_ctx_destroy": (None, [vp]),
    "hm_ctx_generation": (ctypes.c_uint64, [vp]),
    "hm_ctx_trim": (ctypes.c_int, [vp]),
    "hm_ctx_mask_bytes": (ctypes.c_uint32, [vp]),
    "hm_random_bytes": (ctypes.c_int, [vp, vp, ctypes.c_size_t]),
    "hm_ctx_set_stream": (ctypes.c_int, [vp, vp]),
    "hm_ctx_stream": (vp, [vp]),
    "hm_ctx_parameters": (ctypes.c_int, [vp, u16p, u16p, u16p, u16p]),
    "hm_ctx_set_secret_key": (ctypes.c_int, [vp, u64p, ctypes.c_size_t]),
    "hm_ctx_set_public_key": (ctypes.c_int, [vp, u64p, ctypes.c_uint32, ctypes.c_uint32]),
    "hm_ctx_seed_rng": (ctypes.c_int, [vp, ctypes.c_uint64]),
    "hm_ctx_generate_secret_key": (ctypes.c_int, [vp]),
    "hm_ctx_generate_public_key": (ctypes.c_int, [vp]),
    "hm_ctx_get_secret_key": (ctypes.c_int, [vp, u64p, ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_size_t)]),
    "hm_ctx_get_public_key": (ctypes.c_int, [vp, u64p, ctypes.c_size_t, u32p, u32p]),
    "hm_validate_operation": (ctypes.c_int, [vp, ctypes.c_int, u16p]),
    "hm_ctx_set_mul_options": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32]),
    "hm_ctx_set_mul_scratch": (ctypes.c_int, [vp, ctypes.c_uint64]),
    "hm_ctx_set_add_options": (ctypes.c_int, [vp, ctypes.c_uint32]),
    "hm_ctx_set_mul_products": (ctypes.c_int, [vp, ctypes.c_uint32]),
    "hm_ctx_set_add_pipeline": (ctypes.c_int, [vp, ctypes.c_int]),
    "hm_ctx_set_kernel_timing": (ctypes.c_int, [vp, ctypes.c_int]),
    "hm_ctx_clear_kernel_timing": (ctypes.c_int, [vp]),
    "hm_ctx_kernel_timing": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double), u32p]),
    "hm_fresh_bound": (ctypes.c_uint32, [vp]),
    "hm_add_out_bounds": (ctypes.c_int, [ctypes.c_uint32, u32p, u32p, u32p]),
    "hm_mul_out_bounds": (ctypes.c_int, [ctypes.c_uint32, u32p, u32p, ctypes.c_int, u32p]),
    "hm_mul_cost": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_double)]),
    "hm_mul_plan_work": (ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_double)]),
    "hm_gate_out_bounds": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, u32p, u32p, u32p]),
    "hm_batch_stride": (ctypes.c_uint64, [ctypes.c_uint32, u32p]),
    "hm_encrypt_batch": (ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, ctypes.POINTER(HmBatch)]),
    "hm_decrypt_batch": (ctypes.c_int, [vp, ctypes.POINTER(HmBatch), vp]),
    "hm_add_batch": (ctypes.c_int, [vp] + [ctypes.POINTER(HmBatch)] * 3),
    "hm_mul_batch": (ctypes.c_int, [vp, ctypes.POINTER(HmBatch), ctypes.POINTER(HmBatch),
                                    ctypes.c_int, ctypes.POINTER(HmBatch)]),
    "hm_mul_low_batch": (ctypes.c_int, [vp, ctypes.POINTER(HmBatch), ctypes.POINTER(HmBatch),
                                        ctypes.c_uint32, ctypes.POINTER(HmBatch)]),
    "hm_gate_batch": (ctypes.c_int, [vp, ctypes.c_int] + [ctypes.POINTER(HmBatch)] * 3),
    "hm_poly_add_batch": (ctypes.c_int, [vp] + [ctypes.POINTER(HmPolys)] * 3),
    "hm_poly_mul_batch": (ctypes.c_int, [vp] + [ctypes.POINTER(HmPolys)] * 3),
    "hm_poly_rem_batch": (ctypes.c_int, [vp, ctypes.POINTER(HmPolys), u64p, ctypes.c_size_t,
                                         ctypes.POINTER(HmPolys)]),
    "hm_wire_bytes": (ctypes.c_uint64, [ctypes.c_uint32, u32p, ctypes.c_uint64]),
    "hm_wire_peek": (ctypes.c_int, [vp, ctypes.c_size_t, u32p, ctypes.POINTER(ctypes.c_uint64),
                                    u32p]),
    "hm_wire_encode": (ctypes.c_int, [vp, ctypes.POINTER(HmBatch), vp, ctypes.c_size_t]),
    "hm_wire_decode": (ctypes.c_int, [vp, vp, ctypes.c_size_t, ctypes.POINTER(HmBatch)]),
    "hm_ctx_synchronize": (ctypes.c_int, [vp]),
    "hm_ctx_last_hip_error": (ctypes.c_int32, [vp]),
}

_lib = None


class LibraryMissing(RuntimeError):
    pass


def lib():
    """Load the HIP engine; raise loudly if it is not built (no fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LibraryMissing(
                f"{LIB_PATH} not found: build the gfx950 engine first "
                "(make -C homomorph-rust_amd, or python -c 'import __graft_entry__ as g; g.build()')")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def status_string(st: int) -> str:
    return lib().hm_status_string(st).decode()
