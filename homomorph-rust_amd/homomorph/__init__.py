"""homomorph — MI355X (gfx950) engine for mathisbot/homomorph-rust's bit-level homomorphic scheme.

Host-side mirror of the reference crate's public surface, batched over the GPU engine's C ABI
(include/homomorph_gpu.h).  Names, argument meaning and error behaviour follow the reference:

  Parameters(d, dp, delta, tau)          src/context.rs:33-119   (asserts -> ValueError)
  SecretKey / PublicKey  to/from_bytes   src/context.rs:121-298
  Context.generate_secret_key/public_key src/context.rs:421-454
  Context.encrypt / decrypt              src/context.rs:463-488  (ContextCryptoError)
  Context.apply1 / apply2                src/context.rs:496-527  (OperationError.InvalidParameters)
  HomomorphicAddition, ...Multiplication src/impls/numbers.rs:9-50 (MIN_D_OVER_DELTA)
  Ciphered                               src/cipher.rs:125-259   (a BATCH of Ciphered<T> here)

Everything below the API runs in hand-written HIP kernels; there is no CPU fallback — if the
engine library is not built, the first call raises `LibraryMissing`.  PyTorch is used only for
device memory and stream plumbing.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import HmBatch, HmPolys, LibraryMissing, lib

__all__ = [
    "Parameters", "SecretKey", "PublicKey", "Context", "Ciphered", "Polys",
    "HomomorphicAndGate", "HomomorphicOrGate", "HomomorphicXorGate", "HomomorphicNotGate",
    "HomomorphicAddition", "HomomorphicMultiplication",
    "OperationError", "ContextCryptoError", "CipherError", "EngineError", "LibraryMissing",
    "EngineGraph",
    "add_out_bounds", "mul_out_bounds", "gate_out_bounds", "batch_stride", "caps",
]


# ------------------------------------------------------------------ errors (reference enums)
class EngineError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {_lib.status_string(status)} (status {status})")


class OperationError(EngineError):
    """OperationError::InvalidParameters (src/operations.rs:11-18)."""

    def __init__(self, required_min_d_over_delta: int, actual_d: int, actual_delta: int):
        self.required_min_d_over_delta = required_min_d_over_delta
        self.actual_d = actual_d
        self.actual_delta = actual_delta
        RuntimeError.__init__(self, f"InvalidParameters {{ required_min_d_over_delta: "
                                    f"{required_min_d_over_delta}, actual_d: {actual_d}, "
                                    f"actual_delta: {actual_delta} }}")
        self.status = _lib.ERR_INVALID_PARAMETERS


class ContextCryptoError(EngineError):
    """ContextCryptoError::{SecretKeyUnset, PublicKeyUnset, Cipher} (src/context.rs:41-46)."""


class CipherError(EngineError):
    """CipherError (src/cipher.rs:17-24)."""


def _check(st: int, what: str):
    if st == _lib.OK:
        return
    if st in (_lib.ERR_SECRET_KEY_UNSET, _lib.ERR_PUBLIC_KEY_UNSET):
        raise ContextCryptoError(st, what)
    if st in (_lib.ERR_INVALID_CIPHERED_LENGTH, _lib.ERR_RANDOMNESS):
        raise CipherError(st, what)
    if st == _lib.ERR_DIVIDE_BY_ZERO:
        raise ZeroDivisionError("attempt to divide by zero")  # polynomial.rs:319-322
    if st == _lib.ERR_OUT_OF_MEMORY:
        raise MemoryError(f"{what}: {_lib.status_string(st)}")
    raise EngineError(st, what)


# ------------------------------------------------------------------ operation markers
class _Op:
    MIN_D_OVER_DELTA: int
    CODE: int


class HomomorphicAndGate(_Op):
    MIN_D_OVER_DELTA, CODE = 2, _lib.OP_AND


class HomomorphicOrGate(_Op):
    MIN_D_OVER_DELTA, CODE = 2, _lib.OP_OR


class HomomorphicXorGate(_Op):
    MIN_D_OVER_DELTA, CODE = 1, _lib.OP_XOR


class HomomorphicNotGate(_Op):
    MIN_D_OVER_DELTA, CODE = 1, _lib.OP_NOT


class HomomorphicAddition(_Op):
    MIN_D_OVER_DELTA, CODE = 21, _lib.OP_ADD


class HomomorphicMultiplication(_Op):
    MIN_D_OVER_DELTA, CODE = 64, _lib.OP_MUL


# ------------------------------------------------------------------ parameters / keys
@dataclass(frozen=True)
class Parameters:
    """Parameters::new (src/context.rs:87-94): all strictly positive u16, delta < d."""
    d: int
    dp: int
    delta: int
    tau: int

    def __post_init__(self):
        for k in ("d", "dp", "delta", "tau"):
            v = getattr(self, k)
            if not (0 <= v < 1 << 16):
                raise ValueError(f"{k} must fit in u16")
        if self.d == 0 or self.dp == 0 or self.delta == 0 or self.tau == 0:
            raise ValueError("Parameters must be strictly positive")
        if self.delta >= self.d:
            raise ValueError("Delta must be less than d (delta < d)")


class SecretKey:
    """SecretKey(Polynomial) with the reference's byte format: little-endian u64 limbs."""

    def __init__(self, limbs: np.ndarray):
        self.limbs = np.ascontiguousarray(limbs, dtype=np.uint64)

    @classmethod
    def from_bytes(cls, b: bytes) -> "SecretKey":  # context.rs:153-155 / polynomial.rs:108-122
        if len(b) == 0:
            raise ValueError("The vector of bytes must not be empty.")
        pad = (-len(b)) % 8
        return cls(np.frombuffer(bytes(b) + b"\0" * pad, dtype="<u8").copy())

    def to_bytes(self) -> bytes:
        return self.limbs.astype("<u8").tobytes()

    def __eq__(self, o):
        return isinstance(o, SecretKey) and _poly_eq(self.limbs, o.limbs)


class PublicKey:
    def __init__(self, limbs: np.ndarray):
        """limbs: (tau, limbs_per_poly) uint64."""
        self.limbs = np.ascontiguousarray(limbs, dtype=np.uint64)

    @classmethod
    def from_bytes(cls, rows: list[bytes]) -> "PublicKey":  # context.rs:239-245
        polys = [SecretKey.from_bytes(r).limbs for r in rows]
        w = max(len(p) for p in polys)
        out = np.zeros((len(polys), w), dtype=np.uint64)
        for i, p in enumerate(polys):
            out[i, : len(p)] = p
        return cls(out)

    def to_bytes(self) -> list[bytes]:
        return [r.astype("<u8").tobytes() for r in self.limbs]

    def __eq__(self, o):
        return isinstance(o, PublicKey) and len(self.limbs) == len(o.limbs) and all(
            _poly_eq(a, b) for a, b in zip(self.limbs, o.limbs))


def _deg(limbs) -> int:
    nz = np.nonzero(limbs)[0]
    if nz.size == 0:
        return 0
    k = int(nz[-1])
    return 64 * k + int(limbs[k]).bit_length() - 1


def _poly_eq(a, b) -> bool:  # PartialEq, polynomial.rs:417-426
    da, db = _deg(a), _deg(b)
    return da == db and np.array_equal(a[: da // 64 + 1], b[: db // 64 + 1])


# ------------------------------------------------------------------ bounds / layout helpers
def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint32)


def caps(bound) -> np.ndarray:
    return _u32(bound) // 64 + 1


def batch_stride(bound) -> int:
    return int(caps(bound).sum())


def add_out_bounds(a_bound, b_bound) -> np.ndarray:
    a, b = _u32(a_bound), _u32(b_bound)
    out = np.zeros_like(a)
    _check(lib().hm_add_out_bounds(a.size, _p32(a), _p32(b), _p32(out)), "hm_add_out_bounds")
    return out


def mul_out_bounds(a_bound, b_bound, signed=False) -> np.ndarray:
    a, b = _u32(a_bound), _u32(b_bound)
    out = np.zeros_like(a)
    _check(lib().hm_mul_out_bounds(a.size, _p32(a), _p32(b), int(signed), _p32(out)),
           "hm_mul_out_bounds")
    return out


def mul_cost(a_bound, b_bound, k=None, signed=False) -> dict:
    """hm_mul_cost: the planner's price of the low k output bits of the carry-save multiplier
    (all bits when k is None) -- word_pairs (32x32 carry-less word products), out_bytes,
    max_degree.  Host only; works for circuits far beyond what any device can run."""
    a, b = _u32(a_bound), _u32(b_bound)
    k = a.size if k is None else int(k)
    w, o, m = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    _check(lib().hm_mul_cost(a.size, k, _p32(a), _p32(b), int(signed), ctypes.byref(w),
                             ctypes.byref(o), ctypes.byref(m)), "hm_mul_cost")
    return {"word_pairs": w.value, "out_bytes": o.value, "max_degree": m.value}


def wire_info(data: bytes) -> dict:
    """hm_wire_peek: {"nbits", "n", "bound"} of a wire image (host only)."""
    nb, n = ctypes.c_uint32(), ctypes.c_uint64()
    bound = np.zeros(_lib.HM_MAX_BITS, dtype=np.uint32)
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    _check(lib().hm_wire_peek(buf, len(data), ctypes.byref(nb), ctypes.byref(n), _p32(bound)),
           "hm_wire_peek")
    return {"nbits": nb.value, "n": n.value, "bound": bound[: nb.value].copy()}


def gate_out_bounds(op, a_bound, b_bound=None) -> np.ndarray:
    a = _u32(a_bound)
    b = _u32(b_bound) if b_bound is not None else None
    out = np.zeros_like(a)
    _check(lib().hm_gate_out_bounds(op.CODE, a.size, _p32(a), _p32(b) if b is not None else None,
                                    _p32(out)), "hm_gate_out_bounds")
    return out


def _p32(a):
    return a.ctypes.data_as(_lib.u32p)


def _p64(a):
    return a.ctypes.data_as(_lib.u64p)


# ------------------------------------------------------------------ device buffers
def _torch():
    import torch
    return torch


class Ciphered:
    """A batch of n `Ciphered<T>` values, nbits ciphertext bits each, resident on one GPU.

    limbs: int64 tensor (raw u64 limbs, batch layout of include/homomorph_gpu.h);
    degree: int32 tensor (n, nbits) of exact degrees; bound: per-bit degree bounds (host).
    `len(c)` is nbits, like the reference's `Deref<Target=[CipheredBit]>` (cipher.rs:253-259).
    """

    def __init__(self, limbs, degree, bound, nbits: int, n: int, plain_dtype=None):
        self.limbs = limbs
        self.degree = degree
        self.bound = _u32(bound)
        self.nbits = int(nbits)
        self.n = int(n)
        self.plain_dtype = plain_dtype
        assert self.bound.size == self.nbits

    @classmethod
    def empty(cls, n: int, bound, device, plain_dtype=None) -> "Ciphered":
        torch = _torch()
        bound = _u32(bound)
        stride = batch_stride(bound)
        limbs = torch.empty(n * stride, dtype=torch.int64, device=device)
        degree = torch.empty((n, bound.size), dtype=torch.int32, device=device)
        return cls(limbs, degree, bound, bound.size, n, plain_dtype)

    @classmethod
    def from_host(cls, limbs: np.ndarray, degree: np.ndarray, bound, n: int, device,
                  plain_dtype=None) -> "Ciphered":
        torch = _torch()
        bound = _u32(bound)
        l = torch.from_numpy(np.ascontiguousarray(limbs, dtype=np.uint64).view(np.int64)).to(device)
        d = torch.from_numpy(np.ascontiguousarray(degree, dtype=np.uint32).view(np.int32)
                             .reshape(n, bound.size)).to(device)
        return cls(l, d, bound, bound.size, n, plain_dtype)

    def __len__(self):
        return self.nbits

    @property
    def stride(self) -> int:
        return batch_stride(self.bound)

    def _c(self) -> HmBatch:
        self._bound_keep = self.bound  # keep the host array alive for the call
        return HmBatch(self.limbs.data_ptr(), self.degree.data_ptr(), _p32(self.bound), self.nbits,
                       self.n)

    def to_host(self) -> tuple[np.ndarray, np.ndarray]:
        l = self.limbs.cpu().numpy().view(np.uint64)
        d = self.degree.cpu().numpy().view(np.uint32).reshape(self.n * self.nbits)
        return l, d

    def nbytes(self) -> int:
        return self.stride * 8 * self.n

    def to_wire(self, ctx: "Context") -> bytes:
        """The batch's wire image (include/homomorph_gpu.h "wire format"; synchronous)."""
        size = int(lib().hm_wire_bytes(self.nbits, _p32(self.bound), self.n))
        if size == 0:
            raise EngineError(_lib.ERR_UNSUPPORTED, "to_wire")
        buf = (ctypes.c_uint8 * size)()
        c = self._c()
        _check(lib().hm_wire_encode(ctx._h, ctypes.byref(c), buf, size), "hm_wire_encode")
        return bytes(buf)

    @classmethod
    def from_wire(cls, ctx: "Context", data: bytes, plain_dtype=None) -> "Ciphered":
        """A device batch from a wire image (validated on the host: HM_ERR_BAD_INPUT)."""
        info = wire_info(data)
        out = cls.empty(info["n"], info["bound"], ctx.device, plain_dtype)
        c = out._c()
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        ctx._launch(lambda: lib().hm_wire_decode(ctx._h, buf, len(data), ctypes.byref(c)),
                    "hm_wire_decode")
        return out


class Polys:
    """n independent polynomials of `cap` limbs on one GPU (unit-parity primitives)."""

    def __init__(self, limbs, degree, cap: int, n: int):
        self.limbs, self.degree, self.cap, self.n = limbs, degree, int(cap), int(n)

    @classmethod
    def from_host(cls, limbs: np.ndarray, device) -> "Polys":
        torch = _torch()
        limbs = np.ascontiguousarray(limbs, dtype=np.uint64)
        n, cap = limbs.shape
        deg = np.array([_deg(r) for r in limbs], dtype=np.uint32)
        return cls(torch.from_numpy(limbs.view(np.int64)).to(device),
                   torch.from_numpy(deg.view(np.int32)).to(device), cap, n)

    @classmethod
    def empty(cls, n: int, cap: int, device) -> "Polys":
        torch = _torch()
        return cls(torch.empty(n * cap, dtype=torch.int64, device=device),
                   torch.empty(n, dtype=torch.int32, device=device), cap, n)

    def _c(self) -> HmPolys:
        return HmPolys(self.limbs.data_ptr(), self.degree.data_ptr(), self.cap, self.n)

    def to_host(self):
        return (self.limbs.cpu().numpy().view(np.uint64).reshape(self.n, self.cap),
                self.degree.cpu().numpy().view(np.uint32))


_NP_PLAIN = {np.dtype(t).name: np.dtype(t) for t in
             (np.uint8, np.uint16, np.uint32, np.uint64, np.int8, np.int16, np.int32, np.int64)}


class Context:
    """Context (src/context.rs:300-596) bound to one GPU; every call is batched over values."""

    def __init__(self, parameters: Parameters, device=None):
        torch = _torch()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self._params = parameters
        h = ctypes.c_void_p()
        st = lib().hm_ctx_create(parameters.d, parameters.dp, parameters.delta, parameters.tau,
                                 self.device.index or 0, ctypes.byref(h))
        _check(st, "hm_ctx_create")
        self._h = h
        # The engine launches on a dedicated torch-created stream.  Every launching call first
        # makes that stream wait for the caller's current stream and afterwards makes the caller's
        # stream wait for it (event record + wait, asynchronous), so torch-side producers and
        # consumers of the buffers are ordered with the kernels whatever stream the caller uses.
        self._stream = torch.cuda.Stream(device=self.device)
        _check(lib().hm_ctx_set_stream(self._h, ctypes.c_void_p(self._stream.cuda_stream)),
               "hm_ctx_set_stream")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                lib().hm_ctx_destroy(h)
            except Exception:
                pass
            self._h = None

    def _launch(self, fn, what: str):
        torch = _torch()
        if torch.cuda.is_current_stream_capturing():
            # inside Context.graph: the engine stream is the capture stream
            self._check_hip(fn(), what)
            return
        cur = torch.cuda.current_stream(self.device)
        self._stream.wait_stream(cur)
        st = fn()
        cur.wait_stream(self._stream)
        self._check_hip(st, what)

    def _check_hip(self, st: int, what: str):
        if st == _lib.ERR_HIP:  # name the runtime's own code (hm_ctx_last_hip_error)
            what = f"{what} (hipError_t {lib().hm_ctx_last_hip_error(self._h)})"
        _check(st, what)

    def graph(self, fn, warmup: int = 1) -> "EngineGraph":
        """Capture the engine launches `fn` makes into one HIP graph on the engine stream and
        return it (`.replay()` re-runs it over the same buffers).  `fn` runs `warmup` times
        first, so that workspaces and decrypt tables are allocated outside the capture;
        launch-bound sequences (encrypt + decrypt of a batch) then cost one graph launch instead
        of one host round trip per kernel.  The graph holds raw pointers to the context's
        buffers: it refuses to replay once the context has replaced any of them
        (hm_ctx_generation, e.g. after a bigger batch or a new key)."""
        torch = _torch()
        for _ in range(warmup):
            fn()
        self.synchronize()
        gen = self.generation()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self._stream):
            fn()
        if self.generation() != gen:
            raise EngineError(_lib.ERR_INVALID_ARGUMENT,
                              "graph capture: the context replaced a buffer during capture "
                              "(run more warm-up calls)")
        return EngineGraph(self, g, gen)

    ADD_CHAINS = {"auto": 0, "mfma": 1, "valu": 2}

    def set_add_options(self, chain: str = "auto"):
        """hm_ctx_set_add_options: where the adder's carry products run -- "mfma" (fp4 matrix
        cores, a {0,1} Toeplitz product reduced mod 2), "valu" (scalar-decided XORs) or "auto"
        (MFMA when the plan fits).  Results are identical either way (every product is exact);
        "mfma" on a plan it cannot run makes the add raise EngineError (HM_ERR_UNSUPPORTED)."""
        _check(lib().hm_ctx_set_add_options(self._h, self.ADD_CHAINS[chain]),
               "hm_ctx_set_add_options")

    def set_add_pipeline(self, enable: bool = True):
        """hm_ctx_set_add_pipeline: run big MFMA-chain adds as two halves whose second prep
        overlaps the first chain (default off: no faster on configs[1]).  Results are identical
        either way."""
        _check(lib().hm_ctx_set_add_pipeline(self._h, int(bool(enable))), "hm_ctx_set_add_pipeline")

    TIMED_KERNELS = {"add_chain": 1, "encrypt": 2, "decrypt": 3}

    def set_kernel_timing(self, enable: bool = True, kernel: str = "add_chain"):
        """hm_ctx_set_kernel_timing: time the launches of `kernel` ("add_chain": the adder's
        carry chain, "encrypt", "decrypt") made or captured from now on (one record slot each,
        up to 128; a captured launch's slot is valid for one replay, see clear_kernel_timing)
        by device wall-clock stamps; kernel_timing() reads them back.  Resets the record."""
        k = self.TIMED_KERNELS[kernel] if enable else 0
        _check(lib().hm_ctx_set_kernel_timing(self._h, k), "hm_ctx_set_kernel_timing")

    def clear_kernel_timing(self):
        """hm_ctx_clear_kernel_timing: clear every slot's stamps, keeping the slots, so that the
        next replay of a graph captured under timing can be read on its own."""
        _check(lib().hm_ctx_clear_kernel_timing(self._h), "hm_ctx_clear_kernel_timing")

    def kernel_timing(self):
        """(summed kernel ms, launches) of the timed kernel since set_kernel_timing."""
        t = ctypes.c_double(0.0)
        n = ctypes.c_uint32(0)
        _check(lib().hm_ctx_kernel_timing(self._h, ctypes.byref(t), ctypes.byref(n)),
               "hm_ctx_kernel_timing")
        return t.value, n.value

    def set_mul_options(self, karatsuba_min_words: int = 256, karatsuba_leaf_words: int = 256):
        """hm_ctx_set_mul_options: which carry products of the multiplier run as Karatsuba
        recursions (shorter operand >= karatsuba_min_words words; 0 = never) and their leaf
        size.  Results are identical either way (every product is exact)."""
        _check(lib().hm_ctx_set_mul_options(self._h, karatsuba_min_words, karatsuba_leaf_words),
               "hm_ctx_set_mul_options")

    def set_mul_scratch(self, words_per_value: int = 200_000_000):
        """hm_ctx_set_mul_scratch: the Karatsuba scratch (32-bit words per value and lane) above
        which a product's recursion is planned one subtree at a time.  Results are identical
        either way."""
        _check(lib().hm_ctx_set_mul_scratch(self._h, words_per_value), "hm_ctx_set_mul_scratch")

    MUL_PRODUCTS = {"auto": 0, "mfma": 1, "valu": 2}

    def set_mul_products(self, products: str = "auto"):
        """hm_ctx_set_mul_products: where the multiplier's products run -- "mfma" (fp4 matrix
        cores, {0,1} Toeplitz GEMMs reduced mod 2) or "valu".  It covers every product kind of
        the carry-save plan: Karatsuba leaves, schoolbook carry products and the partial products
        of fresh operands (operands below 4 words and the signed circuit's flipped partial
        products stay on the VALU).  "auto" (the default) = MFMA on a gfx950 device, VALU
        elsewhere; "mfma" without the fp4 MFMA raises EngineError (HM_ERR_UNSUPPORTED).  Results
        are identical either way (every product is exact)."""
        _check(lib().hm_ctx_set_mul_products(self._h, self.MUL_PRODUCTS[products]),
               "hm_ctx_set_mul_products")

    def generation(self) -> int:
        return int(lib().hm_ctx_generation(self._h))

    def trim(self):
        """Free retired device buffers (no graph captured earlier may be replayed after)."""
        _check(lib().hm_ctx_trim(self._h), "hm_ctx_trim")

    def mask_bytes(self) -> int:
        """Mask bytes per ciphertext bit: ceil(tau/8) for the LOADED public key's tau."""
        return int(lib().hm_ctx_mask_bytes(self._h))

    def random_bytes(self, n: int):
        """n bytes of the context's device CSPRNG (ChaCha20) as a uint8 device tensor."""
        torch = _torch()
        out = torch.empty(n, dtype=torch.uint8, device=self.device)
        self._launch(lambda: lib().hm_random_bytes(self._h, out.data_ptr(), n), "random_bytes")
        return out

    @property
    def stream(self):
        """The torch stream the engine's kernels run on."""
        return self._stream

    @property
    def parameters(self) -> Parameters:
        return self._params

    def fresh_bound(self) -> int:
        return int(lib().hm_fresh_bound(self._h))

    # ---- keys
    def seed_rng(self, seed: int):
        _check(lib().hm_ctx_seed_rng(self._h, seed & (2**64 - 1)), "hm_ctx_seed_rng")

    def generate_secret_key(self):
        _check(lib().hm_ctx_generate_secret_key(self._h), "generate_secret_key")

    def generate_public_key(self):
        _check(lib().hm_ctx_generate_public_key(self._h), "generate_public_key")

    def set_secret_key(self, sk: SecretKey):
        _check(lib().hm_ctx_set_secret_key(self._h, _p64(sk.limbs), sk.limbs.size),
               "set_secret_key")

    def set_public_key(self, pk: PublicKey):
        _check(lib().hm_ctx_set_public_key(self._h, _p64(pk.limbs), pk.limbs.shape[0],
                                           pk.limbs.shape[1]), "set_public_key")

    def get_secret_key(self) -> SecretKey | None:
        n = ctypes.c_size_t()
        st = lib().hm_ctx_get_secret_key(self._h, None, 0, ctypes.byref(n))
        if st == _lib.ERR_SECRET_KEY_UNSET:
            return None
        _check(st, "get_secret_key")
        out = np.zeros(n.value, dtype=np.uint64)
        _check(lib().hm_ctx_get_secret_key(self._h, _p64(out), out.size, None), "get_secret_key")
        return SecretKey(out)

    def get_public_key(self) -> PublicKey | None:
        tau, lpp = ctypes.c_uint32(), ctypes.c_uint32()
        st = lib().hm_ctx_get_public_key(self._h, None, 0, ctypes.byref(tau), ctypes.byref(lpp))
        if st == _lib.ERR_PUBLIC_KEY_UNSET:
            return None
        _check(st, "get_public_key")
        out = np.zeros((tau.value, lpp.value), dtype=np.uint64)
        _check(lib().hm_ctx_get_public_key(self._h, _p64(out), out.size, None, None),
               "get_public_key")
        return PublicKey(out)

    # ---- cipher
    def encrypt(self, data, masks=None, bound=None) -> Ciphered:
        """Context::encrypt over a batch.  data: 1-D array of one integer dtype (the bincode fixint
        LE image of each value is its little-endian bytes) or an (n, nbytes) uint8 array.  masks:
        (n, 8*nbytes, ceil(tau/8)) uint8 subset masks with tau = the loaded public key's row count
        (the bytes CipheredBit::part draws, cipher.rs:92-97) -- the parity-test contract; when
        omitted the engine draws them from its CSPRNG, as the reference draws from getrandom."""
        torch = _torch()
        plain_dtype = None
        if isinstance(data, torch.Tensor):
            data = data.cpu().numpy()
        arr = np.asarray(data)
        if arr.ndim == 2 and arr.dtype == np.uint8:
            raw = np.ascontiguousarray(arr)
        else:
            plain_dtype = arr.dtype
            raw = np.ascontiguousarray(arr.astype(arr.dtype.newbyteorder("<"))).view(np.uint8)
            raw = raw.reshape(arr.shape[0], arr.dtype.itemsize)
        n, nbytes = raw.shape
        nbits = 8 * nbytes
        mb = self.mask_bytes()
        if mb == 0:
            _check(_lib.ERR_PUBLIC_KEY_UNSET, "encrypt")
        dev_data = torch.from_numpy(raw).to(self.device)
        if masks is None:
            dev_masks = None
        elif isinstance(masks, torch.Tensor):
            dev_masks = masks.to(self.device, torch.uint8).contiguous()
        else:
            dev_masks = torch.from_numpy(np.ascontiguousarray(masks, dtype=np.uint8)).to(self.device)
        if dev_masks is not None and dev_masks.numel() != n * nbits * mb:
            raise ValueError(f"masks must be (n, 8*nbytes, {mb}) bytes: ceil(tau/8) per bit for "
                             f"the loaded public key's tau")
        if bound is None:
            bound = np.full(nbits, self.fresh_bound(), dtype=np.uint32)
        out = Ciphered.empty(n, bound, self.device, plain_dtype)
        c = out._c()
        mptr = None if dev_masks is None else dev_masks.data_ptr()
        self._launch(lambda: lib().hm_encrypt_batch(self._h, dev_data.data_ptr(), nbytes, mptr,
                                                    ctypes.byref(c)), "encrypt")
        out._keep = (dev_data, dev_masks)
        return out

    def decrypt_bytes(self, c: Ciphered):
        """Context::decrypt over a batch -> (n, nbits/8) uint8 device tensor."""
        torch = _torch()
        if c.nbits % 8:
            raise CipherError(_lib.ERR_INVALID_CIPHERED_LENGTH, "decrypt")
        out = torch.empty((c.n, c.nbits // 8), dtype=torch.uint8, device=self.device)
        cb = c._c()
        self._launch(lambda: lib().hm_decrypt_batch(self._h, ctypes.byref(cb), out.data_ptr()),
                     "decrypt")
        return out

    def decrypt(self, c: Ciphered, dtype=None) -> np.ndarray:
        raw = self.decrypt_bytes(c).cpu().numpy()
        dt = np.dtype(dtype) if dtype is not None else c.plain_dtype
        if dt is None:
            return raw
        return raw.view(dt.newbyteorder("<")).reshape(c.n).astype(dt)

    # ---- operations (Context::apply1 / apply2, src/context.rs:496-527)
    def validate_operation(self, op) -> None:
        """Context::validate_operation (src/context.rs:310-323).  Built-in operations ask the
        engine (hm_validate_operation); a user operation supplies MIN_D_OVER_DELTA itself."""
        if not hasattr(op, "CODE"):
            req = int(op.MIN_D_OVER_DELTA)
            if self._params.d < req * self._params.delta:
                raise OperationError(req, self._params.d, self._params.delta)
            return
        req = ctypes.c_uint16()
        st = lib().hm_validate_operation(self._h, op.CODE, ctypes.byref(req))
        if st == _lib.ERR_INVALID_PARAMETERS:
            raise OperationError(req.value, self._params.d, self._params.delta)
        _check(st, "validate_operation")

    def apply2(self, op, a: Ciphered, b: Ciphered, out_bound=None, signed=None) -> Ciphered:
        self.validate_operation(op)
        if op is HomomorphicAddition:
            need = add_out_bounds(a.bound, b.bound)
        elif op is HomomorphicMultiplication:
            if signed is None:
                signed = a.plain_dtype is not None and np.issubdtype(a.plain_dtype, np.signedinteger)
            need = mul_out_bounds(a.bound, b.bound, signed)
        else:
            need = gate_out_bounds(op, a.bound, b.bound)
        out = Ciphered.empty(a.n, need if out_bound is None else out_bound, self.device,
                             a.plain_dtype)
        ca, cb, co = a._c(), b._c(), out._c()
        if op is HomomorphicAddition:
            fn = lambda: lib().hm_add_batch(self._h, ctypes.byref(ca), ctypes.byref(cb),  # noqa
                                            ctypes.byref(co))
        elif op is HomomorphicMultiplication:
            fn = lambda: lib().hm_mul_batch(self._h, ctypes.byref(ca), ctypes.byref(cb),  # noqa
                                            int(signed), ctypes.byref(co))
        else:
            fn = lambda: lib().hm_gate_batch(self._h, op.CODE, ctypes.byref(ca),  # noqa
                                             ctypes.byref(cb), ctypes.byref(co))
        self._launch(fn, op.__name__)
        return out

    def mul_plan_work(self, a_bound, b_bound, k=None, signed=False) -> float:
        """hm_mul_plan_work: the carry products' word pairs as this context's plan runs them
        (Karatsuba products by their leaves) for the low k output bits (all when k is None)."""
        a, b = _u32(a_bound), _u32(b_bound)
        k = a.size if k is None else int(k)
        w = ctypes.c_double()
        _check(lib().hm_mul_plan_work(self._h, a.size, k, _p32(a), _p32(b), int(signed),
                                      ctypes.byref(w)), "hm_mul_plan_work")
        return w.value

    def mul_low(self, a: Ciphered, b: Ciphered, k: int) -> Ciphered:
        """Low k bits of HomomorphicMultiplication on a and b: bit-exact
        equal to the k-bit carry-save circuit on the low k bits (common.rs:66-105), which is how
        a u32 multiply's first k result bits are obtained when the full u32 circuit is
        infeasible (its output alone is ~8.4 GiB per value)."""
        self.validate_operation(HomomorphicMultiplication)
        if not 1 <= k <= a.nbits:
            raise ValueError("k must be in 1..nbits")
        need = mul_out_bounds(a.bound[:k], b.bound[:k])
        out = Ciphered.empty(a.n, need, self.device, None)
        ca, cb, co = a._c(), b._c(), out._c()
        self._launch(lambda: lib().hm_mul_low_batch(self._h, ctypes.byref(ca), ctypes.byref(cb),
                                                    k, ctypes.byref(co)), "mul_low")
        return out

    def apply1(self, op, a: Ciphered) -> Ciphered:
        """Context::apply1 (src/context.rs:496-510): validate, then HomomorphicOperation1::apply
        on `&mut a` -- IN PLACE, as the reference mutates its argument (the NOT gate keeps every
        bound, so the kernel writes each bit over the one it read).  Returns `a` itself."""
        self.validate_operation(op)
        need = gate_out_bounds(op, a.bound)
        if not np.array_equal(need, a.bound):
            raise ValueError(f"{op.__name__} changes the bounds: not an in-place operation")
        ca = a._c()
        self._launch(lambda: lib().hm_gate_batch(self._h, op.CODE, ctypes.byref(ca), None,
                                                 ctypes.byref(ca)), op.__name__)
        return a

    def apply_n(self, op, args) -> Ciphered:
        """Context::apply_n (src/context.rs:535-546): validate `op`'s MIN_D_OVER_DELTA, then call
        the user operation `op.apply(ctx, args)` (HomomorphicOperation<N>, operations.rs:204-213:
        the crate ships no N-ary operation of its own; a user op composes the batched ones)."""
        self.validate_operation(op)
        return op.apply(self, list(args))

    # ---- polynomial primitives
    def poly_add(self, a: Polys, b: Polys) -> Polys:
        out = Polys.empty(a.n, max(a.cap, b.cap), self.device)
        ca, cb, co = a._c(), b._c(), out._c()
        self._launch(lambda: lib().hm_poly_add_batch(self._h, ctypes.byref(ca), ctypes.byref(cb),
                                              ctypes.byref(co)), "poly_add")
        return out

    def poly_mul(self, a: Polys, b: Polys) -> Polys:
        out = Polys.empty(a.n, a.cap + b.cap, self.device)
        ca, cb, co = a._c(), b._c(), out._c()
        self._launch(lambda: lib().hm_poly_mul_batch(self._h, ctypes.byref(ca), ctypes.byref(cb),
                                              ctypes.byref(co)), "poly_mul")
        return out

    def poly_rem(self, a: Polys, s_limbs) -> Polys:
        s = np.ascontiguousarray(s_limbs, dtype=np.uint64)
        out = Polys.empty(a.n, a.cap, self.device)
        ca, co = a._c(), out._c()
        self._launch(lambda: lib().hm_poly_rem_batch(self._h, ctypes.byref(ca), _p64(s), s.size,
                                                     ctypes.byref(co)), "poly_rem")
        return out

    def synchronize(self):
        """Wait for the engine's stream; raise the first device-side error flagged since the
        last check (capacity / bad input)."""
        _check(lib().hm_ctx_synchronize(self._h), "device")


class EngineGraph:
    """A captured sequence of engine launches (Context.graph).  Replays only while the context
    still owns the buffers the capture recorded (hm_ctx_generation unchanged)."""

    def __init__(self, ctx: Context, graph, generation: int):
        self._ctx, self._g, self._gen = ctx, graph, generation

    def replay(self):
        """Replay on the context's stream, so the replay is ordered with the context's other
        launches (before it and after it) like the calls it captured."""
        if self._ctx.generation() != self._gen:
            raise EngineError(_lib.ERR_INVALID_ARGUMENT,
                              "graph replay: the context replaced a buffer this graph uses "
                              "(capture it again)")
        with _torch().cuda.stream(self._ctx.stream):
            self._g.replay()


def add_into(ctx: Context, a: Ciphered, b: Ciphered, out: Ciphered) -> None:
    """hm_add_batch into a preallocated output (no allocation on the launch path)."""
    ca, cb, co = a._c(), b._c(), out._c()
    ctx._launch(lambda: lib().hm_add_batch(ctx._h, ctypes.byref(ca), ctypes.byref(cb),
                                           ctypes.byref(co)), "hm_add_batch")


def mul_into(ctx: Context, a: Ciphered, b: Ciphered, out: Ciphered, signed=False) -> None:
    ca, cb, co = a._c(), b._c(), out._c()
    ctx._launch(lambda: lib().hm_mul_batch(ctx._h, ctypes.byref(ca), ctypes.byref(cb),
                                           int(signed), ctypes.byref(co)), "hm_mul_batch")


def mul_low_into(ctx: Context, a: Ciphered, b: Ciphered, k: int, out: Ciphered) -> None:
    """hm_mul_low_batch into a preallocated k-bit output (bounds: mul_out_bounds of the first k
    input bounds)."""
    ca, cb, co = a._c(), b._c(), out._c()
    ctx._launch(lambda: lib().hm_mul_low_batch(ctx._h, ctypes.byref(ca), ctypes.byref(cb), k,
                                               ctypes.byref(co)), "hm_mul_low_batch")


def value_slice(c: Ciphered, lo: int, hi: int) -> Ciphered:
    """Values [lo, hi) of a batch as a view (one value's limbs and degrees are contiguous)."""
    s = c.stride
    return Ciphered(c.limbs[lo * s: hi * s], c.degree[lo:hi], c.bound, c.nbits, hi - lo,
                    c.plain_dtype)


def pad_bits(c: Ciphered, nbits: int) -> Ciphered:
    """A copy of c widened to nbits ciphertext bits per value, the new bits null polynomials
    (bound 0, one zero limb): e.g. a k-bit product decrypted as a 16-bit value."""
    torch = _torch()
    extra = int(nbits) - c.nbits
    if extra < 0:
        raise ValueError("pad_bits only widens")
    limbs = torch.cat([c.limbs.view(c.n, c.stride),
                       torch.zeros((c.n, extra), dtype=c.limbs.dtype, device=c.limbs.device)],
                      dim=1).reshape(-1)
    deg = torch.cat([c.degree.view(c.n, c.nbits),
                     torch.zeros((c.n, extra), dtype=c.degree.dtype, device=c.degree.device)], dim=1)
    bound = np.concatenate([c.bound, np.zeros(extra, dtype=np.uint32)])
    return Ciphered(limbs, deg, bound, nbits, c.n, c.plain_dtype)
