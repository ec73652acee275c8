// capi.cpp — host side of the C ABI declared in include/homomorph_gpu.h.
//
// Owns the per-device context (keys, derived decrypt table, workspace, stream), validates every
// call the way the reference's safe wrappers do (Context::validate_operation, src/context.rs:
// 310-323; Parameters::new asserts, :87-94), computes static degree bounds and per-wave LDS carve-
// outs, and launches the kernels of kernels.hip.  Never throws across the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include <sys/random.h>

#include "ctx.h"

using namespace hm;

namespace {

uint64_t splitmix64(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

size_t degree_of(const uint64_t *c, size_t n) {
    for (size_t k = n; k-- > 0;)
        if (c[k]) return 64 * k + 63 - (size_t)__builtin_clzll(c[k]);
    return 0;
}

// getrandom(2) into buf (the reference's getrandom::fill, src/polynomial.rs:87, cipher.rs:95)
bool os_random(void *buf, size_t n) {
    uint8_t *p = (uint8_t *)buf;
    while (n) {
        const ssize_t r = getrandom(p, n, 0);
        if (r < 0) return false;
        p += r, n -= (size_t)r;
    }
    return true;
}

// Polynomial::random(degree) (src/polynomial.rs:73-96): limbs from getrandom, or from the
// context's SplitMix64 stream once hm_ctx_seed_rng fixed it (test contract); top bit forced,
// bits above it cleared (:89-90).
bool random_poly(hm_ctx *c, size_t degree, std::vector<uint64_t> &v) {
    v.assign(degree / 64 + 1, 0);
    if (c->seeded) {
        for (auto &w : v) w = splitmix64(c->rng);
    } else if (!os_random(v.data(), v.size() * 8)) {
        return false;
    }
    v.back() &= (1ull << (degree % 64)) - 1;
    v.back() |= 1ull << (degree % 64);
    return true;
}

void wipe(void *p, size_t n) {
    volatile uint8_t *q = (volatile uint8_t *)p;
    for (size_t i = 0; i < n; ++i) q[i] = 0;
}

// Host carry-less product for key generation only (setup path, runs once per key).
std::vector<uint64_t> clmul_host(const std::vector<uint64_t> &a, const std::vector<uint64_t> &b) {
    std::vector<uint64_t> r(a.size() + b.size(), 0);
    for (size_t i = 0; i < a.size(); ++i) {
        for (size_t j = 0; j < b.size(); ++j) {
            uint64_t lo = 0, hi = 0, x = a[i], y = b[j];
            while (x) {
                unsigned k = (unsigned)__builtin_ctzll(x);
                lo ^= y << k;
                if (k) hi ^= y >> (64 - k);
                x &= x - 1;
            }
            r[i + j] ^= lo;
            r[i + j + 1] ^= hi;
        }
    }
    return r;
}

// 64x64 bit-matrix transpose in place: bit j of m[u] moves to bit u of m[j] (block swaps of
// halving size; the remainder table's columns are built as rows of X^k mod S)
void transpose64(uint64_t m[64]) {
    uint64_t mask = 0x00000000FFFFFFFFull;
    for (unsigned s = 32; s; s >>= 1, mask ^= mask << s)
        for (unsigned u = 0; u < 64; u = ((u | s) + 1) & ~s) {
            const uint64_t x = ((m[u] >> s) ^ m[u | s]) & mask;
            m[u] ^= x << s;
            m[u | s] ^= x;
        }
}

uint16_t min_d_over_delta(hm_op op) { // src/impls/numbers.rs:27-50
    switch (op) {
    case HM_OP_AND: case HM_OP_OR: return 2;
    case HM_OP_XOR: case HM_OP_NOT: return 1;
    case HM_OP_ADD: return 21;
    case HM_OP_MUL: case HM_OP_MUL_SIGNED: return 64;
    }
    return 0xFFFF;
}

// the bound of an output must cover the computed bound, bit by bit
bool covers(const hm_batch *out, const std::vector<uint32_t> &need) {
    for (uint32_t i = 0; i < out->nbits; ++i)
        if (out->bound[i] < need[i]) return false;
    return true;
}

// Uploads the public key rows, and (when it fits an LDS budget) the encryption nibble table:
// for every group g of four rows, the 16 XOR combinations T[g][n] = XOR_{k: bit k of n} T_{4g+k}
// (rows past tau are zero).  Built once per key, so encryption blocks only copy it into LDS.
// Layout [g][limb pair p][n][2 limbs] (a missing last limb is zero): the 16 entries' copies of
// one limb pair are 16 B apart, so a wave's per-lane lookups (any n per lane) of one pair are a
// conflict-free ds_read_b128 -- 16 distinct addresses cover the 64 LDS banks exactly once.
hm_status upload_pk(hm_ctx *c) {
    DeviceGuard g(c->device);
    HM_HIP(c, hipStreamSynchronize(c->stream));
    retire(c, c->d_pk, 0, false), c->d_pk = nullptr;
    retire(c, c->d_pk_tab, 0, false), c->d_pk_tab = nullptr;
    retire(c, c->d_pk_tab1, 0, false), c->d_pk_tab1 = nullptr;
    HM_HIP(c, hipMalloc(&c->d_pk, c->pk.size() * 8));
    HM_HIP(c, hipMemcpy(c->d_pk, c->pk.data(), c->pk.size() * 8, hipMemcpyHostToDevice));
    const uint32_t G = (c->pk_tau + 3) / 4, PC = c->pk_cap, NP = (PC + 1) / 2;
    const size_t words = (size_t)G * NP * 16 * 2;
    if (words * 8 <= kEncTableBytes) {
        std::vector<uint64_t> tab(words, 0);
        for (uint32_t grp = 0; grp < G; ++grp)
            for (uint32_t n = 0; n < 16; ++n)
                for (uint32_t k = 0; k < 4; ++k)
                    if (((n >> k) & 1u) && 4 * grp + k < c->pk_tau)
                        for (uint32_t l = 0; l < PC; ++l)
                            tab[(((size_t)grp * NP + l / 2) * 16 + n) * 2 + l % 2] ^=
                                c->pk[(size_t)(4 * grp + k) * PC + l];
        HM_HIP(c, hipMalloc(&c->d_pk_tab, words * 8));
        HM_HIP(c, hipMemcpy(c->d_pk_tab, tab.data(), words * 8, hipMemcpyHostToDevice));
        if (c->pk_top1) {
            // the same table without the one-bit top limb (EncArgs::top1): pairs of limbs
            // 0 .. PC-2 only, NP1 = (PC - 1 + 1) / 2 pairs per group -- a third smaller at PC = 5
            const uint32_t NP1 = PC / 2;
            std::vector<uint64_t> tab1((size_t)G * NP1 * 32, 0);
            for (uint32_t grp = 0; grp < G; ++grp)
                for (uint32_t p = 0; p < NP1; ++p)
                    for (uint32_t k = 0; k < 32; ++k)
                        if (2 * p + k % 2 < PC - 1)
                            tab1[((size_t)grp * NP1 + p) * 32 + k] = tab[((size_t)grp * NP + p) * 32 + k];
            HM_HIP(c, hipMalloc(&c->d_pk_tab1, tab1.size() * 8));
            HM_HIP(c, hipMemcpy(c->d_pk_tab1, tab1.data(), tab1.size() * 8, hipMemcpyHostToDevice));
        }
    }
    return HM_OK;
}

void drop_secret(hm_ctx *c) {
    // SecretKey's Drop zeroizes (src/context.rs:197-206): zero host copy and device tables
    if (!c->sk.empty()) {
        volatile uint64_t *p = c->sk.data();
        for (size_t i = 0; i < c->sk.size(); ++i) p[i] = 0;
    }
    c->sk.clear();
    if (c->d_z) {
        (void)hipStreamSynchronize(c->stream);
        retire(c, c->d_z, (size_t)c->z_limbs * 8, true);
        c->d_z = nullptr;
        c->z_limbs = 0;
    }
    c->has_sk = false;
}

// z_k = (X^k mod S)(0) for k < 64*limbs: the decrypt functional (DESIGN.md "Decryption").
hm_status ensure_ztable(hm_ctx *c, uint32_t max_bound) {
    const uint32_t need = max_bound / 64 + 1;
    if (c->d_z && c->z_limbs >= need) return HM_OK;
    const size_t ds = degree_of(c->sk.data(), c->sk.size());
    bool nonzero = false;
    for (auto w : c->sk) nonzero |= (w != 0);
    if (!nonzero) return HM_ERR_DIVIDE_BY_ZERO;
    if (ds == 0) return HM_ERR_DIVISOR_IS_ONE;
    const size_t sl = ds / 64 + 1;
    std::vector<uint64_t> r(sl, 0), z(need, 0);
    r[0] = 1; // X^0
    for (size_t k = 0; k < (size_t)need * 64; ++k) {
        if (r[0] & 1) z[k / 64] |= 1ull << (k % 64);
        // r = X*r mod S  (r has degree < ds)
        uint64_t carry = 0;
        for (size_t w = 0; w < sl; ++w) {
            uint64_t nc = r[w] >> 63;
            r[w] = (r[w] << 1) | carry;
            carry = nc;
        }
        if ((r[ds / 64] >> (ds % 64)) & 1)
            for (size_t w = 0; w < sl; ++w) r[w] ^= c->sk[w];
    }
    DeviceGuard g(c->device);
    size_t have = (size_t)c->z_limbs * 8;
    HM_HIP(c, grow(c, c->d_z, have, (size_t)need * 8, true));
    HM_HIP(c, hipMemcpy(c->d_z, z.data(), (size_t)need * 8, hipMemcpyHostToDevice));
    wipe(z.data(), z.size() * 8);
    wipe(r.data(), r.size() * 8);
    c->z_limbs = need;
    return HM_OK;
}

// n bytes of the context's ChaCha20 keystream into device memory: the kernel reads the nonce
// from device memory and a second launch advances it, so every draw -- also every replay of a
// captured graph that contains one -- uses a fresh keystream (DESIGN.md "Randomness").
hm_status draw_random(hm_ctx *c, uint8_t *dst, size_t n, bool bump = true) {
    if (!n) return HM_OK;
    RandArgs R{};
    std::memcpy(R.key, c->chacha_key, sizeof(R.key));
    R.nonce = c->d_nonce, R.out = dst, R.nbytes = n;
    const int r = launch_random(R, c->stream, bump);
    wipe(R.key, sizeof(R.key));
    return r ? hip_fail(c, hipGetLastError()) : HM_OK;
}

} // namespace

// The context's auxiliary stream and its fork / mid / join events (the add pipeline, the
// multiplier's second Karatsuba lane), created on first use into locals and stored only when all
// of them exist.
hm_status hm::ensure_aux_stream(hm_ctx *c) {
    if (c->aux_stream) return HM_OK;
    hipStream_t s = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming);
    if (e != hipSuccess) {
        for (hipEvent_t x : ev)
            if (x) (void)hipEventDestroy(x);
        if (s) (void)hipStreamDestroy(s);
        return hip_fail(c, e);
    }
    c->aux_stream = s, c->ev_fork = ev[0], c->ev_mid = ev[1], c->ev_join = ev[2];
    return HM_OK;
}

// The status an hm_* entry returns for the exception its function-try-block caught (HM_ABI_CATCH,
// ctx.h): host containers throw std::bad_alloc; nothing is allowed to unwind into a C, Rust or
// ctypes caller.
hm_status hm::exception_status() noexcept {
    try {
        throw;
    } catch (const std::bad_alloc &) {
        return HM_ERR_OUT_OF_MEMORY;
    } catch (...) {
        return HM_ERR_INTERNAL;
    }
}

// =============================================================================================
extern "C" {

const char *hm_status_string(int s) { // int: any value a foreign caller passes is defined
    switch (s) {
    case HM_OK: return "ok";
    case HM_ERR_INVALID_PARAMETERS: return "invalid parameters (d < min_d_over_delta * delta)";
    case HM_ERR_SECRET_KEY_UNSET: return "secret key unset";
    case HM_ERR_PUBLIC_KEY_UNSET: return "public key unset";
    case HM_ERR_DIVIDE_BY_ZERO: return "attempt to divide by zero";
    case HM_ERR_DIVISOR_IS_ONE: return "divisor is the constant 1";
    case HM_ERR_CAPACITY: return "output exceeds its capacity";
    case HM_ERR_UNSUPPORTED: return "unsupported size";
    case HM_ERR_HIP: return "HIP runtime error";
    case HM_ERR_INVALID_ARGUMENT: return "invalid argument";
    case HM_ERR_INVALID_CIPHERED_LENGTH: return "ciphered length is not a multiple of 8";
    case HM_ERR_BAD_INPUT: return "input degree does not match its limbs";
    case HM_ERR_RANDOMNESS: return "the OS random source failed";
    case HM_ERR_OUT_OF_MEMORY: return "host memory allocation failed";
    case HM_ERR_INTERNAL: return "internal error (C++ exception caught at the ABI)";
    }
    return "unknown status";
}

uint32_t hm_abi_version(void) { return HM_ABI_VERSION; }

hm_status hm_ctx_create(uint16_t d, uint16_t dp, uint16_t delta, uint16_t tau, int device,
                        hm_ctx **out) try {
    if (!out) return HM_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    if (d == 0 || dp == 0 || delta == 0 || tau == 0 || delta >= d) return HM_ERR_INVALID_PARAMETERS;
    hm_ctx *c = new (std::nothrow) hm_ctx();
    if (!c) return HM_ERR_OUT_OF_MEMORY;
    c->d = d, c->dp = dp, c->delta = delta, c->tau = tau, c->device = device;
    uint64_t nonce0 = 0;
    if (!os_random(c->chacha_key, sizeof(c->chacha_key)) || !os_random(&nonce0, sizeof(nonce0))) {
        delete c;
        return HM_ERR_RANDOMNESS; // CipherError::Randomness (src/cipher.rs:18-24)
    }
    DeviceGuard g(device);
    hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&c->d_status, sizeof(int));
    if (e == hipSuccess) e = hipMemset(c->d_status, 0, sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&c->d_nonce, sizeof(uint64_t));
    if (e == hipSuccess) e = hipMemcpy(c->d_nonce, &nonce0, sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (c->d_status) (void)hipFree(c->d_status);
        if (c->d_nonce) (void)hipFree(c->d_nonce);
        if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
        wipe(c->chacha_key, sizeof(c->chacha_key));
        delete c;
        return HM_ERR_HIP;
    }
    c->stream = c->own_stream;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        cus = 256;
    c->cus = (uint32_t)std::max(cus, 1);
    // fp4 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4) is a gfx950 instruction: AUTO strategies use
    // the matrix cores only there, and an explicit MFMA request elsewhere is HM_ERR_UNSUPPORTED
    hipDeviceProp_t prop{};
    c->fp4_mfma = hipGetDeviceProperties(&prop, device) == hipSuccess &&
                  std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
    // test hook: HM_TEST_NO_FP4_MFMA=1 makes this context behave as on a device without the fp4
    // MFMA, so the VALU fallbacks and the explicit-MFMA error path run on the gfx950 test box
    if (const char *v = std::getenv("HM_TEST_NO_FP4_MFMA"); v && v[0] == '1') c->fp4_mfma = false;
    *out = c;
    return HM_OK;
} HM_ABI_CATCH

void hm_ctx_destroy(hm_ctx *c) try {
    if (!c) return;
    DeviceGuard g(c->device);
    (void)hipStreamSynchronize(c->stream);
    drop_secret(c);
    if (c->d_masks) (void)hipMemset(c->d_masks, 0, c->masks_bytes);
    mul_plans_release(c);
    for (void *p : {(void *)c->d_pk, (void *)c->d_pk_tab, (void *)c->d_pk_tab1, (void *)c->d_s,
                    (void *)c->d_ws_add, (void *)c->d_status, (void *)c->d_nonce,
                    (void *)c->d_masks, (void *)c->d_mws, (void *)c->d_kt})
        if (p) (void)hipFree(p);
    for (auto &r : c->retired) (void)hipFree(r.p);
    for (hipEvent_t e : {c->ev_fork, c->ev_mid, c->ev_join})
        if (e) (void)hipEventDestroy(e);
    if (c->aux_stream) (void)hipStreamDestroy(c->aux_stream);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    wipe(c->chacha_key, sizeof(c->chacha_key));
    wipe(&c->rng, sizeof(c->rng));
    delete c;
} catch (...) {
}

uint64_t hm_ctx_generation(const hm_ctx *c) { return c ? c->generation : 0; }

hm_status hm_ctx_trim(hm_ctx *c) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    DeviceGuard g(c->device);
    HM_HIP(c, hipStreamSynchronize(c->stream));
    for (auto &r : c->retired) (void)hipFree(r.p);
    c->retired.clear();
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_set_stream(hm_ctx *c, void *s) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    c->stream = (hipStream_t)s; // NULL = the device's default (null) stream, as in HIP
    return HM_OK;
} HM_ABI_CATCH

void *hm_ctx_stream(const hm_ctx *c) { return c ? (void *)c->stream : nullptr; }

hm_status hm_ctx_parameters(const hm_ctx *c, uint16_t *d, uint16_t *dp, uint16_t *delta,
                            uint16_t *tau) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    if (d) *d = c->d;
    if (dp) *dp = c->dp;
    if (delta) *delta = c->delta;
    if (tau) *tau = c->tau;
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_set_secret_key(hm_ctx *c, const uint64_t *limbs, size_t n) try {
    if (!c || !limbs || n == 0) return HM_ERR_INVALID_ARGUMENT; // from_bytes asserts non-empty
    drop_secret(c);
    c->sk.assign(limbs, limbs + n);
    c->has_sk = true;
    c->has_pk = false; // set_secret_key clears the public key (src/context.rs:568-571)
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_set_public_key(hm_ctx *c, const uint64_t *limbs, uint32_t tau, uint32_t lpp) try {
    if (!c || !limbs || tau == 0 || lpp == 0) return HM_ERR_INVALID_ARGUMENT;
    c->pk.assign(limbs, limbs + (size_t)tau * lpp);
    c->pk_tau = tau, c->pk_cap = lpp;
    c->pk_maxdeg = 0;
    for (uint32_t i = 0; i < tau; ++i)
        c->pk_maxdeg = std::max<uint32_t>(c->pk_maxdeg, (uint32_t)degree_of(&c->pk[(size_t)i * lpp], lpp));
    c->pk_top1 = tau <= 128 && lpp > 1;
    std::memset(c->pk_topcol, 0, sizeof(c->pk_topcol));
    for (uint32_t i = 0; i < tau && c->pk_top1; ++i) {
        const uint64_t top = c->pk[(size_t)i * lpp + lpp - 1];
        if (top > 1) c->pk_top1 = false;
        else c->pk_topcol[i / 32] |= (uint32_t)top << (i % 32);
    }
    hm_status st = upload_pk(c);
    if (st == HM_OK) c->has_pk = true;
    return st;
} HM_ABI_CATCH

hm_status hm_ctx_seed_rng(hm_ctx *c, uint64_t seed) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    // test contract: keys from SplitMix64(seed), masks from ChaCha20 keyed by SplitMix64(seed ^ K)
    c->seeded = true;
    c->rng = seed;
    uint64_t ks = seed ^ 0x6D61736B73636861ull; // "masksCha"
    for (int i = 0; i < 4; ++i) {
        const uint64_t w = splitmix64(ks);
        c->chacha_key[2 * i] = (uint32_t)w, c->chacha_key[2 * i + 1] = (uint32_t)(w >> 32);
    }
    const uint64_t nonce0 = splitmix64(ks);
    DeviceGuard g(c->device);
    HM_HIP(c, hipMemcpyAsync(c->d_nonce, &nonce0, sizeof(nonce0), hipMemcpyHostToDevice, c->stream));
    HM_HIP(c, hipStreamSynchronize(c->stream));
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_generate_secret_key(hm_ctx *c) try { // src/context.rs:421-424
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    std::vector<uint64_t> s;
    if (!random_poly(c, c->d, s)) return HM_ERR_RANDOMNESS;
    hm_status st = hm_ctx_set_secret_key(c, s.data(), s.size());
    wipe(s.data(), s.size() * 8);
    return st;
} HM_ABI_CATCH

hm_status hm_ctx_generate_public_key(hm_ctx *c) try { // src/context.rs:249-261, :444-454
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    if (!c->has_sk) return HM_ERR_SECRET_KEY_UNSET;
    // T_i = S*Q_i + X*R_i.  deg S is d for generated keys but any degree for a key set with
    // set_secret_key (the reference's own example, SecretKey::from_bytes(&[5, 14, 8]) at d = 6,
    // has degree 19): rows are as wide as the widest T_i needs.
    std::vector<std::vector<uint64_t>> rows(c->tau);
    size_t cap = 1;
    for (uint32_t i = 0; i < c->tau; ++i) {
        std::vector<uint64_t> q, r;
        if (!random_poly(c, c->dp, q) || !random_poly(c, c->delta, r)) return HM_ERR_RANDOMNESS;
        std::vector<uint64_t> t = clmul_host(c->sk, q);
        t.resize(std::max(t.size(), r.size() + 1), 0);
        for (size_t w = 0; w < r.size(); ++w) { // + X * R
            t[w] ^= r[w] << 1;
            t[w + 1] ^= r[w] >> 63;
        }
        wipe(q.data(), q.size() * 8);
        wipe(r.data(), r.size() * 8);
        cap = std::max(cap, (size_t)degree_of(t.data(), t.size()) / 64 + 1);
        rows[i] = std::move(t);
    }
    std::vector<uint64_t> all((size_t)c->tau * cap, 0);
    for (uint32_t i = 0; i < c->tau; ++i)
        for (size_t w = 0; w < cap && w < rows[i].size(); ++w) all[(size_t)i * cap + w] = rows[i][w];
    return hm_ctx_set_public_key(c, all.data(), c->tau, (uint32_t)cap);
} HM_ABI_CATCH

hm_status hm_ctx_get_secret_key(const hm_ctx *c, uint64_t *limbs, size_t cap, size_t *n) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    if (!c->has_sk) return HM_ERR_SECRET_KEY_UNSET;
    if (n) *n = c->sk.size();
    if (limbs) {
        if (cap < c->sk.size()) return HM_ERR_CAPACITY;
        std::memcpy(limbs, c->sk.data(), c->sk.size() * 8);
    }
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_get_public_key(const hm_ctx *c, uint64_t *limbs, size_t cap, uint32_t *tau,
                                uint32_t *lpp) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    if (!c->has_pk) return HM_ERR_PUBLIC_KEY_UNSET;
    if (tau) *tau = c->pk_tau;
    if (lpp) *lpp = c->pk_cap;
    if (limbs) {
        if (cap < c->pk.size()) return HM_ERR_CAPACITY;
        std::memcpy(limbs, c->pk.data(), c->pk.size() * 8);
    }
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_set_kernel_timing(hm_ctx *c, int enable) try {
    if (!c || enable < HM_TIME_OFF || enable > HM_TIME_DECRYPT) return HM_ERR_INVALID_ARGUMENT;
    DeviceGuard g(c->device);
    HM_HIP(c, hipStreamSynchronize(c->stream));
    const size_t half = (size_t)kTimedLaunches * kTimerWaves * sizeof(unsigned long long);
    if (enable && !c->d_kt) {
        void *p = nullptr;
        HM_HIP(c, hipMalloc(&p, 2 * half));
        c->d_kt = (unsigned long long *)p;
    }
    if (c->d_kt) { // reset: starts at the maximum (atomic min), ends at 0 (atomic max)
        HM_HIP(c, hipMemset(c->d_kt, 0xFF, half));
        HM_HIP(c, hipMemset((char *)c->d_kt + half, 0, half));
    }
    c->time_kernel = (uint32_t)enable;
    c->kt_next = 0;
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_clear_kernel_timing(hm_ctx *c) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    if (!c->d_kt) return HM_OK;
    DeviceGuard g(c->device);
    HM_HIP(c, hipStreamSynchronize(c->stream));
    const size_t half = (size_t)kTimedLaunches * kTimerWaves * sizeof(unsigned long long);
    HM_HIP(c, hipMemsetAsync(c->d_kt, 0xFF, half, c->stream));
    HM_HIP(c, hipMemsetAsync((char *)c->d_kt + half, 0, half, c->stream));
    HM_HIP(c, hipStreamSynchronize(c->stream));
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_kernel_timing(hm_ctx *c, double *total_ms, uint32_t *launches) try {
    if (!c || !total_ms || !launches) return HM_ERR_INVALID_ARGUMENT;
    *total_ms = 0.0, *launches = 0;
    if (!c->d_kt || !c->kt_next) return HM_OK;
    DeviceGuard g(c->device);
    HM_HIP(c, hipStreamSynchronize(c->stream));
    const size_t n = (size_t)c->kt_next * kTimerWaves;
    std::vector<unsigned long long> t0(n), t1(n);
    HM_HIP(c, hipMemcpy(t0.data(), c->d_kt, n * 8, hipMemcpyDeviceToHost));
    HM_HIP(c, hipMemcpy(t1.data(), c->d_kt + (size_t)kTimedLaunches * kTimerWaves, n * 8,
                        hipMemcpyDeviceToHost));
    int rate_khz = 0; // the wall clock's frequency (100 MHz on gfx9)
    HM_HIP(c, hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, c->device));
    if (rate_khz <= 0) return HM_ERR_UNSUPPORTED;
    double ticks = 0.0;
    uint32_t k = 0;
    for (uint32_t s = 0; s < c->kt_next; ++s) {
        unsigned long long lo = ~0ull, hi = 0ull;
        for (size_t w = (size_t)s * kTimerWaves; w < (size_t)(s + 1) * kTimerWaves; ++w)
            lo = std::min(lo, t0[w]), hi = std::max(hi, t1[w]);
        if (lo == ~0ull || hi < lo) continue; // (a slot whose launch has not run)
        ticks += (double)(hi - lo);
        ++k;
    }
    *total_ms = ticks / rate_khz;
    *launches = k;
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_set_add_options(hm_ctx *c, uint32_t chain) try {
    if (!c || chain > HM_ADD_CHAIN_VALU) return HM_ERR_INVALID_ARGUMENT;
    c->add_chain = chain;
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_set_mul_options(hm_ctx *c, uint32_t ka_min, uint32_t ka_leaf) try {
    if (!c || (ka_min && (ka_leaf < 32 || ka_leaf > 512))) return HM_ERR_INVALID_ARGUMENT;
    c->ka_min = ka_min;
    c->ka_leaf = ka_leaf & ~31u;
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_set_mul_scratch(hm_ctx *c, uint64_t words) try {
    if (!c || words == 0 || words > (1ull << 27) + (1ull << 26)) return HM_ERR_INVALID_ARGUMENT;
    c->ka_scratch = words;
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_set_add_pipeline(hm_ctx *c, int enable) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    c->add_pipe = enable != 0;
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_set_mul_products(hm_ctx *c, uint32_t products) try {
    if (!c || products > HM_MUL_PRODUCTS_VALU) return HM_ERR_INVALID_ARGUMENT;
    if (products == HM_MUL_PRODUCTS_MFMA && !c->fp4_mfma) return HM_ERR_UNSUPPORTED;
    c->mul_products = products;
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_validate_operation(const hm_ctx *c, hm_op op, uint16_t *req) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    const uint16_t m = min_d_over_delta(op);
    if (req) *req = m;
    if ((uint32_t)c->d < (uint32_t)m * (uint32_t)c->delta) return HM_ERR_INVALID_PARAMETERS;
    return HM_OK;
} HM_ABI_CATCH

// A fresh ciphertext bit is a subset sum of public-key rows (plus the plaintext bit), so its
// degree is at most max(d + dp, deg T_i): d + dp for generated keys, more for a loaded key.
uint32_t hm_fresh_bound(const hm_ctx *c) {
    if (!c) return 0;
    const uint32_t b = (uint32_t)c->d + c->dp;
    return c->has_pk ? std::max(b, c->pk_maxdeg) : b;
}

uint32_t hm_ctx_mask_bytes(const hm_ctx *c) { return (c && c->has_pk) ? (c->pk_tau + 7) / 8 : 0; }

uint64_t hm_batch_stride(uint32_t nbits, const uint32_t *bound) {
    uint64_t s = 0;
    for (uint32_t i = 0; i < nbits; ++i) s += cap_of(bound[i]);
    return s;
}

// Degree bounds of common.rs:37-56 (deg(xy) = deg x + deg y, deg(x+y) <= max).
hm_status hm_add_out_bounds(uint32_t L, const uint32_t *a, const uint32_t *b, uint32_t *out) try {
    if (!a || !b || !out || L == 0 || L > HM_MAX_BITS) return HM_ERR_INVALID_ARGUMENT;
    int64_t c = -1; // null carry
    for (uint32_t i = 0; i < L; ++i) {
        const int64_t x = std::max<int64_t>(a[i], b[i]);
        const int64_t s = std::max(x, c);
        if (s >= (int64_t)1 << 30) return HM_ERR_UNSUPPORTED;
        out[i] = (uint32_t)s;
        if (i + 1 < L) {
            const int64_t ab = (int64_t)a[i] + b[i];
            const int64_t p = x + ab;
            c = (c < 0) ? ab : std::max(ab, p + c);
        }
    }
    return HM_OK;
} HM_ABI_CATCH

} // extern "C"

extern "C" {

hm_status hm_mul_out_bounds(uint32_t L, const uint32_t *a, const uint32_t *b, int is_signed,
                            uint32_t *out) try {
    if (!a || !b || !out || L == 0 || L > HM_MAX_BITS) return HM_ERR_INVALID_ARGUMENT;
    std::vector<int64_t> res;
    if (!mul_result_bounds(L, L, a, b, is_signed != 0, res)) return HM_ERR_UNSUPPORTED;
    for (uint32_t i = 0; i < L; ++i) out[i] = (uint32_t)std::max<int64_t>(res[i], 0);
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_mul_cost(uint32_t L, uint32_t k, const uint32_t *a, const uint32_t *b, int is_signed,
                      double *word_pairs, double *out_bytes, double *max_degree) try {
    if (!a || !b || L == 0 || L > HM_MAX_BITS || k == 0 || k > L) return HM_ERR_INVALID_ARGUMENT;
    (void)is_signed; // the signed corners (+1 in column L-1) change no bound
    double w, o, m;
    mul_cost_model(L, k, a, b, w, o, m);
    if (word_pairs) *word_pairs = w;
    if (out_bytes) *out_bytes = o;
    if (max_degree) *max_degree = m;
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_mul_plan_work(hm_ctx *c, uint32_t L, uint32_t k, const uint32_t *a, const uint32_t *b,
                          int is_signed, double *word_pairs) try {
    if (!c || !a || !b || !word_pairs || L == 0 || L > HM_MAX_BITS || k == 0 || k > L)
        return HM_ERR_INVALID_ARGUMENT;
    return mul_plan_work(c, L, k, a, b, is_signed != 0 && k == L, *word_pairs);
} HM_ABI_CATCH

hm_status hm_gate_out_bounds(hm_op g, uint32_t L, const uint32_t *a, const uint32_t *b,
                             uint32_t *out) try {
    if (!a || !out || L == 0 || L > HM_MAX_BITS) return HM_ERR_INVALID_ARGUMENT;
    if (g != HM_OP_NOT && !b) return HM_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < L; ++i) {
        uint64_t v;
        switch (g) {
        case HM_OP_AND: case HM_OP_OR: v = (uint64_t)a[i] + b[i]; break;
        case HM_OP_XOR: v = std::max(a[i], b[i]); break;
        case HM_OP_NOT: v = a[i]; break;
        default: return HM_ERR_INVALID_ARGUMENT;
        }
        if (v >= (1u << 30)) return HM_ERR_UNSUPPORTED;
        out[i] = (uint32_t)v;
    }
    return HM_OK;
} HM_ABI_CATCH

// ------------------------------------------------------------------ cipher
hm_status hm_encrypt_batch(hm_ctx *c, const uint8_t *data, uint32_t nbytes, const uint8_t *masks,
                           hm_batch *out) try {
    if (!c || !out) return HM_ERR_INVALID_ARGUMENT;
    if (!c->has_pk) return HM_ERR_PUBLIC_KEY_UNSET;
    if (hm_status st = check_batch(out); st) return st;
    if (nbytes == 0 || out->nbits != 8 * nbytes) return HM_ERR_INVALID_ARGUMENT;
    if (out->n && !data) return HM_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < out->nbits; ++i)
        if (out->bound[i] < c->pk_maxdeg) return HM_ERR_INVALID_ARGUMENT;
    if (out->n == 0) return HM_OK;
    // launch_encrypt instantiates pk_cap <= 17 limbs; reject the rest BEFORE a mask draw (the
    // encryption kernel advances the CSPRNG nonce: a draw without it would repeat its keystream)
    if (c->pk_cap == 0 || c->pk_cap > 17) return HM_ERR_UNSUPPORTED;
    DeviceGuard g(c->device);
    EncArgs E{};
    E.pk = c->d_pk, E.tau = c->pk_tau, E.pk_cap = c->pk_cap;
    E.pk_tab = c->d_pk_tab;
    E.pk_tab1 = c->d_pk_tab1;
    E.cus = c->cus;
    E.lognbits = -1;
    for (int s = 0; s < 8; ++s)
        if ((8u * nbytes) == (1u << s)) E.lognbits = s;
    E.data = data, E.nbytes = nbytes;
    E.out = batch_arg(out);
    E.n = out->n;
    E.status = c->d_status;
    fill_bounds(E.ob, out);
    E.uniform_cap = 1;
    for (uint32_t i = 0, o = 0; i < out->nbits; ++i) {
        E.ooff.b[i] = o, o += cap_of(out->bound[i]);
        E.uniform_cap &= cap_of(out->bound[i]) == c->pk_cap;
    }
#ifndef HM_ENC_NO_TOP1
    E.top1 = c->pk_top1 && c->d_pk_tab1 ? 1u : 0u;
#endif
    std::memcpy(E.topcol, c->pk_topcol, sizeof(E.topcol));
    if (!masks) {
        // CipheredBit::part draws ceil(tau/8) random bytes per bit (cipher.rs:92-97): here the
        // device ChaCha20 stream, drawn into the context's mask buffer right before the launch;
        // the encryption kernel advances the nonce (no bump launch of its own)
        const size_t mb = (size_t)out->n * out->nbits * ((c->pk_tau + 7) / 8);
        const size_t need = (mb + 63) & ~(size_t)63;
        if (need > c->masks_bytes && c->d_masks) (void)hipMemset(c->d_masks, 0, c->masks_bytes);
        HM_HIP(c, grow(c, c->d_masks, c->masks_bytes, need));
        if (hm_status st = draw_random(c, c->d_masks, mb, false); st) return st;
        masks = c->d_masks;
        E.nonce_bump = c->d_nonce;
    }
    E.masks = masks;
    E.kt = c->ktimer(HM_TIME_ENCRYPT);
    int r = launch_encrypt(E, c->stream);
    if (r == HM_ERR_UNSUPPORTED) return HM_ERR_UNSUPPORTED;
    return r ? hip_fail(c, hipGetLastError()) : HM_OK;
} HM_ABI_CATCH

hm_status hm_random_bytes(hm_ctx *c, uint8_t *dst, size_t nbytes) try {
    if (!c || (nbytes && !dst)) return HM_ERR_INVALID_ARGUMENT;
    DeviceGuard g(c->device);
    return draw_random(c, dst, nbytes);
} HM_ABI_CATCH

hm_status hm_decrypt_batch(hm_ctx *c, const hm_batch *in, uint8_t *out) try {
    if (!c || !in) return HM_ERR_INVALID_ARGUMENT;
    if (!c->has_sk) return HM_ERR_SECRET_KEY_UNSET;
    if (in->nbits % 8) return HM_ERR_INVALID_CIPHERED_LENGTH; // cipher.rs:218-220
    if (hm_status st = check_batch(in); st) return st;
    if (in->n == 0) return HM_OK;
    if (!out) return HM_ERR_INVALID_ARGUMENT;
    uint32_t mb = 0;
    for (uint32_t i = 0; i < in->nbits; ++i) mb = std::max(mb, in->bound[i]);
    if (hm_status st = ensure_ztable(c, mb); st) return st;
    DecArgs D{};
    D.in = batch_arg(in);
    D.n = in->n, D.nbits = in->nbits;
    D.z = c->d_z, D.zlimbs = c->z_limbs;
    D.out = out;
    D.status = c->d_status;
    fill_bounds(D.ib, in);
    for (uint32_t i = 0, o = 0; i < in->nbits; ++i) {
        D.ioff.b[i] = o;
        o += cap_of(in->bound[i]);
        D.maxcap = std::max(D.maxcap, cap_of(in->bound[i]));
    }
    D.ucap = cap_of(in->bound[0]) <= 8 ? cap_of(in->bound[0]) : 0;
    for (uint32_t i = 1; i < in->nbits; ++i)
        if (cap_of(in->bound[i]) != D.ucap) D.ucap = 0;
    D.kt = c->ktimer(HM_TIME_DECRYPT);
    DeviceGuard g(c->device);
    return launch_decrypt(D, c->stream) ? hip_fail(c, hipGetLastError()) : HM_OK;
} HM_ABI_CATCH

// ------------------------------------------------------------------ operations
hm_status hm_add_batch(hm_ctx *c, const hm_batch *a, const hm_batch *b, hm_batch *out) try {
    if (!c || !a || !b || !out) return HM_ERR_INVALID_ARGUMENT;
    if (hm_status st = hm_validate_operation(c, HM_OP_ADD, nullptr); st) return st;
    for (const hm_batch *x : {a, b, (const hm_batch *)out})
        if (hm_status st = check_batch(x); st) return st;
    if (a->nbits != b->nbits || a->nbits != out->nbits || a->n != b->n || a->n != out->n)
        return HM_ERR_INVALID_ARGUMENT;
    const uint32_t L = a->nbits;
    std::vector<uint32_t> need(L);
    if (hm_status st = hm_add_out_bounds(L, a->bound, b->bound, need.data()); st) return st;
    if (!covers(out, need)) return HM_ERR_INVALID_ARGUMENT;
    if (a->n == 0) return HM_OK;

    // Workspace slots (words) and LDS plans, from the static bounds
    uint32_t cntA = 0, cntB = 0, cntAB = 0, cntP = 0, cntX = 1, SC = 2, maxPw = 0;
    int64_t maxb = 0; // the largest input bound
    int64_t cb = -1;
    for (uint32_t i = 0; i < L; ++i) {
        const int64_t ba = a->bound[i], bb = b->bound[i];
        cntA = std::max(cntA, 2 * cap_of(a->bound[i]));
        cntB = std::max(cntB, 2 * cap_of(b->bound[i]));
        cntX = std::max(cntX, words_of_bound(std::max(ba, bb)));
        maxb = std::max(maxb, std::max(ba, bb));
        if (i + 1 < L) {
            const int64_t x = std::max(ba, bb), ab = ba + bb, p = x + ab;
            cntAB = std::max(cntAB, words_of_bound(ab));
            cntP = std::max(cntP, words_of_bound(p));
            maxPw = std::max(maxPw, words_of_bound(p));
            SC = std::max(SC, std::max(words_of_bound(p) + words_of_bound(cb), words_of_bound(ab)) + 2);
            cb = (cb < 0) ? ab : std::max(ab, p + cb);
        }
    }
    cntAB = std::max(cntAB, 1u), cntP = std::max(cntP, 1u);
    auto even = [](uint32_t v) { return (v + 1) & ~1u; };
    AddArgs A{};
    A.cntA = cntA, A.cntB = cntB, A.cntAB = cntAB, A.cntP = cntP, A.cntX = cntX;
    // prep: enough waves per value to keep the chip busy, and at least enough that one wave's
    // product rows (bits x multiplier words) fit its 64 lanes in two passes (bits are dealt in
    // contiguous ranges)
    {
        const uint64_t want = (16384 + a->n - 1) / a->n;
        // (rows_fit: waves per value for one pass of a wave's rows; big batches take two passes
        // per wave -- half the waves: configs[4]'s prep 7.8 -> 5.7 ms per 131,072 adds, the
        // headline's 4 waves per value unchanged, since its `want` is 4 already)
        auto waves = [&](uint32_t rows) { // rows: product rows per bit
            const uint64_t rows_fit = (L + std::max<uint32_t>(1, 64 / rows) - 1) /
                                      std::max<uint32_t>(1, 64 / rows);
            return (uint32_t)std::max<uint64_t>(
                1, std::min<uint64_t>({std::max(want, (rows_fit + 1) / 2), 8, (uint64_t)L}));
        };
        // the top word of every a_i, b_i, x_i holds at most bit 32 (cntX - 1) = maxb: the prep can
        // add its multiples as shifted copies instead of product rows -- worth it when the shorter
        // rows save waves per value or row passes per wave (waves x passes; the headline: 2 passes
        // -> 1 at 4 waves; one wave and one pass per value only pays for the copy passes, +8 us
        // per 65,536 u8 adds)
        const bool t1ok = cntX >= 2 && maxb % 32 == 0;
        // row passes per wave at w waves per value (rows per bit)
        auto passes = [&](uint32_t w, uint32_t rows) { return (((L + w - 1) / w) * rows + 63) / 64; };
        const uint32_t w0 = waves(cntX), w1 = t1ok ? waves(cntX - 1) : w0;
        A.top1 = t1ok && (uint64_t)w1 * passes(w1, cntX - 1) < (uint64_t)w0 * passes(w0, cntX);
        A.wpv = waves(cntX - A.top1);
        // one wave per value already (short values, big batch): several whole values per wave
        // instead when their rows fit one pass (L a power of two: configs[0]'s u8 add, 2 values
        // of 8 bits x 4 rows with the top-word copies; its prep cost is per wave)
        A.vpw = 1, A.lgL = 0;
        if (A.wpv == 1 && (L & (L - 1)) == 0 && a->n >= 16384) {
            const uint32_t rows = cntX - (t1ok ? 1u : 0u);
            const uint32_t v = std::min<uint32_t>(8, 64 / std::max<uint32_t>(1, L * rows));
            if (v >= 2) {
                A.vpw = v, A.top1 = t1ok;
                while ((1u << A.lgL) < L) ++A.lgL;
            }
        }
        const uint32_t bpw = A.vpw > 1 ? A.vpw * L : (L + A.wpv - 1) / A.wpv;
        // (+ 2 bpw: with dAB / dP, stage_ab's bound / offset tables; a wave's range is at most 64 bits)
        if (bpw > 64) return HM_ERR_UNSUPPORTED;
        A.prep_lds = even(bpw * (cntA + cntB + cntX + cntAB + cntP) + 6 * bpw);
        if ((size_t)A.prep_lds * 4 * 4 > 160 * 1024) return HM_ERR_UNSUPPORTED;
    }
    // chain: a carry buffer holds a whole tile of the widest width instantiated (PAD mode);
    // each buffer sits above a zero halo of kHalo words
    const uint32_t need_w = (SC + 63) / 64;
    const uint32_t wmax = need_w <= 4 ? 4 : need_w <= 8 ? 8 : need_w <= 12 ? 12 : need_w <= 16 ? 16 : 24;
    // PAD needs one tile per product (need_w <= 24) and one uniform chunk (P within kQBig
    // words) so that window reads stay inside [-kHalo, 64*wmax)
    A.pad = need_w <= 24 && maxPw <= 25;
    uint32_t cw = SC;
    if (A.pad) cw = std::max(cw, 64 * wmax);
    A.cw = even(cw);
    // staged chain (PAD only): one in-place carry buffer, and everything the chain reads per bit
    // (x_i, ab_i, P_i, degrees) in LDS, so the loop issues no global loads at all
    const uint32_t staged_lds =
        even(A.cw + kHalo + (L - 1) * (cntP + cntAB) + L * cntX + 2 * L);
    A.staged = A.pad && (size_t)staged_lds * 4 * kAddWavesPerBlock <= 160 * 1024;
    A.chain_lds = A.staged ? staged_lds : even(2 * (A.cw + kHalo) + (L - 1) * cntP);
    A.max_prod_words = SC;
    if ((size_t)A.chain_lds * 4 * kAddWavesPerBlock > 160 * 1024) return HM_ERR_UNSUPPORTED;
    // MFMA chain (adder_mfma.hip): P_i within 2*kMfmaChunks-1 words, ab_i within 64 words (two
    // tiles), a bit's workspace record (x, P, ab, two degrees) within one 64-lane LDS-DMA; carry
    // bits for every tile plus the 64-word window overhang of the ring fill
    {
        const uint32_t tiles = (SC + 31) / 32;
        const uint32_t mf_cw = 32 * tiles + 64;
        // the smallest chunk count whose plan fits: P_i within 2 NC - 1 words, ab_i within 64
        // words (two tiles), the bit's record within kRecWords, and x_i below 32 words (the
        // kernel XORs x into sum words 0..31 only; words from 32 up are the carry's, stored by the
        // tiles), for the last bit as for every other; LDS (dynamic + the static record stage)
        // for one block
        auto plan = [&](auto cfg) -> uint32_t {
            using Cfg = decltype(cfg);
            const uint32_t lds = Cfg::kHalo + mf_cw + Cfg::kRingWords + Cfg::kRsWords;
            const bool fits = maxPw <= 2 * Cfg::kChunks - 1 && cntAB <= 64 && cntX <= 32 &&
                              cntX + cntP + cntAB + 2 <= (uint32_t)Cfg::kRecWords &&
                              (256 + (size_t)lds * kAddWavesPerBlock + Cfg::kStageWords) * 4 <=
                                  160 * 1024;
            return fits ? lds : 0u;
        };
        uint32_t nc = 0, lds = 0;
        if ((lds = plan(MfmaCfg<7>{}))) nc = 7;
        else if ((lds = plan(MfmaCfg<13>{}))) nc = 13;
        else if ((lds = plan(MfmaCfg<25>{}))) nc = 25;
        if (!c->fp4_mfma) nc = 0;
        A.mfma = c->add_chain != HM_ADD_CHAIN_VALU ? nc : 0u;
        if (c->add_chain == HM_ADD_CHAIN_MFMA && !nc) return HM_ERR_UNSUPPORTED;
        if (A.mfma) A.mf_cw = mf_cw, A.chain_lds = lds;
    }
    A.ws_stride = ((uint64_t)L * (cntAB + cntP + 2 + cntX) + 63) & ~(uint64_t)63;
    const size_t bytes = (size_t)A.ws_stride * 4 * a->n;
    DeviceGuard g(c->device);
    HM_HIP(c, grow(c, c->d_ws_add, c->ws_add_bytes, bytes));
    A.ws = c->d_ws_add;
    A.a = batch_arg(a), A.b = batch_arg(b), A.out = batch_arg(out);
    A.n = a->n, A.nbits = L;
    A.status = c->d_status;
    fill_bounds(A.ab, a), fill_bounds(A.bb, b), fill_bounds(A.ob, out);
    A.kt = c->ktimer(HM_TIME_ADD_CHAIN);
    // Two-stage pipeline (not while timing the chain): the batch in two halves, the second
    // half's prep on the auxiliary stream right after the first half's, so it runs beside the
    // first half's chain (the chain is matrix-core and latency bound, the prep VALU bound); the
    // halves use disjoint workspace and outputs.  Fork / join by events, so a graph captured on
    // the context stream holds both branches.
    if (c->add_pipe && !A.kt.t0 && A.mfma && a->n >= 2 * kAddPipeMin) {
        if (hm_status st = ensure_aux_stream(c); st) return st;
        const uint64_t h = (a->n / 2 + kAddWavesPerBlock - 1) / kAddWavesPerBlock * kAddWavesPerBlock;
        const AddArgs A1 = add_args_slice(A, 0, h), A2 = add_args_slice(A, h, a->n - h);
        HM_HIP(c, hipEventRecord(c->ev_fork, c->stream));
        HM_HIP(c, hipStreamWaitEvent(c->aux_stream, c->ev_fork, 0));
        if (launch_add_prep(A1, c->stream)) return hip_fail(c, hipGetLastError());
        HM_HIP(c, hipEventRecord(c->ev_mid, c->stream));
        if (launch_add_chain_mfma(A1, c->stream)) return hip_fail(c, hipGetLastError());
        HM_HIP(c, hipStreamWaitEvent(c->aux_stream, c->ev_mid, 0));
        if (launch_add_prep(A2, c->aux_stream)) return hip_fail(c, hipGetLastError());
        if (launch_add_chain_mfma(A2, c->aux_stream)) return hip_fail(c, hipGetLastError());
        HM_HIP(c, hipEventRecord(c->ev_join, c->aux_stream));
        HM_HIP(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
        return HM_OK;
    }
    return launch_add(A, c->stream) ? hip_fail(c, hipGetLastError()) : HM_OK;
} HM_ABI_CATCH

hm_status hm_mul_batch(hm_ctx *c, const hm_batch *a, const hm_batch *b, int is_signed,
                       hm_batch *out) try {
    if (!c || !a || !b || !out) return HM_ERR_INVALID_ARGUMENT;
    if (hm_status st = hm_validate_operation(c, is_signed ? HM_OP_MUL_SIGNED : HM_OP_MUL, nullptr); st)
        return st;
    for (const hm_batch *x : {a, b, (const hm_batch *)out})
        if (hm_status st = check_batch(x); st) return st;
    if (a->nbits != b->nbits || a->nbits != out->nbits || a->n != b->n || a->n != out->n)
        return HM_ERR_INVALID_ARGUMENT;
    return mul_columns(c, a, b, a->nbits, is_signed != 0, out);
} HM_ABI_CATCH

hm_status hm_mul_low_batch(hm_ctx *c, const hm_batch *a, const hm_batch *b, uint32_t k,
                           hm_batch *out) try {
    if (!c || !a || !b || !out) return HM_ERR_INVALID_ARGUMENT;
    if (hm_status st = hm_validate_operation(c, HM_OP_MUL, nullptr); st) return st;
    for (const hm_batch *x : {a, b, (const hm_batch *)out})
        if (hm_status st = check_batch(x); st) return st;
    if (a->nbits != b->nbits || k == 0 || k > a->nbits || out->nbits != k || a->n != b->n ||
        a->n != out->n)
        return HM_ERR_INVALID_ARGUMENT;
    return mul_columns(c, a, b, k, false, out);
} HM_ABI_CATCH

hm_status hm_gate_batch(hm_ctx *c, hm_op gate, const hm_batch *a, const hm_batch *b,
                        hm_batch *out) try {
    if (!c || !a || !out) return HM_ERR_INVALID_ARGUMENT;
    if (gate > HM_OP_NOT) return HM_ERR_INVALID_ARGUMENT;
    if (hm_status st = hm_validate_operation(c, gate, nullptr); st) return st;
    if (hm_status st = check_batch(a); st) return st;
    if (hm_status st = check_batch(out); st) return st;
    if (gate != HM_OP_NOT) {
        if (!b) return HM_ERR_INVALID_ARGUMENT;
        if (hm_status st = check_batch(b); st) return st;
        if (b->nbits != a->nbits || b->n != a->n) return HM_ERR_INVALID_ARGUMENT;
    }
    if (out->nbits != a->nbits || out->n != a->n) return HM_ERR_INVALID_ARGUMENT;
    const uint32_t L = a->nbits;
    std::vector<uint32_t> need(L);
    if (hm_status st = hm_gate_out_bounds(gate, L, a->bound, gate == HM_OP_NOT ? nullptr : b->bound,
                                          need.data());
        st)
        return st;
    if (!covers(out, need)) return HM_ERR_INVALID_ARGUMENT;
    if (a->n == 0) return HM_OK;
    uint32_t SA = 0, SB = 2;
    for (uint32_t i = 0; i < L; ++i) {
        SA = std::max(SA, 2 * cap_of(a->bound[i]));
        if (gate != HM_OP_NOT) SB = std::max(SB, 2 * cap_of(b->bound[i]));
    }
    GateArgs G{};
    G.op = gate;
    G.oA = 0, G.oB = SA + 2, G.oT = G.oB + SB + 2;
    G.lds_per_wave = G.oT + 2 * (SA + SB) + 8;
    if ((size_t)G.lds_per_wave * 16 > 160 * 1024) return HM_ERR_UNSUPPORTED;
    G.a = batch_arg(a);
    if (gate != HM_OP_NOT) G.b = batch_arg(b);
    G.out = batch_arg(out);
    G.n = a->n, G.nbits = L;
    G.status = c->d_status;
    fill_bounds(G.ab, a);
    if (gate != HM_OP_NOT) fill_bounds(G.bb, b);
    fill_bounds(G.ob, out);
    DeviceGuard g(c->device);
    return launch_gate(G, c->stream) ? hip_fail(c, hipGetLastError()) : HM_OK;
} HM_ABI_CATCH

// ------------------------------------------------------------------ polynomial primitives
static PolyArgs poly_args(hm_ctx *c, const hm_polys *a, const hm_polys *b, hm_polys *out) {
    PolyArgs P{};
    P.a = a->limbs, P.adeg = a->degree, P.acap = a->cap;
    if (b) P.b = b->limbs, P.bdeg = b->degree, P.bcap = b->cap;
    P.out = out->limbs, P.odeg = out->degree, P.ocap = out->cap;
    P.n = a->n;
    P.status = c->d_status;
    return P;
}

hm_status hm_poly_add_batch(hm_ctx *c, const hm_polys *a, const hm_polys *b, hm_polys *out) try {
    if (!c || !a || !b || !out || a->n != b->n || a->n != out->n) return HM_ERR_INVALID_ARGUMENT;
    if (!a->cap || !b->cap || out->cap < std::max(a->cap, b->cap)) return HM_ERR_INVALID_ARGUMENT;
    DeviceGuard g(c->device);
    return launch_poly_add(poly_args(c, a, b, out), c->stream) ? hip_fail(c, hipGetLastError()) : HM_OK;
} HM_ABI_CATCH

hm_status hm_poly_mul_batch(hm_ctx *c, const hm_polys *a, const hm_polys *b, hm_polys *out) try {
    if (!c || !a || !b || !out || a->n != b->n || a->n != out->n) return HM_ERR_INVALID_ARGUMENT;
    if (!a->cap || !b->cap || out->cap < a->cap + b->cap) return HM_ERR_INVALID_ARGUMENT;
    DeviceGuard g(c->device);
    return launch_poly_mul(poly_args(c, a, b, out), c->stream) ? hip_fail(c, hipGetLastError()) : HM_OK;
} HM_ABI_CATCH

hm_status hm_poly_rem_batch(hm_ctx *c, const hm_polys *a, const uint64_t *s, size_t sn,
                            hm_polys *out) try {
    if (!c || !a || !out || !s || sn == 0 || a->n != out->n) return HM_ERR_INVALID_ARGUMENT;
    if (!a->cap || out->cap < a->cap) return HM_ERR_INVALID_ARGUMENT;
    bool nz = false;
    for (size_t i = 0; i < sn; ++i) nz |= s[i] != 0;
    if (!nz) return HM_ERR_DIVIDE_BY_ZERO;           // polynomial.rs:319-322
    const size_t ds = degree_of(s, sn);
    if (ds == 0) return HM_ERR_DIVISOR_IS_ONE;       // the reference never terminates
    DeviceGuard g(c->device);
    const size_t acap = a->cap, kmax = 64 * acap;
    RemTable T{nullptr, 0, 0, 0};
    if (ds < kmax) {
        // Remainder table (poly_rem_kernel): row j < deg S, bit k = bit j of X^k mod S.  Columns
        // k < deg S are the identity (X^k mod S = X^k), so rows hold only the limbs from
        // l0 = deg S / 64 on; size and build time are bounded by the dividend's capacity whatever
        // the divisor's degree (a divisor above every dividend needs no table: zt = null).
        const size_t l0 = ds / 64, tcols = acap - l0, sl = ds / 64 + 1;
        if ((double)ds * tcols * 8 > 1.0 * (1ull << 30)) return HM_ERR_UNSUPPORTED; // host memory
        const bool cached = c->d_s && c->rem_acap == acap && c->rem_gen == c->generation &&
                            c->rem_key.size() == sl && std::equal(s, s + sl, c->rem_key.begin());
        if (cached) {
            T = RemTable{c->d_s, (uint32_t)ds, (uint32_t)l0, (uint32_t)tcols};
            const int rc = launch_poly_rem(poly_args(c, a, nullptr, out), T, c->stream);
            return rc ? hip_fail(c, hipGetLastError()) : HM_OK;
        }
        // the cache is invalid from here until the new table is complete (a failed rebuild must
        // not leave the old key matching a half-overwritten d_s)
        c->rem_key.clear();
        std::vector<uint64_t> zt(ds * tcols, 0);
        // X^k mod S for the 64 k of column limb l0 + t: unit bits below deg S, then r = X * r mod
        // S; each block of 64 vectors is transposed word by word into the rows
        std::vector<uint64_t> r(sl, 0), blk(64 * sl);
        bool iter = false;
        for (size_t t = 0; t < tcols; ++t) {
            for (size_t u = 0; u < 64; ++u) {
                const size_t k = 64 * (l0 + t) + u;
                uint64_t *v = &blk[u * sl];
                if (k < ds) {
                    std::fill(v, v + sl, 0ull);
                    v[k / 64] = 1ull << (k % 64);
                    continue;
                }
                if (!iter) { // X^ds mod S = S - X^ds
                    std::copy(s, s + sl, r.begin());
                    r[ds / 64] &= ~(1ull << (ds % 64));
                    iter = true;
                } else {
                    uint64_t carry = 0;
                    for (size_t w = 0; w < sl; ++w) {
                        const uint64_t nc = r[w] >> 63;
                        r[w] = (r[w] << 1) | carry;
                        carry = nc;
                    }
                    if ((r[ds / 64] >> (ds % 64)) & 1)
                        for (size_t w = 0; w < sl; ++w) r[w] ^= s[w];
                }
                std::copy(r.begin(), r.end(), v);
            }
            uint64_t m[64];
            for (size_t w = 0; w < sl; ++w) {
                for (size_t u = 0; u < 64; ++u) m[u] = blk[u * sl + w];
                transpose64(m); // m[jb] bit u = bit jb of word w of X^(64(l0+t)+u) mod S
                for (size_t jb = 0; jb < 64 && 64 * w + jb < ds; ++jb) zt[(64 * w + jb) * tcols + t] = m[jb];
            }
        }
        size_t have = c->d_s_limbs * 8;
        HM_HIP(c, grow(c, c->d_s, have, zt.size() * 8));
        c->d_s_limbs = have / 8;
        // d_s is rewritten in place for another divisor: a graph captured with the old table
        // (the cached path has no sync, so it is capturable) must refuse to replay
        ++c->generation;
        HM_HIP(c, hipMemcpyAsync(c->d_s, zt.data(), zt.size() * 8, hipMemcpyHostToDevice, c->stream));
        HM_HIP(c, hipStreamSynchronize(c->stream)); // host buffer is released after return
        T = RemTable{c->d_s, (uint32_t)ds, (uint32_t)l0, (uint32_t)tcols};
        c->rem_key.assign(s, s + sl), c->rem_acap = acap, c->rem_gen = c->generation;
    }
    const int rc = launch_poly_rem(poly_args(c, a, nullptr, out), T, c->stream);
    return rc ? hip_fail(c, hipGetLastError()) : HM_OK;
} HM_ABI_CATCH

hm_status hm_ctx_synchronize(hm_ctx *c) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    DeviceGuard g(c->device);
    HM_HIP(c, hipStreamSynchronize(c->stream));
    int st = 0;
    HM_HIP(c, hipMemcpy(&st, c->d_status, sizeof(int), hipMemcpyDeviceToHost));
    if (st) HM_HIP(c, hipMemset(c->d_status, 0, sizeof(int)));
    if (c->last_hip != hipSuccess) {
        c->last_hip = hipSuccess;
        return HM_ERR_HIP;
    }
    return (hm_status)st;
} HM_ABI_CATCH

int32_t hm_ctx_last_hip_error(const hm_ctx *c) { return c ? (int32_t)c->last_hip : 0; }

} // extern "C"
