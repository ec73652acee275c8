// ctx.h — internal to the engine library: the context object behind hm_ctx* and the host helpers
// shared by capi.cpp and mul_host.cpp.  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "engine.h"
#include "gf2_wave.h"

namespace hm {
struct MulPlan; // mul_host.cpp
// default Karatsuba scratch limit, words per value and lane (hm_ctx_set_mul_scratch): above it a
// product is planned one subtree at a time (mul_host.cpp); every K <= 20 plan stays below it
constexpr uint64_t kKaScratchWords = 200000000u;
}

struct hm_ctx {
    uint16_t d, dp, delta, tau;
    int device;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // Randomness.  Unseeded (the default): key polynomials come straight from getrandom(2), as
    // Polynomial::random does (src/polynomial.rs:73-96), and encryption masks from a device
    // ChaCha20 keystream keyed with 32 getrandom bytes.  hm_ctx_seed_rng switches both to a
    // reproducible test contract: SplitMix64 for keys, a ChaCha20 key derived from the seed.
    bool seeded = false;
    uint64_t rng = 0;
    uint32_t chacha_key[8] = {};
    uint64_t *d_nonce = nullptr;       // device ChaCha20 nonce counter, advanced by every draw
    // keys (host copies; SecretKey / PublicKey)
    bool has_sk = false, has_pk = false;
    std::vector<uint64_t> sk;          // limbs of S
    std::vector<uint64_t> pk;          // tau * pk_cap limbs
    uint32_t pk_tau = 0, pk_cap = 0;
    uint32_t pk_maxdeg = 0;
    // the rows' top limbs are all 0 or 1 (tau <= 128): their bits as a column (EncArgs::topcol)
    bool pk_top1 = false;
    uint32_t pk_topcol[4] = {0, 0, 0, 0};
    // device state
    uint64_t *d_pk = nullptr;
    uint64_t *d_pk_tab = nullptr;      // encryption nibble table (upload_pk), or null
    uint64_t *d_pk_tab1 = nullptr;     // the same without the one-bit top limb (pk_top1), or null
    uint64_t *d_z = nullptr;           // decrypt parity table z_k = (X^k mod S)(0)
    uint32_t z_limbs = 0;
    uint64_t *d_s = nullptr;           // divisor scratch for hm_poly_rem_batch
    size_t d_s_limbs = 0;
    // hm_poly_rem_batch's remainder table in d_s is cached for (divisor, dividend capacity):
    // a repeated divisor skips the host build and the upload
    std::vector<uint64_t> rem_key;
    size_t rem_acap = 0;
    uint64_t rem_gen = 0;
    uint32_t *d_ws_add = nullptr;      // adder workspace (validated inputs, per-bit a_i*b_i)
    size_t ws_add_bytes = 0;
    uint32_t *d_mws = nullptr;         // column multiplier arena (mul_columns)
    size_t mws_bytes = 0;
    uint8_t *d_masks = nullptr;        // engine-drawn encryption masks (hm_encrypt_batch, masks NULL)
    size_t masks_bytes = 0;
    int *d_status = nullptr;
    uint32_t cus = 256;                // compute units of the device (grid sizing)
    bool fp4_mfma = false;             // the device has the gfx950 fp4 MFMA (set at creation)
    hipError_t last_hip = hipSuccess;
    // Device buffers the kernels read are never freed while the context lives: a HIP graph
    // captured over the engine's launches holds their raw pointers.  A buffer that has to be
    // replaced (grown, or keyed by a new key) is retired instead -- zeroed first when it holds
    // secret-derived data -- and `generation` advances, so a graph wrapper can refuse to replay
    // across the change (hm_ctx_generation).  hm_ctx_trim / hm_ctx_destroy free retired buffers.
    struct Retired {
        void *p;
        size_t bytes;
    };
    std::vector<Retired> retired;
    uint64_t generation = 0;
    // column multiplier plans (device task tables), keyed by the operand bounds; see mul_host.cpp
    std::vector<hm::MulPlan *> mul_plans; // owned; freed by mul_plans_release
    // Karatsuba carry products (hm_ctx_set_mul_options): shorter operand >= ka_min words (0 =
    // never), recursion down to leaves of at most ka_leaf words
    uint32_t ka_min = 256, ka_leaf = 256;
    // Karatsuba scratch per value and lane above which a product is planned one subtree at a
    // time (hm_ctx_set_mul_scratch; mul_host.cpp kKaScratchWords)
    uint64_t ka_scratch = hm::kKaScratchWords;
    // where the Karatsuba leaf products run (hm_ctx_set_mul_products): HM_MUL_PRODUCTS_*
    uint32_t mul_products = 0;
    // carry chain of the adder (hm_ctx_set_add_options): HM_ADD_CHAIN_AUTO / _MFMA / _VALU
    uint32_t add_chain = 0;
    // adder pipelining (hm_ctx_set_add_pipeline, off by default): batches of at least
    // 2 * kAddPipeMin values run as two halves, the second half's prep on aux_stream beside the
    // first half's chain
    bool add_pipe = false;
    hipStream_t aux_stream = nullptr;  // created on first use
    hipEvent_t ev_fork = nullptr, ev_mid = nullptr, ev_join = nullptr;
    // per-launch timing of one kernel (hm_ctx_set_kernel_timing, HM_TIME_*): device wall-clock
    // stamps (engine.h KTimer) in d_kt: [kTimedLaunches][kTimerWaves] starts, then as many ends;
    // kt_next = the next launch's slot
    uint32_t time_kernel = HM_TIME_OFF;
    unsigned long long *d_kt = nullptr;
    uint32_t kt_next = 0;
    hm::KTimer ktimer(uint32_t which) {
        if (time_kernel != which || !d_kt || kt_next >= hm::kTimedLaunches) return hm::KTimer{nullptr, nullptr};
        const size_t slot = (size_t)kt_next++ * hm::kTimerWaves;
        return hm::KTimer{d_kt + slot, d_kt + (size_t)hm::kTimedLaunches * hm::kTimerWaves + slot};
    }
};

namespace hm {

struct DeviceGuard {
    int prev = 0;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (cur != prev) (void)hipSetDevice(prev);
    }
};

inline uint32_t cap_of(uint32_t bound) { return bound / 64 + 1; }

// hm_ctx_set_mul_products: MFMA, or AUTO on a device with the fp4 MFMA (gfx950)
inline bool mul_on_mfma(const hm_ctx *c) {
    return c->mul_products == HM_MUL_PRODUCTS_MFMA ||
           (c->mul_products == HM_MUL_PRODUCTS_AUTO && c->fp4_mfma);
}
inline uint32_t words_of_bound(int64_t b) { return b < 0 ? 0u : (uint32_t)(b / 32 + 1); }

inline void retire(hm_ctx *c, void *p, size_t bytes, bool secret) {
    if (!p) return;
    if (secret) (void)hipMemset(p, 0, bytes); // SecretKey's Drop zeroizes (context.rs:197-206)
    c->retired.push_back({p, bytes});
    ++c->generation;
}

// Grow-only device buffer (see hm_ctx::retired).  Allocation is synchronous, outside any
// capture: callers size buffers on a warm-up call before a graph is captured.
template <class T>
hipError_t grow(hm_ctx *c, T *&p, size_t &have, size_t need, bool secret = false) {
    if (need <= have && p) return hipSuccess;
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return e;
    retire(c, p, have, secret);
    p = nullptr, have = 0;
    e = hipMalloc(&p, need);
    if (e != hipSuccess) return e;
    have = need;
    ++c->generation;
    return hipSuccess;
}

inline hm_status hip_fail(hm_ctx *c, hipError_t e) {
    if (c) c->last_hip = e;
    return HM_ERR_HIP;
}

// Every hm_* entry returning hm_status is a function-try-block ending in HM_ABI_CATCH, so no C++
// exception (std::bad_alloc from a host container above all) crosses the C ABI
// (include/homomorph_gpu.h: HM_ERR_OUT_OF_MEMORY, HM_ERR_INTERNAL).
hm_status exception_status() noexcept;
hm_status ensure_aux_stream(hm_ctx *c);
#define HM_ABI_CATCH                                                                              \
    catch (...) {                                                                                 \
        return hm::exception_status();                                                            \
    }

#define HM_HIP(ctx, expr)                                                                         \
    do {                                                                                          \
        hipError_t _e = (expr);                                                                   \
        if (_e != hipSuccess) return hip_fail((ctx), _e);                                         \
    } while (0)

inline bool fill_bounds(Bounds &dst, const hm_batch *b) {
    if (!b || !b->bound || b->nbits == 0 || b->nbits > HM_MAX_BITS) return false;
    std::memset(&dst, 0, sizeof(dst));
    for (uint32_t i = 0; i < b->nbits; ++i) dst.b[i] = b->bound[i];
    return true;
}

inline BatchArg batch_arg(const hm_batch *b) {
    BatchArg a;
    a.limbs = b->limbs;
    a.degree = b->degree;
    a.stride = hm_batch_stride(b->nbits, b->bound);
    a.dstride = b->nbits;
    return a;
}

inline hm_status check_batch(const hm_batch *b, bool need_limbs = true) {
    if (!b || !b->bound || b->nbits == 0 || b->nbits > HM_MAX_BITS) return HM_ERR_INVALID_ARGUMENT;
    if (b->n && need_limbs && (!b->limbs || !b->degree)) return HM_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < b->nbits; ++i)
        if (b->bound[i] > (1u << 30)) return HM_ERR_UNSUPPORTED;
    return HM_OK;
}

// The column-parallel carry-save multiplier (mul_host.cpp): the low K output bits of the
// nbits-bit circuit over a and b (K = nbits for the full product; flip = the signed circuit's
// constant terms, applied only when K == nbits).
hm_status mul_columns(hm_ctx *c, const hm_batch *a, const hm_batch *b, uint32_t K, bool is_signed,
                      hm_batch *out);
void mul_plans_release(hm_ctx *c);
// The word pairs of the carry products as the context's plan runs them (Karatsuba products by
// their leaves), for the low K output bits of the nbits-bit circuit (hm_mul_plan_work).
hm_status mul_plan_work(hm_ctx *c, uint32_t nbits, uint32_t K, const uint32_t *a, const uint32_t *b,
                        bool is_signed, double &executed);
// Degree bounds of the K low output bits of the nbits-bit circuit (-1 = always null); false when a
// bound exceeds the engine's 2^30 limit.  The same symbolic walk as the plan.
bool mul_result_bounds(uint32_t nbits, uint32_t K, const uint32_t *a, const uint32_t *b,
                       bool is_signed, std::vector<int64_t> &res);
// The same walk over bounds only, without limits: word-pair products, output bytes, max degree.
void mul_cost_model(uint32_t nbits, uint32_t K, const uint32_t *a, const uint32_t *b,
                    double &pairs, double &out_bytes, double &maxdeg);

} // namespace hm
