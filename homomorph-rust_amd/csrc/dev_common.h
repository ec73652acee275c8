// dev_common.h — device helpers shared by the gfx950 kernel translation units (kernels.hip,
// mul_engine.hip): status flags, wave-scope fences, ciphertext-bit load/store with validation, and
// per-lane carry-less products of "holey" operands.
#pragma once
#include <hip/hip_runtime.h>

#include "engine.h"
#include "gf2_wave.h"

namespace hm {

__device__ __forceinline__ void flag(int *status, int code) {
    if (status) atomicCAS(status, 0, code);
}

// wsync: order this wave's LDS writes before its later LDS reads by other lanes.  A wave's LDS
// instructions execute in order, so only the compiler must be kept from reordering (wavefront
// scope emits no wait).  gsync: the same for GLOBAL memory, where a lane's load must not overtake
// another lane's earlier store: workgroup scope drains vmcnt/lgkmcnt.
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void gsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t cap_of(uint32_t bound) { return bound / 64 + 1; }

// ---------------------------------------------------------------------------------------------
// By-value argument arrays (Bounds) are indexed with WAVE-UNIFORM indices only.  A lane-varying
// index into a kernel argument compiles to vector loads from the kernarg segment (an address off
// the kernarg SGPR pair, `v_lshl_add_u64 v, v, 2, s[0:1]` + `global_load_dword`) instead of scalar
// loads -- the construct behind round 5's non-deterministic decrypt misreads.
// tools/kernarg_audit.py checks every kernel of the library for it (tests/test_kernarg_audit.py).
// Per-lane lookups go through LDS copies made here: the array is read with scalar loads
// (uniform indices) and written to LDS by one lane.

// the first n (wave-uniform, <= HM_MAX_BITS) entries of a into lds[0:n) (lds: HM_MAX_BITS words,
// 16-byte aligned; entries past n up to the next multiple of 16 are written too), by the calling
// wave: 16 entries per s_load_dwordx16, stored by lane 0 as four ds_write_b128.  Order them before
// other lanes' (wsync) or other waves' (__syncthreads) reads.
__device__ __forceinline__ void arg_to_lds(const uint32_t (&a)[HM_MAX_BITS], uint32_t n, uint32_t *lds) {
    static_assert(HM_MAX_BITS % 16 == 0, "whole 16-entry chunks");
    n = rfl(n);
    const bool l0 = (threadIdx.x & 63u) == 0;
    for (uint32_t c = 0; c < n; c += 16) { // uniform; c + 16 <= HM_MAX_BITS
        uint32_t v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = a[c + j];
        if (l0) {
            uint4 *d = (uint4 *)(lds + c);
#pragma unroll
            for (int q = 0; q < 4; ++q) d[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
        }
    }
}

// Load one ciphertext bit (u64 limbs, exact degree `deg`) into 32-bit words at dst.
// The degree word is validated against the limbs (top bit set, nothing above it).
// Returns the word count (0 for the null polynomial).
__device__ __forceinline__ int load_bit(const uint64_t *__restrict__ src, uint32_t deg, uint32_t bound,
                        uint32_t *__restrict__ dst, int *status) {
    const int lane = lane_id();
    if (deg > bound) {
        if (lane == 0) flag(status, HM_ERR_BAD_INPUT);
        return 0;
    }
    const int nl = (int)(deg / 64) + 1;
    const int cap = (int)(bound / 64) + 1;
    const uint32_t tb = deg % 64;
    bool bad = false;
    for (int g = lane; g < cap; g += kWave) {
        uint64_t v = src[g];
        if (g >= nl) { // limbs above the degree must be zero (layout invariant)
            bad |= v != 0;
            continue;
        }
        if (g == nl - 1) {
            const uint64_t keep = (~0ull) >> (63 - tb);
            bad |= (v & ~keep) != 0;
            v &= keep;
            if (deg > 0 && !((v >> tb) & 1ull)) bad = true;
        }
        dst[2 * g] = (uint32_t)v;
        dst[2 * g + 1] = (uint32_t)(v >> 32);
    }
    if (__any(bad) && lane == 0) flag(status, HM_ERR_BAD_INPUT);
    if (deg == 0) {
        const uint32_t w0 = rfl((uint32_t)src[0]);
        if (!(w0 & 1u)) return 0;
    }
    return (int)(deg / 32) + 1;
}

// dst (cap limbs) = X ^ C; writes the exact degree; returns it (-1 = null).
__device__ __forceinline__ int store_xor_bit(const uint32_t *X, int nx, const uint32_t *C, int nc,
                             uint64_t *__restrict__ dst, uint32_t bound, uint32_t *deg_out,
                             int *status) {
    const int lane = lane_id();
    const int cap = (int)cap_of(bound);
    const int n = max(nx, nc);
    const int total = max(cap, (n + 1) / 2);
    int ldeg = -1;
    for (int g = lane; g < total; g += kWave) {
        const int w = 2 * g;
        uint32_t lo = (w < nx ? X[w] : 0u) ^ (w < nc ? C[w] : 0u);
        uint32_t hi = (w + 1 < nx ? X[w + 1] : 0u) ^ (w + 1 < nc ? C[w + 1] : 0u);
        uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
        if (g < cap) dst[g] = v;
        if (v) ldeg = g * 64 + 63 - __builtin_clzll(v);
    }
    const int deg = wave_max_i32(ldeg);
    if (lane == 0) {
        if (deg > (int)bound) flag(status, HM_ERR_CAPACITY);
        *deg_out = (uint32_t)max(deg, 0);
    }
    return deg;
}

// s = X ^ C for the adder's sum bit (x_i from the prep workspace, carry words C); writes the
// output limbs and the exact degree.
__device__ __forceinline__ int store_sum_x(const uint32_t *X, int nx, const uint32_t *C, int nc,
                           uint64_t *__restrict__ dst, uint32_t bound, uint32_t *deg_out,
                           int *status) {
    const int lane = lane_id();
    const int cap = (int)cap_of(bound);
    const int total = max(cap, (max(nx, nc) + 1) / 2);
    int ldeg = -1;
    for (int g = lane; g < total; g += kWave) {
        const int w = 2 * g;
        const uint32_t lo = (w < nx ? X[w] : 0u) ^ (w < nc ? C[w] : 0u);
        const uint32_t hi = (w + 1 < nx ? X[w + 1] : 0u) ^ (w + 1 < nc ? C[w + 1] : 0u);
        const uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
        if (g < cap) dst[g] = v;
        if (v) ldeg = g * 64 + 63 - __builtin_clzll(v);
    }
    const int deg = wave_max_i32(ldeg);
    if (lane == 0) {
        if (deg > (int)bound) flag(status, HM_ERR_CAPACITY);
        *deg_out = (uint32_t)max(deg, 0);
    }
    return deg;
}

__device__ __forceinline__ int words_of(int deg) { return deg >= 0 ? nwords(deg) : 0; }

// dst (cap limbs) = A ^ B ^ C (output bit of the adder); writes the exact degree.
__device__ __forceinline__ int store_xor3_bit(const uint32_t *Aw, int na, const uint32_t *Bw, int nb,
                              const uint32_t *C, int nc, uint64_t *__restrict__ dst,
                              uint32_t bound, uint32_t *deg_out, int *status) {
    const int lane = lane_id();
    const int cap = (int)cap_of(bound);
    const int n = max(max(na, nb), nc);
    const int total = max(cap, (n + 1) / 2);
    int ldeg = -1;
    for (int g = lane; g < total; g += kWave) {
        const int w = 2 * g;
        uint32_t lo = (w < na ? Aw[w] : 0u) ^ (w < nb ? Bw[w] : 0u) ^ (w < nc ? C[w] : 0u);
        uint32_t hi = (w + 1 < na ? Aw[w + 1] : 0u) ^ (w + 1 < nb ? Bw[w + 1] : 0u) ^
                      (w + 1 < nc ? C[w + 1] : 0u);
        uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
        if (g < cap) dst[g] = v;
        if (v) ldeg = g * 64 + 63 - __builtin_clzll(v);
    }
    const int deg = wave_max_i32(ldeg);
    if (lane == 0) {
        if (deg > (int)bound) flag(status, HM_ERR_CAPACITY);
        *deg_out = (uint32_t)max(deg, 0);
    }
    return deg;
}

// Small products (fresh operands: 9 words at d+dp = 256) use a short uniform chunk; the carry
// product P * carry uses a chunk that covers P (25 words at d+dp = 256) in one pass.
constexpr int kQSmall = 10;
constexpr int kQBig = 25;

// ---------------------------------------------------------------------------------------------
// Per-lane carry-less product word by integer multiplication of "holey" operands.
// Split u and v by bit position mod 4 (u_a = u & M_a, M_a = 0x11111111 << a).  In the integer
// product u_a * v_b every set bit pair lands on a position == a+b (mod 4), and at most 8 pairs
// land on any one position (8 bits per holey word), so the column counts never carry out of
// their 4-bit field: bit p of u_a*v_b is the GF(2) coefficient sum at p.  XOR the 4 products of
// each residue class c, keep the positions == c:  clmul(u, v) = OR_c (M_c & XOR_{a+b=c} u_a v_b).
// v_mul_lo_u32 / v_mul_hi_u32 give the two halves of the 64-bit product at the rate of a shift
// (measured), i.e. 16 multiplies replace 32 (funnel + bfe + bitop3) bit steps.
// Masking commutes with XOR, so classes are accumulated over q and masked once per word.
struct Holey {
    uint32_t h[4];
    __device__ __forceinline__ explicit Holey(uint32_t v) {
#pragma unroll
        for (int a = 0; a < 4; ++a) h[a] = v & (0x11111111u << a);
    }
};

// z[c] ^= low halves of U (x) V1  ^  high halves of U (x) V0   (residue class c)
__device__ __forceinline__ void holey_acc(uint32_t z[4], const Holey &U, const Holey &V1,
                                          const Holey &V0) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        uint32_t lo[4], hi[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const int b = (c - a) & 3;
            lo[a] = U.h[a] * V1.h[b];
            hi[a] = __umulhi(U.h[a], V0.h[b]);
        }
        // nine-term XOR as four three-input v_bitop3
        z[c] = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(z[c], lo[0], lo[1], 0x96),
                                           __builtin_amdgcn_bitop3_b32(lo[2], lo[3], hi[0], 0x96),
                                           __builtin_amdgcn_bitop3_b32(hi[1], hi[2], hi[3], 0x96), 0x96);
    }
}

// a ^ b ^ c ^ d as one three-input v_bitop3 (truth table 0x96) and one XOR (the compiler does not
// form bitop3 from XOR chains on its own)
__device__ __forceinline__ uint32_t xor4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96) ^ d;
}

__device__ __forceinline__ uint32_t holey_fold(const uint32_t z[4]) {
    return (z[0] & 0x11111111u) | (z[1] & 0x22222222u) | (z[2] & 0x44444444u) |
           (z[3] & 0x88888888u);
}

// Word m of U*V (U: nu words, V: nv words): XOR over q of low(U_q V_{m-q}) ^ high(U_q V_{m-q-1}).
// Used where lanes work on DIFFERENT products (no uniform operand), i.e. the adder's pre-phase.
__device__ __forceinline__ uint32_t clmul_word(const uint32_t *__restrict__ pu, int nu,
                                               const uint32_t *__restrict__ pv, int nv, int m) {
    uint32_t z[4] = {0u, 0u, 0u, 0u};
    const int qlo = max(0, m - nv), qhi = min(nu - 1, m);
    if (qlo > qhi) return 0u;
    int k = m - qlo;
    Holey V1(k < nv ? pv[k] : 0u);
    for (int q = qlo; q <= qhi; ++q, --k) {
        const Holey V0((k >= 1 && k - 1 < nv) ? pv[k - 1] : 0u);
        holey_acc(z, Holey(pu[q]), V1, V0);
        V1 = V0; // V_{m-q-1} is the next q's V_{m-q}
    }
    return holey_fold(z);
}

// One row of a product: out[k] ^= word k of u * V for k = 0..nv (out in LDS, shared by the
// lanes that own the other rows, hence ds_xor).  Each 32x32 product is formed whole: 16
// v_mad_u64_u32 give both halves, the low half goes to word k and the high half to word k+1.
__device__ __forceinline__ void clmul_row_xor(uint32_t u, const uint32_t *__restrict__ pv, int nv,
                                              uint32_t *out) {
    const Holey U(u);
    uint32_t hiprev = 0u;
    // pv[k] is read one step ahead (the LDS latency hides under the step before), and each
    // residue class XORs its four products as one expression (v_bitop3 three-input XORs)
#ifndef HM_CLMUL_PEEL
#define HM_CLMUL_PEEL 1 // (A/B knob) last step peeled, clamped read-ahead, unconditional ds_xor
#endif
    if (HM_CLMUL_PEEL) {
        if (nv <= 0) return;
        uint32_t vnext = pv[0];
        for (int k = 0; k < nv; ++k) {
            const Holey V(vnext);
            vnext = pv[min(k + 1, nv - 1)];
            uint32_t zl[4], zh[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                uint64_t p[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) p[a] = (uint64_t)U.h[a] * V.h[(c - a) & 3];
                zl[c] = xor4((uint32_t)p[0], (uint32_t)p[1], (uint32_t)p[2], (uint32_t)p[3]);
                zh[c] = xor4((uint32_t)(p[0] >> 32), (uint32_t)(p[1] >> 32), (uint32_t)(p[2] >> 32),
                             (uint32_t)(p[3] >> 32));
            }
            atomicXor(&out[k], holey_fold(zl) ^ hiprev);
            hiprev = holey_fold(zh);
        }
        if (hiprev) atomicXor(&out[nv], hiprev);
        return;
    }
    uint32_t vnext = nv > 0 ? pv[0] : 0u;
    for (int k = 0; k <= nv; ++k) {
        uint32_t lo = 0u, hi = 0u;
        if (k < nv) {
            const Holey V(vnext);
            vnext = k + 1 < nv ? pv[k + 1] : 0u;
            uint32_t zl[4], zh[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                uint64_t p[4];
#pragma unroll
                for (int a = 0; a < 4; ++a) p[a] = (uint64_t)U.h[a] * V.h[(c - a) & 3];
                zl[c] = xor4((uint32_t)p[0], (uint32_t)p[1], (uint32_t)p[2], (uint32_t)p[3]);
                zh[c] = xor4((uint32_t)(p[0] >> 32), (uint32_t)(p[1] >> 32), (uint32_t)(p[2] >> 32),
                             (uint32_t)(p[3] >> 32));
            }
            lo = holey_fold(zl), hi = holey_fold(zh);
        }
        const uint32_t w = lo ^ hiprev;
        if (w) atomicXor(&out[k], w);
        hiprev = hi;
    }
}

// The same row with a compile-time multiplicand length NV (its LDS slot is zero-padded to NV
// words, so words past the degree multiply as zeros): fully unrolled, every multiplicand word read
// before the first product (NV LDS reads in flight, no read-ahead bookkeeping), no loop control.
template <int NV>
__device__ __forceinline__ void clmul_row_xor_fixed(uint32_t u, const uint32_t *__restrict__ pv,
                                                    uint32_t *out) {
    const Holey U(u);
    uint32_t v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = pv[k];
    uint32_t hiprev = 0u;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const Holey V(v[k]);
        uint32_t zl[4], zh[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            uint64_t p[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) p[a] = (uint64_t)U.h[a] * V.h[(c - a) & 3];
            zl[c] = xor4((uint32_t)p[0], (uint32_t)p[1], (uint32_t)p[2], (uint32_t)p[3]);
            zh[c] = xor4((uint32_t)(p[0] >> 32), (uint32_t)(p[1] >> 32), (uint32_t)(p[2] >> 32),
                         (uint32_t)(p[3] >> 32));
        }
        atomicXor(&out[k], holey_fold(zl) ^ hiprev);
        hiprev = holey_fold(zh);
    }
    if (hiprev) atomicXor(&out[NV], hiprev); // (zero whenever the product fits its slot)
}

// Kernel timer (engine.h KTimer): lane 0 of every wave stamps the device wall clock (100 MHz)
// at the kernel's entry and at its exit.  Fire-and-forget atomics on per-wave addresses: no
// barrier, no LDS, no contention (an earlier form counted blocks out on one global counter with
// a static LDS word; the LDS word misaligned the kernels' dynamic LDS and the counter serialised).
__device__ __forceinline__ uint32_t kt_wave() {
    return (blockIdx.x * ((blockDim.x + 63u) >> 6) + (threadIdx.x >> 6)) & (kTimerWaves - 1);
}
__device__ __forceinline__ void kt_start(const KTimer &k) {
    if (k.t0 && (threadIdx.x & 63u) == 0)
        __hip_atomic_fetch_min(&k.t0[kt_wave()], (unsigned long long)wall_clock64(),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void kt_finish(const KTimer &k) {
    if (k.t1 && (threadIdx.x & 63u) == 0)
        __hip_atomic_fetch_max(&k.t1[kt_wave()], (unsigned long long)wall_clock64(),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int bitwords(int degp1) { return degp1 ? ((degp1 - 1) >> 5) + 1 : 0; }

} // namespace hm
