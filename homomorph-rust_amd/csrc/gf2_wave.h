// gf2_wave.h — wave-level GF(2)[X] primitives for gfx950 (CDNA4, wave64).
//
// A polynomial here is a little-endian array of 32-bit words: coefficient of X^k is bit k%32 of
// word k/32 (the same bit order as the reference's u64 limbs, src/polynomial.rs:142-150, read as
// two u32 halves).  One wavefront owns one polynomial operation; its 64 lanes split the OUTPUT
// words: in a tile starting at word `base`, lane l owns words base + l*W ... base + l*W + W-1.
//
// Carry-less product (replaces Polynomial::mul, src/polynomial.rs:252-310).  gfx950 has no
// carry-less multiply instruction, and MFMA is the wrong tool for XOR/AND work, so the product is
// built from VALU funnel shifts and XORs with one operand made WAVE-UNIFORM:
//     out = sum_q sum_r [bit r of U_q] * X^(32q + r) * V
//         = Horner over r:  t = X*t + S_r,   S_r = sum_{q : bit r of U_q} X^(32q) V
// U's words live in SGPRs (readfirstlane), so "is bit r of U_q set" is a scalar branch, and the
// word shift X^(32q) V is a compile-time register index into a per-lane window `cx` of V.  Per
// set bit of U a lane does W XORs; per Horner step W funnel shifts (v_alignbit_b32) plus one DPP
// wave_shr:1 that carries the top bit across lanes.  That is ~0.5 VALU op per (set bit, word) —
// about 2x fewer than the reference-style bit-serial shift-XOR (2 ops per set bit and word).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hm {

constexpr int kWave = 64;
constexpr int kHalo = 32; // zero words below a padded V buffer (>= the uniform chunk QC)

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// The lane index through a volatile asm: values derived from it cannot be hoisted out of the
// kernel's outer loops.  Without this, LICM precomputes the per-lane addresses of every inlined
// tile width at kernel entry and keeps ~170 VGPRs live for the whole kernel.
__device__ __forceinline__ int lane_id_local() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// lane l receives lane l-1's value; lane 0 receives `old`
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138 /*wave_shr:1*/, 0xf, 0xf,
                                                 false);
}

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);
}

// acc ^ (x & m) in one v_bitop3_b32 (truth table index = S0*4 + S1*2 + S2 with S0 = x,
// S1 = acc, S2 = m  ->  0x6c; the compiler does not always fuse the and/xor pair itself).
__device__ __forceinline__ uint32_t xor_and(uint32_t acc, uint32_t x, uint32_t m) {
    return __builtin_amdgcn_bitop3_b32(x, acc, m, 0x6c);
}

// in-place t ^= a and t ^= a ^ b, tied so the register allocator keeps t where it is (the
// two-bit Horner loop otherwise copies every updated word back after each XOR)
__device__ __forceinline__ void xor_in(uint32_t &t, uint32_t a) {
    asm volatile("v_xor_b32 %0, %0, %1" : "+v"(t) : "v"(a));
}
__device__ __forceinline__ void xor3_in(uint32_t &t, uint32_t a, uint32_t b) {
    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(t) : "v"(a), "v"(b));
}

// Max over the wave, all in VALU (DPP), no LDS round trips (a __shfl_xor butterfly is six
// ds_bpermute + s_waitcnt pairs): row_shr 1/2/4/8 leave each row's max in its lane 15,
// row_bcast:15 / :31 fold the rows into lane 63.  Lanes without a DPP source take INT_MIN.
__device__ __forceinline__ int wave_max_i32(int v) {
    constexpr int kMin = -2147483647 - 1;
    auto mx = [](int a, int b) { return a > b ? a : b; };
    v = mx(v, __builtin_amdgcn_update_dpp(kMin, v, 0x111, 0xf, 0xf, false)); // row_shr:1
    v = mx(v, __builtin_amdgcn_update_dpp(kMin, v, 0x112, 0xf, 0xf, false)); // row_shr:2
    v = mx(v, __builtin_amdgcn_update_dpp(kMin, v, 0x114, 0xf, 0xf, false)); // row_shr:4
    v = mx(v, __builtin_amdgcn_update_dpp(kMin, v, 0x118, 0xf, 0xf, false)); // row_shr:8
    v = mx(v, __builtin_amdgcn_update_dpp(kMin, v, 0x142, 0xa, 0xf, false)); // row_bcast:15
    v = mx(v, __builtin_amdgcn_update_dpp(kMin, v, 0x143, 0xc, 0xf, false)); // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63); // uniform: sizes derived from it stay in SGPRs
}

__device__ __forceinline__ uint32_t wave_xor_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v ^= (uint32_t)__shfl_xor((int)v, o, 64);
    return rfl(v);
}

__device__ __forceinline__ int nwords(int deg) { return (deg >> 5) + 1; }

// Exact degree of a polynomial whose words are distributed in ascending lane order (lane l's
// words all precede lane l+1's).  ldeg = the lane's highest set bit index or -1.  Returns -1 for
// null.
__device__ __forceinline__ int wave_top_ordered(int ldeg) {
    uint64_t m = __ballot(ldeg >= 0);
    if (m == 0) return -1;
    int hl = 63 - __builtin_clzll(m);
    return __builtin_amdgcn_readlane(ldeg, hl);
}

// One output tile of  Dst = Add ^ U*V.
//  U  : nu uniform-operand words (any address space; read with wave-uniform addresses)
//  V  : nv words, read per lane (bounds-checked unless PAD)
//  Add: nadd words XORed into the result (may be nullptr with nadd = 0)
//  tile covers output words [base, base + 64*W) ∩ [0, nout)
// MULTI: the tile does not start at word 0, so lane 0 tracks word base-1 to shift its top bit in.
// PAIR: two bit positions per Horner step (t = X^2 t + X S_{r+1} + S_r) with a pre-shifted copy
//   of the V window (cx1 = X*window).  When both bits of a (q, pair) are set the two windows are
//   folded with one v_bitop3 xor3, so the XOR work per pair drops from 1.0 W to 0.75 W on average,
//   and the half-rate v_alignbit shifts run once per pair instead of once per bit.
// Returns the tile's highest set bit index (global), or -1.
template <int W, int QC, bool MULTI, int PAIR, bool PAD>
__device__ __forceinline__ int mul_tile(const uint32_t *__restrict__ U, int nu,
                                        const uint32_t *V, int nv,
                                        const uint32_t *__restrict__ Add, int nadd,
                                        uint32_t *Dst, int nout, int base) {
    // sizes are wave-uniform; say so, so every size test below is a scalar branch
    nu = (int)rfl((uint32_t)nu), nv = (int)rfl((uint32_t)nv), nadd = (int)rfl((uint32_t)nadd);
    nout = (int)rfl((uint32_t)nout), base = (int)rfl((uint32_t)base);
    const int lane = lane_id_local();
    const int w0 = base + lane * W;
    // PAD: the host guarantees nu <= QC, so there is exactly one chunk and Add is folded in after
    // it (W fewer registers live across the Horner loop)
    uint32_t acc[W];
#pragma unroll
    for (int j = 0; j < W; ++j) acc[j] = (!PAD && w0 + j < nadd) ? Add[w0 + j] : 0u;

    const int tile_end = base + kWave * W; // exclusive
    for (int q0 = 0; q0 < (PAD ? 1 : nu); q0 += QC) {
        // U chunk words [q0, q0+QC) reach output words [q0, q0 + QC + nv)
        if (q0 >= tile_end || base >= q0 + QC + nv) continue;
        // window: cx[k] = V[w0 - q0 - QC - 1 + k], k in [0, W+QC+1); the word for (j, q) is
        // cx[j - q + QC + 1]; word base-1 (MULTI) uses cx[QC - q]
        constexpr int NX = W + QC + 1;
        uint32_t cx[NX];
        const int cb = w0 - q0 - QC - 1;
#pragma unroll
        for (int k = 0; k < NX; ++k) {
            const int idx = cb + k;
            if constexpr (PAD) cx[k] = V[idx]; // zero halo below, zeros above nv
            else cx[k] = (idx >= 0 && idx < nv) ? V[idx] : 0u;
        }
        // cx1[k] = word k+1 of X * window: (cx[k+1] << 1) | (cx[k] >> 31)
        uint32_t cx1[PAIR ? NX - 1 : 1];
        if constexpr (PAIR) {
#pragma unroll
            for (int k = 0; k < NX - 1; ++k) cx1[k] = funnel(cx[k + 1], cx[k], 31);
        }
        // Decision bits, transposed: lane r holds col_r = sum_q bit r of U[q0+q] << q, so each
        // (q, r) decision is one scalar bit test of a readlane'd column (s_bitcmp + s_cbranch).
        uint32_t colv = 0u;
#pragma unroll
        for (int q = 0; q < QC; ++q) {
            const uint32_t uq = (q0 + q < nu) ? U[q0 + q] : 0u; // uniform address: broadcast read
            colv |= ((uq >> (lane & 31)) & 1u) << q;
        }

        uint32_t t[W];
#pragma unroll
        for (int j = 0; j < W; ++j) t[j] = 0u;
        uint32_t tlo = 0u; // word base-1 (lane 0 only meaningful), MULTI only
        if constexpr (PAIR) {
            for (int r = 30; r >= 0; r -= 2) {
                // t <<= 2 across the whole distributed polynomial
                const uint32_t prev = wave_shr1(t[W - 1], MULTI ? tlo : 0u);
#pragma unroll
                for (int j = W - 1; j >= 1; --j) t[j] = funnel(t[j], t[j - 1], 30);
                t[0] = funnel(t[0], prev, 30);
                if (MULTI) tlo <<= 2;
                const uint32_t chi = (uint32_t)__builtin_amdgcn_readlane((int)colv, r + 1);
                const uint32_t clo = (uint32_t)__builtin_amdgcn_readlane((int)colv, r);
                // three exclusive scalar masks and three flat ifs: a nested if/else is
                // structurised into VCC branches plus register copies
                const uint32_t both = PAIR == 1 ? chi & clo : 0u;
                const uint32_t hi = PAIR == 1 ? chi & ~clo : chi, lo = PAIR == 1 ? clo & ~chi : clo;
#pragma unroll
                for (int q = 0; q < QC; ++q) {
                    if (PAIR == 1 && __builtin_expect((both & (1u << q)) != 0, 1)) {
#pragma unroll
                        for (int j = 0; j < W; ++j) xor3_in(t[j], cx[j - q + QC + 1], cx1[j - q + QC]);
                        if (MULTI) tlo ^= cx[QC - q] ^ cx1[QC - 1 - q];
                    }
                    if (__builtin_expect((hi & (1u << q)) != 0, 1)) {
#pragma unroll
                        for (int j = 0; j < W; ++j) xor_in(t[j], cx1[j - q + QC]);
                        if (MULTI) tlo ^= cx1[QC - 1 - q];
                    }
                    if (__builtin_expect((lo & (1u << q)) != 0, 1)) {
#pragma unroll
                        for (int j = 0; j < W; ++j) xor_in(t[j], cx[j - q + QC + 1]);
                        if (MULTI) tlo ^= cx[QC - q];
                    }
                }
            }
        } else {
            for (int r = 31; r >= 0; --r) {
                // t <<= 1 across the whole distributed polynomial
                const uint32_t prev = wave_shr1(t[W - 1], MULTI ? tlo : 0u);
#pragma unroll
                for (int j = W - 1; j >= 1; --j) t[j] = funnel(t[j], t[j - 1], 31);
                t[0] = funnel(t[0], prev, 31);
                if (MULTI) tlo <<= 1;
                const uint32_t col = (uint32_t)__builtin_amdgcn_readlane((int)colv, r);
#pragma unroll
                for (int q = 0; q < QC; ++q) {
                    if (__builtin_expect((col & (1u << q)) != 0, 1)) {
                        asm volatile("" ::);
#pragma unroll
                        for (int j = 0; j < W; ++j) t[j] ^= cx[j - q + QC + 1];
                        if (MULTI) tlo ^= cx[QC - q];
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < W; ++j) acc[j] ^= t[j];
    }
    if constexpr (PAD) {
#pragma unroll
        for (int j = 0; j < W; ++j) acc[j] ^= (w0 + j < nadd) ? Add[w0 + j] : 0u;
    }
    int ldeg = -1;
#pragma unroll
    for (int j = 0; j < W; ++j) {
        if (PAD || w0 + j < nout) { // PAD: the whole tile is written (zeros past nout)
            Dst[w0 + j] = acc[j];
            if (acc[j]) ldeg = (w0 + j) * 32 + 31 - __builtin_clz(acc[j]);
        }
    }
    return wave_top_ordered(ldeg);
}

// Horner step form: 0 = one bit per step; 1 = two bits per step with the both-set case folded
// into one xor3 (three exclusive tests per word); 2 = two bits per step, two independent tests.
#ifndef HM_PAIR
#define HM_PAIR 2
#endif
constexpr int kPair = HM_PAIR;
// Tiles at least this wide are VALU-bound, where folding both-set pairs into one xor3 pays for
// its extra (taken) scalar branch; narrower tiles are branch-bound and keep two tests per word.
#ifndef HM_XOR3_MIN_W
#define HM_XOR3_MIN_W 99
#endif
template <int W> constexpr int pair_mode() { return (kPair == 2 && W >= HM_XOR3_MIN_W) ? 1 : kPair; }

template <int QC, int W, int WMAX, bool PAD>
__device__ __forceinline__ int mul_tiles(const uint32_t *U, int nu, const uint32_t *V, int nv,
                                         const uint32_t *Add, int nadd, uint32_t *Dst, int nout) {
    int top = mul_tile<W, QC, false, pair_mode<W>(), PAD>(U, nu, V, nv, Add, nadd, Dst, nout, 0);
    if constexpr (W == WMAX && !PAD) { // only the widest tile ever needs more than one pass
        for (int base = kWave * W; base < nout; base += kWave * W) {
            int t = mul_tile<W, QC, true, pair_mode<W>(), false>(U, nu, V, nv, Add, nadd, Dst, nout,
                                                                 base);
            if (t >= 0) top = t;
        }
    }
    return top;
}

// Dst[0..nout) = Add ^ U*V with nout = max(nu+nv, nadd).  Returns the exact degree (-1 = null).
// Dst must not alias U or Add; it may alias V only in PAD mode (one chunk, one tile: every window
// word is read into registers before the tile is written).  The per-lane tile width W is picked from nout among the
// instantiated widths <= WMAX (the kernel's VGPR budget is set by WMAX + QC); longer outputs are
// produced in several WMAX-wide tiles.
// PAD (caller guarantees): V has >= kHalo zero words below it and zeros from nv up to 64*WMAX,
// Dst has room for 64*W words, and nout <= 64*WMAX (one tile).
template <int QC, int WMAX, bool PAD = false>
__device__ __forceinline__ int wave_mul(const uint32_t *U, int nu, const uint32_t *V, int nv,
                                        const uint32_t *Add, int nadd, uint32_t *Dst,
                                        int *nout_p) {
    nu = (int)rfl((uint32_t)nu), nv = (int)rfl((uint32_t)nv), nadd = (int)rfl((uint32_t)nadd);
    const int nout = max(nu + nv, nadd);
    *nout_p = nout;
    const int w = (nout + kWave - 1) / kWave;
#define HM_TRY_W(WW)                                                                              \
    if constexpr (WW < WMAX) {                                                                    \
        if (w <= WW) return mul_tiles<QC, WW, WMAX, PAD>(U, nu, V, nv, Add, nadd, Dst, nout);          \
    }
    HM_TRY_W(1)
    HM_TRY_W(2)
    HM_TRY_W(3)
    HM_TRY_W(4)
    HM_TRY_W(5)
    HM_TRY_W(6)
    HM_TRY_W(7)
    HM_TRY_W(8)
    HM_TRY_W(9)
    HM_TRY_W(10)
    HM_TRY_W(11)
    HM_TRY_W(12)
    HM_TRY_W(16)
#undef HM_TRY_W
    return mul_tiles<QC, WMAX, WMAX, PAD>(U, nu, V, nv, Add, nadd, Dst, nout);
}

// Dst[0..n) = A ^ B (n = max(na, nb)); exact degree (-1 = null).  Strided lane loop.
__device__ __forceinline__ int wave_xor(const uint32_t *A, int na, const uint32_t *B, int nb,
                                        uint32_t *Dst) {
    const int n = max(na, nb);
    int ldeg = -1;
    for (int w = lane_id(); w < n; w += kWave) {
        uint32_t v = (w < na ? A[w] : 0u) ^ (w < nb ? B[w] : 0u);
        Dst[w] = v;
        if (v) ldeg = w * 32 + 31 - __builtin_clz(v);
    }
    return wave_max_i32(ldeg);
}

} // namespace hm
