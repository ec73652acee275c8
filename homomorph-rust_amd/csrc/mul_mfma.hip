// mul_mfma.hip — the multiplier's carry products on the gfx950 matrix cores: out = U * V over
// GF(2)[X] as {0,1} Toeplitz GEMMs on fp4 MFMA (mfma_gf2.h), replacing the scalar-decided VALU
// XORs of mul_engine.hip (mul_prod_kernel, mul_vprod_kernel).  Same products as the reference's
// Polynomial::mul (src/polynomial.rs:252-310): exact, so every bit is identical.
//
// Two kinds of task, one kernel body:
//   LEAF  the Karatsuba leaves (mul_host.cpp "Karatsuba"): arena views with explicit sizes;
//   SLOT  the schoolbook carry products p_t * x_t of the column plan: slots whose exact sizes come
//         from their degree rows (deg1), U = the operand with fewer words.
// One wavefront per (value, task, output span of `span` tiles of 32 words).  U is taken in blocks
// of kUB words (U * V = sum_b X^(32 kUB b) U_b * V).  Per block, in the wave's LDS slice:
//   RS   the bit-reversed nibble image of U_b over R = ub + 2 words (+ zero nibbles the last
//        chunk's window reaches),
//   VI   the nibble image (16 B per word) of the V words the span's windows reach, zero outside V,
// and across blocks OUT, the span's output words, XOR-accumulated.  Chunks (floor(ub/2) + 1 of
// K = 64) are taken in groups of G (16, then 4, then 1 for the tail): the group's A fragments are
// built once, then every tile of the span that the group reaches is swept, two tiles at a time
// (independent accumulator chains), one B read per chunk and tile.  Each (tile, group) starts its
// accumulators at 2^23, so its parities are its part of the product mod 2; parts of different
// groups and blocks meet in OUT by XOR (the parity of a sum is the XOR of the parities of its
// parts).
#include <hip/hip_runtime.h>

#include "mfma_gf2.h"

namespace hm {

constexpr int kMfG = 16;      // chunks per full A group (64 VGPRs of A fragments)

// Phase timers (diagnostic builds with -DHM_MF_PROFILE only; the library never has them): per
// launch class (the instance's template key), s_memtime deltas summed over waves for the record
// loads, the operand images, the chunk groups (A fragments + tiles) and the copy-out, plus the
// wave count; read back with hm_debug_mf_prof (scripts/mf_phases.py).
#ifdef HM_MF_PROFILE
__device__ unsigned long long g_mf_prof[8][8];
#define HM_MF_PT(v)                                                                               \
    asm volatile("" ::: "memory");                                                                \
    const unsigned long long v = __builtin_amdgcn_s_memtime();                                    \
    asm volatile("" ::: "memory")
#else
#define HM_MF_PT(v)
#endif
#ifndef HM_MF_PF
#define HM_MF_PF 3
#endif
constexpr int kMfPf = HM_MF_PF; // B reads issued ahead of their MFMA
constexpr int kVPad = 2 * kMfG + 32; // V words read beyond V's ends (zero)

// U blocks of at most ub = min(umax, kMfUB) words: the launch's LDS slices are sized for them
// (a launch of narrow schoolbook products reserves no 256-word U image, so more waves fit a CU)
__host__ __device__ constexpr uint32_t mf_ub(uint32_t umax) { return umax < kMfUB ? umax : kMfUB; }
__host__ __device__ constexpr uint32_t mf_rs_words(uint32_t umax) { return 4 * (mf_ub(umax) + 2) + 16; }
// V words one (block, span) reaches: 32 span + 32 + 2 NC (NC <= ub/2 + 1), or all of V plus its
// zero pads when that is fewer
__host__ __device__ constexpr uint32_t mf_vi_words(uint32_t vmax, uint32_t span, uint32_t umax) {
    const uint32_t a = 32 * span + 32 + 2 * (mf_ub(umax) / 2 + 1), b = vmax + 2 * kVPad;
    return 4 * ((a < b ? a : b) + 8);
}
__host__ __device__ constexpr uint32_t mf_wave_words(uint32_t vmax, uint32_t span, uint32_t umax) {
    return mf_rs_words(umax) + mf_vi_words(vmax, span, umax) + 32 * span;
}

__device__ __forceinline__ int floor_div32(int x) { return x >= 0 ? x / 32 : -((31 - x) / 32); }

// Tiles T0 .. T0 + NT - 1 (NT = 1, 2) against G chunks from c0: one accumulator set per tile,
// one B read per chunk and tile (window word 32T + col - D + h + 2c of VI, whose first word is
// vlo), the parities XORed into OUT (span-relative tile T - Ts).
template <int G, int NT>
__device__ __forceinline__ void mf_tiles(const v8i (&Af)[G], const uint32_t *VI, int vlo, int T0,
                                         int Ts, int c0, int D, uint32_t *OUT) {
    const int lane = lane_opaque(), col = lane & 31, h = lane >> 5;
    const uint4 *bt[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
        bt[t] = (const uint4 *)VI + (32 * (T0 + t) + col - D + h + 2 * c0 - vlo);
    v16f acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[t][j] = 8388608.0f;
    constexpr int P = G < kMfPf ? G : kMfPf;
    uint4 bq[NT][G];
#pragma unroll
    for (int c = 0; c < P; ++c)
#pragma unroll
        for (int t = 0; t < NT; ++t) bq[t][c] = bt[t][2 * c];
#pragma unroll
    for (int c = 0; c < G; ++c) {
        if (c + P < G) {
#pragma unroll
            for (int t = 0; t < NT; ++t) bq[t][c + P] = bt[t][2 * (c + P)];
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            acc[t] = mfma_fp4(Af[c], b_fragment(bq[t][c]), acc[t]);
            // keep the reads of later chunks below this MFMA (adder_mfma.hip tile_mfma)
            asm volatile("" : "+v"(acc[t])::"memory");
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        // row-permuted tiles (mfma_gf2.h row_bit): accumulator j is output bit j + 16h
        const uint32_t word = join_halves(acc_parities_hi16(acc[t]) >> (16 - 16 * h));
        if (h == 0) atomicXor(&OUT[32 * (T0 + t - Ts) + col], word); // this wave's slice only
    }
}

// One tile at a time with accumulators that keep counting across all of a wave's (tile, group)
// sweeps (HM_MF_CONT): a sweep's parities are bit 0 of the accumulators now XOR bit 0 before it
// (as the adder's chain does across tiles), so no 16 accumulator moves to 2^23 per tile -- a narrow
// product's tile is only ~9 MFMAs.  Counts stay exact: 2^23 + 64 per MFMA of the wave < 2^24.
#ifndef HM_MF_CONT
#define HM_MF_CONT 0 // (narrow instance: measured -1 % on the u8 multiply, its spills)
#endif
struct MfCont {
    v16f acc;
    uint32_t prev; // bit 16 + j = bit 0 of accumulator j after the last sweep
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = 8388608.0f;
        prev = 0u;
    }
};

template <int G>
__device__ __forceinline__ void mf_tile_cont(const v8i (&Af)[G], const uint32_t *VI, int vlo, int T0,
                                             int Ts, int c0, int D, uint32_t *OUT, MfCont &cs) {
    const int lane = lane_opaque(), col = lane & 31, h = lane >> 5;
    const uint4 *bt = (const uint4 *)VI + (32 * T0 + col - D + h + 2 * c0 - vlo);
    constexpr int P = G < kMfPf ? G : kMfPf;
    uint4 bq[G];
#pragma unroll
    for (int c = 0; c < P; ++c) bq[c] = bt[2 * c];
#pragma unroll
    for (int c = 0; c < G; ++c) {
        if (c + P < G) bq[c + P] = bt[2 * (c + P)];
        cs.acc = mfma_fp4(Af[c], b_fragment(bq[c]), cs.acc);
        asm volatile("" : "+v"(cs.acc)::"memory");
    }
    const uint32_t tnow = acc_parities_hi16(cs.acc);
    const uint32_t word = join_halves((tnow ^ cs.prev) >> (16 - 16 * h));
    cs.prev = tnow;
    if (h == 0) atomicXor(&OUT[32 * (T0 - Ts) + col], word); // this wave's slice only
}

// The A fragments of chunks c0 .. c0 + G - 1 from the U image RS (R words)
template <int G>
__device__ __forceinline__ void mf_afrags(const uint32_t *RS, int R, int D, int c0, v8i (&Af)[G]) {
    const int lane = lane_opaque(), col = lane & 31, h = lane >> 5;
    const int jb = 32 * (R - D + h) - 1 - row_bit(col); // (row-permuted tiles)
    const uint32_t *rw0 = RS + (jb >> 3) + 8 * c0;
    const uint32_t sh = 4u * (uint32_t)(jb & 7);
#pragma unroll
    for (int c = 0; c < G; ++c) Af[c] = a_fragment(rw0 + 8 * c, sh);
}

// Every tile of the span Ts .. Te - 1 that the group of G chunks from c0 reaches: two tiles at a
// time (two accumulator chains), or (PAIRS false: 16 + 12 fewer VGPRs) one at a time
template <int G, bool PAIRS = true, bool CONT = false>
__device__ __forceinline__ void mf_sweep(const v8i (&Af)[G], const uint32_t *VI, int vlo, int D,
                                         int nv, int Ts, int Te, int c0, uint32_t *OUT, MfCont &cs) {
    // tiles whose windows (words 32T - D + 2c0 .. 32T + 31 - D + 2(c0 + G) - 1) meet [0, nv)
    const int tlo = max(Ts, floor_div32(D - 2 * c0 - 2 * G + 1));
    const int thi = min(Te - 1, floor_div32(nv - 1 + D - 2 * c0));
    int T = tlo;
    if constexpr (PAIRS) {
        for (; T + 1 <= thi; T += 2) mf_tiles<G, 2>(Af, VI, vlo, T, Ts, c0, D, OUT);
        if (T <= thi) mf_tiles<G, 1>(Af, VI, vlo, T, Ts, c0, D, OUT);
    } else if constexpr (CONT) {
        for (; T <= thi; ++T) mf_tile_cont<G>(Af, VI, vlo, T, Ts, c0, D, OUT, cs);
    } else {
        for (; T <= thi; ++T) mf_tiles<G, 1>(Af, VI, vlo, T, Ts, c0, D, OUT);
    }
}

// One group of G chunks from c0 over the tiles tlo .. thi of the span
template <int G, bool PAIRS, bool CONT>
__device__ __forceinline__ void mf_group(const uint32_t *RS, const uint32_t *VI, int vlo, int R, int D,
                                         int nv, int Ts, int Te, int c0, uint32_t *OUT, MfCont &cs) {
    v8i Af[G];
    mf_afrags<G>(RS, R, D, c0, Af);
    mf_sweep<G, PAIRS, CONT>(Af, VI, vlo, D, nv, Ts, Te, c0, OUT, cs);
}

#ifndef HM_MF_IMG_BATCH
#define HM_MF_IMG_BATCH 4
#endif
constexpr int kMfImgBatch = HM_MF_IMG_BATCH; // operand words per lane loaded together (images)
// RS quad R-1-q = the nibbles of bitreverse(U[q]) for q < ub, zero up to R, then zero to rs_words
// (U2: a second view XORed in below ub2, a fused Karatsuba sum; ub2 <= 0: none)
__device__ __forceinline__ void mf_u_image(const uint32_t *U, int ub, int R, uint32_t rs_words,
                                           const uint32_t *tab, uint32_t *RS,
                                           const uint32_t *U2 = nullptr, int ub2 = 0) {
    const int lane = lane_id();
    // the lane's words are all loaded before any is converted (kMfImgBatch in flight per lane)
    for (int q0 = 0; q0 < R; q0 += kWave * kMfImgBatch) {
        uint32_t u[kMfImgBatch];
#pragma unroll
        for (int k = 0; k < kMfImgBatch; ++k) {
            const int q = q0 + lane + kWave * k;
            u[k] = q < ub ? U[q] ^ (q < ub2 ? U2[q] : 0u) : 0u;
        }
#pragma unroll
        for (int k = 0; k < kMfImgBatch; ++k) {
            const int q = q0 + lane + kWave * k;
            if (q >= R) break;
            const uint32_t rev = __builtin_bitreverse32(u[k]);
            uint4 x;
            x.x = tab[rev & 0xFFu], x.y = tab[(rev >> 8) & 0xFFu];
            x.z = tab[(rev >> 16) & 0xFFu], x.w = tab[rev >> 24];
            ((uint4 *)RS)[R - 1 - q] = x;
        }
    }
    for (int k = 4 * R + lane; k < (int)rs_words; k += kWave) RS[k] = 0u;
}

// VI quad i = the nibbles of V word vlo + i (zero outside [0, nv)) for i < vhi - vlo
__device__ __forceinline__ void mf_v_image(const uint32_t *V, int nv, int vlo, int vhi,
                                           const uint32_t *tab, uint32_t *VI,
                                           const uint32_t *V2 = nullptr, int nv2 = 0) {
    const int lane = lane_id();
    for (int i0 = 0; i0 < vhi - vlo; i0 += kWave * kMfImgBatch) {
        uint32_t v[kMfImgBatch];
#pragma unroll
        for (int k = 0; k < kMfImgBatch; ++k) {
            const int w = vlo + i0 + lane + kWave * k;
            v[k] = (w >= 0 && w < nv && w < vhi) ? V[w] ^ (w < nv2 ? V2[w] : 0u) : 0u;
        }
#pragma unroll
        for (int k = 0; k < kMfImgBatch; ++k) {
            const int i = i0 + lane + kWave * k;
            if (i >= vhi - vlo) break;
            uint4 q;
            q.x = tab[v[k] & 0xFFu], q.y = tab[(v[k] >> 8) & 0xFFu];
            q.z = tab[(v[k] >> 16) & 0xFFu], q.w = tab[v[k] >> 24];
            ((uint4 *)VI)[i] = q;
        }
    }
}

// One group of G chunks from c0 whose A fragments come from a window of the U image built for
// this group alone (the lean leaf instance keeps no whole-U image): RS quads Qlo = 2 c0 + 1 ..
// Qlo + 2G + 1, i.e. U words q = R - 1 - Q (zero outside [0, ub)), are all its fragments read
__host__ __device__ constexpr uint32_t mf_win_words(int G) { return 4u * (2u * (uint32_t)G + 2u) + 16u; }
// lane k's U word of the window of the group of G chunks from c0 (k < 2G + 2 <= 36 lanes)
__device__ __forceinline__ uint32_t mf_win_word(const uint32_t *Ub, int ub, int R, int c0, int G,
                                                const uint32_t *Ub2, int ub2) {
    const int lane = lane_id();
    const int q = R - 1 - (2 * c0 + 1 + lane);
    return (lane < 2 * G + 2 && q >= 0 && q < ub) ? Ub[q] ^ (q < ub2 ? Ub2[q] : 0u) : 0u;
}
// wword: this lane's window word (mf_win_word, loaded ahead); the next group's is loaded here,
// before the sweep, into *next (G2 chunks from c0 + G; G2 = 0: none)
template <int G, bool CONT>
__device__ __forceinline__ void mf_group_win(uint32_t wword, const uint32_t *Ub, int ub, int G2,
                                             uint32_t *next, uint32_t *RSW, const uint32_t *tab,
                                             const uint32_t *VI, int vlo, int R, int D, int nv,
                                             int Ts, int Te, int c0, uint32_t *OUT,
                                             const uint32_t *Ub2, int ub2, MfCont &cs) {
    const int lane = lane_id();
    const int Qlo = 2 * c0 + 1;
    wsync(); // the previous group's fragment reads are done
    if (lane < 2 * G + 2) {
        const uint32_t rev = __builtin_bitreverse32(wword);
        uint4 x;
        x.x = tab[rev & 0xFFu], x.y = tab[(rev >> 8) & 0xFFu];
        x.z = tab[(rev >> 16) & 0xFFu], x.w = tab[rev >> 24];
        ((uint4 *)RSW)[lane] = x;
    }
    wsync();
    v8i Af[G];
    mf_afrags<G>(RSW - 4 * Qlo, R, D, c0, Af);
    if (G2) *next = mf_win_word(Ub, ub, R, c0 + G, G2, Ub2, ub2);
    mf_sweep<G, false, CONT>(Af, VI, vlo, D, nv, Ts, Te, c0, OUT, cs);
}

#ifndef HM_MF_WPE
#define HM_MF_WPE 3
#endif
#ifndef HM_MF_WPE_MIN
#define HM_MF_WPE_MIN 2
#endif
#ifndef HM_MFN_WPE
#define HM_MFN_WPE 4
#endif
// LEAN instances trade the paired tile chains for occupancy: one tile at a time, <= 128 VGPRs,
// 4 waves per SIMD.
//  - schoolbook (LEAF false): the launches whose U has at most kMfNarrowWords words (mul_host.cpp).
//    Such a wave is short (a 33-word U is 17 chunks: ~76 MFMAs) and waits on its record and operand
//    loads for much of its life; the host sizes the narrow spans so 16 waves' LDS slices fit.
//  - leaves (LEAF true): no whole-U image either, only each group's window (mf_group_win), so a
//    256-word leaf's LDS slice is ~9 KB instead of ~12.5 KB and 16 waves fit a CU.
//  - wide schoolbook products (LEAF false, WIN true: U above kMfNarrowWords) the same way as the
//    leaves: per-group U windows, spans of kMfWideLeanSpan tiles.
#ifndef HM_MFT_WPE
#define HM_MFT_WPE 5
#endif
// GMAX: the most chunks any task of the launch has (the tiny class: kMfTinyChunks; otherwise any
// count, in groups of GS and one tail group of at most GS + 1)
#ifndef HM_MFNS_WPE
#define HM_MFNS_WPE 5 // waves per SIMD of the narrow instance with groups smaller than kMfG
#endif
#ifndef HM_MFN_GS
#define HM_MFN_GS 16 // chunks per group of the narrow instance (A fragments held: GS + 1)
#endif
// One work item of mul_mfma_kernel: a leaf's whole output or one span of a schoolbook product,
// for value e, in the wave's LDS slice (lds: the block's LDS, tab: its nibble table)
template <bool LEAF, bool LEAN, bool WIN, int GMAX, int GS>
__device__ __forceinline__ void mf_item(const MulMfmaArgs &P, uint64_t e, uint32_t item, uint32_t *lds,
                                        const uint32_t *tab, int wave) {
    HM_MF_PT(tp0);
    uint32_t *arena = P.B.arena + e * P.B.astride;
    const uint32_t *U, *V, *U2 = nullptr, *V2 = nullptr;
    uint32_t *O;
    int nu, nv, nout, base, nu2 = 0, nv2 = 0;
    if constexpr (LEAF) {
        const MulVTask t = ((const MulVTask *)P.tasks)[item / P.nspans];
        base = (int)(item % P.nspans) * 32 * (int)P.span;
        U = arena + t.u, V = arena + t.v, O = arena + t.out;
        nu = (int)rfl(t.nu), nv = (int)rfl(t.nv), nout = (int)rfl(t.nout);
        // a fused Karatsuba sum: the operand is u ^ u2 (second view nu2 <= nu words)
        nu2 = (int)rfl(t.nu2), nv2 = (int)rfl(t.nv2);
        U2 = arena + (nu2 ? t.u2 : t.u), V2 = arena + (nv2 ? t.v2 : t.v);
        if (base >= nout) return;
    } else {
        // one host-resolved record (MulSpanRec): the operands' degrees are the only loads that
        // depend on it (u8 multiply, batch 16384: 4.74 -> 4.82e6/s against the span -> task ->
        // slot chain; sizes from the static bounds instead of the degrees measured 4.61e6/s)
        const MulSpanRec r = P.recs[item];
        base = (int)rfl(r.base);
        U = arena + r.uoff, V = arena + r.voff, O = arena + r.ooff;
        nout = (int)rfl(r.nout);
        const uint32_t du = rfl(P.B.deg1[(uint64_t)r.uslot * P.B.nv + e]);
        const uint32_t dv = rfl(P.B.deg1[(uint64_t)r.vslot * P.B.nv + e]);
        nu = bitwords((int)du), nv = bitwords((int)dv);
        if (base == 0 && lane_id() == 0)
            P.B.deg1[(uint64_t)r.oslot * P.B.nv + e] = (du && dv) ? du + dv - 1 : 0u;
    }
    if (!nu2) U2 = U; // (never read: a valid pointer all the same)
    if (!nv2) V2 = V;
    const int lane = lane_id();
    const int span = (int)P.span;
    const int wend = min(nout, base + 32 * span); // this span's output words [base, wend)
    if (nu == 0 || nv == 0) {
        for (int w = base + lane; w < wend; w += kWave) O[w] = 0u;
        return;
    }
    static_assert(!WIN || LEAN, "windows come with the lean instance");
    uint32_t *RS = lds + 256 + (size_t)wave * P.wave_words;
    const uint32_t rs_words = WIN ? mf_win_words(kMfG + 1) : mf_rs_words(P.umax);
    uint32_t *VI = RS + rs_words;
    uint32_t *OUT = VI + mf_vi_words(P.vmax, P.span, P.umax);
    for (int w = lane; w < wend - base; w += kWave) OUT[w] = 0u; // the span's live words
    const int T0 = base >> 5;
#ifdef HM_MF_PROFILE
    (void)rfl((uint32_t)(uintptr_t)U); // the record loads have landed
    HM_MF_PT(tp1);
    unsigned long long t_img = 0, t_grp = 0;
#endif
    // (the one-tile-at-a-time instances: accumulators counting across the wave's sweeps)
    constexpr bool CONT = LEAN && !LEAF && !WIN && GMAX > GS && HM_MF_CONT; // (narrow: spills elsewhere)
    MfCont cs;
    if constexpr (CONT) cs.init();
    for (int b0 = 0; b0 < nu; b0 += kMfUB) {
        // U_b = words [b0, b0 + ub) of U: its product with V lands kb = b0/32 tiles up
        const int ub = min(kMfUB, nu - b0), kb = b0 >> 5;
        const int Ts = T0 - kb, Te = Ts + span;      // the span in U_b * V's tiles
        if (Te <= 0) break;                          // this and later blocks land above the span
        const int D = ub, R = ub + 2, nc = ub / 2 + 1;
        const int vlo = max(32 * Ts - D, -kVPad);
        const int vhi = min(32 * Te + 32 - D + 2 * nc, nv + kVPad);
        wsync(); // the previous block's reads of RS / VI are done
        // RS quad R-1-q = the nibbles of bitreverse(U_b[q]) (one load, one 16-B store per word)
        HM_MF_PT(tpa);
        if constexpr (!WIN) mf_u_image(U + b0, ub, R, rs_words, tab, RS, U2 + b0, nu2 - b0);
        mf_v_image(V, nv, vlo, vhi, tab, VI, V2, nv2);
        wsync();
#ifdef HM_MF_PROFILE
        __builtin_amdgcn_s_waitcnt(0); // (the image stores)
        HM_MF_PT(tpb);
        t_img += tpb - tpa;
#endif
        const int tlo = max(Ts, 0);
        uint32_t *OUTs = OUT + 32 * (tlo - Ts);
        // groups of 16 chunks while more than 17 are left, then the rest as ONE group of 1..17
        // chunks: every group costs a parity gather per tile it reaches, so a narrow U (the
        // 17-word partial products at d + d' = 512: 9 chunks) takes one gather per tile instead of
        // one per 4-chunk group, and a 256-word leaf's 129 chunks end in a 17-chunk group
        int c0 = 0;
        // (lean leaves) each group's U window words are loaded one group ahead
        auto gsize = [&](int c) { return nc - c > GS + 1 ? GS : nc - c; };
        uint32_t ww = WIN ? mf_win_word(U + b0, ub, R, 0, gsize(0), U2 + b0, nu2 - b0) : 0u;
        static_assert(!WIN || GS == kMfG, "the windowed instances' LDS is sized for kMfG + 1");
        if constexpr (GMAX <= GS) {
            if (nc > GMAX) { // (the plan's class bound)
                if (lane == 0) flag(P.B.status, HM_ERR_BAD_INPUT);
                c0 = nc;
            }
        }
        for (; GMAX > GS && nc - c0 > GS + 1; c0 += GS) {
            if constexpr (WIN)
                mf_group_win<GS, CONT>(ww, U + b0, ub, gsize(c0 + GS), &ww, RS, tab, VI, vlo, R, D,
                                       nv, tlo, Te, c0, OUTs, U2 + b0, nu2 - b0, cs);
            else mf_group<GS, !LEAN, CONT>(RS, VI, vlo, R, D, nv, tlo, Te, c0, OUTs, cs);
        }
        switch (nc - c0) {
#define HM_MF_TAIL(G) \
    case G:                                                                                      \
        if constexpr (G > GMAX || G > GS + 1) {                                                  \
        } else if constexpr (WIN)                                                                \
            mf_group_win<G, CONT>(ww, U + b0, ub, 0, &ww, RS, tab, VI, vlo, R, D, nv, tlo, Te, c0,  \
                                  OUTs, U2 + b0, nu2 - b0, cs);                                  \
        else mf_group<G, !LEAN, CONT>(RS, VI, vlo, R, D, nv, tlo, Te, c0, OUTs, cs);           \
        break;
            HM_MF_TAIL(1) HM_MF_TAIL(2) HM_MF_TAIL(3) HM_MF_TAIL(4) HM_MF_TAIL(5) HM_MF_TAIL(6)
            HM_MF_TAIL(7) HM_MF_TAIL(8) HM_MF_TAIL(9) HM_MF_TAIL(10) HM_MF_TAIL(11) HM_MF_TAIL(12)
            HM_MF_TAIL(13) HM_MF_TAIL(14) HM_MF_TAIL(15) HM_MF_TAIL(16) HM_MF_TAIL(17)
#undef HM_MF_TAIL
        default: break;
        }
#ifdef HM_MF_PROFILE
        HM_MF_PT(tpc);
        t_grp += tpc - tpb;
#endif
    }
    wsync();
    for (int w = base + lane; w < wend; w += kWave) O[w] = OUT[w - base];
#ifdef HM_MF_PROFILE
    __builtin_amdgcn_s_waitcnt(0);
    HM_MF_PT(tp9);
    if (lane == 0) {
        // class: 0 leaves, 1 lean leaves, 2 tiny, 3 narrow, 4 wide (windowed), 5 wide
        const int cls = LEAF ? (LEAN ? 1 : 0) : (GMAX <= kMfG ? 2 : (LEAN && !WIN) ? 3 : WIN ? 4 : 5);
        atomicAdd(&g_mf_prof[cls][0], 1ull);
        atomicAdd(&g_mf_prof[cls][1], tp1 - tp0);       // records, degrees, OUT zero
        atomicAdd(&g_mf_prof[cls][2], t_img);           // operand images
        atomicAdd(&g_mf_prof[cls][3], t_grp);           // A fragments + tiles
        atomicAdd(&g_mf_prof[cls][4], tp9 - tp1 - t_img - t_grp); // copy-out and the rest
    }
#endif
}


template <bool LEAF, bool LEAN = false, bool WIN = LEAF && LEAN, int GMAX = kMfG + 1, int GS = kMfG>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(GMAX <= kMfG ? HM_MFT_WPE : GS < kMfG ? HM_MFNS_WPE : LEAN ? HM_MFN_WPE : HM_MF_WPE_MIN,
                                   GMAX <= kMfG ? HM_MFT_WPE : GS < kMfG ? HM_MFNS_WPE : LEAN ? HM_MFN_WPE : HM_MF_WPE)))
mul_mfma_kernel(MulMfmaArgs P) {
    extern __shared__ uint32_t lds[];
    uint32_t *tab = lds;
    nibble_table(tab);
    __syncthreads();
    const int wave = (int)rfl(threadIdx.x >> 6);
    // P.per_wave consecutive items per wave (the tiny and narrow classes: more work per wave for
    // its nibble table, launch and LDS slice; the next item's record loads issue under this one's)
    if constexpr (LEAF || WIN) { // (one item per wave: no loop around the big instances)
        const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
        const uint64_t e = g / P.nitems;
        if (e >= P.B.nv) return; // whole wave exits together
        mf_item<LEAF, LEAN, WIN, GMAX, GS>(P, e, (uint32_t)(g % P.nitems), lds, tab, wave);
        return;
    }
    const uint32_t per = P.per_wave;
    const uint64_t g0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + wave) * per;
    for (uint32_t k = 0; k < per; ++k) {
        const uint64_t g = g0 + k;
        const uint64_t e = g / P.nitems;
        if (e >= P.B.nv) return; // whole wave exits together
        mf_item<LEAF, LEAN, WIN, GMAX, GS>(P, e, (uint32_t)(g % P.nitems), lds, tab, wave);
        wsync(); // (the item's last LDS reads precede the next item's writes)
    }
}

// Partial products a_j * b_k grouped by a_j (MulPPGroup): one wave per (value, group).  a_j has
// at most kMfPPGWords words, so its chunks (nu/2 + 1 <= 17) are one group: the A fragments are
// built once, then every product of the group gets its V image, its tiles (the whole output:
// span tiles) and its output words and degree.  Same products as mul_mfma_kernel<false>.
// A product is only 2 x (nu/2 + 1) MFMAs, so its loads are staged per batch of kPPGBatch items
// instead of per product: the items' records (one lane each), then their degrees and slots, then
// every item's b_k words into the wave's VW slice (one word per lane and item, all in flight
// together) -- three dependent loads per batch where a product at a time took three each.
constexpr int kPPGBatch = (int)kMfPPGBatch;
static_assert(kMfPPGWords <= 64, "one word per lane");

template <int G, bool PAIRS>
__device__ __forceinline__ void ppg_products(const MulPPGArgs &P, uint64_t e, const MulPPGroup &grp,
                                             const uint32_t *RS, int nu, uint32_t du,
                                             const uint32_t *tab, uint32_t *VW, uint32_t *VI,
                                             uint32_t *OUT) {
    const int lane = lane_id();
    uint32_t *arena = P.B.arena + e * P.B.astride;
    const int D = nu, R = nu + 2;
    const int vlo = -D; // D <= kMfPPGWords < kVPad
    v8i Af[G];
    mf_afrags<G>(RS, R, D, 0, Af);
    MfCont cs0; // (unused: the paired sweeps reset their accumulators per tile)
    for (uint32_t i0 = 0; i0 < grp.count; i0 += kPPGBatch) {
        const int nb = (int)min((uint32_t)kPPGBatch, grp.count - i0);
        uint32_t dv = 0u, voff = 0u, ooff = 0u, ow = 0u, oslot = 0u;
        if (lane < nb) {
            const MulPPItem it = P.items[grp.first + i0 + lane];
            dv = P.B.deg1[(uint64_t)it.v * P.B.nv + e];
            voff = P.B.slots[it.v].off;
            ooff = P.B.slots[it.out].off;
            ow = P.B.slots[it.out].words;
            oslot = it.out;
        }
        uint32_t vw[kPPGBatch];
#pragma unroll
        for (int k = 0; k < kPPGBatch; ++k) {
            const int nvk = bitwords((int)__builtin_amdgcn_readlane(dv, k));
            const uint32_t vo = __builtin_amdgcn_readlane(voff, k);
            vw[k] = (k < nb && lane < nvk) ? arena[vo + lane] : 0u;
        }
        wsync(); // the previous batch's reads of VW are done
#pragma unroll
        for (int k = 0; k < kPPGBatch; ++k) VW[64 * k + lane] = vw[k];
        for (int k = 0; k < nb; ++k) {
            const uint32_t dvk = __builtin_amdgcn_readlane(dv, k);
            const int nv = bitwords((int)dvk);
            uint32_t *O = arena + __builtin_amdgcn_readlane(ooff, k);
            const int nout = (int)__builtin_amdgcn_readlane(ow, k);
            if (lane == 0)
                P.B.deg1[(uint64_t)__builtin_amdgcn_readlane(oslot, k) * P.B.nv + e] = dvk ? du + dvk - 1 : 0u;
            if (nv == 0) {
                for (int w = lane; w < nout; w += kWave) O[w] = 0u;
                continue;
            }
            const int Te = min((int)P.span, (nout + 31) >> 5);
            const int vhi = min(32 * Te + 32 - D + 2 * G, nv + kVPad);
            wsync(); // VW written; the previous product's reads of VI and OUT are done
            for (int j = lane; j < vhi - vlo; j += kWave) {
                const int w = vlo + j;
                const uint32_t v = (w >= 0 && w < nv) ? VW[64 * k + w] : 0u;
                uint4 q;
                q.x = tab[v & 0xFFu], q.y = tab[(v >> 8) & 0xFFu];
                q.z = tab[(v >> 16) & 0xFFu], q.w = tab[v >> 24];
                ((uint4 *)VI)[j] = q;
            }
            for (int w = lane; w < nout; w += kWave) OUT[w] = 0u;
            wsync();
            mf_sweep<G, PAIRS>(Af, VI, vlo, D, nv, 0, Te, 0, OUT, cs0);
            wsync();
            for (int w = lane; w < nout; w += kWave) O[w] = OUT[w];
        }
    }
}

#ifndef HM_PPG_NO_TINY
#define HM_PPG_NO_TINY 0 // (A/B knob) the partial products on the general instance only
#endif
#ifndef HM_PPGT_WPE
#define HM_PPGT_WPE 4
#endif
// GMAX: the most chunks of any a_j (kMfTinyChunks: a_j within kMfTinyWords words, the fresh
// operands of d + d' <= 512 -- an instance with 11 A fragments and one tile at a time, the products'
// outputs being one or two tiles, at HM_MFT_WPE waves per SIMD instead of 3)
template <int GMAX>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(GMAX <= kMfG ? HM_PPGT_WPE : HM_MF_WPE_MIN, GMAX <= kMfG ? HM_PPGT_WPE : HM_MF_WPE)))
mul_ppg_kernel(MulPPGArgs P) {
    extern __shared__ uint32_t lds[];
    uint32_t *tab = lds;
    nibble_table(tab);
    __syncthreads();
    const int wave = (int)rfl(threadIdx.x >> 6);
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    const uint64_t e = g / P.ngroups;
    if (e >= P.B.nv) return; // whole wave exits together
    const MulPPGroup grp = P.groups[g % P.ngroups];
    const int lane = lane_id();
    uint32_t *arena = P.B.arena + e * P.B.astride;
    const uint32_t du = rfl(P.B.deg1[(uint64_t)grp.u * P.B.nv + e]);
    const int nu = bitwords((int)du);
    constexpr int kUMax = GMAX <= kMfG ? (int)kMfTinyWords : (int)kMfPPGWords; // (the plan's bound)
    if (nu == 0 || nu > kUMax) { // null a_j: every product of the group is null
        for (uint32_t it = 0; it < grp.count; ++it) {
            const MulPPItem item = P.items[grp.first + it];
            uint32_t *O = arena + P.B.slots[item.out].off;
            for (int w = lane; w < (int)P.B.slots[item.out].words; w += kWave) O[w] = 0u;
            if (lane == 0) P.B.deg1[(uint64_t)item.out * P.B.nv + e] = 0u;
        }
        if (nu > kUMax && lane == 0) flag(P.B.status, HM_ERR_BAD_INPUT); // (plan bound)
        return;
    }
    uint32_t *RS = lds + 256 + (size_t)wave * P.wave_words;
    const uint32_t rs_words = mf_rs_words(P.umax);
    uint32_t *VI = RS + rs_words;
    uint32_t *OUT = VI + mf_vi_words(P.vmax, P.span, P.umax);
    uint32_t *VW = OUT + 32 * P.span; // kPPGBatch x 64 staged b_k words
    mf_u_image(arena + P.B.slots[grp.u].off, nu, nu + 2, rs_words, tab, RS);
    wsync();
    switch (nu / 2 + 1) {
#define HM_PPG(G) \
    case G:                                                                                      \
        if constexpr (G <= GMAX) ppg_products<G, (GMAX > kMfG)>(P, e, grp, RS, nu, du, tab, VW, VI, OUT); \
        break;
        HM_PPG(1) HM_PPG(2) HM_PPG(3) HM_PPG(4) HM_PPG(5) HM_PPG(6) HM_PPG(7) HM_PPG(8) HM_PPG(9)
        HM_PPG(10) HM_PPG(11) HM_PPG(12) HM_PPG(13) HM_PPG(14) HM_PPG(15) HM_PPG(16) HM_PPG(17)
#undef HM_PPG
    default: break;
    }
}

int launch_mul_ppg(const MulPPGArgs &a, void *stream) {
    const uint64_t waves = a.B.nv * a.ngroups;
    if (!waves) return 0;
    const size_t lds = (256 + (size_t)a.wave_words * 4) * 4;
    if (a.umax <= kMfTinyWords && !HM_PPG_NO_TINY)
        hipLaunchKernelGGL(mul_ppg_kernel<kMfTinyChunks>, dim3((unsigned)((waves + 3) / 4)), dim3(256), lds,
                           (hipStream_t)stream, a);
    else hipLaunchKernelGGL(mul_ppg_kernel<kMfG + 1>, dim3((unsigned)((waves + 3) / 4)), dim3(256), lds,
                       (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#ifndef HM_MF_PER
#define HM_MF_PER 4
#endif
int launch_mul_mfma(const MulMfmaArgs &args, bool leaf, void *stream) {
    MulMfmaArgs a = args;
    // the tiny and narrow schoolbook classes: HM_MF_PER spans per wave (their waves are short)
    a.per_wave = (!leaf && a.umax <= kMfNarrowWords) ? HM_MF_PER : 1u; // (LEAF / WIN: 1)
    const uint64_t items = a.B.nv * a.nitems;
    if (!items) return 0;
    const uint64_t waves = (items + a.per_wave - 1) / a.per_wave;
    const size_t lds = (256 + (size_t)a.wave_words * 4) * 4;
    const dim3 grid((unsigned)((waves + 3) / 4)), block(256);
    if (leaf && a.lean)
        hipLaunchKernelGGL((mul_mfma_kernel<true, true>), grid, block, lds, (hipStream_t)stream, a);
    else if (leaf) hipLaunchKernelGGL(mul_mfma_kernel<true>, grid, block, lds, (hipStream_t)stream, a);
    else if (a.umax <= kMfTinyWords)
        hipLaunchKernelGGL((mul_mfma_kernel<false, true, false, kMfTinyChunks>), grid, block, lds,
                           (hipStream_t)stream, a);
    else if (a.umax <= kMfNarrowWords)
        hipLaunchKernelGGL((mul_mfma_kernel<false, true, false, kMfG + 1, HM_MFN_GS>), grid, block, lds,
                           (hipStream_t)stream, a);
    else if (a.lean)
        hipLaunchKernelGGL((mul_mfma_kernel<false, true, true>), grid, block, lds, (hipStream_t)stream, a);
    else hipLaunchKernelGGL(mul_mfma_kernel<false>, grid, block, lds, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

uint32_t mul_mfma_wave_words(uint32_t vmax, uint32_t span, uint32_t umax) {
    return mf_wave_words(vmax, span, umax);
}

uint32_t mul_mfma_lean_leaf_wave_words(uint32_t vmax, uint32_t span, uint32_t umax) {
    return mf_win_words(kMfG + 1) + mf_vi_words(vmax, span, umax) + 32 * span;
}

} // namespace hm

#ifdef HM_MF_PROFILE
extern "C" int hm_debug_mf_prof(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hm::g_mf_prof), sizeof(hm::g_mf_prof)) != hipSuccess) return -1;
    if (reset) {
        static unsigned long long zero[8][8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(hm::g_mf_prof), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
