// adder_mfma.hip — the ripple-carry adder's carry chain on the matrix cores (gfx950 fp4 MFMA).
//
// The chain (src/impls/numbers/common.rs:37-56) is  carry_{i+1} = ab_i ^ P_i * carry_i  with one
// carry-less product per bit (adder.hip derives the identity; add_prep_kernel computes ab_i, P_i
// and x_i).  A GF(2)[X] product is a {0,1} convolution reduced mod 2:
//     bit k of P*C = ( sum_j P[j] C[k-j] ) mod 2,
// and v_mfma_scale_f32_32x32x64_f8f6f4 with fp4 (e2m1) operands multiplies {0,1} matrices exactly
// (products 0/1, f32 accumulation exact below 2^24).  So the product runs as a Toeplitz GEMM:
//
//   output tile T = 32 carry words W = 32T + n (MFMA column n) x 32 bit positions m (MFMA row m).
//   K runs over the carry window of W: words w = W - D + 2c + h (chunk c, lane half h) and their
//   bits e, so that
//       out[32W + m] = sum_{c,h,e} A_c[m][(h,e)] * B_c[(h,e)][n]
//       A_c[m][(h,e)] = P[32(D - 2c - h) + m - e]      (independent of the tile: built once per bit)
//   (with the rows permuted, mfma_gf2.h row_bit: A row m computes output bit row_bit(m), so that
//   each lane's 16 accumulators are one contiguous half of the output word)
//       B_c[(h,e)][n] = C[32(32T + n - D + 2c + h) + e]
//   with D = np (np = words of P_i: output word W takes carry words W-np .. W, since word q of P
//   times word w of the carry reaches output words q+w and q+w+1) and NC = floor(np/2) + 1
//   chunks of K = 64.  At d+d' = 256 (P_i < 2^769, 25 words) that is 13 MFMAs per 32 output
//   words, 8 % above the dense bit-pair count.
//
// tools/fp4_mfma_probe.hip pins what this relies on: lane l holds A row l%32 and B column l%32,
// element e of lane half h of A meets element e of lane half h of B, and fp4 reads only the low 4
// operand VGPRs.  Element e of a fragment is nibble e%8 of VGPR e/8.
//
// Per value (one wave), in LDS:
//   C     the carry as bits (u32 words), zero halo below, updated in place tile by tile from the
//         top (tile T's output words are no longer read by tiles < T);
//   ring  nibble images of the carry words the next tiles read (fp4 1.0 per set bit, 16 B per
//         word, 128 slots, the first kMirror of them mirrored past the end): a B fragment is one
//         ds_read_b128;
//   RS    the nibble image of P_i bit-reversed: an A fragment is a 128-bit window of it.
// A 1 KB table per block maps a byte to its 8 nibbles.
//
// Parity: every accumulator starts at 2^23, so after the MFMAs it holds 2^23 + count exactly and
// bit 0 of its f32 encoding is the coefficient.  One v_alignbit per accumulator gathers them.
#include <hip/hip_runtime.h>

#include "mfma_gf2.h"

namespace hm {
// Per chunk count NC (engine.h MfmaCfg: 13 chunks for P_i up to 25 words, d + d' <= 256; 25 for
// up to 49 words, d + d' <= 512):
//   RS    P_i bit-reversed over kRevWords words (> max np + 1), as nibble words, plus the zero
//         nibble words that the windows of the chunks past P reach;
//   halo  zero carry words below C (>= the deepest window reach, np words);
//   rec   words of one bit's workspace record (one or two 64-lane LDS-DMAs).

// Phase timers (tools/chain_check.hip builds with HM_MFMA_PROFILE; the library never does):
// per-wave sums of s_memtime deltas for the sum store, the A build and the tile loop.
#ifdef HM_MFMA_PROFILE
__device__ unsigned long long *g_mfma_prof; // 4 per wave, set by the harness
#define HM_PT(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define HM_PACC(k, a, b) prof[k] += (b) - (a)
#else
#define HM_PT(v)
#define HM_PACC(k, a, b)
#endif

// acc += A * B over the kMfmaChunks chunks of one tile; rb = the tile's window slot (chunk c's B
// fragment at rb[2c]).  The reads run kPrefetch chunks ahead of the MFMAs.  Left alone, the
// compiler hoists all 13 reads (13 x 4 VGPRs beside A's 52: spills) and sinks the MFMAs below
// them; an empty asm after each MFMA that names acc (so the MFMA stays above it: no instruction,
// no wait) and clobbers memory (so later reads stay below it) pins the interleaving.
#ifndef HM_MFMA_PREFETCH
#define HM_MFMA_PREFETCH 3
#endif
// the 25-chunk chain reads 4 ahead: configs[4] 925-929 -> 922-923 ms per 2^20 (2: 932-936,
// 5: 926-927), measured when it ran at 2 waves per SIMD; re-measured in round 5 at its current
// 3 waves per SIMD (168 VGPRs, HM_MFMA25_WPE): 3 ahead 881.1-883.7 ms, 4 ahead 881.4-884.4,
// 5 ahead 898.4-898.5 (alternating on one box)
#ifndef HM_MFMA_PREFETCH25
#define HM_MFMA_PREFETCH25 4
#endif
// (NC = 7, configs[0]'s d + d' = 128: 2 ahead, so that the ring fill's three stages fit before
// the next tile's reads)
template <int NC> constexpr int kPrefetchOf = NC > 16 ? HM_MFMA_PREFETCH25 : NC <= 8 ? 2 : HM_MFMA_PREFETCH;
// side(k) runs after MFMA kStage<NC>(k) = 1, 4, 7 (NC = 7: 0, 2, 4): the next tile's ring fill in
// three stages, its LDS latency hidden under this tile's MFMAs instead of stalling the wave between
// tiles
template <int NC> constexpr int kStage(int k) { return NC <= 8 ? 2 * k : 1 + 3 * k; }
template <int NC, class Side, int kPrefetch = kPrefetchOf<NC>>
__device__ __forceinline__ v16f tile_mfma(const v8i (&Af)[NC], const uint4 *rb, const uint4 *rbn,
                                          uint4 (&pf)[kPrefetch], v16f acc, Side &&side) {
    // pf holds this tile's first kPrefetch B fragments (read during the tile before); the last
    // kPrefetch reads of this tile fetch the next tile's (window base rbn; its ring fill is side
    // stage 2, issued above them), so the next tile's first MFMA does not wait for the LDS
    static_assert(NC - kPrefetch > kStage<NC>(2), "next tile's B reads must follow its ring fill (stage 2)");
    uint4 bq[NC];
#pragma unroll
    for (int c = 0; c < kPrefetch; ++c) bq[c] = pf[c];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        if (c + kPrefetch < NC) bq[c + kPrefetch] = rb[2 * (c + kPrefetch)];
        else pf[c + kPrefetch - NC] = rbn[2 * (c + kPrefetch - NC)];
        const v8i Bf = {(int)bq[c].x, (int)bq[c].y, (int)bq[c].z, (int)bq[c].w, 0, 0, 0, 0};
        acc = mfma_fp4(Af[c], Bf, acc);
        asm volatile("" : "+v"(acc)::"memory");
        if (c == kStage<NC>(0)) side(0);
        if (c == kStage<NC>(1)) side(1);
        if (c == kStage<NC>(2)) side(2);
    }
    return acc;
}

// Ring slot of carry word w: its nibble image at slot w % kMfmaRingSlots, and slots below
// kMirror once more past the end, so a tile's window [slot, slot + 2*NC - 1) is contiguous
// wherever it starts: its B reads share one address and differ by immediates.
template <int kMirror>
__device__ __forceinline__ void ring_put(uint32_t *ring, int w, int h, uint2 nb) {
    const int s = w & (kMfmaRingSlots - 1);
    uint32_t *slot = &ring[s * 4 + 2 * h];
    *(uint2 *)slot = nb;
    if (kMirror >= kMfmaRingSlots || s < kMirror) *(uint2 *)(slot + 4 * kMfmaRingSlots) = nb;
}

// Nibble images of carry words [base, base + count) into the ring (count <= 64).  Lane l writes
// bytes 2h, 2h+1 of word base + k (k = l/2 + 32*pass, h = l%2) as two table lookups: a lane pair
// fills one 16-byte slot, so a wave's 8-byte stores are contiguous (no LDS bank conflicts; lane
// halves h = l/32 wrote 16-byte-strided pieces, two-way conflicted)
#ifndef HM_RING_PAIRS
#define HM_RING_PAIRS 1 // (A/B knob) 0: lane halves h = l/32 fill the slots' halves
#endif
template <int kMirror>
__device__ __forceinline__ void ring_fill(const uint32_t *C, uint32_t *ring, const uint32_t *tab,
                                          int base, int count, int lane) {
    const int h = HM_RING_PAIRS ? lane & 1 : lane >> 5;
    for (int k = HM_RING_PAIRS ? lane >> 1 : lane & 31; k < count; k += 32) {
        const int w = base + k;
        const uint32_t v = C[w] >> (16 * h);
        uint2 nb;
        nb.x = tab[v & 0xFFu];
        nb.y = tab[(v >> 8) & 0xFFu];
        ring_put<kMirror>(ring, w, h, nb);
    }
}

// Wait for bit i's record DMA (stage_rec) but not for the `young` sum stores the previous bit's
// tiles issued after it: gfx9 vector memory operations complete in order, loads and stores alike
// (the compiler itself waits with vmcnt(N) on a load that younger stores follow), so vmcnt(N) with
// N <= young guarantees the older DMA has landed.  young is a lower bound the tile loop counts
// (one store instruction per tile on the uniform full-tile branch).
#ifndef HM_REC_WAIT_YOUNG
#define HM_REC_WAIT_YOUNG 0 // (A/B knob, measured slower: r06 chain 463-472 us with vmcnt(0) against 472-476 us)
#endif
__device__ __forceinline__ void wait_record(int young) {
    if (!HM_REC_WAIT_YOUNG || young <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (young >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (young >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (young >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (young >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
}

// waves per block (<= kAddWavesPerBlock, which the host plan's LDS check assumes)
#ifndef HM_MFMA_WPB
#define HM_MFMA_WPB kAddWavesPerBlock
#endif
constexpr int kMfmaWpb = HM_MFMA_WPB;
static_assert(kMfmaWpb <= kAddWavesPerBlock, "host LDS plan");

// NC = 7: 4 waves per SIMD (HM_MFMA7_WPE: 108 VGPRs, no spills; 5 or 6 spill 18 / 28); NC = 13: 4 waves per SIMD (configs[1]'s 4096 waves
// fill the chip at that), 128 VGPRs;
// NC = 25: 3 waves per SIMD, 168 VGPRs (the 25 A fragments alone are 100; engine.h HM_MFMA25_WPE)
template <int NC>
__global__ void __launch_bounds__(64 * kMfmaWpb)
__attribute__((amdgpu_waves_per_eu(MfmaCfg<NC>::kWavesPerEU, MfmaCfg<NC>::kWavesPerEU)))
add_chain_mfma_kernel(AddArgs A) {
    kt_start(A.kt);
    using Cfg = MfmaCfg<NC>;
    constexpr int kRevWords = Cfg::kRevWords, kRsWords = Cfg::kRsWords, kRec = Cfg::kRecWords;
    extern __shared__ uint32_t lds[];
    __shared__ uint32_t stage[kMfmaWpb][2][kRec];
    uint32_t *tab = lds; // byte -> 8 nibbles, fp4 1.0 (0b0010) per set bit
    for (uint32_t k = threadIdx.x; k < 256; k += blockDim.x) {
        uint32_t v = 0u;
#pragma unroll
        for (int t = 0; t < 8; ++t) v |= ((k >> t) & 1u) << (4 * t + 1);
        tab[k] = v;
    }
    __syncthreads();
    const int wave = (int)rfl(threadIdx.x >> 6); // wave-uniform by construction
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (e >= A.n) { // whole wave exits together
        kt_finish(A.kt);
        return;
    }
    const int lane = lane_id();
    const uint32_t L = A.nbits;
    // LDS per wave: [halo][C: mf_cw][ring: kRingWords][RS: kRsWords]
    uint32_t *Ls = lds + 256 + (size_t)wave * A.chain_lds;
    uint32_t *C = Ls + Cfg::kHalo;
    uint32_t *ring = C + A.mf_cw;
    uint32_t *RS = ring + Cfg::kRingWords;
    const uint32_t *ws = A.ws + e * A.ws_stride;
    uint64_t *po = A.out.limbs + e * A.out.stride;
    uint32_t *dout = A.out.degree + e * L;
    // Bit i's workspace record, copied into stage[wave][i&1] by one LDS-DMA a bit ahead (its
    // latency hides behind the previous bit's tiles): [x_i: cntX][P_i: cntP][ab_i: cntAB][deg P_i]
    // [deg ab_i] (host plan: at most kRec words, one DMA per 64).  The DMA is asm: the compiler cannot tell the
    // dynamic LDS from stage and would wait for the DMA before the next LDS write; instead each
    // bit starts with one vmcnt(0), when the DMA and the previous bit's stores are a bit old.
    const uint32_t oP = A.cntX, oAB = oP + A.cntP, oD = oAB + A.cntAB;
    // record word u of bit i is workspace word base(u) + i * step(u) (words past the record
    // re-read deg P_i); lane l loads words l and (kRec = 128) 64 + l
    auto rec_word = [&](uint32_t u, uint32_t &base, uint32_t &step) {
        const uint32_t offD = L * (A.cntAB + A.cntP);
        if (u < oP) base = offD + 2 * L + u, step = A.cntX;
        else if (u < oAB) base = L * A.cntAB + (u - oP), step = A.cntP;
        else if (u < oD) base = u - oAB, step = A.cntAB;
        else if (u == oD + 1) base = offD, step = 1;
        else base = offD + L, step = 1;
    };
    uint32_t lbase, lstep, lbase2 = 0, lstep2 = 0;
    rec_word((uint32_t)lane, lbase, lstep);
    if constexpr (kRec > 64) rec_word(64u + (uint32_t)lane, lbase2, lstep2);
    const bool two = kRec > 64 && oD + 2 > 64; // wave-uniform
    const uint64_t wsu = ((uint64_t)rfl((uint32_t)((uintptr_t)ws >> 32)) << 32) |
                         rfl((uint32_t)(uintptr_t)ws); // wave-uniform: SGPR base of the DMA
    auto stage_rec = [&](uint32_t i) {
        const uint32_t voff = 4u * (lbase + i * lstep);
        const uint32_t m0 = (uint32_t)(uintptr_t)&stage[wave][i & 1][0]; // LDS byte offset
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1"
                     :
                     : "v"(voff), "s"(wsu), "s"(m0)
                     : "memory", "m0");
        if (two) {
            const uint32_t voff2 = 4u * (lbase2 + i * lstep2);
            asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %0, %1"
                         :
                         : "v"(voff2), "s"(wsu), "s"(m0 + 256u)
                         : "memory", "m0");
        }
    };
    stage_rec(0);

#ifdef HM_MFMA_PROFILE
    unsigned long long prof[4] = {0, 0, 0, 0};
#endif
    for (uint32_t k = lane; k < Cfg::kHalo + A.mf_cw; k += kWave) Ls[k] = 0u;
    for (int k = 4 * kRevWords + lane; k < kRsWords; k += kWave) RS[k] = 0u; // P below bit 0
    wsync();
    int nc = 0;    // carry words (0 = null carry, common.rs:39)
    int degc = -1; // the carry's degree
    int tw = -1;   // > 0: the previous bit's tiles stored sum words [cntX, min(tw, cap words))
    int young = 0; // store instructions issued after bit i's record DMA (a lower bound)
    uint32_t offo = 0;
    for (uint32_t i = 0; i < L; ++i) {
        HM_PT(tw0);
        wait_record(young); // bit i's record has landed
        young = 0;
        const uint32_t *rec = &stage[wave][i & 1][0];
        // s_i = x_i ^ carry_i (common.rs:43-47)
        HM_PT(t0);
        HM_PACC(3, tw0, t0);
        if (tw < 0) {
            store_sum_x(rec, (int)A.cntX, C, nc, po + offo, A.ob.b[i], dout + i, A.status);
        } else {
            // the tiles T >= 1 wrote s_i's words from 32 up (= carry words there); left: words
            // 0..31 (x_i ^ carry; stored here rather than by tile 0, whose stores would still be
            // in flight at this bit's vmcnt wait), zeros above the tiles, the degree
            const int capw = 2 * (int)cap_of(A.ob.b[i]);
            uint32_t *so = (uint32_t *)(po + offo);
            int ldeg = -1;
            if (lane < 32) { // C is valid up to tw >= 32 words; cntX < 32
                const uint32_t v = (lane < (int)A.cntX ? rec[lane] : 0u) ^ C[lane];
                if (lane < capw) so[lane] = v;
                // (a word past the capacity still counts: the degree check below flags it)
                if (v) ldeg = lane * 32 + 31 - (int)__builtin_clz(v);
            }
            for (int w = tw + lane; w < capw; w += kWave) so[w] = 0u;
            int deg = wave_max_i32(ldeg);
            if (nc > 32) deg = degc; // the carry's top word is above the words stored here
            if (lane == 0) {
                if (deg > (int)A.ob.b[i]) flag(A.status, HM_ERR_CAPACITY);
                dout[i] = (uint32_t)max(deg, 0);
            }
        }
        offo += cap_of(A.ob.b[i]);
        HM_PT(t1);
        HM_PACC(0, t0, t1);
        if (i + 1 == L) break;
        const int np = bitwords((int)rfl(rec[oD])), nab = bitwords((int)rfl(rec[oD + 1]));
        const uint32_t *abi = rec + oAB;
        wsync(); // the sum bit's reads of C precede the carry update
        if (np == 0 || nc == 0) {
            // P_i * carry_i = 0: carry_{i+1} = ab_i, stale words above it cleared
            const int n = max(nc, nab);
            for (int w = lane; w < n; w += kWave) C[w] = w < nab ? abi[w] : 0u;
            nc = nab;
            degc = (int)rfl(rec[oD + 1]) - 1; // carry_{i+1} = ab_i
            tw = -1;
            wsync();
            stage_rec(i + 1);
            continue;
        }
        // RS = nibble image of P_i bit-reversed over kRevWords words: nibble j = P[32*kRevWords-1-j]
        // (nibble words >= 4*kRevWords stay zero: P below bit 0).
        const uint32_t *pi = rec + oP;
        for (int k = lane; k < 4 * kRevWords; k += kWave) {
            const int q = kRevWords - 1 - (k >> 2); // the P word behind nibble word k
            const uint32_t rev = __builtin_bitreverse32(q < np ? pi[q] : 0u);
            RS[k] = tab[(rev >> (8 * (k & 3))) & 0xFFu];
        }
        wsync();
        // bit i+1's record goes to the other buffer (this one is read until the last tile)
        stage_rec(i + 1);
        // All kMfmaChunks chunks run whatever np is: chunks past floor(np/2) have all-zero A (their
        // P indices are negative), so the chunk loop has no branches and its reads can be issued
        // ahead of the MFMAs.
        const int D = np;
        const int lane = lane_opaque(), col = lane & 31, h = lane >> 5;
        // A fragments: lane (row m = col, half h), chunk c holds P[s - e], s = 32(D-2c-h) + m,
        // i.e. RS nibbles j0 .. j0+31 with j0 = 32*kRevWords - 1 - s: five words, four funnels
        // j0 of chunk c = jb + 64c (jb >= 64 since D <= 2 NC - 1 < kRevWords - 2): one base word per
        // lane, chunk c at +8c words (immediate offsets), one shift for all chunks
        v8i Af[NC];
        const int jb = 32 * (kRevWords - D + h) - 1 - row_bit(col); // (row-permuted tiles)
        const uint32_t *rw0 = RS + (jb >> 3);
        const uint32_t sh = 4u * (uint32_t)(jb & 7);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const uint32_t *rw = rw0 + 8 * c;
            const uint32_t w0 = rw[0], w1 = rw[1], w2 = rw[2], w3 = rw[3], w4 = rw[4];
            Af[c] = (v8i){(int)funnel(w1, w0, sh), (int)funnel(w2, w1, sh), (int)funnel(w3, w2, sh),
                          (int)funnel(w4, w3, sh), 0, 0, 0, 0};
        }
        HM_PT(t2);
        HM_PACC(1, t1, t2);
        const int nout = max(nc + np, nab);
        const int tiles = (nout + 31) >> 5;
        // s_{i+1}'s words from 32 up are carry_{i+1}'s (x_{i+1} < 32 words): tiles T >= 1 store
        // them (u32 words of the output limbs) below the output's capacity; bit i+1 does the rest
        uint32_t *son = (uint32_t *)(po + offo);
        const int capn = 2 * (int)cap_of(A.ob.b[i + 1]);
        const int wlo = 32;
        // the top tile's whole window: words 32(tiles-1) - D .. + 32 + 2 NC
        ring_fill<Cfg::kMirror>(C, ring, tab, 32 * (tiles - 1) - D, 32 + 2 * NC, lane);
        int ldeg = -1;
        // deg(P_i * carry_i) = deg P_i + deg carry_i exactly (GF(2)[X] has no zero divisors), so
        // when that is above deg ab_i it is carry_{i+1}'s degree; only otherwise (a short carry:
        // ab_i may reach the top word) do the tiles track the highest set bit (wave-uniform)
        const int alg = (int)rfl(rec[oD]) - 1 + degc;
        const bool track = alg <= (int)rfl(rec[oD + 1]) - 1;
        // The accumulators start at 2^23 once per bit and keep accumulating tile after tile
        // (2^23 + every count stays below 2^24, exact): a tile's parities are bit 0 of its
        // accumulators XOR bit 0 before the tile.
        v16f acc;
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = 8388608.0f;
        uint32_t gprev = 0u;
        // window words 32T + col - D + h + 2c: one base slot, chunk c at +2c slots (32 B)
        auto rbase = [&](int T) {
            return (const uint4 *)&ring[((32 * T + col - D + h) & (kMfmaRingSlots - 1)) * 4];
        };
        wsync(); // the first tile's ring images are written
        constexpr int kPrefetch = kPrefetchOf<NC>;
        uint4 pf[kPrefetch];
#pragma unroll
        for (int c = 0; c < kPrefetch; ++c) pf[c] = rbase(tiles - 1)[2 * c];
        // (NC = 13: the window base carries over, this tile's is the previous tile's next)
        const uint4 *rb = rbase(tiles - 1);
        for (int T = tiles - 1; T >= 0; --T) {
            wsync(); // ring images of this tile's window are written
            if constexpr (NC > 16) rb = rbase(T); // (NC = 25: carried over, it spilled)
            const uint4 *rbn = rbase(T - 1); // (T = 0: rbn reads are not used)
            // the next tile's 32 new window words (old carry: below 32T; their ring slots are not
            // in this tile's window), one per lane pair, staged between this tile's MFMAs
            // (tile 0 stages words -32-D+col too: its ring slots are outside tile 0's window, C
            // reads below the halo stay inside the block's LDS, and the next bit refills its window
            // before reading it, so no per-tile test is needed)
            // (lane pair 2j, 2j + 1: word j's two halves, contiguous stores as in ring_fill)
            const int fh = HM_RING_PAIRS ? lane & 1 : h;
            const int fw = 32 * (T - 1) - D + (HM_RING_PAIRS ? lane >> 1 : col);
            uint32_t fv;
            uint2 fn;
            // ab_i's word of this tile's output, read before the MFMAs (ab_i < 64 words: host plan;
            // a wave-uniform branch: tiles 0 and 1 at most)
            const int W = 32 * T + col;
            uint32_t abw = 0u;
            if (32 * T < nab) {
                asm volatile("" ::: "memory");
                abw = W < nab ? abi[W] : 0u;
            }
            __builtin_amdgcn_s_setprio(1); // the MFMA phase keeps the pipe
            acc = tile_mfma<NC>(Af, rb, rbn, pf, acc, [&](int stage) {
                // (the empty asm keep each stage's arithmetic from being hoisted into an earlier
                // stage, where it would wait for the read of the stage before)
                if (stage == 0) fv = C[fw];
                else if (stage == 1) {
                    asm volatile("" : "+v"(fv));
                    fv >>= 16 * fh;
                    fn.x = tab[fv & 0xFFu], fn.y = tab[(fv >> 8) & 0xFFu];
                } else {
                    asm volatile("" : "+v"(fn.x), "+v"(fn.y));
                    ring_put<Cfg::kMirror>(ring, fw, fh, fn);
                }
            });
            __builtin_amdgcn_s_setprio(0);
            // accumulator j of lane half h is output bit j + 16h (row-permuted tiles): its parity
            // is bit 16 + j of tnow; XOR the bits of the accumulators before this tile
            const uint32_t tnow = acc_parities_hi16(acc);
            const uint32_t t = (tnow ^ gprev) >> (16 - 16 * h);
            // the two lane halves' bits meet by one v_permlane32_swap (VALU; no LDS round trip):
            // lanes 0-31 keep their t in the first result and receive lanes 32-63's t in the
            // second; only lanes 0-31 use the word (stores, degree), so the second operand is the
            // dead previous gprev rather than a copy of t
            const auto sw = __builtin_amdgcn_permlane32_swap(t, gprev, false, false);
            gprev = tnow;
            const uint32_t word = sw[0] | sw[1];
            const uint32_t v = word ^ abw;
            // (wave-uniform first: a tile wholly inside [wlo, capn) needs no per-lane test; it
            // issues exactly one store instruction, counted for the next bit's record wait)
            const bool full = T >= 1 && 32 * T + 32 <= capn;
            young += full ? 1 : 0;
            if (h == 0) {
                C[W] = v;
                if (full) {
                    asm volatile("" ::: "memory");
                    son[W] = v;
                } else if (W >= wlo && W < capn) son[W] = v;
            }
            // a wave-uniform branch (the empty volatile asm keeps the compiler from if-converting
            // it into per-lane selects that run on every tile)
            if (track) {
                asm volatile("" ::: "memory");
                int Wq = W; // (opaque: its bit position is not strength-reduced into every tile)
                asm volatile("" : "+v"(Wq));
                if (h == 0 && v) ldeg = max(ldeg, Wq * 32 + 31 - (int)__builtin_clz(v));
            }
            rb = rbn;
        }
        const int deg = track ? wave_max_i32(ldeg) : alg;
        nc = deg >= 0 ? (deg >> 5) + 1 : 0;
        degc = deg;
        tw = 32 * tiles;
        wsync();
        HM_PT(t3);
        HM_PACC(2, t2, t3);
    }
#ifdef HM_MFMA_PROFILE
    if (lane == 0)
        for (int k = 0; k < 4; ++k) g_mfma_prof[e * 4 + k] = prof[k];
#endif
    kt_finish(A.kt);
}

int launch_add_chain_mfma(const AddArgs &a, void *stream) {
    const int wpb = kMfmaWpb;
    const uint64_t blocks = (a.n + wpb - 1) / wpb;
    const size_t lds = (256 + (size_t)a.chain_lds * wpb) * 4;
#define HM_LAUNCH_CHAIN(NCV)                                                                      \
    hipLaunchKernelGGL((add_chain_mfma_kernel<NCV>), dim3((unsigned)blocks), dim3(64 * wpb), lds,  \
                       (hipStream_t)stream, a)
    if (a.mfma == MfmaCfg<7>::kChunks) HM_LAUNCH_CHAIN(7);
    else if (a.mfma == MfmaCfg<13>::kChunks) HM_LAUNCH_CHAIN(13);
    else if (a.mfma == MfmaCfg<25>::kChunks) HM_LAUNCH_CHAIN(25);
    else return -1;
#undef HM_LAUNCH_CHAIN
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace hm
