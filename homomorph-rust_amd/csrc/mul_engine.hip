// mul_engine.hip — gfx950 kernels of the column-parallel carry-save multiplier
// (mul_unsigned_internal / mul_signed_internal, src/impls/numbers/common.rs:66-155).
//
// The reference walks column i's items x_0..x_{n-1} (partial products a_j b_{i-j}, then the
// previous column's carries) sequentially:  carries.push(result * x_t); result ^= x_t.  The
// carry pushed before item t is p_t * x_t with p_t = x_0 ^ .. ^ x_{t-1} (the running result), so
// once the prefixes are materialised every carry of a column is an independent product and the
// whole batch's column runs as three wide launches:
//   mul_pp_kernel     partial products a_j * b_{i-j} (fresh x fresh, per-lane holey multiplies)
//   mul_scan_kernel   prefixes p_1..p_{n-1} and the output bit p_n (XOR streams over 256-word
//                     chunks, lanes over words, one uint4 per lane)
//   mul_prod_kernel   carries p_t * x_t, one wavefront per (value, 64*W-word output tile):
//                     Horner over the uniform operand's bits with scalar decisions (gf2_wave.h)
// The products are exact (GF(2)[X] has no zero divisors: deg = deg u + deg v), the prefixes'
// degrees come from the words, so every polynomial is bit-identical to the reference's.
#include "dev_common.h"

namespace hm {

__device__ __forceinline__ uint32_t *slot_ptr(const MulBase &B, uint32_t s, uint64_t e) {
    return B.arena + e * B.astride + B.slots[s].off;
}

// one ciphertext bit (u64 limbs + exact degree) -> arena slot (u32 words, zero-filled to the
// slot's capacity), validated as load_bit does; writes deg1.
__device__ __forceinline__ void stage_one(const MulBase &B, const uint64_t *src, uint32_t deg, uint32_t bound,
                          uint32_t slot, uint64_t e) {
    const int lane = lane_id();
    uint32_t *dst = slot_ptr(B, slot, e);
    const uint32_t words = B.slots[slot].words;
    const uint32_t cap = bound / 64 + 1;
    bool bad = deg > bound;
    const uint32_t nl = bad ? 0u : deg / 64 + 1, tb = deg % 64;
    uint32_t w0 = 0u;
    for (uint32_t g = lane; 2 * g < words; g += kWave) {
        uint64_t v = (g < cap) ? src[g] : 0ull;
        if (g >= nl) {
            bad |= v != 0;
            v = 0;
        } else if (g == nl - 1) {
            const uint64_t keep = (~0ull) >> (63 - tb);
            bad |= (v & ~keep) != 0;
            v &= keep;
            if (deg > 0 && !((v >> tb) & 1ull)) bad = true;
        }
        if (g == 0) w0 = (uint32_t)v;
        dst[2 * g] = (uint32_t)v;
        if (2 * g + 1 < words) dst[2 * g + 1] = (uint32_t)(v >> 32);
    }
    for (uint32_t g = (words + 1) / 2 + lane; g < cap; g += kWave) bad |= src[g] != 0;
    if (__any(bad) && lane == 0) flag(B.status, HM_ERR_BAD_INPUT);
    w0 = (uint32_t)__shfl((int)w0, 0, 64);
    if (lane == 0) {
        const bool null = deg == 0 && !(w0 & 1u);
        B.deg1[(uint64_t)slot * B.nv + e] = (bad || null) ? 0u : deg + 1;
    }
}

// one wave per (value, input bit): a_j -> slot j, b_j -> slot K + j
__global__ void __launch_bounds__(256) mul_stage_kernel(MulStageArgs S) {
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + rfl(threadIdx.x >> 6);
    const uint64_t e = g / (2 * S.K);
    const uint32_t t = (uint32_t)(g % (2 * S.K));
    if (e >= S.B.nv) return;
    const bool isb = t >= S.K;
    const uint32_t j = isb ? t - S.K : t;
    const BatchArg &A = isb ? S.b : S.a;
    const Bounds &bd = isb ? S.bb : S.ab;
    uint32_t off = 0;
    for (uint32_t q = 0; q < j; ++q) off += cap_of(bd.b[q]);
    const uint64_t ge = S.B.e0 + e;
    stage_one(S.B, A.limbs + ge * A.stride + off, rfl(A.degree[ge * A.dstride + j]), bd.b[j], t, e);
}

// The same staging with one wave per VALUE: lanes over (input bit, limb pair of its slot), so a
// u8 multiply's 16 bits take two passes of one wave instead of 16 one-pass waves (the per-bit
// form is latency-bound: 110 us per 16384 u8 pairs).  Per-bit tables in the wave's LDS: slot
// offset / words, limb offset / capacity in the value, degree, and the OR of its bad flags and its
// word 0 (ds_or) -- the bounds come in through arg_to_lds (never indexed per lane).
// LDS per wave: kStageTab * 2K words.
constexpr uint32_t kStageTab = 8;
__global__ void __launch_bounds__(256) mul_stage_value_kernel(MulStageArgs S) {
    extern __shared__ uint32_t lds[];
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    const uint32_t lane = (uint32_t)lane_id(), nb = 2 * S.K;
    uint32_t *tab = lds + (size_t)wave * kStageTab * nb;
    uint32_t *bnd = tab, *loff = tab + nb, *soff = tab + 2 * nb, *sw = tab + 3 * nb;
    uint32_t *dg = tab + 4 * nb, *badw = tab + 5 * nb, *w0 = tab + 6 * nb;
    // (bounds 16-byte aligned for arg_to_lds: nb words each, written up to a multiple of 16)
    __shared__ __attribute__((aligned(16))) uint32_t sb[4][2 * HM_MAX_BITS];
    arg_to_lds(S.ab.b, S.K, sb[wave]);
    arg_to_lds(S.bb.b, S.K, sb[wave] + HM_MAX_BITS);
    wsync();
    if (e >= S.B.nv) return; // whole wave exits together (after its LDS writes: no barrier below)
    const uint64_t ge = S.B.e0 + e;
    for (uint32_t t = lane; t < nb; t += kWave) {
        const bool isb = t >= S.K;
        const uint32_t j = isb ? t - S.K : t;
        const uint32_t *bd = sb[wave] + (isb ? HM_MAX_BITS : 0);
        uint32_t off = 0;
        for (uint32_t q = 0; q < j; ++q) off += cap_of(bd[q]);
        bnd[t] = bd[j], loff[t] = off;
        const MulSlot sl = S.B.slots[t];
        soff[t] = sl.off, sw[t] = sl.words;
        dg[t] = isb ? S.b.degree[ge * S.b.dstride + j] : S.a.degree[ge * S.a.dstride + j];
        badw[t] = 0u, w0[t] = 0u;
    }
    wsync();
    uint32_t *dst0 = S.B.arena + e * S.B.astride;
    // lanes over (bit t, limb g): the slot's (words + 1) / 2 limb pairs, and every limb up to the
    // bit's capacity (limbs past the slot must be zero, as stage_one checks)
    uint32_t maxp = 0;
    for (uint32_t t = 0; t < nb; ++t) maxp = max(maxp, max((sw[t] + 1) / 2, cap_of(bnd[t])));
    for (uint32_t f = lane; f < nb * maxp; f += kWave) {
        const uint32_t t = f / maxp, g = f % maxp;
        const uint32_t bound = bnd[t], deg = dg[t], words = sw[t], cap = cap_of(bound);
        const bool isb = t >= S.K;
        const uint64_t *src = (isb ? S.b.limbs : S.a.limbs) + ge * (isb ? S.b.stride : S.a.stride) + loff[t];
        bool bad = deg > bound;
        const uint32_t nl = bad ? 0u : deg / 64 + 1, tb = deg % 64;
        uint64_t v = g < cap ? src[g] : 0ull;
        if (2 * g < words) {
            if (g >= nl) {
                bad |= v != 0;
                v = 0;
            } else if (g == nl - 1) {
                const uint64_t keep = (~0ull) >> (63 - tb);
                bad |= (v & ~keep) != 0;
                v &= keep;
                if (deg > 0 && !((v >> tb) & 1ull)) bad = true;
            }
            uint32_t *dst = dst0 + soff[t];
            dst[2 * g] = (uint32_t)v;
            if (2 * g + 1 < words) dst[2 * g + 1] = (uint32_t)(v >> 32);
            if (g == 0) w0[t] = (uint32_t)v; // (one lane per bit)
        } else if (g < cap) {
            bad |= v != 0; // a limb past the slot's capacity must be zero
        }
        if (bad) atomicOr(&badw[t], 1u);
    }
    wsync();
    bool anybad = false;
    for (uint32_t t = lane; t < nb; t += kWave) {
        const bool bad = badw[t] != 0 || dg[t] > bnd[t];
        anybad |= bad;
        const bool null = dg[t] == 0 && !(w0[t] & 1u);
        S.B.deg1[(uint64_t)t * S.B.nv + e] = (bad || null) ? 0u : dg[t] + 1;
    }
    if (__any(anybad) && lane == 0) flag(S.B.status, HM_ERR_BAD_INPUT);
}

#ifndef HM_STAGE_VALUE
#define HM_STAGE_VALUE 1 // (A/B knob) 0: one wave per (value, input bit)
#endif
int launch_mul_stage(const MulStageArgs &S, void *stream) {
    if (HM_STAGE_VALUE && 2 * S.K <= 64) {
        if (!S.B.nv) return 0;
        hipLaunchKernelGGL(mul_stage_value_kernel, dim3((unsigned)((S.B.nv + 3) / 4)), dim3(256),
                           (size_t)kStageTab * 2 * S.K * 4 * 4, (hipStream_t)stream, S);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    const uint64_t waves = S.B.nv * 2 * S.K;
    if (!waves) return 0;
    hipLaunchKernelGGL(mul_stage_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, S);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// exact top bit of a word range spread over the wave (lane-local top word index `tw`, -1 = none)
__device__ __forceinline__ int wave_topbit(int tw, uint32_t v) {
    const int lb = tw >= 0 ? tw * 32 + 31 - __builtin_clz(v) : -1;
    return wave_max_i32(lb);
}

// one wave per (value, partial product): out = a * b (+1), lanes over output words
__global__ void __launch_bounds__(256) mul_pp_kernel(MulPPArgs P) {
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + rfl(threadIdx.x >> 6);
    const uint64_t e = g / P.ntasks;
    const uint32_t k = (uint32_t)(g % P.ntasks);
    if (e >= P.B.nv) return;
    const MulPPTask T = P.tasks[k];
    const uint32_t da = P.B.deg1[(uint64_t)T.a * P.B.nv + e], db = P.B.deg1[(uint64_t)T.b * P.B.nv + e];
    const int na = bitwords((int)rfl(da)), nb = bitwords((int)rfl(db));
    const uint32_t *A = slot_ptr(P.B, T.a, e), *Bp = slot_ptr(P.B, T.b, e);
    uint32_t *O = slot_ptr(P.B, T.out, e);
    const uint32_t words = P.B.slots[T.out].words;
    int tw = -1;
    uint32_t tv = 0;
    for (uint32_t m = lane_id(); m < words; m += kWave) {
        uint32_t w = (na && nb) ? clmul_word(A, na, Bp, nb, (int)m) : 0u;
        if (m == 0 && T.flip) w ^= 1u;
        O[m] = w;
        if (w) tw = (int)m, tv = w;
    }
    const int top = wave_topbit(tw, tv);
    if (lane_id() == 0) P.B.deg1[(uint64_t)T.out * P.B.nv + e] = (uint32_t)(top + 1);
}

// Partial products by rows (engine.h MulPPVArgs): one wave per value.  LDS per wave:
// [IN: nin x inw words][deg1 of the inputs: nin][OUT: ntasks x outw words].  Row (t, q) XORs word
// q of a_j times b_k into OUT_t from word q up (clmul_row_xor: one 32x32 product per step as 16
// v_mad_u64_u32 of holey operands, dev_common.h); the products are exact, so the words equal the
// MFMA form's (mul_ppg_kernel) and the reference's (polynomial.rs:252-310).
__global__ void __launch_bounds__(256) mul_ppv_kernel(MulPPVArgs P) {
    extern __shared__ uint32_t lds[];
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (e >= P.B.nv) return; // whole wave exits together
    const uint32_t lane = (uint32_t)lane_id();
    uint32_t *IN = lds + (size_t)wave * P.wave_words, *DIN = IN + P.nin * P.inw;
    uint32_t *OUT = DIN + P.nin;
    const uint32_t *arena = P.B.arena + e * P.B.astride;
    // inputs: every slot's words up to inw (zero past its capacity; slots are zero above their
    // degree), and their degrees
    for (uint32_t f = lane; f < P.nin * P.inw; f += kWave) {
        const uint32_t s = f / P.inw, w = f % P.inw;
        const MulSlot sl = P.B.slots[s];
        IN[f] = w < sl.words ? arena[sl.off + w] : 0u;
    }
    for (uint32_t s = lane; s < P.nin; s += kWave) DIN[s] = P.B.deg1[(uint64_t)s * P.B.nv + e];
    for (uint32_t f = lane; f < P.ntasks * P.outw; f += kWave) OUT[f] = 0u;
    wsync();
    // rows: lanes over (task t, word q of its a_j)
    for (uint32_t f = lane; f < P.ntasks * P.qw; f += kWave) {
        const uint32_t t = f / P.qw, q = f % P.qw;
        const MulPPTask T = P.tasks[t];
        const int nu = bitwords((int)DIN[T.a]), nv = bitwords((int)DIN[T.b]);
        if ((int)q < nu && nv)
            clmul_row_xor(IN[T.a * P.inw + q], IN + T.b * P.inw, nv, OUT + t * P.outw + q);
    }
    wsync();
    uint32_t *aw = P.B.arena + e * P.B.astride;
    // lanes over (task, word): every output slot's words (outw >= its capacity), then the degrees
    for (uint32_t f = lane; f < P.ntasks * P.outw; f += kWave) {
        const uint32_t t = f / P.outw, w = f % P.outw;
        const MulSlot so = P.B.slots[P.tasks[t].out];
        if (w < so.words) aw[so.off + w] = OUT[f];
    }
    for (uint32_t t = lane; t < P.ntasks; t += kWave) {
        const MulPPTask T = P.tasks[t];
        const uint32_t du = DIN[T.a], dv = DIN[T.b];
        P.B.deg1[(uint64_t)T.out * P.B.nv + e] = (du && dv) ? du + dv - 1 : 0u;
    }
}

int launch_mul_ppv(const MulPPVArgs &P, void *stream) {
    if (!P.B.nv || !P.ntasks) return 0;
    const uint64_t blocks = (P.B.nv + 3) / 4;
    hipLaunchKernelGGL(mul_ppv_kernel, dim3((unsigned)blocks), dim3(256), (size_t)P.wave_words * 4 * 4,
                       (hipStream_t)stream, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// A column's small carry products by rows (engine.h MulRowArgs): one wave per value.  LDS per
// wave: per task [u: uw][v: vw][out: ow][deg u, deg v]; the products exact (= mul_mfma_kernel's).
__global__ void __launch_bounds__(256) mul_rows_kernel(MulRowArgs P) {
    extern __shared__ uint32_t lds[];
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (e >= P.B.nv) return; // whole wave exits together
    const uint32_t lane = (uint32_t)lane_id();
    const uint32_t tw = P.uw + P.vw + P.ow + 2; // LDS words per task
    uint32_t *W = lds + (size_t)wave * P.wave_words;
    uint32_t *R = W + P.ntasks * tw; // per task: uoff voff ooff nout words oslot (6 words)
    uint32_t *aw = P.B.arena + e * P.B.astride;
    // the host-resolved records (one load), then the operands' degrees (one dependent load)
    for (uint32_t t = lane; t < P.ntasks; t += kWave) {
        const MulSpanRec r = P.recs[t];
        uint32_t *Rt = R + 6 * t;
        Rt[0] = r.uoff, Rt[1] = r.voff, Rt[2] = r.ooff, Rt[3] = r.nout, Rt[4] = r.base, Rt[5] = r.oslot;
        W[t * tw + tw - 2] = P.B.deg1[(uint64_t)r.uslot * P.B.nv + e];
        W[t * tw + tw - 1] = P.B.deg1[(uint64_t)r.vslot * P.B.nv + e];
    }
    wsync();
    // operands (zero past their slot capacity; slots are zero above their degree) and zeroed
    // products: lanes over (task, word of the task's block)
    for (uint32_t f = lane; f < P.ntasks * tw; f += kWave) {
        const uint32_t t = f / tw, w = f % tw;
        if (w >= tw - 2) continue;
        const uint32_t *Rt = R + 6 * t;
        const uint32_t uw = Rt[4] & 0xFFFFu, vw = Rt[4] >> 16;
        uint32_t v = 0u;
        if (w < P.uw) v = w < uw ? aw[Rt[0] + w] : 0u;
        else if (w < P.uw + P.vw) v = w - P.uw < vw ? aw[Rt[1] + w - P.uw] : 0u;
        W[f] = v;
    }
    wsync();
    for (uint32_t f = lane; f < P.ntasks * P.qw; f += kWave) {
        const uint32_t t = f / P.qw, q = f % P.qw;
        uint32_t *Tw = W + t * tw;
        const int nu = bitwords((int)Tw[tw - 2]), nv = bitwords((int)Tw[tw - 1]);
        if ((int)q < nu && nv) clmul_row_xor(Tw[q], Tw + P.uw, nv, Tw + P.uw + P.vw + q);
    }
    wsync();
    for (uint32_t f = lane; f < P.ntasks * P.ow; f += kWave) {
        const uint32_t t = f / P.ow, w = f % P.ow;
        const uint32_t *Rt = R + 6 * t;
        if (w < Rt[3]) aw[Rt[2] + w] = W[t * tw + P.uw + P.vw + w];
    }
    for (uint32_t t = lane; t < P.ntasks; t += kWave) {
        const uint32_t du = W[t * tw + tw - 2], dv = W[t * tw + tw - 1];
        P.B.deg1[(uint64_t)R[6 * t + 5] * P.B.nv + e] = (du && dv) ? du + dv - 1 : 0u;
    }
}

int launch_mul_rows(const MulRowArgs &P, void *stream) {
    if (!P.B.nv || !P.ntasks) return 0;
    const uint64_t blocks = (P.B.nv + 3) / 4;
    hipLaunchKernelGGL(mul_rows_kernel, dim3((unsigned)blocks), dim3(256), (size_t)P.wave_words * 4 * 4,
                       (hipStream_t)stream, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_mul_pp(const MulPPArgs &P, void *stream) {
    const uint64_t waves = P.B.nv * P.ntasks;
    if (!waves) return 0;
    hipLaunchKernelGGL(mul_pp_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// one wave per (value, 256-word chunk): acc ^= x_t chunk, store p_{t+1} chunk, track degrees.
// Slots are zero above their degree and capacities are multiples of 4 words, so every item and
// prefix is read / written as whole uint4s up to its capacity.
//   - The column's slot records (item t, and the slot that receives p_{t+1} or the output bit)
//     are copied into LDS once per block: read per item through items[] -> slots[], they were
//     two dependent scalar loads each, twice per item, and the kernel waited ~90 % of its cycles.
//   - Items live in the pp / carry regions and prefixes in their own region (mul_host.cpp
//     build_plan), so no store aliases a later item: kScanBatch item loads are issued together,
//     ahead of the XORs and stores.
constexpr uint32_t kScanBatch = 8;

__global__ void __launch_bounds__(256) mul_scan_kernel(MulScanArgs S) {
    extern __shared__ uint32_t lds[]; // [item off][item words][dest off][dest words][dest slot] x nitems
    uint32_t *ioff = lds, *iwords = lds + S.nitems, *doff = lds + 2 * S.nitems, *dwords = lds + 3 * S.nitems;
    uint32_t *dslots = lds + 4 * S.nitems;
    for (uint32_t t = threadIdx.x; t < S.nitems; t += blockDim.x) {
        const MulSlot si = S.B.slots[S.items[t]];
        ioff[t] = si.off, iwords[t] = si.words;
        if (t + 1 < S.nitems) {
            const MulSlot sp = S.B.slots[S.prefix[t]];
            doff[t] = sp.off, dwords[t] = sp.words, dslots[t] = S.prefix[t];
        } else {
            doff[t] = 0u, dwords[t] = 0u, dslots[t] = S.res; // the output bit
        }
    }
    __syncthreads();
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + rfl(threadIdx.x >> 6);
    const uint64_t e = g / S.chunks;
    const uint32_t c0 = (uint32_t)(g % S.chunks) * 256u;
    if (e >= S.B.nv) return;
    const int lane = lane_id();
    const uint32_t w = c0 + 4u * (uint32_t)lane;
    uint32_t *const arena = S.B.arena + e * S.B.astride;
    uint4 acc = make_uint4(0u, 0u, 0u, 0u);
    for (uint32_t t0 = 0; t0 < S.nitems; t0 += kScanBatch) {
        const uint32_t nb = min(kScanBatch, S.nitems - t0);
        uint4 v[kScanBatch];
#pragma unroll
        for (uint32_t k = 0; k < kScanBatch; ++k) {
            v[k] = make_uint4(0u, 0u, 0u, 0u);
            if (k < nb && w < iwords[t0 + k]) v[k] = *(const uint4 *)(arena + ioff[t0 + k] + w);
        }
#pragma unroll
        for (uint32_t k = 0; k < kScanBatch; ++k) {
            if (k >= nb) break;
            const uint32_t t = t0 + k;
            acc.x ^= v[k].x, acc.y ^= v[k].y, acc.z ^= v[k].z, acc.w ^= v[k].w;
            int tw = -1;
            uint32_t tv = 0;
            if (acc.x) tw = (int)w, tv = acc.x;
            if (acc.y) tw = (int)w + 1, tv = acc.y;
            if (acc.z) tw = (int)w + 2, tv = acc.z;
            if (acc.w) tw = (int)w + 3, tv = acc.w;
            if (t + 1 < S.nitems) {
                if (w < dwords[t]) *(uint4 *)(arena + doff[t] + w) = acc;
            } else {
                // the output bit: u32 words into the u64 limbs (little-endian), zeros up to capacity
                uint32_t *o = (uint32_t *)(S.out.limbs + (S.B.e0 + e) * S.out.stride + S.out_off);
                const uint32_t ow = 2 * S.out_cap;
                if (w < ow) *(uint2 *)(o + w) = make_uint2(acc.x, acc.y);
                if (w + 2 < ow) *(uint2 *)(o + w + 2) = make_uint2(acc.z, acc.w);
            }
            // degree + 1 of this prefix: the chunk's top bit, max over chunks
            const uint64_t m = __ballot(tw >= 0);
            if (m) {
                const uint32_t dslot = dslots[t];
                const int hl = 63 - __builtin_clzll(m);
                if (lane == hl) atomicMax(&S.B.deg1[(uint64_t)dslot * S.B.nv + e],
                                          (uint32_t)(tw * 32 + 32 - __builtin_clz(tv)));
            }
        }
    }
}

int launch_mul_scan(const MulScanArgs &S, void *stream) {
    const uint64_t waves = S.B.nv * S.chunks;
    if (!waves || !S.nitems) return 0;
    if ((size_t)S.nitems * 20 > 64 * 1024) return -1; // slot records staged in LDS
    hipLaunchKernelGGL(mul_scan_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256),
                       (size_t)S.nitems * 20, (hipStream_t)stream, S);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// One wave per (value, tile): output words [base, base + 64 W) of u * v.  The operand with fewer
// words is the uniform one (its bits become scalar decisions); QC words of it per Horner pass.
constexpr int kMulQC = 10;

template <int W>
__global__ void __launch_bounds__(256) mul_prod_kernel(MulProdArgs P) {
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + rfl(threadIdx.x >> 6);
    const uint64_t e = g / P.ntiles;
    const uint32_t k = (uint32_t)(g % P.ntiles);
    if (e >= P.B.nv) return;
    const MulTile tl = P.tiles[k];
    const MulProdTask T = P.tasks[tl.task];
    const uint32_t du = rfl(P.B.deg1[(uint64_t)T.u * P.B.nv + e]);
    const uint32_t dv = rfl(P.B.deg1[(uint64_t)T.v * P.B.nv + e]);
    uint32_t *O = slot_ptr(P.B, T.out, e);
    const int nout = (int)P.B.slots[T.out].words;
    const int base = (int)rfl(tl.base);
    if (du == 0 || dv == 0) { // a null operand: the carry is null (zero-filled slot)
        for (int j = 0; j < W; ++j) {
            const int w = base + lane_id() * W + j;
            if (w < nout) O[w] = 0u;
        }
    } else {
        const uint32_t *U = slot_ptr(P.B, T.u, e), *V = slot_ptr(P.B, T.v, e);
        const int nu = bitwords((int)du), nv = bitwords((int)dv);
        if (base == 0)
            mul_tile<W, kMulQC, false, pair_mode<W>(), false>(U, nu, V, nv, nullptr, 0, O, nout, 0);
        else
            mul_tile<W, kMulQC, true, pair_mode<W>(), false>(U, nu, V, nv, nullptr, 0, O, nout, base);
    }
    if (base == 0 && lane_id() == 0)
        P.B.deg1[(uint64_t)T.out * P.B.nv + e] = (du && dv) ? du + dv - 1 : 0u;
}

int launch_mul_prod(const MulProdArgs &P, uint32_t w, void *stream) {
    const uint64_t waves = P.B.nv * P.ntiles;
    if (!waves) return 0;
    const dim3 grid((unsigned)((waves + 3) / 4)), block(256);
    switch (w) {
    case 1: hipLaunchKernelGGL(mul_prod_kernel<1>, grid, block, 0, (hipStream_t)stream, P); break;
    case 2: hipLaunchKernelGGL(mul_prod_kernel<2>, grid, block, 0, (hipStream_t)stream, P); break;
    case 4: hipLaunchKernelGGL(mul_prod_kernel<4>, grid, block, 0, (hipStream_t)stream, P); break;
    case 8: hipLaunchKernelGGL(mul_prod_kernel<8>, grid, block, 0, (hipStream_t)stream, P); break;
    case 12: hipLaunchKernelGGL(mul_prod_kernel<12>, grid, block, 0, (hipStream_t)stream, P); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------------------------
// Karatsuba over arena views (mul_host.cpp "Karatsuba").  All offsets and h are multiples of 4
// words, so every access is a whole uint4; one wave per (value, task, 256-word chunk).

// dst[0:h) = src[0:h) ^ src[h:2h), words at or past `valid` of src read as zero
__global__ void __launch_bounds__(256) ka_sum_kernel(KaSumArgs A) {
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + rfl(threadIdx.x >> 6);
    const uint32_t chunks = (A.h + 255) / 256;
    const uint64_t per_value = (uint64_t)A.nt * chunks;
    const uint64_t e = g / per_value;
    if (e >= A.B.nv) return;
    const uint32_t r = (uint32_t)(g % per_value);
    const KaSum t = A.t[r / chunks];
    const uint32_t w = (r % chunks) * 256 + 4u * (uint32_t)lane_id();
    if (w >= A.h) return;
    const uint32_t *base = A.B.arena + e * A.B.astride;
    uint4 lo = make_uint4(0u, 0u, 0u, 0u), hi = lo;
    if (w < t.valid) lo = *(const uint4 *)(base + t.src + w);
    if (A.h + w < t.valid) hi = *(const uint4 *)(base + t.src + A.h + w);
    *(uint4 *)(A.B.arena + e * A.B.astride + t.dst + w) =
        make_uint4(lo.x ^ hi.x, lo.y ^ hi.y, lo.z ^ hi.z, lo.w ^ hi.w);
}

int launch_ka_sum(const KaSumArgs &A, void *stream) {
    const uint64_t waves = A.B.nv * A.nt * ((A.h + 255) / 256);
    if (!waves) return 0;
    hipLaunchKernelGGL(ka_sum_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, A);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// leaf products over views: one wave per (value, 64*W-word output tile), as mul_prod_kernel
template <int W>
__global__ void __launch_bounds__(256) mul_vprod_kernel(MulVProdArgs P) {
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + rfl(threadIdx.x >> 6);
    const uint64_t e = g / P.ntiles;
    const uint32_t k = (uint32_t)(g % P.ntiles);
    if (e >= P.B.nv) return;
    const MulVTile tl = P.tiles[k];
    const MulVTask T = P.tasks[tl.task];
    uint32_t *arena = P.B.arena + e * P.B.astride;
    uint32_t *O = arena + T.out;
    const int nout = (int)rfl(T.nout), base = (int)rfl(tl.base);
    const int nu = (int)rfl(T.nu), nv = (int)rfl(T.nv);
    if (nu == 0 || nv == 0) {
        for (int j = 0; j < W; ++j) {
            const int w = base + lane_id() * W + j;
            if (w < nout) O[w] = 0u;
        }
        return;
    }
    const uint32_t *U = arena + T.u, *V = arena + T.v;
    if (base == 0)
        mul_tile<W, kMulQC, false, pair_mode<W>(), false>(U, nu, V, nv, nullptr, 0, O, nout, 0);
    else
        mul_tile<W, kMulQC, true, pair_mode<W>(), false>(U, nu, V, nv, nullptr, 0, O, nout, base);
}

int launch_mul_vprod(const MulVProdArgs &P, uint32_t w, void *stream) {
    const uint64_t waves = P.B.nv * P.ntiles;
    if (!waves) return 0;
    const dim3 grid((unsigned)((waves + 3) / 4)), block(256);
    switch (w) {
    case 1: hipLaunchKernelGGL(mul_vprod_kernel<1>, grid, block, 0, (hipStream_t)stream, P); break;
    case 2: hipLaunchKernelGGL(mul_vprod_kernel<2>, grid, block, 0, (hipStream_t)stream, P); break;
    case 4: hipLaunchKernelGGL(mul_vprod_kernel<4>, grid, block, 0, (hipStream_t)stream, P); break;
    case 8: hipLaunchKernelGGL(mul_vprod_kernel<8>, grid, block, 0, (hipStream_t)stream, P); break;
    case 12: hipLaunchKernelGGL(mul_vprod_kernel<12>, grid, block, 0, (hipStream_t)stream, P); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// r[0:min(4h, rcap)) = z0 + (z0 + z1 + z2) X^h + z1 X^2h  (z* are 2h words; X^h = h words).
// One lane per 4-word offset o of the half: it reads z0, z1, z2 at o and h + o once each and
// writes r at o, h + o, 2h + o, 3h + o (10h words of traffic; a lane per output word re-read the
// middle terms: 14h)
__global__ void __launch_bounds__(256) ka_comb_kernel(KaCombArgs A) {
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + rfl(threadIdx.x >> 6);
    const uint32_t h = A.h, chunks = (h + 255) / 256;
    const uint64_t per_value = (uint64_t)A.nt * chunks;
    const uint64_t e = g / per_value;
    if (e >= A.B.nv) return;
    const uint32_t r = (uint32_t)(g % per_value);
    const KaComb t = A.t[r / chunks];
    const uint32_t o = (r % chunks) * 256 + 4u * (uint32_t)lane_id();
    if (o >= h || o >= t.rcap) return;
    uint32_t *base = A.B.arena + e * A.B.astride;
    const uint4 zero = make_uint4(0u, 0u, 0u, 0u);
    auto ld = [&](uint32_t off, uint32_t i) -> uint4 {
        return off == kKaNone ? zero : *(const uint4 *)(base + off + i);
    };
    auto x = [](uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); };
    const bool s1 = h + o < t.rcap, s2 = 2 * h + o < t.rcap, s3 = 3 * h + o < t.rcap;
    const uint4 a0 = ld(t.z0, o);
    uint4 a1 = zero, b0 = zero, c0 = zero, b1 = zero, c1 = zero;
    if (s1) a1 = ld(t.z0, h + o), b0 = ld(t.z1, o), c0 = ld(t.z2, o);
    if (s2) b1 = ld(t.z1, h + o), c1 = ld(t.z2, h + o);
    uint4 *R = (uint4 *)(base + t.r + o);
    R[0] = a0;
    if (s1) *(uint4 *)(base + t.r + h + o) = x(x(a0, a1), x(b0, c0));
    if (s2) *(uint4 *)(base + t.r + 2 * h + o) = x(x(b0, a1), x(b1, c1));
    if (s3) *(uint4 *)(base + t.r + 3 * h + o) = b1;
}

int launch_ka_comb(const KaCombArgs &A, void *stream) {
    const uint64_t waves = A.B.nv * A.nt * ((A.h + 255) / 256);
    if (!waves) return 0;
    hipLaunchKernelGGL(ka_comb_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, A);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// deg(u*v) = deg u + deg v exactly (GF(2)[X] has no zero divisors); null if either is null
__global__ void __launch_bounds__(256) mul_deg_kernel(MulDegArgs A) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= A.B.nv) return;
    const uint32_t du = A.B.deg1[(uint64_t)A.u * A.B.nv + e], dv = A.B.deg1[(uint64_t)A.v * A.B.nv + e];
    A.B.deg1[(uint64_t)A.out * A.B.nv + e] = (du && dv) ? du + dv - 1 : 0u;
}

int launch_mul_deg(const MulDegArgs &A, void *stream) {
    if (!A.B.nv) return 0;
    hipLaunchKernelGGL(mul_deg_kernel, dim3((unsigned)((A.B.nv + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, A);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// output degree words (exact; null -> 0) and the capacity check
__global__ void __launch_bounds__(256) mul_final_kernel(MulFinalArgs F) {
    // the lane's output bit i indexes an LDS copy of F.ob (a by-value argument array is never
    // indexed per lane, dev_common.h)
    __shared__ __attribute__((aligned(16))) uint32_t sob[HM_MAX_BITS];
    if (threadIdx.x < 64) arg_to_lds(F.ob.b, F.K, sob);
    __syncthreads();
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t e = t / F.K;
    const uint32_t i = (uint32_t)(t % F.K);
    if (e >= F.B.nv) return;
    const uint32_t d1 = F.B.deg1[(uint64_t)F.res[i] * F.B.nv + e];
    const uint32_t d = d1 ? d1 - 1 : 0u;
    if (d > sob[i]) flag(F.B.status, HM_ERR_CAPACITY);
    F.out.degree[(F.B.e0 + e) * F.out.dstride + i] = d;
}

int launch_mul_final(const MulFinalArgs &F, void *stream) {
    const uint64_t threads = F.B.nv * F.K;
    if (!threads) return 0;
    hipLaunchKernelGGL(mul_final_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, F);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace hm
