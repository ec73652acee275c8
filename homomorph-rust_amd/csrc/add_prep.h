// add_prep.h — the adder's carry-independent part (src/impls/numbers/common.rs:37-56 as
// carry' = ab_i ^ P_i * carry, adder.hip): staging and validating input bits, and the per-bit
// products ab_i = a_i b_i and P_i = x_i (1 ^ ab_i).  Shared by add_prep_kernel (adder.hip: a
// separate launch writing a workspace) and the fused MFMA chain (adder_mfma.hip: the same work
// done by the chain's own wave, a group of bits at a time, into LDS records).
#pragma once
#include <hip/hip_runtime.h>

#include "dev_common.h"

#ifndef HM_FUSE_DIAG
#define HM_FUSE_DIAG 0
#endif

namespace hm {

__device__ __forceinline__ uint32_t limb_off(const Bounds &B, uint32_t i) {
    uint32_t o = 0;
    for (uint32_t j = 0; j < i; ++j) o += cap_of(B.b[j]);
    return o;
}

// Stage bits [i0, i0+nb) of one value's input (u64 limbs, exact degrees) into LDS words: bit
// i0+t at dst + t*cnt, its word count at nw[t] (0 = null).  Lanes stride over the range's
// contiguous limbs (all its bits at once, coalesced); every limb is validated against its bit's
// degree word as in load_bit.  src/deg point at the value's first limb / degree word.
__device__ __forceinline__ void stage_bits(const uint64_t *__restrict__ src, const uint32_t *__restrict__ deg,
                           const Bounds &B, uint32_t i0, uint32_t nb, uint32_t *dst, uint32_t cnt,
                           uint32_t *nw, int *status) {
    const int lane = lane_id();
    src += limb_off(B, i0);
    deg += i0;
    uint32_t total = 0;
    for (uint32_t t = 0; t < nb; ++t) total += cap_of(B.b[i0 + t]);
    uint32_t t = 0, lo = 0, hi = nb ? cap_of(B.b[i0]) : 0;
    bool bad = false;
    for (uint32_t g = lane; g < total; g += kWave) {
        while (g >= hi) ++t, lo = hi, hi += cap_of(B.b[i0 + t]);
        const uint32_t d = deg[t], k = g - lo;
        uint64_t v = src[g];
        if (d > B.b[i0 + t]) {
            bad = true;
            continue;
        }
        const uint32_t nl = d / 64 + 1;
        if (k >= nl) {
            bad |= v != 0; // limbs above the degree must be zero (layout invariant)
            continue;
        }
        if (k == nl - 1) {
            const uint32_t tb = d % 64;
            const uint64_t keep = (~0ull) >> (63 - tb);
            bad |= (v & ~keep) != 0;
            v &= keep;
            if (d > 0 && !((v >> tb) & 1ull)) bad = true;
        }
        dst[t * cnt + 2 * k] = (uint32_t)v;
        dst[t * cnt + 2 * k + 1] = (uint32_t)(v >> 32);
    }
    if (__any(bad) && lane == 0) flag(status, HM_ERR_BAD_INPUT);
    wsync();
    for (uint32_t k = lane; k < nb; k += kWave) {
        const uint32_t d = deg[k];
        uint32_t n = d / 32 + 1;
        if (d > B.b[i0 + k] || (d == 0 && !(dst[k * cnt] & 1u))) n = 0;
        nw[k] = n;
    }
}

// One wave computes the chain's records of bits [i0, i0 + nb) of value e: record t (at
// rec + t * recw) = [x_i: cntX][P_i: cntP][ab_i: cntAB][deg P_i + 1][deg ab_i + 1] (0 = null),
// i = i0 + t, the layout the chain reads.  Products only for bits < nbits - 1 (the last bit has
// no outgoing carry).  Lanes work over (bit t, multiplier word q) rows, each row one
// clmul_row_xor (holey integer products, ds_xor into the record), as add_prep_kernel does.
// scratch: nb * (cntA + cntB) + 2 nb words (the staged input words and their word counts).
__device__ __forceinline__ void prep_records(const AddArgs &A, uint64_t e, uint32_t i0, uint32_t nb,
                                             uint32_t *rec, uint32_t recw, uint32_t *scratch) {
    const int lane = lane_id();
    const uint32_t L = A.nbits;
    const uint32_t oP = A.cntX, oAB = oP + A.cntP, oD = oAB + A.cntAB;
    uint32_t *Al = scratch, *Bl = Al + nb * A.cntA, *nAl = Bl + nb * A.cntB, *nBl = nAl + nb;
    const uint64_t *pa = A.a.limbs + e * A.a.stride, *pb = A.b.limbs + e * A.b.stride;
    const uint32_t *da = A.a.degree + e * A.a.dstride, *db = A.b.degree + e * A.b.dstride;
    // products and degrees accumulate by ds_xor / ds_max: zero them first
    for (uint32_t k = lane; k < nb * recw; k += kWave) rec[k] = 0u;
#if HM_FUSE_DIAG == 1
    return; // diagnostic: no prep at all (wrong results)
#endif
    stage_bits(pa, da, A.ab, i0, nb, Al, A.cntA, nAl, A.status);
    stage_bits(pb, db, A.bb, i0, nb, Bl, A.cntB, nBl, A.status);
    wsync();
#if HM_FUSE_DIAG == 2
    return; // diagnostic: staging only
#endif
    const uint32_t nprod = min(nb, (L - 1) - min(i0, L - 1));
    // x_i = a_i ^ b_i (inputs masked and validated by stage_bits)
    for (uint32_t f = lane; f < nb * A.cntX; f += kWave) {
        const uint32_t t = f / A.cntX, m = f % A.cntX;
        const int na = (int)nAl[t], nbw = (int)nBl[t];
        rec[t * recw + m] = ((int)m < na ? Al[t * A.cntA + m] : 0u) ^
                            ((int)m < nbw ? Bl[t * A.cntB + m] : 0u);
    }
    const uint32_t cq = A.cntX; // multiplier words: a_i (phase 1) and x_i (phase 2) fit in cntX
    auto for_rows = [&](auto &&row) {
        const uint32_t dt = kWave / cq, dq = kWave % cq;
        uint32_t t = (uint32_t)lane / cq, q = (uint32_t)lane % cq;
        for (uint32_t f0 = 0; f0 < nprod * cq; f0 += kWave) {
            if (t < nprod) row(t, q);
            t += dt, q += dq;
            if (q >= cq) q -= cq, ++t;
        }
    };
    wsync();
    // phase 1: ab_i = a_i * b_i
    for_rows([&](uint32_t t, uint32_t q) {
        if ((int)q < (int)nAl[t])
            clmul_row_xor(Al[t * A.cntA + q], Bl + t * A.cntB, (int)nBl[t], rec + t * recw + oAB + q);
    });
    wsync();
    for (uint32_t f = lane; f < nprod * A.cntAB; f += kWave) {
        const uint32_t t = f / A.cntAB, m = f % A.cntAB;
        const uint32_t w = rec[t * recw + oAB + m];
        if (w) atomicMax(&rec[t * recw + oD + 1], m * 32 + 32 - __builtin_clz(w));
    }
    wsync();
    // phase 2: P_i = x_i ^ x_i * ab_i
    for_rows([&](uint32_t t, uint32_t q) {
        const int nx = max((int)nAl[t], (int)nBl[t]);
        if ((int)q < nx)
            clmul_row_xor(rec[t * recw + q], rec + t * recw + oAB, bitwords((int)rec[t * recw + oD + 1]),
                          rec + t * recw + oP + q);
    });
    wsync();
    for (uint32_t f = lane; f < nprod * A.cntP; f += kWave) {
        const uint32_t t = f / A.cntP, m = f % A.cntP;
        uint32_t *pw = &rec[t * recw + oP + m];
        const uint32_t w = *pw ^ (m < A.cntX ? rec[t * recw + m] : 0u);
        *pw = w;
        if (w) atomicMax(&rec[t * recw + oD], m * 32 + 32 - __builtin_clz(w));
    }
    wsync();
}

} // namespace hm
