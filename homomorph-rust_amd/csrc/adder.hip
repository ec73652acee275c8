// adder.hip — gfx950 kernels of the ripple-carry adder (src/impls/numbers/common.rs:37-56):
//   add_prep_kernel          carry-independent part: ab_i, P_i, x_i for every bit, lanes over
//                            (bit, word), several waves per value
//   add_chain_staged_kernel / add_chain_kernel
//                            the carry chain carry' = ab_i ^ P_i * carry, one wavefront per
//                            value, carry kept in LDS, products by scalar-decided VALU XORs
//                            (the matrix-core chain is adder_mfma.hip)
#include <hip/hip_runtime.h>

#include "dev_common.h"

namespace hm {

// ---------------------------------------------------------------------------------------------
// Ripple-carry adder (common.rs:37-56).  Per bit i (common.rs:43-53):
//   x = a_i ^ b_i;  s_i = x ^ carry;
//   carry' = (x & carry) ^ (a_i & b_i) & ((x & carry) ^ 1)
//          = ab_i ^ P_i * carry,   ab_i = a_i b_i,   P_i = x (1 ^ ab_i)   (GF(2)[X] ring identity)
// ab_i and P_i do not depend on the carry: add_prep_kernel computes all of them in parallel
// (several waves per value, lanes over (bit, output word), branch-free per-lane products), then
// add_chain_kernel runs the sequential chain with ONE product per bit, P_i * carry, where P_i is
// wave-uniform (scalar loads, scalar branches over its bits, Horner over bit positions) and the
// carry stays in LDS for the whole chain.

__device__ __forceinline__ uint32_t limb_off(const Bounds &B, uint32_t i) {
    uint32_t o = 0;
    for (uint32_t j = 0; j < i; ++j) o += cap_of(B.b[j]);
    return o;
}

// Validate limb v = limb k of a bit of degree d and bound bnd (as load_bit): limbs above the
// degree must be zero, the top limb's bits above the degree too, and a nonzero degree's bit must be
// set; returns the limb masked at the degree (0 for an invalid bit, whose staged words are zeros).
__device__ __forceinline__ uint64_t checked_limb(uint64_t v, uint32_t d, uint32_t bnd, uint32_t k, bool &bad) {
    const uint32_t nl = d / 64 + 1;
    if (d > bnd) {
        bad = true;
        return 0; // (every staged word is written: the fixed-length product rows read them all)
    }
    if (k >= nl) {
        bad |= v != 0; // limbs above the degree must be zero (layout invariant)
        return 0;
    }
    if (k == nl - 1) {
        const uint32_t top = d % 64;
        const uint64_t keep = (~0ull) >> (63 - top);
        bad |= (v & ~keep) != 0;
        v &= keep;
        if (d > 0 && !((v >> top) & 1ull)) bad = true;
    }
    return v;
}

// Stage bits [i0, i0+nb) of both operands of one value (u64 limbs, exact degrees) into LDS words,
// validating every limb against its bit's degree word: bit i0+t of a at Al + t*cntA, its word
// count at nAl[t] (0 = null), of b at Bl + t*cntB / nBl[t].  Lanes stride over each range's
// contiguous limbs (coalesced).  One global round trip: the bits' degrees (one per lane) and each
// lane's first limb of both operands are all in flight before the first wait (round 6; the
// per-operand form waited for limbs, then for degrees, twice).  nAl / nBl hold the degrees until
// the last pass turns them into word counts.  tb: 4 nb LDS words for both ranges' bounds and limb
// end offsets -- the per-lane bit cursors read them there, never from the by-value Bounds
// (dev_common.h: by-value argument arrays).  pa/da, pb/db: the value's first limb / degree word.
// bmask: L - 1 when the range spans several whole values (L a power of two; consecutive values'
// limbs and degree words are contiguous), so slot t is bit t & bmask.
__device__ __forceinline__ void stage_ab(const uint64_t *__restrict__ pa, const uint32_t *__restrict__ da,
                                         const Bounds &BA, const uint64_t *__restrict__ pb,
                                         const uint32_t *__restrict__ db, const Bounds &BB, uint32_t i0,
                                         uint32_t nb, uint32_t *Al, uint32_t cntA, uint32_t *nAl,
                                         uint32_t *Bl, uint32_t cntB, uint32_t *nBl, uint32_t *tb,
                                         int *status, uint32_t bmask = ~0u) {
    const uint32_t lane = (uint32_t)lane_id();
    i0 = rfl(i0), nb = rfl(nb);
    pa += limb_off(BA, i0), pb += limb_off(BB, i0);
    da += i0, db += i0;
    uint32_t dga = 0, dgb = 0;
    if (lane < nb) dga = da[lane], dgb = db[lane];
    // uniform pass: bounds and inclusive limb end offsets of both ranges, scalar reads only
    uint32_t tota = 0, totb = 0, vba = 0, vea = 0, vbb = 0, veb = 0;
    for (uint32_t t = 0; t < nb; ++t) {
        const uint32_t j = (i0 + t) & bmask; // (bmask = L - 1: several whole values per wave)
        const uint32_t ba = BA.b[j], bb = BB.b[j];
        tota += cap_of(ba), totb += cap_of(bb);
        if (lane == t) vba = ba, vea = tota, vbb = bb, veb = totb;
    }
    const uint64_t fa = lane < tota ? pa[lane] : 0ull, fb = lane < totb ? pb[lane] : 0ull;
    uint32_t *bnda = tb, *enda = tb + nb, *bndb = tb + 2 * nb, *endb = tb + 3 * nb;
    if (lane < nb) {
        bnda[lane] = vba, enda[lane] = vea, bndb[lane] = vbb, endb[lane] = veb;
        nAl[lane] = dga, nBl[lane] = dgb;
    }
    // slot words past a bit's own capacity (bits of smaller bounds than the slot's) read as zero
    for (uint32_t k = lane; k < nb * cntA; k += kWave) Al[k] = 0u;
    for (uint32_t k = lane; k < nb * cntB; k += kWave) Bl[k] = 0u;
    wsync();
    bool bad = false;
    auto one = [&](const uint64_t *src, uint64_t first, uint32_t total, const uint32_t *bnd,
                   const uint32_t *ends, const uint32_t *deg, uint32_t *dst, uint32_t cnt) {
        uint32_t t = 0, lo = 0, hi = nb ? ends[0] : 0;
        for (uint32_t g = lane; g < total; g += kWave) {
            while (g >= hi) ++t, lo = hi, hi = ends[t];
            const uint32_t k = g - lo;
            const uint64_t v = checked_limb(g == lane ? first : src[g], deg[t], bnd[t], k, bad);
            dst[t * cnt + 2 * k] = (uint32_t)v;
            dst[t * cnt + 2 * k + 1] = (uint32_t)(v >> 32);
        }
    };
    one(pa, fa, tota, bnda, enda, nAl, Al, cntA);
    one(pb, fb, totb, bndb, endb, nBl, Bl, cntB);
    if (__any(bad) && lane == 0) flag(status, HM_ERR_BAD_INPUT);
    wsync();
    if (lane < nb) {
        const uint32_t d1 = nAl[lane], d2 = nBl[lane];
        uint32_t n1 = d1 / 32 + 1, n2 = d2 / 32 + 1;
        if (d1 > bnda[lane] || (d1 == 0 && !(Al[lane * cntA] & 1u))) n1 = 0;
        if (d2 > bndb[lane] || (d2 == 0 && !(Bl[lane * cntB] & 1u))) n2 = 0;
        nAl[lane] = n1, nBl[lane] = n2;
    }
}

// NB, NAB > 0: the plan's b_i and ab_i slots hold exactly NB and NAB words (d + d' = 128 / 256 /
// 512: 6 / 10 / 18 and 9 / 17 / 33), and the product rows run at those fixed lengths
// (clmul_row_xor_fixed: unrolled, zero-padded); 0: lengths from the degrees
// TOP1: AddArgs.top1 (the top-word copies below), a separate instance so that the plain one keeps
// its code (the copies' dead branch cost configs[0]'s prep 1.3 % as a runtime flag)
// MULTI: AddArgs.vpw > 1 -- a wave holds vpw whole values (L = 2^lgL bits each; configs[0]'s
// one-wave-per-value prep paid a per-wave cost, not a per-bit one): slot t is bit t & (L - 1) of
// value e + (t >> lgL), and the last bit of every value has no product.
template <int NB, int NAB, bool TOP1 = false, bool MULTI = false>
__global__ void __launch_bounds__(256) add_prep_kernel(AddArgs A) {
    extern __shared__ uint32_t lds[];
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    const int lane = lane_id();
    const uint32_t L = A.nbits;
    uint64_t e;
    uint32_t bpw, i0, nmine; // bit slots per wave; this wave's: slots [0, nmine) = bits [i0, i0 + nmine)
    if constexpr (MULTI) {
        e = gw * A.vpw;
        if (e >= A.n) return;
        bpw = A.vpw * L;
        i0 = 0;
        nmine = (uint32_t)min((uint64_t)A.vpw, A.n - e) * L;
    } else {
        e = gw / A.wpv;
        const uint32_t part = (uint32_t)(gw % A.wpv);
        if (e >= A.n) return;
        bpw = (L + A.wpv - 1) / A.wpv;
        i0 = min(L, part * bpw), nmine = min(L, i0 + bpw) - i0;
    }
    // slot t's value (relative to e) and bit
    auto val_of = [&](uint32_t t) -> uint32_t { return MULTI ? t >> A.lgL : 0u; };
    auto bit_of = [&](uint32_t t) -> uint32_t { return MULTI ? t & (L - 1) : i0 + t; };
    // LDS: [a: bpw cntA][b: bpw cntB][x: bpw cntX][ab: bpw cntAB][P: bpw cntP][na nb dAB dP]
    //      [2 bpw more: with dAB / dP (zeroed after it), stage_ab's bound / end-offset tables]
    uint32_t *Ls = lds + (size_t)wave * A.prep_lds;
    uint32_t *Al = Ls, *Bl = Al + bpw * A.cntA, *Xl = Bl + bpw * A.cntB;
    uint32_t *ABl = Xl + bpw * A.cntX, *Pl = ABl + bpw * A.cntAB;
    uint32_t *nAl = Pl + bpw * A.cntP, *nBl = nAl + bpw, *dAB = nBl + bpw, *dP = dAB + bpw;
    // a value's workspace: [ab: L cntAB][P: L cntP][deg ab: L][deg P: L][x: L cntX]
    const size_t oP = (size_t)L * A.cntAB, oDA = oP + (size_t)L * A.cntP, oDP = oDA + L, oX = oDP + L;
    uint32_t *ws = A.ws + e * A.ws_stride;
    auto wsv = [&](uint32_t t) { return MULTI ? ws + (size_t)val_of(t) * A.ws_stride : ws; };
    const uint64_t *pa = A.a.limbs + e * A.a.stride, *pb = A.b.limbs + e * A.b.stride;
    const uint32_t *da = A.a.degree + e * L, *db = A.b.degree + e * L;

    // stage + validate this wave's bits (every bit is validated, the last one too)
    stage_ab(pa, da, A.ab, pb, db, A.bb, i0, nmine, Al, A.cntA, nAl, Bl, A.cntB, nBl, dAB, A.status,
             MULTI ? L - 1 : ~0u);
    for (uint32_t k = lane; k < 2 * bpw; k += kWave) dAB[k] = 0u;
    wsync();
    // products only for bits < L-1 (the last bit has no outgoing carry): slots [0, nprod) with
    // has_prod (MULTI: every value's last slot skipped)
    const uint32_t nprod = MULTI ? nmine : min(nmine, (L - 1) - min(i0, L - 1));
    auto has_prod = [&](uint32_t t) { return !MULTI || bit_of(t) + 1 < L; };

    // x_i = a_i ^ b_i for every bit: LDS for the P products, workspace for the chain's sum bits
    for (uint32_t f = lane; f < nmine * A.cntX; f += kWave) {
        const uint32_t t = f / A.cntX, m = f % A.cntX, i = bit_of(t);
        const int na = (int)nAl[t], nb = (int)nBl[t];
        const uint32_t x = ((int)m < na ? Al[t * A.cntA + m] : 0u) ^
                           ((int)m < nb ? Bl[t * A.cntB + m] : 0u);
        Xl[t * A.cntX + m] = x;
        wsv(t)[oX + (size_t)i * A.cntX + m] = x;
    }

    // Products by rows: lanes over (slot t, multiplier word q) -- every lane of a slot runs the
    // same number of steps (the multiplicand's length), rows meet in LDS through ds_xor.
    // Multiplier words: a_i (phase 1) and x_i (phase 2) fit in cntX.  With top1 their word
    // cntX - 1 is 0 or 1, so its row is the multiplicand shifted by cntX - 1 words: top_rows adds
    // it as a copy (ds_xor), and the rows cover words 0 .. cntX - 2 (for_rows).
    const uint32_t cq = A.cntX - (TOP1 ? 1u : 0u);
    const uint32_t qt = A.cntX - 1; // (top1) the top word's index
    auto top_rows = [&](uint32_t cnt, auto &&len, auto &&set, const uint32_t *src, uint32_t scnt,
                        uint32_t *dst, uint32_t dcnt) {
        // lanes over (slot t, multiplicand word k): dst_t[qt + k] ^= src_t[k] where the top bit is set
        const uint32_t dt = kWave / cnt, dk = kWave % cnt;
        uint32_t t = (uint32_t)lane / cnt, k = (uint32_t)lane % cnt;
        for (uint32_t f0 = 0; f0 < nprod * cnt; f0 += kWave) {
            if (t < nprod && has_prod(t) && k < len(t) && set(t))
                atomicXor(&dst[t * dcnt + qt + k], src[t * scnt + k]);
            t += dt, k += dk;
            if (k >= cnt) k -= cnt, ++t;
        }
    };
    auto for_rows = [&](auto &&row) {
        const uint32_t dt = kWave / cq, dq = kWave % cq;
        uint32_t t = (uint32_t)lane / cq, q = (uint32_t)lane % cq;
        for (uint32_t f0 = 0; f0 < nprod * cq; f0 += kWave) {
            if (t < nprod && has_prod(t)) row(t, q);
            t += dt, q += dq;
            if (q >= cq) q -= cq, ++t;
        }
    };
    // phase 1: ab_i = a_i * b_i
    for (uint32_t k = lane; k < nprod * A.cntAB; k += kWave) ABl[k] = 0u;
    for (uint32_t k = lane; k < nprod * A.cntP; k += kWave) Pl[k] = 0u;
    wsync();
    for_rows([&](uint32_t t, uint32_t q) {
        if ((int)q < (int)nAl[t]) {
            if constexpr (NB > 0) {
                if (nBl[t]) clmul_row_xor_fixed<NB>(Al[t * A.cntA + q], Bl + t * NB, ABl + t * NAB + q);
            } else {
                clmul_row_xor(Al[t * A.cntA + q], Bl + t * A.cntB, (int)nBl[t], ABl + t * A.cntAB + q);
            }
        }
    });
    if constexpr (TOP1) // a_i's word qt is 1 exactly when a_i has cntX words (exact degrees)
        top_rows(A.cntB, [&](uint32_t t) { return nBl[t]; }, [&](uint32_t t) { return nAl[t] == A.cntX; },
                 Bl, A.cntB, ABl, A.cntAB);
    wsync();
    for (uint32_t f = lane; f < nprod * A.cntAB; f += kWave) {
        const uint32_t t = f / A.cntAB, m = f % A.cntAB;
        const uint32_t w = ABl[f];
        if (has_prod(t)) wsv(t)[(size_t)bit_of(t) * A.cntAB + m] = w;
        if (w) atomicMax(&dAB[t], m * 32 + 32 - __builtin_clz(w));
    }
    wsync();
    // phase 2: P_i = x_i ^ x_i * ab_i
    for_rows([&](uint32_t t, uint32_t q) {
        const int nx = max((int)nAl[t], (int)nBl[t]);
        if ((int)q < nx) {
            if constexpr (NAB > 0) {
                if (dAB[t]) clmul_row_xor_fixed<NAB>(Xl[t * A.cntX + q], ABl + t * NAB, Pl + t * A.cntP + q);
            } else {
                clmul_row_xor(Xl[t * A.cntX + q], ABl + t * A.cntAB, bitwords((int)dAB[t]),
                              Pl + t * A.cntP + q);
            }
        }
    });
    if constexpr (TOP1) // x_i's word qt (a_i's and b_i's top bits may cancel)
        top_rows(A.cntAB, [&](uint32_t t) { return (uint32_t)bitwords((int)dAB[t]); },
                 [&](uint32_t t) { return (Xl[t * A.cntX + qt] & 1u) != 0; }, ABl, A.cntAB, Pl, A.cntP);
    wsync();
    for (uint32_t f = lane; f < nprod * A.cntP; f += kWave) {
        const uint32_t t = f / A.cntP, m = f % A.cntP;
        const uint32_t w = Pl[f] ^ (m < A.cntX ? Xl[t * A.cntX + m] : 0u);
        if (has_prod(t)) wsv(t)[oP + (size_t)bit_of(t) * A.cntP + m] = w;
        if (w) atomicMax(&dP[t], m * 32 + 32 - __builtin_clz(w));
    }
    wsync();
    for (uint32_t t = lane; t < nprod; t += kWave) {
        if (!has_prod(t)) continue;
        const uint32_t i = bit_of(t);
        wsv(t)[oDA + i] = dAB[t];
        wsv(t)[oDP + i] = dP[t];
    }
}

// s_i = a_i ^ b_i ^ carry, read straight from the input limbs (masked at the degrees, which the
// prep kernel validated) and the LDS carry words; writes the output bit and its exact degree.
__device__ __forceinline__ int store_sum_bit(const uint64_t *pa, uint32_t dga, const uint64_t *pb, uint32_t dgb,
                             const uint32_t *C, int nc, uint64_t *__restrict__ dst, uint32_t bound,
                             uint32_t *deg_out, int *status) {
    const int lane = lane_id();
    const int cap = (int)cap_of(bound);
    const int nla = (int)(dga >> 6) + 1, nlb = (int)(dgb >> 6) + 1;
    const uint64_t ma = (~0ull) >> (63 - (dga & 63)), mb = (~0ull) >> (63 - (dgb & 63));
    const int total = max(max(cap, max(nla, nlb)), (nc + 1) / 2);
    int ldeg = -1;
    for (int g = lane; g < total; g += kWave) {
        uint64_t v = 0;
        if (g < nla) v ^= g == nla - 1 ? (pa[g] & ma) : pa[g];
        if (g < nlb) v ^= g == nlb - 1 ? (pb[g] & mb) : pb[g];
        const int w = 2 * g;
        const uint32_t lo = w < nc ? C[w] : 0u, hi = w + 1 < nc ? C[w + 1] : 0u;
        v ^= (uint64_t)lo | ((uint64_t)hi << 32);
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

template <int WMAX, bool PAD>
__global__ void __launch_bounds__(256) add_chain_kernel(AddArgs A) {
    kt_start(A.kt);
    extern __shared__ uint32_t lds[];
    const int wave = (int)rfl(threadIdx.x >> 6); // wave-uniform by construction
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (e >= A.n) { // whole wave exits together
        kt_finish(A.kt);
        return;
    }
    const int lane = lane_id();
    const uint32_t L = A.nbits;
    uint32_t *Ls = lds + (size_t)wave * A.chain_lds;
    uint32_t *C = Ls + kHalo, *Cn = C + A.cw + kHalo;
    uint32_t *Pl = Cn + A.cw; // P_i slots, copied once from the workspace (uniform reads per step)
    const uint32_t *ws = A.ws + e * A.ws_stride;
    const uint32_t *ABg = ws, *Pg = ws + (size_t)L * A.cntAB;
    const uint32_t *degABg = Pg + (size_t)L * A.cntP, *degPg = degABg + L;
    const uint64_t *pa = A.a.limbs + e * A.a.stride, *pb = A.b.limbs + e * A.b.stride;
    uint64_t *po = A.out.limbs + e * A.out.stride;
    const uint32_t *da = A.a.degree + e * L, *db = A.b.degree + e * L;
    uint32_t *dout = A.out.degree + e * L;

    // zero both carry buffers with their halos: window reads need no bounds checks (PAD)
    const uint32_t ncarry = 2 * (A.cw + kHalo);
    for (uint32_t k = lane; k < ncarry; k += kWave) Ls[k] = 0u;
    for (uint32_t k = lane; k < (L - 1) * A.cntP; k += kWave) Pl[k] = Pg[k];
    wsync();
    int nc = 0; // carry words (0 = null carry, common.rs:39)
    uint32_t offa = 0, offb = 0, offo = 0;
    for (uint32_t i = 0; i < L; ++i) {
        store_sum_bit(pa + offa, rfl(da[i]), pb + offb, rfl(db[i]), C, nc, po + offo, A.ob.b[i],
                      dout + i, A.status);
        if (i + 1 < L) {
            const int np = bitwords((int)degPg[i]), nab = bitwords((int)degABg[i]);
            int nout;
            nc = words_of(wave_mul<kQBig, WMAX, PAD>(Pl + (size_t)i * A.cntP, np, C, nc,
                                                     ABg + (size_t)i * A.cntAB, nab, Cn, &nout));
            wsync();
            uint32_t *t = C;
            C = Cn;
            Cn = t;
        }
        offa += cap_of(A.ab.b[i]);
        offb += cap_of(A.bb.b[i]);
        offo += cap_of(A.ob.b[i]);
    }
    kt_finish(A.kt);
}

// Staged chain (PAD plans whose slots fit in LDS).  Everything the loop reads per bit -- x_i,
// ab_i, P_i and the product degrees -- is copied from the workspace into LDS once, and the carry
// is updated in place (PAD products read their whole window before writing their tile), so the
// only global traffic inside the loop is the output stores: no load ever waits behind them.
template <int WMAX>
__global__ void __launch_bounds__(256) add_chain_staged_kernel(AddArgs A) {
    kt_start(A.kt);
    extern __shared__ uint32_t lds[];
    const int wave = (int)rfl(threadIdx.x >> 6); // wave-uniform by construction
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (e >= A.n) { // whole wave exits together
        kt_finish(A.kt);
        return;
    }
    const int lane = lane_id();
    const uint32_t L = A.nbits;
    // LDS: [halo][C: cw][P: (L-1) cntP][AB: (L-1) cntAB][X: L cntX][degP: L][degAB: L]
    uint32_t *Ls = lds + (size_t)wave * A.chain_lds;
    uint32_t *C = Ls + kHalo;
    uint32_t *Pl = C + A.cw, *ABl = Pl + (size_t)(L - 1) * A.cntP;
    uint32_t *Xl = ABl + (size_t)(L - 1) * A.cntAB, *dPl = Xl + (size_t)L * A.cntX, *dABl = dPl + L;
    const uint32_t *ws = A.ws + e * A.ws_stride;
    const uint32_t *ABg = ws, *Pg = ws + (size_t)L * A.cntAB;
    const uint32_t *degABg = Pg + (size_t)L * A.cntP, *degPg = degABg + L, *Xg = degPg + L;
    uint64_t *po = A.out.limbs + e * A.out.stride;
    uint32_t *dout = A.out.degree + e * L;

    for (uint32_t k = lane; k < kHalo + A.cw; k += kWave) Ls[k] = 0u;
    for (uint32_t k = lane; k < (L - 1) * A.cntP; k += kWave) Pl[k] = Pg[k];
    for (uint32_t k = lane; k < (L - 1) * A.cntAB; k += kWave) ABl[k] = ABg[k];
    for (uint32_t k = lane; k < L * A.cntX; k += kWave) Xl[k] = Xg[k];
    for (uint32_t k = lane; k < L; k += kWave) dPl[k] = degPg[k], dABl[k] = degABg[k];
    wsync();
    int nc = 0; // carry words (0 = null carry, common.rs:39)
    uint32_t offo = 0;
    for (uint32_t i = 0; i < L; ++i) {
        store_sum_x(Xl + (size_t)i * A.cntX, (int)A.cntX, C, nc, po + offo, A.ob.b[i], dout + i,
                    A.status);
        if (i + 1 < L) {
            const int np = bitwords((int)rfl(dPl[i])), nab = bitwords((int)rfl(dABl[i]));
            int nout;
            wsync(); // the sum bit's reads of C precede the in-place product's writes
            nc = words_of(wave_mul<kQBig, WMAX, true>(Pl + (size_t)i * A.cntP, np, C, nc,
                                                      ABl + (size_t)i * A.cntAB, nab, C, &nout));
            wsync();
        }
        offo += cap_of(A.ob.b[i]);
    }
    kt_finish(A.kt);
}

int launch_add_prep(const AddArgs &a, void *stream) {
    if (a.n == 0) return 0;
    // wpv waves per value (or vpw values per wave), 4 waves per block
    const uint64_t waves = a.vpw > 1 ? (a.n + a.vpw - 1) / a.vpw : a.n * a.wpv;
    const uint64_t blocks = (waves + 3) / 4;
    const size_t lds = (size_t)a.prep_lds * 4 * 4;
#ifndef HM_PREP_FIXED
#define HM_PREP_FIXED 0 // (A/B knob) 1: product rows at the slots' fixed lengths (measured neutral, r06)
#endif
    if (a.vpw > 1 && a.top1)
        hipLaunchKernelGGL((add_prep_kernel<0, 0, true, true>), dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, a);
    else if (a.vpw > 1)
        hipLaunchKernelGGL((add_prep_kernel<0, 0, false, true>), dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, a);
    else if (a.top1)
        hipLaunchKernelGGL((add_prep_kernel<0, 0, true>), dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, a);
    else if (HM_PREP_FIXED && a.cntB == 10 && a.cntAB == 17)
        hipLaunchKernelGGL((add_prep_kernel<10, 17>), dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, a);
    else if (HM_PREP_FIXED && a.cntB == 6 && a.cntAB == 9)
        hipLaunchKernelGGL((add_prep_kernel<6, 9>), dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, a);
    else if (HM_PREP_FIXED && a.cntB == 18 && a.cntAB == 33)
        hipLaunchKernelGGL((add_prep_kernel<18, 33>), dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL((add_prep_kernel<0, 0>), dim3((unsigned)blocks), dim3(256), lds, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

AddArgs add_args_slice(const AddArgs &a, uint64_t e0, uint64_t n) {
    AddArgs s = a;
    s.a.limbs += e0 * a.a.stride, s.a.degree += e0 * a.a.dstride;
    s.b.limbs += e0 * a.b.stride, s.b.degree += e0 * a.b.dstride;
    s.out.limbs += e0 * a.out.stride, s.out.degree += e0 * a.out.dstride;
    s.ws += e0 * a.ws_stride;
    s.n = n;
    return s;
}

int launch_add(const AddArgs &a, void *stream) {
    if (a.n == 0) return 0;
    if (launch_add_prep(a, stream)) return -1;
    return a.mfma ? launch_add_chain_mfma(a, stream) : launch_add_chain_valu(a, stream);
}

int launch_add_chain_valu(const AddArgs &a, void *stream) {
    const int wpb = kAddWavesPerBlock;
    const uint64_t blocks = (a.n + wpb - 1) / wpb;
    const size_t lds = (size_t)a.chain_lds * 4 * wpb;
    // the widest per-lane tile the carry chain needs (carry + P words over 64 lanes)
    const uint32_t need = (a.max_prod_words + 63) / 64;
    const bool pad = a.pad != 0;
#define HM_LAUNCH_ADD(WM)                                                                         \
    do {                                                                                          \
        if (a.staged)                                                                             \
            hipLaunchKernelGGL((add_chain_staged_kernel<WM>), dim3((unsigned)blocks),             \
                               dim3(64 * wpb), lds, (hipStream_t)stream, a);                      \
        else if (pad)                                                                             \
            hipLaunchKernelGGL((add_chain_kernel<WM, true>), dim3((unsigned)blocks),              \
                               dim3(64 * wpb), lds, (hipStream_t)stream, a);                      \
        else                                                                                      \
            hipLaunchKernelGGL((add_chain_kernel<WM, false>), dim3((unsigned)blocks),             \
                               dim3(64 * wpb), lds, (hipStream_t)stream, a);                      \
    } while (0)
    if (need <= 4) HM_LAUNCH_ADD(4);
    else if (need <= 8) HM_LAUNCH_ADD(8);
    else if (need <= 12) HM_LAUNCH_ADD(12);
    else if (need <= 16) HM_LAUNCH_ADD(16);
    else HM_LAUNCH_ADD(24);
#undef HM_LAUNCH_ADD
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace hm
