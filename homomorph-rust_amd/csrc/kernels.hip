// kernels.hip — gfx950 kernels of the GF(2)[X] homomorphic engine.
//
//   add_prep_kernel ripple-carry adder, carry-independent part: ab_i, P_i, x_i for every bit,
//                   lanes over (bit, word), several waves per value
//   add_chain_staged_kernel / add_chain_kernel
//                   the carry chain carry' = ab_i ^ P_i * carry, one wavefront per value, carry
//                   kept in LDS (src/impls/numbers/common.rs:37-56 add_internal)
//   gate_kernel     elementwise AND/OR/XOR/NOT (common.rs:5-35)
//   encrypt_kernel  subset-sum of the public key, one lane per ciphertext bit (cipher.rs:99-115)
//   decrypt_kernel  (C mod S)(0) as the parity functional  sum_k c_k z_k, z_k = (X^k mod S)(0):
//                   a linear map, so it equals the reference's long-division remainder evaluated
//                   at 0 (cipher.rs:119-122, polynomial.rs:316-365); one wavefront per value
//   poly_* kernels  single-polynomial primitives for unit parity (polynomial.rs:190-365)
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

// Stage bits [i0, i0+nb) of one value's input (u64 limbs, exact degrees) into LDS words: bit
// i0+t at dst + t*cnt, its word count at nw[t] (0 = null).  Lanes stride over the range's
// contiguous limbs (all its bits at once, coalesced); every limb is validated against its bit's
// degree word as in load_bit.  src/deg point at the value's first limb / degree word.
__device__ void stage_bits(const uint64_t *__restrict__ src, const uint32_t *__restrict__ deg,
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

__global__ void __launch_bounds__(256) add_prep_kernel(AddArgs A) {
    extern __shared__ uint32_t lds[];
    const uint32_t wave = rfl(threadIdx.x >> 6);
    const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    const uint64_t e = gw / A.wpv;
    const uint32_t part = (uint32_t)(gw % A.wpv);
    if (e >= A.n) return;
    const int lane = lane_id();
    const uint32_t L = A.nbits;
    const uint32_t bpw = (L + A.wpv - 1) / A.wpv; // bit slots per wave: bits [i0, i0 + nmine)
    const uint32_t i0 = min(L, part * bpw), nmine = min(L, i0 + bpw) - i0;
    // LDS: [a: bpw cntA][b: bpw cntB][x: bpw cntX][ab: bpw cntAB][P: bpw cntP][na nb dAB dP]
    uint32_t *Ls = lds + (size_t)wave * A.prep_lds;
    uint32_t *Al = Ls, *Bl = Al + bpw * A.cntA, *Xl = Bl + bpw * A.cntB;
    uint32_t *ABl = Xl + bpw * A.cntX, *Pl = ABl + bpw * A.cntAB;
    uint32_t *nAl = Pl + bpw * A.cntP, *nBl = nAl + bpw, *dAB = nBl + bpw, *dP = dAB + bpw;
    uint32_t *ws = A.ws + e * A.ws_stride;
    uint32_t *ABg = ws, *Pg = ws + (size_t)L * A.cntAB;
    uint32_t *degABg = Pg + (size_t)L * A.cntP, *degPg = degABg + L, *Xg = degPg + L;
    const uint64_t *pa = A.a.limbs + e * A.a.stride, *pb = A.b.limbs + e * A.b.stride;
    const uint32_t *da = A.a.degree + e * L, *db = A.b.degree + e * L;

    // stage + validate this wave's bits (every bit is validated, the last one too)
    stage_bits(pa, da, A.ab, i0, nmine, Al, A.cntA, nAl, A.status);
    stage_bits(pb, db, A.bb, i0, nmine, Bl, A.cntB, nBl, A.status);
    for (uint32_t k = lane; k < 2 * bpw; k += kWave) dAB[k] = 0u;
    wsync();
    // products only for bits < L-1 (the last bit has no outgoing carry)
    const uint32_t nprod = min(nmine, (L - 1) - min(i0, L - 1));

    // x_i = a_i ^ b_i for every bit: LDS for the P products, workspace for the chain's sum bits
    for (uint32_t f = lane; f < nmine * A.cntX; f += kWave) {
        const uint32_t t = f / A.cntX, m = f % A.cntX, i = i0 + t;
        const int na = (int)nAl[t], nb = (int)nBl[t];
        const uint32_t x = ((int)m < na ? Al[t * A.cntA + m] : 0u) ^
                           ((int)m < nb ? Bl[t * A.cntB + m] : 0u);
        Xl[t * A.cntX + m] = x;
        Xg[(size_t)i * A.cntX + m] = x;
    }

    // Products by rows: lanes over (slot t, multiplier word q) -- every lane of a slot runs the
    // same number of steps (the multiplicand's length), rows meet in LDS through ds_xor.
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
    // phase 1: ab_i = a_i * b_i
    for (uint32_t k = lane; k < nprod * A.cntAB; k += kWave) ABl[k] = 0u;
    for (uint32_t k = lane; k < nprod * A.cntP; k += kWave) Pl[k] = 0u;
    wsync();
    for_rows([&](uint32_t t, uint32_t q) {
        if ((int)q < (int)nAl[t])
            clmul_row_xor(Al[t * A.cntA + q], Bl + t * A.cntB, (int)nBl[t], ABl + t * A.cntAB + q);
    });
    wsync();
    for (uint32_t f = lane; f < nprod * A.cntAB; f += kWave) {
        const uint32_t t = f / A.cntAB, m = f % A.cntAB;
        const uint32_t w = ABl[f];
        ABg[(size_t)(i0 + t) * A.cntAB + m] = w;
        if (w) atomicMax(&dAB[t], m * 32 + 32 - __builtin_clz(w));
    }
    wsync();
    // phase 2: P_i = x_i ^ x_i * ab_i
    for_rows([&](uint32_t t, uint32_t q) {
        const int nx = max((int)nAl[t], (int)nBl[t]);
        if ((int)q < nx)
            clmul_row_xor(Xl[t * A.cntX + q], ABl + t * A.cntAB, bitwords((int)dAB[t]),
                          Pl + t * A.cntP + q);
    });
    wsync();
    for (uint32_t f = lane; f < nprod * A.cntP; f += kWave) {
        const uint32_t t = f / A.cntP, m = f % A.cntP;
        const uint32_t w = Pl[f] ^ (m < A.cntX ? Xl[t * A.cntX + m] : 0u);
        Pg[(size_t)(i0 + t) * A.cntP + m] = w;
        if (w) atomicMax(&dP[t], m * 32 + 32 - __builtin_clz(w));
    }
    wsync();
    for (uint32_t t = lane; t < nprod; t += kWave) {
        const uint32_t i = i0 + t;
        degABg[i] = dAB[t];
        degPg[i] = dP[t];
    }
}

// s_i = a_i ^ b_i ^ carry, read straight from the input limbs (masked at the degrees, which the
// prep kernel validated) and the LDS carry words; writes the output bit and its exact degree.
__device__ int store_sum_bit(const uint64_t *pa, uint32_t dga, const uint64_t *pb, uint32_t dgb,
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
    extern __shared__ uint32_t lds[];
    const int wave = (int)rfl(threadIdx.x >> 6); // wave-uniform by construction
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (e >= A.n) return; // whole wave exits together
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
}

// Staged chain (PAD plans whose slots fit in LDS).  Everything the loop reads per bit -- x_i,
// ab_i, P_i and the product degrees -- is copied from the workspace into LDS once, and the carry
// is updated in place (PAD products read their whole window before writing their tile), so the
// only global traffic inside the loop is the output stores: no load ever waits behind them.
__device__ int store_sum_x(const uint32_t *X, int nx, const uint32_t *C, int nc,
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

template <int WMAX>
__global__ void __launch_bounds__(256) add_chain_staged_kernel(AddArgs A) {
    extern __shared__ uint32_t lds[];
    const int wave = (int)rfl(threadIdx.x >> 6); // wave-uniform by construction
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (e >= A.n) return; // whole wave exits together
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
}

int launch_add(const AddArgs &a, void *stream) {
    if (a.n == 0) return 0;
    // prep: wpv waves per value, 4 waves per block
    {
        const uint64_t waves = a.n * a.wpv;
        const uint64_t blocks = (waves + 3) / 4;
        hipLaunchKernelGGL(add_prep_kernel, dim3((unsigned)blocks), dim3(256),
                           (size_t)a.prep_lds * 4 * 4, (hipStream_t)stream, a);
        if (hipGetLastError() != hipSuccess) return -1;
    }
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

// ---------------------------------------------------------------------------------------------
// Elementwise gates: one wavefront per value, bit by bit through LDS.
//   AND = a*b, XOR = a+b, OR = a+b+ab, NOT = a+1    (cipher.rs:58-90)
__global__ void __launch_bounds__(256) gate_kernel(GateArgs G) {
    extern __shared__ uint32_t lds[];
    const int wave = (int)rfl(threadIdx.x >> 6); // wave-uniform by construction
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (e >= G.n) return;
    const int lane = lane_id();
    uint32_t *L = lds + (size_t)wave * G.lds_per_wave;
    uint32_t *Ab = L + G.oA, *Bb = L + G.oB, *T = L + G.oT;
    const uint64_t *pa = G.a.limbs + e * G.a.stride;
    const uint64_t *pb = G.op == HM_OP_NOT ? nullptr : G.b.limbs + e * G.b.stride;
    uint64_t *po = G.out.limbs + e * G.out.stride;
    uint32_t offa = 0, offb = 0, offo = 0;
    for (uint32_t i = 0; i < G.nbits; ++i) {
        const int na = load_bit(pa + offa, rfl(G.a.degree[e * G.nbits + i]), G.ab.b[i], Ab, G.status);
        int nb = 0;
        if (G.op == HM_OP_NOT) {
            if (lane == 0) Bb[0] = 1u; // the unit polynomial, CipheredBit::one (cipher.rs:49-51)
            nb = 1;
        } else {
            nb = load_bit(pb + offb, rfl(G.b.degree[e * G.nbits + i]), G.bb.b[i], Bb, G.status);
        }
        wsync();
        int nt = 0, nout;
        const uint32_t *R = T;
        if (G.op == HM_OP_AND) {
            nt = words_of(wave_mul<kQSmall, 8>(Ab, na, Bb, nb, nullptr, 0, T, &nout));
        } else if (G.op == HM_OP_OR) {
            // a + b + ab: first X = a ^ b into T's tail, then T = X ^ a*b
            uint32_t *Xs = T + (na + nb + 2);
            const int nx = words_of(wave_xor(Ab, na, Bb, nb, Xs));
            wsync();
            nt = words_of(wave_mul<kQSmall, 8>(Ab, na, Bb, nb, Xs, nx, T, &nout));
        } else { // XOR, NOT
            nt = words_of(wave_xor(Ab, na, Bb, nb, T));
        }
        wsync();
        store_xor_bit(R, nt, nullptr, 0, po + offo, G.ob.b[i], G.out.degree + e * G.nbits + i,
                      G.status);
        wsync();
        offa += cap_of(G.ab.b[i]);
        if (G.op != HM_OP_NOT) offb += cap_of(G.bb.b[i]);
        offo += cap_of(G.ob.b[i]);
    }
}

int launch_gate(const GateArgs &g, void *stream) {
    const int wpb = 4;
    const uint64_t blocks = (g.n + wpb - 1) / wpb;
    if (blocks == 0) return 0;
    hipLaunchKernelGGL(gate_kernel, dim3((unsigned)blocks), dim3(64 * wpb),
                       (size_t)g.lds_per_wave * 4 * wpb, (hipStream_t)stream, g);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------------------------
// Encryption: one lane per ciphertext bit.  C = XOR_{i : mask bit i} T_i, then C ^= x
// (CipheredBit::cipher, cipher.rs:99-115; Ciphered::try_cipher bit order :180-185).  The public
// key T_i is read with wave-uniform addresses (scalar loads); the mask select is one bitop3
// (acc ^ (t & m)) per 32-bit half.
template <int PC>
__global__ void __launch_bounds__(256) encrypt_kernel(EncArgs E) {
    const uint32_t nbits = E.nbytes * 8;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= E.n * nbits) return;
    const uint64_t e = t / nbits;
    const uint32_t k = (uint32_t)(t % nbits);
    const uint32_t mb = (E.tau + 7) / 8;
    const uint8_t *m = E.masks + t * mb;
    uint32_t lo[PC], hi[PC];
#pragma unroll
    for (int l = 0; l < PC; ++l) lo[l] = hi[l] = 0u;
    for (uint32_t i0 = 0; i0 < E.tau; i0 += 32) {
        uint32_t bits;
        if ((mb & 3u) == 0) {
            bits = *(const uint32_t *)(m + i0 / 8);
        } else {
            bits = 0;
            for (uint32_t b = 0; b < 4 && i0 / 8 + b < mb; ++b) bits |= (uint32_t)m[i0 / 8 + b] << (8 * b);
        }
        const uint32_t cnt = min(32u, E.tau - i0);
        for (uint32_t ii = 0; ii < cnt; ++ii) {
            const uint32_t msk = (uint32_t)__builtin_amdgcn_sbfe((int)bits, ii, 1); // 0 or ~0
            const uint32_t *pk = (const uint32_t *)(E.pk + (size_t)(i0 + ii) * PC);
#pragma unroll
            for (int l = 0; l < PC; ++l) {
                lo[l] ^= pk[2 * l] & msk; // one v_bitop3_b32 each (compiler-formed)
                hi[l] ^= pk[2 * l + 1] & msk;
            }
        }
    }
    lo[0] ^= (E.data[e * E.nbytes + k / 8] >> (k % 8)) & 1u; // add_bool_assign (:112)
    uint32_t off = 0;
    for (uint32_t j = 0; j < k; ++j) off += cap_of(E.ob.b[j]);
    const uint32_t cap = cap_of(E.ob.b[k]);
    uint64_t *dst = E.out.limbs + e * E.out.stride + off;
    int deg = 0;
#pragma unroll
    for (int l = 0; l < PC; ++l) {
        const uint64_t v = (uint64_t)lo[l] | ((uint64_t)hi[l] << 32);
        if (v) deg = l * 64 + 63 - __builtin_clzll(v);
        if ((uint32_t)l < cap) dst[l] = v;
        else if (v) flag(E.status, HM_ERR_CAPACITY);
    }
    for (uint32_t l = PC; l < cap; ++l) dst[l] = 0ull;
    if ((uint32_t)deg > E.ob.b[k]) flag(E.status, HM_ERR_CAPACITY);
    E.out.degree[e * nbits + k] = (uint32_t)deg;
}

// Table form of the same subset sum (four Russians over the mask): the public-key rows are taken
// four at a time, with the 16 XOR combinations of every group precomputed per key (upload_pk:
// T[g][n] = XOR_{k : bit k of n} T_{4g+k}).  Each block copies that table into LDS once and its
// threads stride over ciphertext bits; a bit is one LDS lookup per mask nibble -- tau/4 lookups
// of PC limbs instead of tau masked XORs of PC limbs with a scalar (SGPR) operand, which run at
// ~0.6 rate.  Same output bits: XOR is associative and commutative.
constexpr int kEncBlock = 512;

// one nibble lookup: acc ^= T[g][nib] (NP limb pairs, one conflict-free ds_read_b128 each)
template <int NP>
__device__ __forceinline__ void enc_lookup(uint64_t *acc, const uint4 *tab4, uint32_t g,
                                           uint32_t nib) {
    const uint4 *row = tab4 + (size_t)g * NP * 16 + nib;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const uint4 v = row[p * 16];
        acc[2 * p] ^= (uint64_t)v.x | ((uint64_t)v.y << 32);
        acc[2 * p + 1] ^= (uint64_t)v.z | ((uint64_t)v.w << 32);
    }
}

// GC: compile-time group count (tau/4) for the fully unrolled path with 16-byte-aligned masks
// (tau = 128: one uint4 of mask per ciphertext bit), 0 = any tau
template <int PC, int GC>
__global__ void __launch_bounds__(kEncBlock) encrypt_table_kernel(EncArgs E) {
    constexpr int NP = (PC + 1) / 2;  // limb pairs
    extern __shared__ uint64_t tab[]; // [G][NP][16][2] (upload_pk)
    const uint32_t G = GC ? GC : (E.tau + 3) / 4;
    {
        const uint32_t n16 = G * NP * 16; // 16-byte chunks
        const uint4 *src = (const uint4 *)E.pk_tab;
        uint4 *dst = (uint4 *)tab;
        for (uint32_t f = threadIdx.x; f < n16; f += blockDim.x) dst[f] = src[f];
    }
    __syncthreads();
    const uint4 *tab4 = (const uint4 *)tab;
    uint64_t *stage = tab + (size_t)G * NP * 32; // [waves][64][PC] store transpose
    const uint32_t nbits = E.nbytes * 8;
    const uint32_t mb = (E.tau + 7) / 8;
    const uint64_t total = E.n * nbits;
    // the loop runs per wave (the store transpose is wave-cooperative): lanes past the end of
    // the batch compute on a clamped index and are masked out of every store
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t lane = threadIdx.x & 63u;
    for (uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); t0 < total;
         t0 += step) {
        const bool live = t0 + lane < total;
        const uint64_t t = live ? t0 + lane : total - 1;
        const uint64_t e = E.lognbits >= 0 ? t >> E.lognbits : t / nbits;
        const uint32_t k = (uint32_t)(t - e * nbits);
        const uint8_t *m = E.masks + t * mb;
        uint64_t acc[2 * NP];
#pragma unroll
        for (int l = 0; l < 2 * NP; ++l) acc[l] = 0;
        if constexpr (GC != 0) {
            static_assert(GC % 32 == 0, "GC: whole uint4 mask words");
#pragma unroll
            for (int w4 = 0; w4 < GC / 32; ++w4) {
                const uint4 mw = ((const uint4 *)m)[w4];
                const uint32_t ws[4] = {mw.x, mw.y, mw.z, mw.w};
#pragma unroll
                for (int w = 0; w < 4; ++w)
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        enc_lookup<NP>(acc, tab4, 32 * w4 + 8 * w + j, (ws[w] >> (4 * j)) & 15u);
            }
        } else {
            for (uint32_t g0 = 0; g0 < G; g0 += 8) { // one 32-bit mask word = 8 nibbles
                const uint32_t b0 = g0 / 2;           // first mask byte of this word
                uint32_t bits;
                if ((mb & 3u) == 0) {
                    bits = *(const uint32_t *)(m + b0);
                } else {
                    bits = 0;
                    for (uint32_t b = 0; b < 4 && b0 + b < mb; ++b)
                        bits |= (uint32_t)m[b0 + b] << (8 * b);
                }
                const uint32_t ng = min(8u, G - g0);
                for (uint32_t j = 0; j < ng; ++j)
                    enc_lookup<NP>(acc, tab4, g0 + j, (bits >> (4 * j)) & 15u);
            }
        }
        // mask bits at or above tau select nothing: the table rows past tau are zero, and the
        // reference reads exactly ceil(tau/8) bytes, bits >= tau unused (cipher.rs:105-110)
        acc[0] ^= (E.data[e * E.nbytes + k / 8] >> (k % 8)) & 1u; // add_bool_assign (:112)
        int deg = 0;
#pragma unroll
        for (int l = 0; l < PC; ++l)
            if (acc[l]) deg = l * 64 + 63 - __builtin_clzll(acc[l]);
        if (live) {
            if ((uint32_t)deg > E.ob.b[k]) flag(E.status, HM_ERR_CAPACITY);
            E.out.degree[e * nbits + k] = (uint32_t)deg;
        }
        if (E.uniform_cap) {
            // the wave's 64 bits own 64*PC consecutive output limbs (limb l of bit t at t*PC + l):
            // transpose through LDS and store them coalesced (lane j writes limb j, j + 64, ...)
            uint64_t *st = stage + (size_t)(threadIdx.x & ~63u) * PC;
#pragma unroll
            for (int l = 0; l < PC; ++l) st[lane * PC + l] = acc[l];
            wsync();
            const uint64_t lim = (total - t0) * PC;
            uint64_t *dst = E.out.limbs + t0 * PC;
#pragma unroll
            for (int r = 0; r < PC; ++r) {
                const uint32_t j = lane + 64 * r;
                if (j < lim) dst[j] = st[j];
            }
            wsync();
        } else if (live) {
            const uint32_t cap = cap_of(E.ob.b[k]);
            uint64_t *dst = E.out.limbs + e * E.out.stride + E.ooff.b[k];
#pragma unroll
            for (int l = 0; l < PC; ++l) {
                if ((uint32_t)l < cap) dst[l] = acc[l];
                else if (acc[l]) flag(E.status, HM_ERR_CAPACITY);
            }
            for (uint32_t l = PC; l < cap; ++l) dst[l] = 0ull;
        }
    }
}

template <int PC>
static void launch_enc_pc(const EncArgs &E, void *stream) {
    const uint64_t threads = E.n * E.nbytes * 8;
    const size_t tab = (size_t)((E.tau + 3) / 4) * ((PC + 1) / 2) * 16 * 16;
    const size_t lds = tab + (size_t)kEncBlock * PC * 8; // + the store transpose
    if (E.pk_tab && tab <= kEncTableBytes && lds <= 64 * 1024) {
        // a few resident blocks per CU, each striding over bits (the table copy is amortised)
        const uint64_t want = (threads + kEncBlock - 1) / kEncBlock;
        const uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>(4, (160 * 1024) / lds));
        const uint64_t blocks = std::min<uint64_t>(want, (uint64_t)E.cus * per_cu);
        if (E.tau == 128 && ((uintptr_t)E.masks & 15u) == 0)
            hipLaunchKernelGGL((encrypt_table_kernel<PC, 32>), dim3((unsigned)blocks),
                               dim3(kEncBlock), lds, (hipStream_t)stream, E);
        else
            hipLaunchKernelGGL((encrypt_table_kernel<PC, 0>), dim3((unsigned)blocks),
                               dim3(kEncBlock), lds, (hipStream_t)stream, E);
        return;
    }
    const uint64_t blocks = (threads + 255) / 256;
    hipLaunchKernelGGL(encrypt_kernel<PC>, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, E);
}

int launch_encrypt(const EncArgs &E, void *stream) {
    if (E.n == 0) return 0;
    switch (E.pk_cap) {
    case 1: launch_enc_pc<1>(E, stream); break;
    case 2: launch_enc_pc<2>(E, stream); break;
    case 3: launch_enc_pc<3>(E, stream); break;
    case 4: launch_enc_pc<4>(E, stream); break;
    case 5: launch_enc_pc<5>(E, stream); break;
    case 6: launch_enc_pc<6>(E, stream); break;
    case 7: launch_enc_pc<7>(E, stream); break;
    case 8: launch_enc_pc<8>(E, stream); break;
    case 9: launch_enc_pc<9>(E, stream); break;
    case 10: launch_enc_pc<10>(E, stream); break;
    case 11: launch_enc_pc<11>(E, stream); break;
    case 12: launch_enc_pc<12>(E, stream); break;
    case 13: launch_enc_pc<13>(E, stream); break;
    case 14: launch_enc_pc<14>(E, stream); break;
    case 15: launch_enc_pc<15>(E, stream); break;
    case 16: launch_enc_pc<16>(E, stream); break;
    case 17: launch_enc_pc<17>(E, stream); break;
    default: return HM_ERR_UNSUPPORTED;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------------------------
// Decryption: bit = parity(C & z) with z_k = (X^k mod S)(0).  Wide ciphertexts (circuit outputs):
// one wavefront per value; lanes stride over the value's limbs (coalesced), accumulate per-bit
// parities, XOR-reduce.
__global__ void __launch_bounds__(256) decrypt_kernel(DecArgs D) {
    const int wave = (int)rfl(threadIdx.x >> 6);
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (e >= D.n) return;
    const int lane = lane_id();
    const uint64_t *src = D.in.limbs + e * D.in.stride;
    const uint32_t total = (uint32_t)D.in.stride;
    uint64_t m0 = 0, m1 = 0;
    // bit i of the value owns limbs [lo, hi); each lane walks its limbs in increasing order
    uint32_t i = 0, lo = 0, hi = cap_of(D.ib.b[0]);
    bool bad = false;
    for (uint32_t g = lane; g < total; g += kWave) {
        while (g >= hi) {
            ++i;
            lo = hi;
            hi += cap_of(D.ib.b[i]);
        }
        const uint64_t v = src[g];
        const uint32_t zi = g - lo;
        uint64_t z = 0;
        if (zi < D.zlimbs) z = D.z[zi];
        else if (v) bad = true;
        const uint64_t p = (uint64_t)(__builtin_popcountll(v & z) & 1);
        if (i < 64) m0 ^= p << i;
        else m1 ^= p << (i - 64);
    }
    if (__any(bad) && lane == 0) flag(D.status, HM_ERR_UNSUPPORTED);
    const uint32_t r0 = wave_xor_u32((uint32_t)m0), r1 = wave_xor_u32((uint32_t)(m0 >> 32));
    const uint32_t r2 = wave_xor_u32((uint32_t)m1), r3 = wave_xor_u32((uint32_t)(m1 >> 32));
    const uint32_t nbytes = D.nbits / 8;
    if ((uint32_t)lane < nbytes) {
        const uint32_t w = lane / 4;
        const uint32_t word = w == 0 ? r0 : w == 1 ? r1 : w == 2 ? r2 : r3;
        D.out[e * nbytes + lane] = (uint8_t)(word >> (8 * (lane % 4)));
    }
}

// Narrow ciphertexts (fresh ones: 5 limbs at d+dp = 256): one lane per ciphertext bit.  A lane
// XORs (limb & z) over its bit's limbs and takes one popcount parity; the wave's 64 parities are
// 64 consecutive plaintext bits (bit g of the flattened stream = byte g/8, bit g%8, because
// nbits = 8 nbytes), so one ballot gives 8 output bytes.  Lanes read consecutive polynomials:
// the loads stream the batch once.
__global__ void __launch_bounds__(256) decrypt_bits_kernel(DecArgs D) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = D.n * D.nbits;
    uint32_t p = 0;
    if (D.ucap) {
        // uniform caps: the wave's 64 bits are 64*C consecutive limbs (bit g at g*C).  Load them
        // coalesced into LDS, then each lane folds its own C limbs.
        __shared__ uint64_t st[256 * 8];
        const uint32_t C = D.ucap, lane = threadIdx.x & 63u;
        uint64_t *sw = st + (threadIdx.x & ~63u) * C;
        const uint64_t g0 = g - lane, lim = g0 < total ? (total - g0) * C : 0;
        const uint64_t *src = D.in.limbs + g0 * C;
        for (uint32_t j = lane; j < 64 * C; j += 64)
            if (j < lim) sw[j] = src[j];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (g < total) {
            uint64_t acc = 0;
            for (uint32_t l = 0; l < C; ++l) acc ^= sw[lane * C + l] & D.z[l];
            p = (uint32_t)__builtin_popcountll(acc) & 1u;
        }
    } else if (g < total) {
        const uint64_t e = g / D.nbits;
        const uint32_t k = (uint32_t)(g % D.nbits);
        const uint64_t *src = D.in.limbs + e * D.in.stride + D.ioff.b[k];
        const uint32_t cap = cap_of(D.ib.b[k]); // <= zlimbs (the host sizes z for the widest bit)
        uint64_t acc = 0;
        for (uint32_t l = 0; l < cap; ++l) acc ^= src[l] & D.z[l];
        p = (uint32_t)__builtin_popcountll(acc) & 1u;
    }
    const uint64_t bits = __ballot(p);
    const uint64_t g0 = g - (uint64_t)lane_id();
    if (lane_id() == 0 && g0 < total) {
        uint8_t *dst = D.out + g0 / 8;
        if (g0 + 64 <= total && ((uintptr_t)dst & 7u) == 0) {
            *(uint64_t *)dst = bits;
        } else {
            for (uint64_t b = 0; b < 8 && g0 + 8 * b < total; ++b) dst[b] = (uint8_t)(bits >> (8 * b));
        }
    }
}

int launch_decrypt(const DecArgs &D, void *stream) {
    if (D.n == 0) return 0;
    if (D.maxcap <= 32) {
        const uint64_t blocks = (D.n * D.nbits + 255) / 256;
        hipLaunchKernelGGL(decrypt_bits_kernel, dim3((unsigned)blocks), dim3(256), 0,
                           (hipStream_t)stream, D);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    const uint32_t wpb = 4u;
    const uint64_t blocks = (D.n + wpb - 1) / wpb;
    hipLaunchKernelGGL(decrypt_kernel, dim3((unsigned)blocks), dim3(64 * wpb), 0, (hipStream_t)stream, D);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------------------------
// Device CSPRNG for encryption masks: ChaCha20 (D. J. Bernstein's original layout: constants,
// 256-bit key, 64-bit block counter, 64-bit nonce), one 64-byte block per thread.  The nonce is
// read from device memory and advanced by rand_bump_kernel after the draw, so a graph replay
// never repeats a keystream.
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return __builtin_amdgcn_alignbit(x, x, 32 - r); }

#define HM_QR(a, b, c, d)                                                                          \
    a += b, d = rotl32(d ^ a, 16), c += d, b = rotl32(b ^ c, 12), a += b, d = rotl32(d ^ a, 8),   \
    c += d, b = rotl32(b ^ c, 7)

__global__ void __launch_bounds__(256) rand_fill_kernel(RandArgs R) {
    const uint64_t blk = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blk * 64 >= R.nbytes) return;
    const uint64_t nonce = *R.nonce;
    uint32_t x[16], s[16];
    s[0] = 0x61707865u, s[1] = 0x3320646eu, s[2] = 0x79622d32u, s[3] = 0x6b206574u;
#pragma unroll
    for (int i = 0; i < 8; ++i) s[4 + i] = R.key[i];
    s[12] = (uint32_t)blk, s[13] = (uint32_t)(blk >> 32);
    s[14] = (uint32_t)nonce, s[15] = (uint32_t)(nonce >> 32);
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = s[i];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        HM_QR(x[0], x[4], x[8], x[12]);
        HM_QR(x[1], x[5], x[9], x[13]);
        HM_QR(x[2], x[6], x[10], x[14]);
        HM_QR(x[3], x[7], x[11], x[15]);
        HM_QR(x[0], x[5], x[10], x[15]);
        HM_QR(x[1], x[6], x[11], x[12]);
        HM_QR(x[2], x[7], x[8], x[13]);
        HM_QR(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] += s[i];
    uint8_t *dst = R.out + blk * 64;
    if (blk * 64 + 64 <= R.nbytes && ((uintptr_t)dst & 15u) == 0) {
        uint4 *d4 = (uint4 *)dst;
#pragma unroll
        for (int i = 0; i < 4; ++i) d4[i] = make_uint4(x[4 * i], x[4 * i + 1], x[4 * i + 2], x[4 * i + 3]);
    } else {
        for (uint64_t k = 0; k < 64 && blk * 64 + k < R.nbytes; ++k)
            dst[k] = (uint8_t)(x[k / 4] >> (8 * (k % 4)));
    }
}
#undef HM_QR

__global__ void rand_bump_kernel(uint64_t *nonce) {
    if (threadIdx.x == 0) atomicAdd((unsigned long long *)nonce, 1ull);
}

int launch_random(const RandArgs &R, void *stream) {
    if (!R.nbytes) return 0;
    const uint64_t blocks = (R.nbytes + 64 * 256 - 1) / (64 * 256);
    hipLaunchKernelGGL(rand_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, R);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(rand_bump_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, R.nonce);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------------------------
// Single-polynomial primitives (unit parity for polynomial.rs).  Inputs must satisfy the layout
// invariant (bits above the degree are zero); word views of the u64 limbs are used directly.
__device__ __forceinline__ int poly_words(const uint64_t *limbs, uint32_t deg) {
    if (deg == 0 && (rfl((uint32_t)limbs[0]) & 1u) == 0) return 0;
    return nwords((int)deg);
}

__device__ void zero_tail_and_degree(uint64_t *out, uint32_t ocap, int deg, uint32_t *odeg,
                                     int written_words) {
    uint32_t *w = (uint32_t *)out;
    for (int k = written_words + lane_id(); k < (int)(2 * ocap); k += kWave) w[k] = 0u;
    if (lane_id() == 0) *odeg = (uint32_t)max(deg, 0);
}

__global__ void __launch_bounds__(256) poly_add_kernel(PolyArgs P) {
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (e >= P.n) return;
    const uint64_t *a = P.a + e * P.acap, *b = P.b + e * P.bcap;
    uint64_t *o = P.out + e * P.ocap;
    const int na = poly_words(a, rfl(P.adeg[e])), nb = poly_words(b, rfl(P.bdeg[e]));
    const int deg = wave_xor((const uint32_t *)a, na, (const uint32_t *)b, nb, (uint32_t *)o);
    zero_tail_and_degree(o, P.ocap, deg, P.odeg + e, max(na, nb));
}

__global__ void __launch_bounds__(256) poly_mul_kernel(PolyArgs P) {
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (e >= P.n) return;
    const uint64_t *a = P.a + e * P.acap, *b = P.b + e * P.bcap;
    uint64_t *o = P.out + e * P.ocap;
    const int na = poly_words(a, rfl(P.adeg[e])), nb = poly_words(b, rfl(P.bdeg[e]));
    int nout;
    int deg;
    if (na <= nb)
        deg = wave_mul<kQBig, 8>((const uint32_t *)a, na, (const uint32_t *)b, nb, nullptr, 0,
                              (uint32_t *)o, &nout);
    else
        deg = wave_mul<kQBig, 8>((const uint32_t *)b, nb, (const uint32_t *)a, na, nullptr, 0,
                              (uint32_t *)o, &nout);
    wsync();
    zero_tail_and_degree(o, P.ocap, deg, P.odeg + e, nout);
}

// Remainder by one divisor S: thread per polynomial, bitwise long division in place on the output
// (polynomial.rs:316-365: XOR S << (r_deg - deg S) while r_deg >= deg S).
__global__ void __launch_bounds__(256) poly_rem_kernel(PolyArgs P, const uint64_t *S, uint32_t sdeg) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= P.n) return;
    const uint64_t *a = P.a + e * P.acap;
    uint64_t *r = P.out + e * P.ocap;
    const uint32_t deg_a = P.adeg[e];
    for (uint32_t k = 0; k < P.ocap; ++k) r[k] = k < P.acap ? a[k] : 0ull;
    const uint32_t sl = sdeg / 64 + 1;
    int rd = (int)deg_a;
    while (rd >= (int)sdeg) {
        if ((r[rd / 64] >> (rd % 64)) & 1ull) {
            const uint32_t sh = (uint32_t)rd - sdeg, ws = sh / 64, bs = sh % 64;
            for (uint32_t k = 0; k < sl; ++k) {
                r[ws + k] ^= S[k] << bs;
                if (bs && ws + k + 1 < P.ocap) r[ws + k + 1] ^= S[k] >> (64 - bs);
            }
        }
        --rd;
    }
    // exact degree of the remainder (< sdeg)
    int d = 0;
    for (int k = (int)min(P.ocap, sl) - 1; k >= 0; --k) {
        if (r[k]) { d = k * 64 + 63 - __builtin_clzll(r[k]); break; }
    }
    P.odeg[e] = (uint32_t)d;
}

int launch_poly_add(const PolyArgs &P, void *stream) {
    if (!P.n) return 0;
    hipLaunchKernelGGL(poly_add_kernel, dim3((unsigned)((P.n + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_poly_mul(const PolyArgs &P, void *stream) {
    if (!P.n) return 0;
    hipLaunchKernelGGL(poly_mul_kernel, dim3((unsigned)((P.n + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, P);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_poly_rem(const PolyArgs &P, const uint64_t *S, uint32_t sdeg, void *stream) {
    if (!P.n) return 0;
    hipLaunchKernelGGL(poly_rem_kernel, dim3((unsigned)((P.n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, P, S, sdeg);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace hm
