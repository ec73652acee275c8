// kernels.hip — gfx950 kernels of the gates and the single-polynomial primitives:
//   gate_kernel     elementwise AND/OR/XOR/NOT (common.rs:5-35)
//   poly_* kernels  single-polynomial primitives for unit parity (polynomial.rs:190-365)
// (adder: adder.hip; cipher: cipher.hip; carry-save multiplier: mul_engine.hip)
#include <hip/hip_runtime.h>

#include "dev_common.h"

namespace hm {

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
// Single-polynomial primitives (unit parity for polynomial.rs).  Inputs must satisfy the layout
// invariant (bits above the degree are zero); word views of the u64 limbs are used directly.
__device__ __forceinline__ int poly_words(const uint64_t *limbs, uint32_t deg) {
    if (deg == 0 && (rfl((uint32_t)limbs[0]) & 1u) == 0) return 0;
    return nwords((int)deg);
}

__device__ __forceinline__ void zero_tail_and_degree(uint64_t *out, uint32_t ocap, int deg, uint32_t *odeg,
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

// Remainder by one divisor S (polynomial.rs:316-365) as a table remainder:
// C mod S = XOR over the set bits k of C of (X^k mod S), so remainder bit j is the parity of
// C AND Z_j, where bit k of the row Z_j is bit j of X^k mod S.  The same linear functional as the
// decrypt table (row j = 0), for every bit of the remainder; identical to the long division's
// remainder, which is unique.  For k < deg S, X^k mod S = X^k: those columns are the identity, so
// the host table (zt, built in hm_poly_rem_batch) holds rows j < deg S over the limbs from
// l0 = deg S / 64 on only (tcols = acap - l0 limbs per row), and remainder word w < l0 starts as
// C's limb w.  zt = null: the divisor is above every dividend's degree, the remainder is C.
// One wave per polynomial: lanes hold C's first 512 limbs in registers (limbs past them are
// re-read from memory for every row, so any dividend size is accepted, as polynomial.rs:316-365
// accepts it), one ballot per remainder bit gives its parity.
constexpr int kRemLimbsPerLane = 8; // limbs held in registers: 512 (32768 coefficients)

__global__ void __launch_bounds__(256) poly_rem_kernel(PolyArgs P, RemTable T) {
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + rfl(threadIdx.x >> 6);
    if (e >= P.n) return;
    const int lane = lane_id();
    const uint64_t *a = P.a + e * P.acap;
    uint64_t *r = P.out + e * P.ocap;
    const uint32_t adeg = rfl(P.adeg[e]);
    const int na = poly_words(a, adeg) ? (int)(adeg / 64 + 1) : 0;
    if (!T.zt) { // deg S above every dividend: C mod S = C
        for (int k = lane; k < (int)P.ocap; k += kWave) r[k] = k < na ? a[k] : 0ull;
        if (lane == 0) P.odeg[e] = na ? adeg : 0u;
        return;
    }
    const int l0 = (int)T.l0;
    uint64_t c[kRemLimbsPerLane];
#pragma unroll
    for (int t = 0; t < kRemLimbsPerLane; ++t) {
        const int k = lane + kWave * t;
        c[t] = k >= l0 && k < na ? a[k] : 0ull;
    }
    // remainder bits, 64 at a time: lane j%64 keeps word j/64's bit j%64; degree < deg S
    const int rl = min((int)(T.rows + 63) / 64, (int)P.ocap);
    int top = -1;
    for (int w = 0; w < rl; ++w) {
        uint64_t word = w < l0 && w < na ? a[w] : 0ull; // the identity columns (wave-uniform)
        for (int jb = 0; jb < 64 && 64 * w + jb < (int)T.rows; ++jb) {
            const uint64_t *z = T.zt + (size_t)(64 * w + jb) * T.tcols - l0; // z[k], k >= l0
            uint32_t par = 0u;
#pragma unroll
            for (int t = 0; t < kRemLimbsPerLane; ++t) {
                const int k = lane + kWave * t;
                if (k >= l0 && k < na) par ^= (uint32_t)__popcll(c[t] & z[k]);
            }
            for (int k = max(kWave * kRemLimbsPerLane, l0) + lane; k < na; k += kWave)
                par ^= (uint32_t)__popcll(a[k] & z[k]);
            const uint64_t m = __ballot(par & 1u);
            word ^= (uint64_t)(__popcll(m) & 1) << jb;
        }
        if (lane == 0) r[w] = word; // word is wave-uniform
        if (word) top = 64 * w + 63 - __builtin_clzll(word);
    }
    for (int k = rl + lane; k < (int)P.ocap; k += kWave) r[k] = 0ull;
    if (lane == 0) P.odeg[e] = (uint32_t)max(top, 0);
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
int launch_poly_rem(const PolyArgs &P, const RemTable &T, void *stream) {
    if (!P.n) return 0;
    hipLaunchKernelGGL(poly_rem_kernel, dim3((unsigned)((P.n + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, P, T);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace hm
