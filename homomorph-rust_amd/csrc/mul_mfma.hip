// mul_mfma.hip — the multiplier's Karatsuba leaf products (mul_host.cpp "Karatsuba") on the
// gfx950 matrix cores: out = U * V over GF(2)[X] as a {0,1} Toeplitz GEMM on fp4 MFMA
// (mfma_gf2.h), replacing mul_vprod_kernel's scalar-decided VALU XORs (mul_engine.hip).
// Same products as the reference's Polynomial::mul (src/polynomial.rs:252-310): exact, so every
// bit is identical.
//
// One wavefront per (value, leaf task).  In its LDS slice the wave builds
//   RS   the bit-reversed nibble image of U over R = nu + 2 words (+ zero nibbles the last chunk's
//        window reaches),
//   VI   the nibble image of V, 16 B per word, with kVHalo zero words below and above,
//   OUT  the product's words, XOR-accumulated.
// Chunks (floor(nu/2) + 1 of K = 64) are taken in groups of kLeafG: the group's A fragments
// (kLeafG x 4 VGPRs) are built once, then every output tile of 32 words that the group reaches is
// swept, two tiles at a time (independent accumulator chains), each tile one B read per chunk.
// Each (tile, group) starts its accumulators at 2^23, so its parities are its part of the product
// mod 2; parts of different groups meet in OUT by XOR (the parity of a sum is the XOR of the
// parities of its parts).
#include <hip/hip_runtime.h>

#include "mfma_gf2.h"

namespace hm {

constexpr int kLeafG = 16;     // chunks per A group (64 VGPRs of A fragments)
constexpr int kVHalo = 64;     // zero V words below and above the image (>= 2 kLeafG + 32)
constexpr int kLeafPf = 3;     // B reads issued ahead of their MFMA

__host__ __device__ constexpr uint32_t leaf_rs_words(uint32_t umax) { return 4 * (umax + 2) + 16; }
__host__ __device__ constexpr uint32_t leaf_vi_words(uint32_t vmax) { return 4 * (vmax + 2 * kVHalo); }
__host__ __device__ constexpr uint32_t leaf_wave_words(uint32_t umax, uint32_t vmax, uint32_t omax) {
    return leaf_rs_words(umax) + leaf_vi_words(vmax) + ((omax + 3) & ~3u);
}

__device__ __forceinline__ int floor_div32(int x) { return x >= 0 ? x / 32 : -((31 - x) / 32); }

// Tiles T0 .. T1 (T1 - T0 = 1 or 2) against G chunks from c0: acc per tile, one B read per chunk
// and tile (window word 32T + col - D + h + 2c of VI), the parities XORed into OUT.
template <int G, int NT>
__device__ __forceinline__ void leaf_tiles(const v8i (&Af)[G], const uint32_t *VI, int T0, int c0,
                                           int D, uint32_t *OUT, int nout) {
    const int lane = lane_opaque(), col = lane & 31, h = lane >> 5;
    const uint4 *bt[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
        bt[t] = (const uint4 *)VI + (32 * (T0 + t) + col - D + h + 2 * c0 + kVHalo);
    v16f acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[t][j] = 8388608.0f;
    constexpr int P = G < kLeafPf ? G : kLeafPf;
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
            // keep the reads of later chunks below this MFMA (see adder_mfma.hip tile_mfma)
            asm volatile("" : "+v"(acc[t])::"memory");
        }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const uint32_t word = join_halves(acc_parities(acc[t]) << (4 * h));
        const int W = 32 * (T0 + t) + col;
        if (h == 0 && W < nout) atomicXor(&OUT[W], word); // ds_xor: this wave's words only
    }
}

// One group of G chunks from c0: A fragments once, then every tile whose window meets V's words
template <int G>
__device__ __forceinline__ void leaf_group(const uint32_t *RS, const uint32_t *VI, int R, int D, int nv,
                                           int tiles, int c0, uint32_t *OUT, int nout) {
    const int lane = lane_opaque(), col = lane & 31, h = lane >> 5;
    const int jb = 32 * (R - D + h) - 1 - col;
    const uint32_t *rw0 = RS + (jb >> 3) + 8 * c0;
    const uint32_t sh = 4u * (uint32_t)(jb & 7);
    v8i Af[G];
#pragma unroll
    for (int c = 0; c < G; ++c) Af[c] = a_fragment(rw0 + 8 * c, sh);
    // tiles whose windows (words 32T - D + 2c0 .. 32T + 31 - D + 2(c0 + G) - 1) meet [0, nv)
    const int tlo = max(0, floor_div32(D - 2 * c0 - 2 * G - 30 + 31));
    const int thi = min(tiles - 1, floor_div32(nv - 1 + D - 2 * c0));
    int T = tlo;
    for (; T + 1 <= thi; T += 2) leaf_tiles<G, 2>(Af, VI, T, c0, D, OUT, nout);
    if (T <= thi) leaf_tiles<G, 1>(Af, VI, T, c0, D, OUT, nout);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 3)))
mul_leaf_mfma_kernel(MulLeafArgs P) {
    extern __shared__ uint32_t lds[];
    uint32_t *tab = lds;
    nibble_table(tab);
    __syncthreads();
    const int wave = (int)rfl(threadIdx.x >> 6);
    const uint64_t g = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    const uint64_t e = g / P.ntasks;
    if (e >= P.B.nv) return; // whole wave exits together
    const MulVTask T = P.tasks[g % P.ntasks];
    uint32_t *arena = P.B.arena + e * P.B.astride;
    uint32_t *O = arena + T.out;
    const int nu = (int)rfl(T.nu), nv = (int)rfl(T.nv), nout = (int)rfl(T.nout);
    const int lane = lane_id();
    if (nu == 0 || nv == 0) {
        for (int w = lane; w < nout; w += kWave) O[w] = 0u;
        return;
    }
    uint32_t *RS = lds + 256 + (size_t)wave * P.wave_words;
    uint32_t *VI = RS + leaf_rs_words(P.umax);
    uint32_t *OUT = VI + leaf_vi_words(P.vmax);
    const uint32_t *U = arena + T.u, *V = arena + T.v;
    // RS: nibble word k (< 4R) = byte (k & 3) of bitreverse(U[R - 1 - k/4]) as nibbles; zeros after
    const int R = nu + 2;
    for (int k = lane; k < (int)leaf_rs_words(P.umax); k += kWave) {
        const int q = R - 1 - (k >> 2);
        const uint32_t rev = (k < 4 * R && q < nu) ? __builtin_bitreverse32(U[q]) : 0u;
        RS[k] = tab[(rev >> (8 * (k & 3))) & 0xFFu];
    }
    // VI: word w (-kVHalo <= w < nv + kVHalo) at quad w + kVHalo
    for (int k = lane; k < 4 * (nv + 2 * kVHalo); k += kWave) {
        const int w = (k >> 2) - kVHalo;
        const uint32_t v = (w >= 0 && w < nv) ? V[w] : 0u;
        VI[k] = tab[(v >> (8 * (k & 3))) & 0xFFu];
    }
    for (int w = lane; w < nout; w += kWave) OUT[w] = 0u;
    wsync();
    const int D = nu, nc = nu / 2 + 1, tiles = (nout + 31) >> 5;
    int c0 = 0;
    for (; c0 + kLeafG <= nc; c0 += kLeafG) leaf_group<kLeafG>(RS, VI, R, D, nv, tiles, c0, OUT, nout);
    for (; c0 < nc; ++c0) leaf_group<1>(RS, VI, R, D, nv, tiles, c0, OUT, nout);
    wsync();
    for (int w = lane; w < nout; w += kWave) O[w] = OUT[w];
}

int launch_mul_leaf_mfma(const MulLeafArgs &a, void *stream) {
    const uint64_t waves = a.B.nv * a.ntasks;
    if (!waves) return 0;
    const size_t lds = (256 + (size_t)a.wave_words * 4) * 4;
    hipLaunchKernelGGL(mul_leaf_mfma_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), lds,
                       (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

uint32_t mul_leaf_wave_words(uint32_t umax, uint32_t vmax, uint32_t omax) {
    return leaf_wave_words(umax, vmax, omax);
}

} // namespace hm
