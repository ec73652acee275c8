// mfma_gf2.h — carry-less products on the gfx950 matrix cores: the pieces shared by the adder's
// carry chain (adder_mfma.hip) and the multiplier's products (mul_mfma.hip).
//
// A GF(2)[X] product is a {0,1} convolution reduced mod 2:  bit k of U*V = (sum_j U[j] V[k-j]) mod 2.
// v_mfma_scale_f32_32x32x64_f8f6f4 with fp4 (e2m1) operands of value 0 or 1 multiplies {0,1}
// matrices exactly (products 0/1, f32 sums exact below 2^24), so a product runs as a Toeplitz GEMM.
// An output tile is 32 output words W = 32T + n (MFMA column n) x 32 bit positions m (MFMA row m);
// K runs over 64-bit windows of V, two 32-bit words per chunk c (lane half h):
//     out[32W + m] = sum_{c,h,e} A_c[m][(h,e)] * B_c[(h,e)][n]
//     A_c[m][(h,e)] = U[32(D - 2c - h) + m - e]          (a Toeplitz block of U, tile-independent)
//     B_c[(h,e)][n] = V[32(32T + n - D + 2c + h) + e]    (a window of V's words)
// with D = the words of U (output word W takes V words W - D .. W) and floor(D/2) + 1 chunks.
//
// Operand images in LDS (fp4 1.0 = 0b0010 per set bit, 8 nibbles per u32 word):
//   U  bit-reversed nibble image over R words: nibble j = U[32R - 1 - j]; lane (col, h)'s A
//      fragment of chunk c is the 32 nibbles from j0 = 32(R - D + h + 2c) - 1 - col: five words
//      read and four funnel shifts;
//   V  nibble image, 16 B per word: a B fragment is one ds_read_b128.
// tools/fp4_mfma_probe.hip pins the operand layout: lane l holds A row l%32 and B column l%32,
// element e of lane half h of A meets element e of lane half h of B, fp4 reads only the low 4
// operand VGPRs, and element e of a fragment is nibble e%8 of VGPR e/8.
//
// Parity without a reduction: an accumulator started at 2^23 holds 2^23 + count exactly, and bit 0
// of its f32 encoding is the coefficient.
#pragma once
#include <hip/hip_runtime.h>

#include "dev_common.h"

namespace hm {

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v16f mfma_fp4(const v8i &a, const v8i &b, const v16f &c) {
    // cbsz = blgp = 4: both operands fp4 e2m1; E8M0 scales 127 = 1.0
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
}

// The lane index as an opaque value: lane-derived addresses computed from it inside a loop stay
// there (hoisted out of it they are live across the whole kernel and spill)
__device__ __forceinline__ int lane_opaque() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// byte -> its 8 bits as fp4 nibbles (1.0 = 0b0010 per set bit); block-cooperative fill
__device__ __forceinline__ void nibble_table(uint32_t *tab) {
    for (uint32_t k = threadIdx.x; k < 256; k += blockDim.x) {
        uint32_t v = 0u;
#pragma unroll
        for (int t = 0; t < 8; ++t) v |= ((k >> t) & 1u) << (4 * t + 1);
        tab[k] = v;
    }
}

// A fragment of chunk c from a bit-reversed U image: 128-bit window of nibbles starting at j0
// = jb + 64c (rw0 = image + (jb >> 3), sh = 4 (jb & 7))
__device__ __forceinline__ v8i a_fragment(const uint32_t *rw, uint32_t sh) {
    const uint32_t w0 = rw[0], w1 = rw[1], w2 = rw[2], w3 = rw[3], w4 = rw[4];
    return (v8i){(int)funnel(w1, w0, sh), (int)funnel(w2, w1, sh), (int)funnel(w3, w2, sh),
                 (int)funnel(w4, w3, sh), 0, 0, 0, 0};
}

__device__ __forceinline__ v8i b_fragment(const uint4 &q) {
    return (v8i){(int)q.x, (int)q.y, (int)q.z, (int)q.w, 0, 0, 0, 0};
}

// Row-permuted tiles (the adder's chain and the multiplier's products): A row m computes output bit row_bit(m) instead of bit m,
// so that lane (col, h)'s accumulator j (D row (j&3) + 8(j>>2) + 4h) holds output bit j + 16h and
// a lane's 16 parities are one contiguous half word: 15 funnel shifts gather them, with no
// per-nibble shifts and ORs (round 4: 26 -> 20 VALU per tile; headline -0.4 %, configs[4]
// -1.5 %, K = 16 -1.1 %).  The A fragments only read their operand from a permuted start.
__host__ __device__ constexpr int row_bit(int m) { return (m & 3) + 4 * (m >> 3) + 16 * ((m >> 2) & 1); }
// bit 16 + j = bit 0 of accumulator j (j = 0..15); bits 0..15 zero
__device__ __forceinline__ uint32_t acc_parities_hi16(const v16f &acc) {
    uint32_t x = __float_as_uint(acc[0]) << 31;
#pragma unroll
    for (int j = 1; j < 16; ++j) x = funnel(__float_as_uint(acc[j]), x, 1);
    return x;
}

// Lane halves joined: lane (col, h) holds its half's bits in place (bits 16h .. 16h + 15); one
// v_permlane32_swap brings the other half's, and both halves return output word col.
__device__ __forceinline__ uint32_t join_halves(uint32_t t_shifted) {
    const auto sw = __builtin_amdgcn_permlane32_swap(t_shifted, t_shifted, false, false);
    return sw[0] | sw[1];
}

} // namespace hm
