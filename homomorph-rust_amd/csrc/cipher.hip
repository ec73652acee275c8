// cipher.hip — gfx950 kernels of the per-bit cipher (src/cipher.rs):
//   encrypt_table_kernel / encrypt_kernel   subset sums of the public key (cipher.rs:99-115)
//   decrypt_bits_kernel / decrypt_kernel    (C mod S)(0) as the parity functional
//                                           sum_k c_k z_k, z_k = (X^k mod S)(0) (cipher.rs:119-122)
//   rand_fill_kernel                        the mask CSPRNG (device ChaCha20; cipher.rs:92-97)
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dev_common.h"

namespace hm {

// ---------------------------------------------------------------------------------------------
// Encryption: one lane per ciphertext bit.  C = XOR_{i : mask bit i} T_i, then C ^= x
// (CipheredBit::cipher, cipher.rs:99-115; Ciphered::try_cipher bit order :180-185).  The public
// key T_i is read with wave-uniform addresses (scalar loads); the mask select is one bitop3
// (acc ^ (t & m)) per 32-bit half.
// The draw that made this launch's masks left its nonce for the encryption to advance (one plain
// store by one thread: nothing in the encryption reads the nonce), saving a launch per encrypt
__device__ __forceinline__ void enc_nonce_bump(const EncArgs &E) {
    if (E.nonce_bump && blockIdx.x == 0 && threadIdx.x == 0) *E.nonce_bump += 1;
}

template <int PC>
__global__ void __launch_bounds__(256) encrypt_kernel(EncArgs E) {
    kt_start(E.kt);
    enc_nonce_bump(E);
    const uint32_t nbits = E.nbytes * 8;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= E.n * nbits) {
        kt_finish(E.kt);
        return;
    }
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
    kt_finish(E.kt);
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

// Two lookups (groups g, g + 1) folded into the 32-bit halves of PC limbs with one three-input
// v_bitop3 XOR each (the compiler splits a ^ b ^ c into two XORs here).  An odd PC's last pair
// holds one live limb: read as 8 B (ds_read_b64, 2 LDS cycles instead of 4) at the same address.
// NP: limb pairs per table group (the table may hold limbs past the PC looked up here).
template <int PC, int NP = (PC + 1) / 2>
__device__ __forceinline__ void enc_lookup2(uint32_t *acc, const uint4 *tab4, uint32_t g,
                                            uint32_t nib0, uint32_t nib1) {
    const uint4 *r0 = tab4 + (size_t)g * NP * 16 + nib0, *r1 = tab4 + (size_t)(g + 1) * NP * 16 + nib1;
#pragma unroll
    for (int p = 0; p < PC / 2; ++p) {
        const uint4 a = r0[p * 16], b = r1[p * 16];
        acc[4 * p] = __builtin_amdgcn_bitop3_b32(acc[4 * p], a.x, b.x, 0x96);
        acc[4 * p + 1] = __builtin_amdgcn_bitop3_b32(acc[4 * p + 1], a.y, b.y, 0x96);
        acc[4 * p + 2] = __builtin_amdgcn_bitop3_b32(acc[4 * p + 2], a.z, b.z, 0x96);
        acc[4 * p + 3] = __builtin_amdgcn_bitop3_b32(acc[4 * p + 3], a.w, b.w, 0x96);
    }
    if constexpr (PC % 2) {
        const uint2 a = *(const uint2 *)&r0[(PC / 2) * 16], b = *(const uint2 *)&r1[(PC / 2) * 16];
        acc[2 * PC - 2] = __builtin_amdgcn_bitop3_b32(acc[2 * PC - 2], a.x, b.x, 0x96);
        acc[2 * PC - 1] = __builtin_amdgcn_bitop3_b32(acc[2 * PC - 1], a.y, b.y, 0x96);
    }
}

#ifndef HM_ENC_NT
#define HM_ENC_NT 0 // non-temporal ciphertext stores (A/B knob)
#endif
#ifndef HM_ENC_LDS_DEPTH
#define HM_ENC_LDS_DEPTH 0 // (A/B knob) lookups per read batch in enc_bits_t128; 0: compiler's
#endif
// The wave's 64 ciphertext bits t0 .. t0 + 63 once their subset sums are in acc: the plaintext
// bit, the degree, and the stores (uniform caps: the wave's 64 * PC consecutive output limbs,
// transposed through its LDS stage and stored coalesced; otherwise per bit at its offset)
// sob / sooff: LDS copies of E.ob / E.ooff (the lane's bit k indexes them; a by-value argument
// array is never indexed per lane, dev_common.h)
template <int PC>
__device__ __forceinline__ void enc_finish(const EncArgs &E, uint64_t *acc, uint64_t *st,
                                           const uint32_t *sob, const uint32_t *sooff,
                                           uint64_t t0, uint64_t total, bool live, uint64_t e,
                                           uint32_t k, uint32_t nbits) {
    const uint32_t lane = threadIdx.x & 63u;
    // mask bits at or above tau select nothing: the table rows past tau are zero, and the
    // reference reads exactly ceil(tau/8) bytes, bits >= tau unused (cipher.rs:105-110)
    acc[0] ^= (E.data[e * E.nbytes + k / 8] >> (k % 8)) & 1u; // add_bool_assign (:112)
    int deg = 0;
#pragma unroll
    for (int l = 0; l < PC; ++l)
        if (acc[l]) deg = l * 64 + 63 - __builtin_clzll(acc[l]);
    if (live) {
        if ((uint32_t)deg > sob[k]) flag(E.status, HM_ERR_CAPACITY);
        E.out.degree[e * nbits + k] = (uint32_t)deg;
    }
    if (E.uniform_cap) {
        // limb l of bit t at t*PC + l: lane j writes limb j, j + 64, ...
#pragma unroll
        for (int l = 0; l < PC; ++l) st[lane * PC + l] = acc[l];
        wsync();
        const uint64_t lim = (total - t0) * PC;
        uint64_t *dst = E.out.limbs + t0 * PC;
#pragma unroll
        for (int r = 0; r < PC; ++r) {
            const uint32_t j = lane + 64 * r;
#if HM_ENC_NT
            if (j < lim) __builtin_nontemporal_store(st[j], dst + j);
#else
            if (j < lim) dst[j] = st[j];
#endif
        }
        wsync();
    } else if (live) {
        const uint32_t cap = cap_of(sob[k]);
        uint64_t *dst = E.out.limbs + e * E.out.stride + sooff[k];
#pragma unroll
        for (int l = 0; l < PC; ++l) {
            if ((uint32_t)l < cap) dst[l] = acc[l];
            else if (acc[l]) flag(E.status, HM_ERR_CAPACITY);
        }
        for (uint32_t l = PC; l < cap; ++l) dst[l] = 0ull;
    }
}

// tau = 128 (one 16-byte mask per ciphertext bit, 32 nibble groups): the lane's subset sum from its
// mask mw, fully unrolled, then enc_finish.  TOP1: every public-key row's top limb (PC - 1) is 0 or
// 1 -- rows of degree <= 64 (PC - 1), i.e. d + dp a multiple of 64 (the bench's 256, configs[4]'s
// 512) -- so that limb of the subset sum is one bit, parity(mask & E.topcol) with topcol bit i =
// row i's bit 64 (PC - 1): five VALU instead of 32 table reads of 8 B and 32 XORs per ciphertext
// bit (a fifth of the LDS traffic at PC = 5).
template <int PC, bool TOP1>
constexpr int kEncTabPairs = ((TOP1 ? PC - 1 : PC) + 1) / 2; // limb pairs per group of the table read

template <int PC, bool TOP1>
__device__ __forceinline__ void enc_bits_t128(const EncArgs &E, const uint4 *tab4, uint64_t *st,
                                              const uint32_t *sob, const uint32_t *sooff,
                                              uint64_t t0, uint64_t total, uint32_t nbits,
                                              const uint4 &mw) {
    constexpr int PL = TOP1 ? PC - 1 : PC;      // limbs looked up (TOP1: E.pk_tab1, without the top)
    constexpr int NP = kEncTabPairs<PC, TOP1>; // the table's limb pairs per group
    const uint32_t lane = threadIdx.x & 63u;
    const bool live = t0 + lane < total;
    const uint64_t t = live ? t0 + lane : total - 1;
    const uint64_t e = E.lognbits >= 0 ? t >> E.lognbits : t / nbits;
    const uint32_t k = (uint32_t)(t - e * nbits);
    uint32_t a32[2 * PC];
#pragma unroll
    for (int l = 0; l < 2 * PC; ++l) a32[l] = 0u;
    const uint32_t ws[4] = {mw.x, mw.y, mw.z, mw.w};
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
            enc_lookup2<PL, NP>(a32, tab4, 8 * w + j, (ws[w] >> (4 * j)) & 15u, (ws[w] >> (4 * j + 4)) & 15u);
#if HM_ENC_LDS_DEPTH
            // (knob) keep the reads of the next lookups below this point
            if (j % (2 * HM_ENC_LDS_DEPTH) == 2 * HM_ENC_LDS_DEPTH - 2) asm volatile("" ::: "memory");
#endif
        }
    if constexpr (TOP1) {
        const uint32_t x = (mw.x & E.topcol[0]) ^ (mw.y & E.topcol[1]) ^ (mw.z & E.topcol[2]) ^
                           (mw.w & E.topcol[3]);
        a32[2 * PC - 2] = (uint32_t)__builtin_popcount(x) & 1u;
    }
    uint64_t acc[PC];
#pragma unroll
    for (int l = 0; l < PC; ++l) acc[l] = (uint64_t)a32[2 * l] | ((uint64_t)a32[2 * l + 1] << 32);
    enc_finish<PC>(E, acc, st, sob, sooff, t0, total, live, e, k, nbits);
}

// Copies a nibble table (G groups of NP limb pairs) into the block's LDS
template <int NP>
__device__ __forceinline__ void enc_table_to_lds(const uint64_t *ptab, uint32_t G, uint64_t *tab) {
    const uint32_t n16 = G * NP * 16; // 16-byte chunks
    const uint4 *src = (const uint4 *)ptab;
    uint4 *dst = (uint4 *)tab;
    for (uint32_t f = threadIdx.x; f < n16; f += blockDim.x) dst[f] = src[f];
    __syncthreads();
}

// GC: compile-time group count (tau/4) for the fully unrolled path with 16-byte-aligned masks
// (tau = 128: one uint4 of mask per ciphertext bit, read one iteration ahead), 0 = any tau
#ifndef HM_ENC_TAB_WPE
#define HM_ENC_TAB_WPE 7 // (A/B knob) waves per SIMD of the table kernel
#endif
template <int PC, int GC, bool TOP1 = false>
__global__ void __launch_bounds__(kEncBlock) __attribute__((amdgpu_waves_per_eu(HM_ENC_TAB_WPE)))
encrypt_table_kernel(EncArgs E) {
    kt_start(E.kt);
    enc_nonce_bump(E);
    constexpr int NP = kEncTabPairs<PC, TOP1>; // limb pairs (TOP1: the table without the top limb)
    extern __shared__ uint64_t tab[];          // [G][NP][16][2] (upload_pk)
    const uint32_t G = GC ? GC : (E.tau + 3) / 4;
    uint64_t *stage = tab + (size_t)G * NP * 32; // [waves][64][PC] store transpose
    uint64_t *st = stage + (size_t)(threadIdx.x & ~63u) * PC;
    const uint32_t nbits = E.nbytes * 8;
    // [HM_MAX_BITS] bounds, [HM_MAX_BITS] limb offsets per bit (after the transposes)
    uint32_t *sob = (uint32_t *)(stage + (size_t)kEncBlock * PC), *sooff = sob + HM_MAX_BITS;
    if (threadIdx.x < 64) {
        arg_to_lds(E.ob.b, nbits, sob);
        arg_to_lds(E.ooff.b, nbits, sooff);
    }
    enc_table_to_lds<NP>(TOP1 ? E.pk_tab1 : E.pk_tab, G, tab); // (its __syncthreads orders sob too)
    const uint4 *tab4 = (const uint4 *)tab;
    const uint32_t mb = (E.tau + 7) / 8;
    const uint64_t total = E.n * nbits;
    // the loop runs per wave (the store transpose is wave-cooperative): lanes past the end of
    // the batch compute on a clamped index and are masked out of every store
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t first = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u);
    if constexpr (GC != 0) {
        static_assert(GC == 32, "GC: tau = 128");
        const uint4 *m4 = (const uint4 *)E.masks;
        uint4 mw = first < total ? m4[min(first + lane, total - 1)] : make_uint4(0, 0, 0, 0);
        for (uint64_t t0 = first; t0 < total; t0 += step) {
            const uint4 cur = mw;
            if (t0 + step < total) mw = m4[min(t0 + step + lane, total - 1)]; // next iteration's
            enc_bits_t128<PC, TOP1>(E, tab4, st, sob, sooff, t0, total, nbits, cur);
        }
    } else {
        for (uint64_t t0 = first; t0 < total; t0 += step) {
            const bool live = t0 + lane < total;
            const uint64_t t = live ? t0 + lane : total - 1;
            const uint64_t e = E.lognbits >= 0 ? t >> E.lognbits : t / nbits;
            const uint32_t k = (uint32_t)(t - e * nbits);
            const uint8_t *m = E.masks + t * mb;
            uint64_t acc[2 * NP];
#pragma unroll
            for (int l = 0; l < 2 * NP; ++l) acc[l] = 0;
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
            enc_finish<PC>(E, acc, st, sob, sooff, t0, total, live, e, k, nbits);
        }
    }
    kt_finish(E.kt);
}

// ChaCha20 block blk of (key, nonce) (D. J. Bernstein's original layout: constants, 256-bit key,
// 64-bit block counter, 64-bit nonce): keystream bytes 64 blk .. 64 blk + 63, little-endian words
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return __builtin_amdgcn_alignbit(x, x, 32 - r); }

#define HM_QR(a, b, c, d)                                                                          \
    a += b, d = rotl32(d ^ a, 16), c += d, b = rotl32(b ^ c, 12), a += b, d = rotl32(d ^ a, 8),   \
    c += d, b = rotl32(b ^ c, 7)

__device__ __forceinline__ void chacha20_init(const uint32_t (&key)[8], uint64_t blk, uint64_t nonce,
                                              uint32_t (&s)[16]) {
    s[0] = 0x61707865u, s[1] = 0x3320646eu, s[2] = 0x79622d32u, s[3] = 0x6b206574u;
#pragma unroll
    for (int i = 0; i < 8; ++i) s[4 + i] = key[i];
    s[12] = (uint32_t)blk, s[13] = (uint32_t)(blk >> 32);
    s[14] = (uint32_t)nonce, s[15] = (uint32_t)(nonce >> 32);
}

// n double rounds (column + diagonal quarter rounds) of the ChaCha state x
template <int N>
__device__ __forceinline__ void chacha20_rounds(uint32_t (&x)[16]) {
#pragma unroll
    for (int r = 0; r < N; ++r) {
        HM_QR(x[0], x[4], x[8], x[12]);
        HM_QR(x[1], x[5], x[9], x[13]);
        HM_QR(x[2], x[6], x[10], x[14]);
        HM_QR(x[3], x[7], x[11], x[15]);
        HM_QR(x[0], x[5], x[10], x[15]);
        HM_QR(x[1], x[6], x[11], x[12]);
        HM_QR(x[2], x[7], x[8], x[13]);
        HM_QR(x[3], x[4], x[9], x[14]);
    }
}

__device__ __forceinline__ void chacha20_block(const uint32_t (&key)[8], uint64_t blk, uint64_t nonce,
                                               uint32_t (&x)[16]) {
    uint32_t s[16];
    chacha20_init(key, blk, nonce, s);
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = s[i];
    chacha20_rounds<10>(x);
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] += s[i];
}
#undef HM_QR

template <int PC>
static void launch_enc_pc(const EncArgs &E, void *stream) {
    const uint64_t threads = E.n * E.nbytes * 8;
    const size_t tab = (size_t)((E.tau + 3) / 4) * ((PC + 1) / 2) * 16 * 16;
    const size_t tab1 = (size_t)((E.tau + 3) / 4) * (PC / 2) * 16 * 16; // (top1: without the top limb)
    const bool t1 = E.tau == 128 && ((uintptr_t)E.masks & 15u) == 0 && E.top1 && PC > 1;
    // + the store transpose + the per-bit bounds and offsets
    const size_t lds = (t1 ? tab1 : tab) + (size_t)kEncBlock * PC * 8 + 2 * HM_MAX_BITS * 4;
    if (E.pk_tab && tab <= kEncTableBytes && lds <= 160 * 1024) { // one CU's LDS at most
        // a few resident blocks per CU, each striding over bits (the table copy is amortised)
        const uint64_t want = (threads + kEncBlock - 1) / kEncBlock;
        const uint64_t per_cu = std::max<uint64_t>(1, std::min<uint64_t>(4, (160 * 1024) / lds));
        const uint64_t blocks = std::min<uint64_t>(want, (uint64_t)E.cus * per_cu);
        if (t1)
            hipLaunchKernelGGL((encrypt_table_kernel<PC, 32, (PC > 1)>), dim3((unsigned)blocks),
                               dim3(kEncBlock), lds, (hipStream_t)stream, E);
        else if (E.tau == 128 && ((uintptr_t)E.masks & 15u) == 0)
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
// one wavefront per value.  The bits are walked in a uniform loop; the lanes stride over the bit's
// limbs (contiguous, so the loads coalesce) with kDecUnroll independent accumulators (that many
// limb + z load pairs in flight per lane), and the bit is the parity of the ballot of the lanes'
// parities.  No lane-dependent control flow besides the strided bounds: every lane runs the same
// bit loop (an earlier form walked a per-lane bit cursor through the flattened limbs; its
// data-dependent inner loops compiled into a schedule that read some limbs wrongly once an
// unrelated argument field was added -- kept out of the way of such codegen).
constexpr uint32_t kDecUnroll = 4;
static_assert(kDecUnroll == 4, "the accumulator fold below names four");
__global__ void __launch_bounds__(256) decrypt_kernel(DecArgs D) {
    kt_start(D.kt);
    const int wave = (int)rfl(threadIdx.x >> 6);
    const uint64_t e = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    if (e < D.n) { // whole wave together
        const uint32_t lane = (uint32_t)lane_id();
        const uint64_t *src = D.in.limbs + e * D.in.stride;
        uint64_t m0 = 0, m1 = 0; // plaintext bits 0..63, 64..127 (wave-uniform)
        bool bad = false;
        for (uint32_t i = 0; i < D.nbits; ++i) {
            const uint32_t cap = cap_of(D.ib.b[i]);
            const uint64_t *p = src + D.ioff.b[i];
            uint64_t acc[kDecUnroll];
#pragma unroll
            for (uint32_t u = 0; u < kDecUnroll; ++u) acc[u] = 0;
            uint32_t k = lane;
            for (; k + (kDecUnroll - 1) * kWave < cap; k += kDecUnroll * kWave) {
                uint64_t v[kDecUnroll], z[kDecUnroll];
#pragma unroll
                for (uint32_t u = 0; u < kDecUnroll; ++u) v[u] = p[k + u * kWave];
#pragma unroll
                for (uint32_t u = 0; u < kDecUnroll; ++u) {
                    const uint32_t kz = k + u * kWave;
                    z[u] = kz < D.zlimbs ? D.z[kz] : 0ull;
                    bad |= kz >= D.zlimbs && v[u] != 0;
                }
#pragma unroll
                for (uint32_t u = 0; u < kDecUnroll; ++u) acc[u] ^= v[u] & z[u];
            }
            for (; k < cap; k += kWave) {
                const uint64_t v = p[k];
                acc[0] ^= v & (k < D.zlimbs ? D.z[k] : 0ull);
                bad |= k >= D.zlimbs && v != 0;
            }
            const uint64_t a = (acc[0] ^ acc[1]) ^ (acc[2] ^ acc[3]);
            const uint64_t par = __ballot(__builtin_popcountll(a) & 1);
            const uint64_t bit = (uint64_t)(__builtin_popcountll(par) & 1);
            if (i < 64) m0 |= bit << i;
            else m1 |= bit << (i - 64);
        }
        if (__any(bad) && lane == 0) flag(D.status, HM_ERR_UNSUPPORTED);
        const uint32_t nbytes = D.nbits / 8;
        if (lane < nbytes) {
            const uint64_t w = lane < 8 ? m0 : m1;
            D.out[e * nbytes + lane] = (uint8_t)(w >> (8 * (lane & 7)));
        }
    }
    kt_finish(D.kt);
}

// Narrow ciphertexts (fresh ones: 5 limbs at d+dp = 256): one lane per ciphertext bit.  A lane
// XORs (limb & z) over its bit's limbs and takes one popcount parity; the wave's 64 parities are
// 64 consecutive plaintext bits (bit g of the flattened stream = byte g/8, bit g%8, because
// nbits = 8 nbytes), so one ballot gives 8 output bytes.  Lanes read consecutive polynomials:
// the loads stream the batch once.
__global__ void __launch_bounds__(256) decrypt_bits_kernel(DecArgs D) {
    kt_start(D.kt);
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
#ifndef HM_DECB_REGS
#define HM_DECB_REGS 1 // (A/B knob) 0: a load -> LDS store loop (one load in flight per lane)
#endif
        if (HM_DECB_REGS) {
            // all C (<= 8) loads of the lane in flight together, then the LDS stores
            uint64_t v[8];
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u) {
                const uint32_t j = lane + 64u * u;
                v[u] = (u < C && j < lim) ? src[j] : 0ull;
            }
#pragma unroll
            for (uint32_t u = 0; u < 8; ++u)
                if (u < C) sw[lane + 64u * u] = v[u];
        } else {
            for (uint32_t j = lane; j < 64 * C; j += 64)
                if (j < lim) sw[j] = src[j];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (g < total) {
            uint64_t acc = 0;
            for (uint32_t l = 0; l < C; ++l) acc ^= sw[lane * C + l] & D.z[l];
            p = (uint32_t)__builtin_popcountll(acc) & 1u;
        }
    } else {
        // lane-varying bit k: its bound and limb offset from LDS copies of D.ib / D.ioff (a
        // by-value argument array is never indexed per lane, dev_common.h)
        __shared__ __attribute__((aligned(16))) uint32_t sb[2 * HM_MAX_BITS];
        if (threadIdx.x < 64) {
            arg_to_lds(D.ib.b, D.nbits, sb);
            arg_to_lds(D.ioff.b, D.nbits, sb + HM_MAX_BITS);
        }
        __syncthreads();
        if (g < total) {
            const uint64_t e = g / D.nbits;
            const uint32_t k = (uint32_t)(g % D.nbits);
            const uint64_t *src = D.in.limbs + e * D.in.stride + sb[HM_MAX_BITS + k];
            const uint32_t cap = cap_of(sb[k]); // <= zlimbs (the host sizes z for the widest bit)
            uint64_t acc = 0;
            for (uint32_t l = 0; l < cap; ++l) acc ^= src[l] & D.z[l];
            p = (uint32_t)__builtin_popcountll(acc) & 1u;
        }
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
    kt_finish(D.kt);
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
// Device CSPRNG for encryption masks: ChaCha20 (chacha20_block above), one 64-byte block per
// thread.  The nonce is read from device memory and advanced by rand_bump_kernel after the draw,
// so a graph replay never repeats a keystream.
#ifndef HM_RAND_BLOCKS
#define HM_RAND_BLOCKS 1 // keystream blocks per thread, computed together (A/B knob: ILP)
#endif
constexpr int kRandBlocks = HM_RAND_BLOCKS;
__global__ void __launch_bounds__(256) rand_fill_kernel(RandArgs R) {
    const uint64_t b0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kRandBlocks;
    if (b0 * 64 >= R.nbytes) return;
    const uint64_t nonce = *R.nonce;
    uint32_t s[kRandBlocks][16], x[kRandBlocks][16];
#pragma unroll
    for (int q = 0; q < kRandBlocks; ++q) {
        chacha20_init(R.key, b0 + q, nonce, s[q]);
#pragma unroll
        for (int i = 0; i < 16; ++i) x[q][i] = s[q][i];
    }
#pragma unroll
    for (int r = 0; r < 10; ++r)
#pragma unroll
        for (int q = 0; q < kRandBlocks; ++q) chacha20_rounds<1>(x[q]);
#pragma unroll
    for (int q = 0; q < kRandBlocks; ++q) {
        const uint64_t blk = b0 + q;
        if (blk * 64 >= R.nbytes) break;
#pragma unroll
        for (int i = 0; i < 16; ++i) x[q][i] += s[q][i];
        uint8_t *dst = R.out + blk * 64;
        if (blk * 64 + 64 <= R.nbytes && ((uintptr_t)dst & 15u) == 0) {
            uint4 *d4 = (uint4 *)dst;
#pragma unroll
            for (int i = 0; i < 4; ++i) d4[i] = make_uint4(x[q][4 * i], x[q][4 * i + 1], x[q][4 * i + 2], x[q][4 * i + 3]);
        } else {
            for (uint64_t k = 0; k < 64 && blk * 64 + k < R.nbytes; ++k)
                dst[k] = (uint8_t)(x[q][k / 4] >> (8 * (k % 4)));
        }
    }
}

__global__ void rand_bump_kernel(uint64_t *nonce) {
    if (threadIdx.x == 0) atomicAdd((unsigned long long *)nonce, 1ull);
}

int launch_random(const RandArgs &R, void *stream, bool bump) {
    if (!R.nbytes) return 0;
    const uint64_t blocks = (R.nbytes + 64 * 256 * kRandBlocks - 1) / (64 * 256 * kRandBlocks);
    hipLaunchKernelGGL(rand_fill_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, R);
    if (hipGetLastError() != hipSuccess) return -1;
    if (!bump) return 0; // the caller's next launch advances the nonce (EncArgs::nonce_bump)
    hipLaunchKernelGGL(rand_bump_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, R.nonce);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace hm
