// engine.h — argument blocks shared by the HIP kernels (kernels.hip) and the C-ABI host code
// (capi.cpp).  Plain structs passed to kernels by value.
#pragma once
#include <stdint.h>

#include "../../include/homomorph_gpu.h"

namespace hm {

// Per-bit-position degree bounds of a batch (cap = bound/64 + 1 limbs).  Passed by value; kernels
// derive limb offsets with a running prefix sum.
struct Bounds {
    uint32_t b[HM_MAX_BITS];
};

// Kernel timer (hm_ctx_set_kernel_timing): device wall-clock stamps of one launch, in the slot
// the host gave it (one slot per launch made or captured while timing is on, so every launch of a
// captured K-step graph has its own).  Each wave's lane 0 stamps its start into t0[w] and its end
// into t1[w] (w = the wave's index in the grid, modulo kTimerWaves; relaxed min / max atomics on
// distinct addresses, nothing waits on them); the host takes the slot's earliest start and latest end.
struct KTimer {
    unsigned long long *t0; // null: timing off
    unsigned long long *t1;
};

struct BatchArg {
    uint64_t *limbs;
    uint32_t *degree;
    uint64_t stride;  // limbs per value
    uint32_t dstride; // degree words per value (the batch's nbits; a low-bits view keeps it)
};

// Fused adder, two launches.  add_prep_kernel (several waves per value, lanes over (bit, word))
// validates the inputs and computes every per-bit product ab_i = a_i b_i and P_i = x_i (1 ^ ab_i)
// into a global workspace; add_chain_kernel (one wave per value) runs the sequential carry chain.
// Workspace per value (ws_stride words): [ab slots: nbits*cntAB][P slots: nbits*cntP]
// [deg(ab)+1: nbits][deg(P)+1: nbits].
struct AddArgs {
    BatchArg a, b, out;
    uint64_t n;
    uint32_t nbits;
    uint32_t *ws;
    uint64_t ws_stride;               // words per value
    uint32_t cntA, cntB, cntAB, cntP; // slot sizes in words (cntA = 2*max cap of a, ...)
    uint32_t cntX;                    // words of x_i = a_i ^ b_i (masked at the degrees)
    uint32_t top1;                    // prep: word cntX - 1 of every a_i, b_i, x_i is 0 or 1 (the
                                      // bounds' maximum is a multiple of 32): no product rows for it
    uint32_t wpv;                     // prep: waves per value (bits are dealt round-robin)
    uint32_t vpw;                     // prep: > 1: values per wave instead (whole values, L = 2^lgL)
    uint32_t lgL;                     // prep: log2 nbits when vpw > 1
    uint32_t prep_lds;                // prep: LDS words per wave
    uint32_t chain_lds;               // chain: LDS words per wave
    uint32_t staged;                  // chain: x, ab, P and degrees staged in LDS, carry in place
    uint32_t cw;                      // chain: carry buffer words
    uint32_t max_prod_words;          // widest carry product along the chain (picks WMAX)
    uint32_t pad;                     // carry buffers zero-padded: unchecked window reads (see capi)
    uint32_t mfma;                    // chain on the matrix cores (adder_mfma.hip): its chunk count
                                      // NC (MfmaCfg), 0 = the VALU chain
    uint32_t mf_cw;                   // MFMA chain: carry bit words (tiles, window overhang)
    int *status;
    Bounds ab, bb, ob;
    KTimer kt; // the carry-chain kernel's launches
};

struct EncArgs {
    const uint64_t *pk;     // tau * pk_cap limbs
    const uint64_t *pk_tab; // nibble table [ceil(tau/4)][limb pair][16][2] (upload_pk), or null
    const uint64_t *pk_tab1; // the same over limbs 0 .. pk_cap - 2 (top1 keys), or null
    uint32_t cus;           // compute units (grid sizing)
    uint32_t tau, pk_cap;
    const uint8_t *data;
    uint32_t nbytes;
    int lognbits;           // log2(8*nbytes) when a power of two, else -1
    uint32_t uniform_cap;   // every output bit has exactly pk_cap limbs: stores go through LDS
    const uint8_t *masks;
    BatchArg out;
    uint64_t n;
    int *status;
    Bounds ob;
    Bounds ooff;            // limb offset of each bit within a value (prefix sums of the caps)
    // every row's top limb (pk_cap - 1) is 0 or 1 (tau <= 128): that limb of a subset sum is
    // parity(mask & topcol), topcol bit i = row i's bit 64 (pk_cap - 1) (cipher.hip enc_bits_t128)
    uint32_t top1;
    uint32_t topcol[4];
    uint64_t *nonce_bump; // non-null: advance this CSPRNG nonce (the masks were just drawn)
    KTimer kt;
};

struct DecArgs {
    BatchArg in;
    uint64_t n;
    uint32_t nbits;
    const uint64_t *z; // z_k = (X^k mod S)(0), bit-packed, zlimbs limbs
    uint32_t zlimbs;
    uint8_t *out;
    int *status;
    Bounds ib;
    Bounds ioff;     // limb offset of each bit within a value (prefix sums of the caps)
    uint32_t maxcap; // widest bit (limbs): picks lane-per-bit or wave-per-value
    uint32_t ucap;   // every bit has exactly ucap <= 8 limbs (fresh ciphertexts), else 0
    KTimer kt;
};

// Gates keep their intermediates in LDS, one wavefront per value.
struct GateArgs {
    int op;
    BatchArg a, b, out;
    uint64_t n;
    uint32_t nbits;
    uint32_t lds_per_wave, oA, oB, oT;
    int *status;
    Bounds ab, bb, ob;
};

// Column-parallel carry-save multiplier (mul_engine.hip, mul_host.cpp).  Column i of
// mul_unsigned_internal (common.rs:66-105) XORs its items x_0..x_{n-1} (the partial products
// a_j b_{i-j}, then the previous column's carries) into result_i and pushes the carry
// (x_0 ^ .. ^ x_{t-1}) * x_t before each XOR.  With the prefixes p_t = x_0 ^ .. ^ x_{t-1}
// materialised (a scan), every carry of a column is an independent product p_t * x_t, so a column
// is three launches over the whole batch: partial products, prefix scan (its last prefix is the
// output bit), and the carry products, tiled over the chip.  Polynomials live in a per-value
// arena of u32 words at static offsets (slots, capacity = bound/32 + 1 rounded up to 4 words,
// always zero above the degree); deg1[slot * nv + e] = degree + 1 of value e (0 = null).
struct MulSlot {
    uint32_t off;   // u32-word offset in a value's arena
    uint32_t words; // capacity (multiple of 4)
};
struct MulBase {
    uint32_t *arena;
    uint64_t astride; // arena words per value
    uint32_t *deg1;
    uint64_t nv;      // values in this chunk (deg1 row length)
    const MulSlot *slots;
    uint64_t e0;      // first value of the chunk in the caller's batches
    int *status;
};
struct MulStageArgs {
    MulBase B;
    BatchArg a, b;
    uint32_t K;       // input bits staged: a_j -> slot j, b_j -> slot K + j
    Bounds ab, bb;
};
struct MulPPTask {
    uint32_t a, b, out, flip; // out = a * b (+1 when flip: mul_signed_internal, common.rs:123-126)
};
struct MulPPArgs {
    MulBase B;
    const MulPPTask *tasks;
    uint32_t ntasks;
};
struct MulScanArgs {
    MulBase B;
    const uint32_t *items;  // nitems slot ids, in the reference's XOR order
    const uint32_t *prefix; // nitems - 1 slot ids: p_1 .. p_{n-1}
    uint32_t nitems;
    uint32_t chunks;        // 256-word chunks per value (of the widest prefix)
    uint32_t res;           // degree slot of the result (output bit i)
    BatchArg out;
    uint32_t out_off, out_cap; // output bit i: limb offset within a value, capacity in limbs
};
struct MulProdTask {
    uint32_t u, v, out; // out = u * v; u is the operand with fewer words (the uniform one)
};
struct MulTile {
    uint32_t task, base; // output words [base, base + 64 W) of task
};
// One span of an MFMA schoolbook product, resolved on the host (mul_host.cpp build_plan): the
// operands' and the output's arena offsets and slots, so a wave's only dependent loads after this
// one record are the operands' degrees (instead of span -> task -> slots -> degrees).
struct MulSpanRec {
    uint32_t uoff, voff, ooff, nout; // arena offsets; output slot capacity (words)
    uint32_t uslot, vslot, oslot;    // slots (the operands' degrees; the output's, written)
    uint32_t base;                   // first output word of the span
};
struct MulProdArgs {
    MulBase B;
    const MulProdTask *tasks;
    const MulTile *tiles;
    uint32_t ntiles;
};
// Karatsuba products (mul_host.cpp "Karatsuba"): the big carries p_t * x_t of the deep columns
// run as a recursion over arena VIEWS (u32-word ranges of a value's arena; words past `valid`
// read as zero).  Level by level: sums of halves (KaSum), leaf products (MulVTask, schoolbook
// tiles), and recombination R = z0 + (z0 + z1 + z2) X^h + z1 X^2h (KaComb).
struct KaSum {
    uint32_t src, valid; // operand view (arena words)
    uint32_t dst;        // dst[0:h) = src[0:h) ^ src[h:2h)
};
struct KaSumArgs {
    MulBase B;
    const KaSum *t;
    uint32_t nt, h;
};
struct MulVTask {
    uint32_t u, nu, v, nv; // operand views (nu, nv valid words; 0 = null)
    uint32_t out, nout;    // out[0:nout) = U * V
    // MFMA leaves of the deepest Karatsuba level read a sum operand lo + hi as two views:
    // U = u[0:nu) ^ u2[0:nu2) (nu2 <= nu; nu2 = 0: no second view), the same for V
    uint32_t u2, nu2, v2, nv2;
};
struct MulVTile {
    uint32_t task, base;
};
struct MulVProdArgs {
    MulBase B;
    const MulVTask *tasks;
    const MulVTile *tiles;
    uint32_t ntiles;
};
// Carry products on the matrix cores (mul_mfma.hip): one wave per (value, task, span of `span`
// output tiles of 32 words; a leaf's whole output, kMfSpan tiles of a schoolbook product), U in
// blocks of kMfUB words.  Tasks are the Karatsuba leaves (MulVTask;
// nspans uniform spans per task) or the column plan's schoolbook products (MulProdTask, with an
// explicit span list {task, first output word}); vmax = the largest V of the launch (words).
constexpr int kMfUB = 256;
constexpr int kMfSpan = 16;
// the narrow class of schoolbook carries: U of at most kMfNarrowWords words, launched apart from
// the wide ones (mul_mfma_kernel<false, true>: 4 waves per SIMD), spans of at most kMfNarrowSpan
// tiles so that 16 waves' LDS slices fit a CU
#ifndef HM_MF_NARROW_WORDS
#define HM_MF_NARROW_WORDS 72
#endif
#ifndef HM_MF_NARROW_SPAN
#define HM_MF_NARROW_SPAN 10
#endif
constexpr uint32_t kMfNarrowWords = HM_MF_NARROW_WORDS;
// ... and within it the tiny class, U of at most kMfTinyWords words (the 17-word partial products
// of fresh d + d' = 512 ciphertexts and carries by them, in slots of 20 words): at most
// kMfTinyWords / 2 + 1 chunks, so its instance (mul_mfma_kernel<false, true, false, 11>) holds
// 11 A fragments, not 17, and fits more waves per SIMD (HM_MFT_WPE)
#ifndef HM_MF_TINY_WORDS
#define HM_MF_TINY_WORDS 20
#endif
constexpr uint32_t kMfTinyWords = HM_MF_TINY_WORDS;
constexpr int kMfTinyChunks = (int)kMfTinyWords / 2 + 1;
constexpr uint32_t kMfNarrowSpan = HM_MF_NARROW_SPAN;
#ifndef HM_MF_WIDE_SPAN
#define HM_MF_WIDE_SPAN 16
#endif
constexpr uint32_t kMfWideSpan = HM_MF_WIDE_SPAN; // tiles per wave of the wide class
// the wide class on the lean windowed instance (mul_mfma_kernel<false, true, true>): configs[4]
// 897.7-901.0 -> 895.4-895.5 ms per 2^20 (spans of 12 tiles: 899-904, 8: 908-909)
#ifndef HM_MF_WIDE_LEAN
#define HM_MF_WIDE_LEAN 1
#endif
constexpr bool kMfWideLean = HM_MF_WIDE_LEAN;
// Karatsuba leaves of at most kMfLeanLeafWords words run on mul_mfma_kernel<true, true> (per-group
// U windows, one tile at a time, 4 waves per SIMD): configs[4]'s 224-word leaves 916-919 -> 911-913
// ms per 2^20; K = 16's 256-word leaves measured 0.5 % slower on it (336-338 -> 338-339 ms), so
// they stay on the 3-wave instance
#ifndef HM_MF_LEAN_LEAF_WORDS
#define HM_MF_LEAN_LEAF_WORDS 224
#endif
constexpr uint32_t kMfLeanLeafWords = HM_MF_LEAN_LEAF_WORDS;
#ifndef HM_MF_LEAN_LEAF_MIN
#define HM_MF_LEAN_LEAF_MIN 193 // leaves narrower than this stay on the 3-wave instance (K = 16: 3,336-3,354 -> 3,389-3,406/s; configs[4]'s 224-word leaves unchanged)
#endif
constexpr uint32_t kMfLeanLeafMin = HM_MF_LEAN_LEAF_MIN;
struct MulMfmaArgs {
    MulBase B;
    const void *tasks;
    const MulTile *spans; // schoolbook products: {task, base}
    const MulSpanRec *recs; // ... the same spans resolved (MulSpanRec), used by the MFMA kernels
    uint32_t nitems;      // work items per value (leaves: tasks x nspans)
    uint32_t nspans;      // leaves: spans per task
    uint32_t span;        // output tiles per span
    uint32_t vmax, wave_words;
    uint32_t umax;        // largest U (words; blocks of at most kMfUB): sizes the U image
    uint32_t lean;        // leaves: the lean instance (per-group U windows, 4 waves per SIMD)
    uint32_t per_wave;    // work items per wave (set by launch_mul_mfma)
};
// Partial products grouped by their shared factor a_j (mul_mfma.hip mul_ppg_kernel): every
// a_j * b_k of the plan in one launch before the columns, one wave per (value, a_j), a_j's A
// fragments built once for all of its products (a_j within kMfPPGWords words: one chunk group).
constexpr uint32_t kMfPPGWords = 34;
// b_k words staged per batch of partial products (mul_ppg_kernel: kMfPPGBatch x 64 LDS words)
constexpr uint32_t kMfPPGBatch = 8;
struct MulPPGroup {
    uint32_t u;            // slot of a_j (the shared factor)
    uint32_t first, count; // its products: items [first, first + count)
};
struct MulPPItem {
    uint32_t v, out;       // b_k's slot, the product's slot
};
struct MulPPGArgs {
    MulBase B;
    const MulPPGroup *groups;
    const MulPPItem *items;
    uint32_t ngroups;                 // groups per value
    uint32_t umax, vmax, span;        // largest factor, other factor (words), output tiles
    uint32_t wave_words;
};
// The same partial products on the VALU by product rows (mul_engine.hip mul_ppv_kernel, the adder
// prep's method): one wave per value stages the input slots 0 .. nin - 1 into its LDS, computes
// every a_j * b_k of the plan (tasks, flattened from the groups) with lanes over (product, word of
// a_j) rows -- 16 v_mad_u64_u32 per 32x32 product, rows meeting in LDS by ds_xor -- and writes
// the products and their degrees.  For fresh operands of at most kPPVWords words (d + d' <= 256),
// where a product is only 5 MFMA chunks and the MFMA form is latency-bound (r05: 0.15 busy).
#ifndef HM_PPV_WORDS
#define HM_PPV_WORDS 12
#endif
constexpr uint32_t kPPVWords = HM_PPV_WORDS;
struct MulPPVArgs {
    MulBase B;
    const MulPPTask *tasks; // {u slot (a_j), v slot (b_k), out slot, 0}
    uint32_t ntasks;
    uint32_t nin;        // input slots staged (2 K: a_j, b_j)
    uint32_t inw;        // LDS words per staged input slot (>= every input slot's capacity)
    uint32_t qw;         // rows per product: the widest a_j (words)
    uint32_t outw;       // LDS words per product (>= qw + the widest b_k + 1)
    uint32_t wave_words; // LDS words per wave
};
// Small schoolbook carry products on the VALU by rows (mul_engine.hip mul_rows_kernel): one wave
// per value, a column's products whose operands fit kRowsU x kRowsV words (slot capacities; the
// 17 x 17 and 17 x 33-word carries of the u8 multiply's columns at d + d' = 256, MFMA "tiny" class
// before), each product's operands staged in the wave's LDS, rows (product, word of u) as in
// mul_ppv_kernel.  LDS per task: uw + vw + ow + 2 words.
#ifndef HM_ROWS_U
#define HM_ROWS_U 20
#endif
#ifndef HM_ROWS_V
#define HM_ROWS_V 36
#endif
constexpr uint32_t kRowsU = HM_ROWS_U, kRowsV = HM_ROWS_V;
struct MulRowArgs {
    MulBase B;
    const MulSpanRec *recs; // resolved tasks: u / v / out offsets, out words, slots; base =
                            // u words | v words << 16 (slot capacities)
    uint32_t ntasks;
    uint32_t uw, vw, ow;      // LDS words per task's u, v and product (slot capacities)
    uint32_t qw;              // rows per task: the widest u's words at its degree bound (<= uw)
    uint32_t wave_words;
};
constexpr uint32_t kKaNone = 0xFFFFFFFFu; // a z1 that is null (the high halves were all zero)
struct KaComb {
    uint32_t z0, z1, z2; // child results, 2h words each (z1 may be kKaNone)
    uint32_t r, rcap;    // parent result: r[0:min(4h, rcap))
};
struct KaCombArgs {
    MulBase B;
    const KaComb *t;
    uint32_t nt, h;
};
struct MulDegArgs { // deg1[out] of an exact product from its operands' deg1 (null -> 0)
    MulBase B;
    uint32_t u, v, out;
};

struct MulFinalArgs {
    MulBase B;
    const uint32_t *res; // K degree slots of the output bits
    uint32_t K;
    BatchArg out;
    Bounds ob;
};

struct PolyArgs {
    const uint64_t *a;
    const uint32_t *adeg;
    uint32_t acap;
    const uint64_t *b;
    const uint32_t *bdeg;
    uint32_t bcap;
    uint64_t *out;
    uint32_t *odeg;
    uint32_t ocap;
    uint64_t n;
    int *status;
};

// Device CSPRNG: ChaCha20 (20 rounds, 256-bit key, 64-bit block counter, 64-bit nonce read from
// *nonce and advanced by one per draw).  Block b of the draw fills bytes [64b, 64b + 64).
struct RandArgs {
    uint32_t key[8];
    uint64_t *nonce;
    uint8_t *out;
    uint64_t nbytes;
};

// host-side launchers (kernels.hip)
// bump false: the nonce is left for the caller's next launch to advance (EncArgs::nonce_bump)
int launch_random(const RandArgs &a, void *stream, bool bump = true);
int launch_add(const AddArgs &a, void *stream);
int launch_add_prep(const AddArgs &a, void *stream);
// the same add over values [e0, e0 + n) of a batch: argument block with every pointer advanced
AddArgs add_args_slice(const AddArgs &a, uint64_t e0, uint64_t n);
int launch_add_chain_mfma(const AddArgs &a, void *stream);
int launch_add_chain_valu(const AddArgs &a, void *stream);
int launch_encrypt(const EncArgs &a, void *stream);
int launch_decrypt(const DecArgs &a, void *stream);
int launch_gate(const GateArgs &a, void *stream);
int launch_mul_stage(const MulStageArgs &a, void *stream);
int launch_mul_pp(const MulPPArgs &a, void *stream);
int launch_mul_scan(const MulScanArgs &a, void *stream);
int launch_mul_prod(const MulProdArgs &a, uint32_t w, void *stream);
int launch_mul_final(const MulFinalArgs &a, void *stream);
int launch_ka_sum(const KaSumArgs &a, void *stream);
int launch_mul_vprod(const MulVProdArgs &a, uint32_t w, void *stream);
int launch_mul_mfma(const MulMfmaArgs &a, bool leaf, void *stream);
int launch_mul_ppg(const MulPPGArgs &a, void *stream);
int launch_mul_ppv(const MulPPVArgs &a, void *stream);
int launch_mul_rows(const MulRowArgs &a, void *stream);
uint32_t mul_mfma_wave_words(uint32_t vmax, uint32_t span, uint32_t umax);
uint32_t mul_mfma_lean_leaf_wave_words(uint32_t vmax, uint32_t span, uint32_t umax);
int launch_ka_comb(const KaCombArgs &a, void *stream);
int launch_mul_deg(const MulDegArgs &a, void *stream);
constexpr uint32_t kMulTileW[] = {1, 2, 4, 8, 12}; // per-lane tile widths of the product launches
int launch_poly_add(const PolyArgs &a, void *stream);
int launch_poly_mul(const PolyArgs &a, void *stream);
// The remainder table of poly_rem_kernel (kernels.hip): rows j < deg S of tcols limbs, row j's
// limb t = bits 64 (l0 + t) .. of Z_j (bit k = bit j of X^k mod S); zt = null: deg S is above
// every dividend (the remainder is the dividend)
struct RemTable {
    const uint64_t *zt;
    uint32_t rows, l0, tcols;
};
int launch_poly_rem(const PolyArgs &a, const RemTable &t, void *stream);

constexpr int kAddWavesPerBlock = 4;
constexpr uint64_t kAddPipeMin = 1024; // values per half of a pipelined add (hm_ctx_set_add_pipeline)
constexpr uint32_t kTimedLaunches = 128;  // launches hm_ctx_set_kernel_timing can record
constexpr uint32_t kTimerWaves = 32768;   // stamp pairs per launch (waves beyond share them)
// MFMA carry chain (adder_mfma.hip), one configuration per chunk count NC: P_i within 2 NC - 1
// words (NC = 7: 13 words, d + d' <= 128, configs[0]; NC = 13: 25 words, d + d' <= 256; NC = 25:
// 49 words, d + d' <= 512), nibble ring slots
// (a power of two above a tile's 32 + 2 NC word window plus the 32 words filled ahead), zero carry
// words below C (the deepest window reach), a bit's workspace record in one or two 64-word
// LDS-DMAs, and the SIMD occupancy the A fragments (4 NC VGPRs) leave.
constexpr int kMfmaRingSlots = 128;
template <int NC> struct MfmaCfg {
    static constexpr int kChunks = NC;
    static constexpr int kRevWords = 2 * NC + 2;            // > max np + 1 (jb >= 64)
    static constexpr int kRsWords = 4 * kRevWords + 8 * NC + 8;
    static constexpr int kHalo = NC <= 16 ? 32 : 64;        // >= 2 NC - 1
    static constexpr int kRecWords = NC <= 16 ? 64 : 128;
// NC = 25: 3 waves per SIMD (168 VGPRs; 23 dwords spill, all outside the tile loop): configs[4]
// 910.5-911.9 -> 902.8-905.1 ms per 2^20 against 2 waves per SIMD at 197 VGPRs (round 4)
#ifndef HM_MFMA25_WPE
#define HM_MFMA25_WPE 3
#endif
// NC = 7: its 7 A fragments leave room for more waves per SIMD (a u8 add at d + d' = 128 is a
// short chain: more waves hide its per-bit phases)
#ifndef HM_MFMA7_WPE
#define HM_MFMA7_WPE 4
#endif
    static constexpr int kWavesPerEU = NC <= 8 ? HM_MFMA7_WPE : NC <= 16 ? 4 : HM_MFMA25_WPE;
    static constexpr int kStageWords = 2 * kRecWords * kAddWavesPerBlock; // static LDS per block
    // ring slots mirrored past the end (slot s < kMirror also at kMfmaRingSlots + s), so every
    // lane's window of 2 NC - 1 slots is contiguous wherever it starts
#ifndef HM_MIRROR13
#define HM_MIRROR13 32
#endif
    // (a whole-ring mirror at NC = 13, whose two copies need no per-lane test, measured 0.5 %
    // slower: 0.5764 against 0.5726 ms per step)
    static constexpr int kMirror = NC <= 16 ? HM_MIRROR13 : 64;
    static constexpr int kRingWords = 4 * (kMfmaRingSlots + kMirror);
    static_assert(2 * NC - 1 <= kMirror, "ring mirror");
    static_assert(32 + 2 * NC + 32 <= kMfmaRingSlots, "ring window");
};
constexpr size_t kEncTableBytes = 96 * 1024; // largest encryption nibble table staged in LDS
                                              // (tau = 256 at d + dp = 512: 80 KB)

} // namespace hm
