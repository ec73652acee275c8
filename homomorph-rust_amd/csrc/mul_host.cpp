// mul_host.cpp — host side of the column-parallel carry-save multiplier (mul_engine.hip).
//
// A plan is the symbolic run of mul_unsigned_internal / mul_signed_internal
// (src/impls/numbers/common.rs:66-155) over static degree bounds: every polynomial the reference
// builds gets a slot (a static offset in a per-value arena of u32 words, capacity from its bound)
// and a degree slot, and every column becomes three launches over the whole batch:
//   partial products  pp_j = a_j * b_{i-j}              (j = 0..i; +1 at the signed corners)
//   prefix scan       p_t = x_0 ^ .. ^ x_{t-1}, result_i = p_n (written to the output bit)
//   carry products    c_t = p_t * x_t                    (t >= 1; column i < K-1 only)
// Items are the column's partial products, then the previous column's carries, in the
// reference's order.  Polynomials that are null by construction (the carry pushed before a
// column's first item: result_i is still zero) are not materialised: XOR with null is the
// identity and a product with null is null, so dropping them changes no output bit.
// Plans (with their device task tables) are cached per context, keyed by the operand bounds.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <memory>

#include "ctx.h"

namespace hm {

namespace {

constexpr int64_t kBoundLimit = (int64_t)1 << 30;
// Karatsuba lanes: a column's Karatsuba products alternate between two scratch regions and two
// streams (the context stream and its auxiliary stream), so one product's HBM-bound operand sums
// and recombinations, and the tail of its leaf launch, overlap the next product's leaves
#ifndef HM_KA_LANES
#define HM_KA_LANES 2
#endif
constexpr uint32_t kKaLanes = HM_KA_LANES;
// the deepest Karatsuba level's operand sums (lo + hi) are not formed in HBM by ka_sum_kernel:
// the MFMA leaves read both halves and XOR them while building their operand images
#ifndef HM_KA_FUSE_SUMS
#define HM_KA_FUSE_SUMS 1
#endif
constexpr bool kFuseLeafSums = HM_KA_FUSE_SUMS;
constexpr uint32_t kNW = sizeof(kMulTileW) / sizeof(kMulTileW[0]);
// schoolbook products whose uniform operand has at least this many words run on the matrix cores
// (mfma plans); narrower ones keep the VALU tiles
#ifndef HM_MF_MIN_WORDS
#define HM_MF_MIN_WORDS 4
#endif
constexpr uint32_t kMfMinWords = HM_MF_MIN_WORDS;

inline uint32_t slot_words(int64_t bound) { return ((uint32_t)(bound / 32) + 1 + 3) & ~3u; }

// signed circuit: pp[0][L-1] and pp[L-1][0] get ^1 (common.rs:123-126); at L = 1 both are pp[0][0]
inline bool pp_flip(bool is_signed, uint32_t L, uint32_t i, uint32_t j) {
    if (!is_signed || i != L - 1) return false;
    const int f = (j == 0) + (j == L - 1);
    return f & 1;
}

} // namespace

// One Karatsuba product (see "Karatsuba" below): its launches, in order.
struct KaProg {
    uint32_t u, v, out;                          // slots (exact degrees: deg1)
    uint32_t lane = 0;                           // scratch region / stream (mul_columns)
    std::vector<std::array<uint32_t, 3>> sums;   // per level 1..k: (first KaSum, count, h)
    uint32_t vtask = 0, nvtask = 0;              // leaf products (MulVTask range)
    uint32_t leaf_umax = 0, leaf_vmax = 0, leaf_omax = 0; // their largest operands and output
    uint32_t tiles[kNW] = {}, ntiles[kNW] = {};  // their tiles (MulVTile ranges) per width class
    std::vector<std::array<uint32_t, 3>> combs;  // per level k..1: (first KaComb, count, h)
    bool deg = true; // then the product's exact degree (false: a subtree of a split product)
};

// One launch of MFMA products (mul_mfma_kernel<false>): spans of `span` output tiles, the LDS
// slices sized by its largest operands.  A column's schoolbook products are split by the shorter
// operand's size into launches of their own, so the narrow products' small slices are not sized
// for the wide products' (and their spans cover their outputs, not 16 tiles of mostly nothing).
struct MfLaunch {
    uint32_t spans = 0, nspans = 0; // MulTile range in mspans
    uint32_t vmax = 0, umax = 0, span = 0;
    bool lean = false; // wide class on the lean windowed instance
};

struct MulPlan {
    // key
    uint32_t L = 0, K = 0;
    bool is_signed = false;
    uint32_t ka_min = 0, ka_leaf = 0;           // Karatsuba options (hm_ctx_set_mul_options)
    uint64_t ka_scratch = 0;                    // ... and hm_ctx_set_mul_scratch
    bool mfma = false;                          // products on the matrix cores (hm_ctx_set_mul_products)
    std::vector<uint32_t> ab, bb;
    // geometry
    std::vector<MulSlot> slots;
    uint64_t astride = 0; // arena words per value
    std::vector<int64_t> res_bound;
    struct Col {
        uint32_t pp, npp;          // MulPPTask offset / count (in tasks): the VALU partial products
        uint32_t ppm;              // MFMA partial products: MulProdTask offset (ppm list)
        MfLaunch ppl;              // ... their launch
        uint32_t items, nitems;    // u32 offset of the item slot ids
        uint32_t prefix;           // u32 offset of the prefix slot ids (nitems - 1)
        uint32_t res;              // result degree slot
        uint32_t maxwords;         // widest prefix / result
        uint32_t prod;             // MulProdTask offset (in tasks)
        uint32_t tiles[kNW], ntiles[kNW]; // MulTile offsets (in tiles) / counts per width class
        MfLaunch mfl[3];                  // MFMA schoolbook products: tiny, narrow, wide
        uint32_t rows = 0, nrows = 0;     // ... small ones on the VALU by rows (row_tasks range)
        uint32_t rows_uw = 0, rows_vw = 0, rows_ow = 0, rows_qw = 0;
        std::vector<KaProg> ka;           // this column's Karatsuba products
    };
    std::vector<Col> cols;
    std::vector<uint32_t> res_slots;
    // host tables, then one device copy
    std::vector<MulPPTask> pp;
    std::vector<uint32_t> lists;
    std::vector<MulProdTask> prod;
    std::vector<MulTile> tiles;
    std::vector<MulTile> mspans; // MFMA spans {task, first output word} of the schoolbook products
    std::vector<MulSpanRec> mrecs; // ... resolved (parallel to mspans; built after the regions)
    std::vector<MulProdTask> ppm; // partial products a_j * b_k run on the matrix cores
    std::vector<MulProdTask> row_tasks; // small carry products on the VALU (Col::rows)
    std::vector<MulSpanRec> row_recs;   // ... resolved (built after the regions)
    size_t off_rows = 0;
    // ... or, when every one fits (kMfPPGWords), all of them in one launch before the columns,
    // grouped by a_j (mul_ppg_kernel)
    bool ppg = false;
    std::vector<MulPPGroup> ppg_groups;
    std::vector<MulPPItem> ppg_items;
    uint32_t ppg_umax = 0, ppg_vmax = 0, ppg_span = 0;
    size_t off_ppg_groups = 0, off_ppg_items = 0;
    // ... or on the VALU by rows (mul_ppv_kernel) when every factor fits kPPVWords words: the same
    // items flattened to tasks {a_j slot, b_k slot, out slot}
    bool ppv = false;
    std::vector<MulPPTask> ppv_tasks;
    uint32_t ppv_inw = 0, ppv_outw = 0;
    size_t off_ppv = 0;
    std::vector<KaSum> ka_sums;
    std::vector<MulVTask> ka_vtasks;
    std::vector<MulVTile> ka_vtiles;
    std::vector<KaComb> ka_combs;
    uint8_t *d_tab = nullptr;
    size_t tab_bytes = 0;
    size_t off_slots = 0, off_pp = 0, off_lists = 0, off_prod = 0, off_tiles = 0, off_res = 0;
    size_t off_mspans = 0, off_ppm = 0, off_mrecs = 0;
    size_t off_ka_sums = 0, off_ka_vtasks = 0, off_ka_vtiles = 0, off_ka_combs = 0;
    uint64_t work = 0; // word-pair products (statistics)
    std::vector<double> prod_pairs; // per carry product (P.prod): its schoolbook word pairs
};

namespace {

struct Region {
    uint64_t used = 0, max = 0;
    uint64_t base = 0;
};

// ---------------------------------------------------------------------------------------------
// Karatsuba.  A carry product u * v whose shorter operand has at least ka_min words is computed
// as a Karatsuba recursion instead of schoolbook tiles: operands padded to N = leaf * 2^k words
// split into halves lo/hi, the three half-size products z0 = lo_u lo_v, z1 = hi_u hi_v,
// z2 = (lo_u + hi_u)(lo_v + hi_v), and u v = z0 + (z0 + z1 + z2) X^h + z1 X^2h (h = half size).
// Exact over GF(2)[X] (the same polynomial as the reference's bit-serial product,
// polynomial.rs:252-310), 3^k leaf products of leaf x leaf words instead of 4^k.  Every node is
// static (slot capacities are static), so the whole recursion is planned here: views into the
// arena, sums and child results in a scratch region (KA) reused product after product.  A
// subtree whose high halves are all padding (zero) is dropped: z1 = 0.
namespace {

// Views while planning: (region << 28) | word offset relative to the region (regions are placed
// after the symbolic run); kKaNone stays as is.
constexpr uint32_t kRegShift = 28, kRelMask = (1u << kRegShift) - 1;

struct KaBuild {
    uint32_t ka_region, leaf;
    bool fuse_leaf_sums = false; // the deepest level's sums are read by the leaves (MFMA plans)
    uint64_t top = 0, max = 0; // scratch bump allocator in the KA region (words)
    std::vector<std::vector<KaSum>> sums;   // by split depth
    std::vector<std::vector<KaComb>> combs; // by split depth
    std::vector<MulVTask> leaves;

    uint32_t alloc(uint64_t words) {
        const uint64_t o = top;
        top += (words + 3) & ~(uint64_t)3;
        max = std::max(max, top);
        return (ka_region << kRegShift) | (uint32_t)o;
    }
    // r[0:min(2n, rcap)) = U * V for views u (un valid words), v (vn), both of logical size n
    // u2 / v2 (nu2 / nv2 valid words): a second view XORed into the operand (fused leaf sums)
    void node(uint32_t lvl, uint32_t uo, uint32_t un, uint32_t vo, uint32_t vn, uint32_t n,
              uint32_t r, uint32_t rcap, uint32_t u2 = kKaNone, uint32_t nu2 = 0,
              uint32_t v2 = kKaNone, uint32_t nv2 = 0) {
        if (n == leaf) {
            leaves.push_back({uo, std::min(un, n), vo, std::min(vn, n), r, std::min(2 * n, rcap),
                              u2, std::min(nu2, n), v2, std::min(nv2, n)});
            return;
        }
        const uint32_t h = n / 2;
        if (un <= h && vn <= h) {
            // both high halves are padding: u v = lo_u lo_v (one child, not three); the
            // recombination with z2 = z0, z1 = 0 copies it and zero-fills r above it
            const uint32_t z0 = alloc(2 * h);
            node(lvl + 1, uo, un, vo, vn, h, z0, 2 * h);
            if (combs.size() <= lvl) combs.resize(lvl + 1);
            combs[lvl].push_back({z0, kKaNone, z0, r, rcap});
            return;
        }
        struct Half {
            uint32_t lo_n, hi_o, hi_n, s_o, s_n;
            uint32_t s2_o = kKaNone, s2_n = 0; // (fused leaf sums) the sum's second view
        };
        // children that are leaves read lo + hi as two views instead of a formed sum
        const bool fuse = fuse_leaf_sums && h == leaf;
        auto half = [&](uint32_t o, uint32_t len) {
            Half x;
            x.lo_n = std::min(len, h);
            x.hi_o = o + h;
            x.hi_n = len > h ? len - h : 0u;
            if (x.hi_n == 0) { // lo + hi = lo: no sum to form
                x.s_o = o, x.s_n = x.lo_n;
            } else if (fuse) { // lo_n = h >= hi_n
                x.s_o = o, x.s_n = x.lo_n, x.s2_o = x.hi_o, x.s2_n = x.hi_n;
            } else {
                x.s_o = alloc(h), x.s_n = h;
                if (sums.size() <= lvl) sums.resize(lvl + 1);
                sums[lvl].push_back({o, len, x.s_o});
            }
            return x;
        };
        const Half U = half(uo, un), V = half(vo, vn);
        const bool has_z1 = U.hi_n && V.hi_n;
        const uint32_t z0 = alloc(2 * h), z2 = alloc(2 * h);
        const uint32_t z1 = has_z1 ? alloc(2 * h) : kKaNone;
        node(lvl + 1, uo, U.lo_n, vo, V.lo_n, h, z0, 2 * h);
        if (has_z1) node(lvl + 1, U.hi_o, U.hi_n, V.hi_o, V.hi_n, h, z1, 2 * h);
        node(lvl + 1, U.s_o, U.s_n, V.s_o, V.s_n, h, z2, 2 * h, U.s2_o, U.s2_n, V.s2_o, V.s2_n);
        if (combs.size() <= lvl) combs.resize(lvl + 1);
        combs[lvl].push_back({z0, z1, z2, r, rcap});
    }

    // The root of node(0, ...) without its recursion, for a product planned one subtree at a time:
    // the root's operand sums (sums[0]; always formed, the children are not leaves), its z buffers
    // and its recombination (combs[0]).  Returns the children, each to be planned into its z
    // (2h words) with scratch above this builder's top.
    struct Child {
        uint32_t uo, un, vo, vn, z;
    };
    std::vector<Child> split(uint32_t uo, uint32_t un, uint32_t vo, uint32_t vn, uint32_t n,
                             uint32_t r, uint32_t rcap) {
        const uint32_t h = n / 2;
        std::vector<Child> ch;
        combs.resize(1);
        if (un <= h && vn <= h) {
            const uint32_t z0 = alloc(2 * h);
            ch.push_back({uo, un, vo, vn, z0});
            combs[0].push_back({z0, kKaNone, z0, r, rcap});
            return ch;
        }
        struct Half {
            uint32_t lo_n, hi_o, hi_n, s_o, s_n;
        };
        auto half = [&](uint32_t o, uint32_t len) {
            Half x;
            x.lo_n = std::min(len, h);
            x.hi_o = o + h;
            x.hi_n = len > h ? len - h : 0u;
            if (x.hi_n == 0) {
                x.s_o = o, x.s_n = x.lo_n;
            } else {
                x.s_o = alloc(h), x.s_n = h;
                sums.resize(1);
                sums[0].push_back({o, len, x.s_o});
            }
            return x;
        };
        const Half U = half(uo, un), V = half(vo, vn);
        const bool has_z1 = U.hi_n && V.hi_n;
        const uint32_t z0 = alloc(2 * h), z2 = alloc(2 * h);
        const uint32_t z1 = has_z1 ? alloc(2 * h) : kKaNone;
        ch.push_back({uo, U.lo_n, vo, V.lo_n, z0});
        if (has_z1) ch.push_back({U.hi_o, U.hi_n, V.hi_o, V.hi_n, z1});
        ch.push_back({U.s_o, U.s_n, V.s_o, V.s_n, z2});
        combs[0].push_back({z0, z1, z2, r, rcap});
        return ch;
    }
};

// A Karatsuba product whose breadth-first recursion needs more scratch than kKaScratchWords (words
// per value, per lane) is planned one subtree at a time: the root's sums and z buffers, then each
// child's own program above them (one after another on the lane's stream, reusing the same
// scratch), then the root's recombination -- recursively.  The planning views hold 28-bit word
// offsets per region, so a breadth-first K = 21 product (3.1e8 words) cannot be planned whole;
// K <= 20 (1.94e8 at most) keeps its one-program plans.
// (The limit is the context's ka_scratch, hm_ctx_set_mul_scratch; default kKaScratchWords, ctx.h.)

} // namespace

// Symbolic run.  Slot offsets are first relative to their region (in / pp / prefix / carries of
// even columns / carries of odd columns); regions are placed once their maxima are known.
bool build_plan(MulPlan &P) {
    const uint32_t K = P.K;
    enum { IN, PP, PRE, CA, CB, KA, PPA, KA2, NREG };
    Region reg[NREG];
    std::vector<uint8_t> slot_reg;
    std::vector<int64_t> slot_bnd; // each slot's degree bound
    auto slot_bound = [&](uint32_t s) { return std::max<int64_t>(slot_bnd[s], 0); };
    auto new_slot = [&](int r, int64_t bound) -> uint32_t {
        slot_bnd.push_back(bound);
        const uint32_t w = bound < 0 ? 0u : slot_words(bound);
        P.slots.push_back({(uint32_t)reg[r].used, w});
        slot_reg.push_back((uint8_t)r);
        reg[r].used += w;
        reg[r].max = std::max(reg[r].max, reg[r].used);
        return (uint32_t)P.slots.size() - 1;
    };
    for (uint32_t j = 0; j < K; ++j) new_slot(IN, P.ab[j]);
    for (uint32_t j = 0; j < K; ++j) new_slot(IN, P.bb[j]);
    struct Item {
        uint32_t slot;
        int64_t bound;
    };
    // Grouped partial products: every a_j * b_k (j + k < K) on the matrix cores, all in one
    // launch, when every factor has at most kMfPPGWords words (and at least kMfMinWords); their
    // slots live in a region of their own (PPA), not reused column by column.  The signed
    // corners (+1, column L-1) stay VALU tasks of their column.
    std::vector<std::vector<uint32_t>> pp_slot(K, std::vector<uint32_t>(K, ~0u));
    P.ppg = P.mfma;
    for (uint32_t j = 0; j < K && P.ppg; ++j) {
        const uint32_t wa = (uint32_t)(P.ab[j] / 32 + 1), wb = (uint32_t)(P.bb[j] / 32 + 1);
        if (std::max(wa, wb) > kMfPPGWords || std::min(wa, wb) < kMfMinWords) P.ppg = false;
    }
    if (P.ppg) {
        uint32_t omax = 0;
        for (uint32_t j = 0; j < K; ++j) {
            MulPPGroup g{j, (uint32_t)P.ppg_items.size(), 0};
            for (uint32_t k = 0; j + k < K; ++k) {
                if (pp_flip(P.is_signed, P.L, j + k, j)) continue;
                const int64_t bnd = (int64_t)P.ab[j] + P.bb[k];
                const uint32_t s = new_slot(PPA, bnd);
                pp_slot[j][k] = s;
                P.ppg_items.push_back({K + k, s});
                omax = std::max(omax, P.slots[s].words);
                P.ppg_vmax = std::max(P.ppg_vmax, (uint32_t)(P.bb[k] / 32 + 1));
            }
            g.count = (uint32_t)P.ppg_items.size() - g.first;
            P.ppg_umax = std::max(P.ppg_umax, (uint32_t)(P.ab[j] / 32 + 1));
            if (g.count) P.ppg_groups.push_back(g);
        }
        P.ppg_span = std::min<uint32_t>(kMfSpan, std::max<uint32_t>(1, (omax + 31) / 32));
#ifndef HM_PPV
#define HM_PPV 1 // (A/B knob) 0: the partial products on the matrix cores (mul_ppg_kernel) always
#endif
        P.ppv = HM_PPV && std::max(P.ppg_umax, P.ppg_vmax) <= kPPVWords;
        if (P.ppv) {
            for (const MulPPGroup &g : P.ppg_groups)
                for (uint32_t it = g.first; it < g.first + g.count; ++it)
                    P.ppv_tasks.push_back({g.u, P.ppg_items[it].v, P.ppg_items[it].out, 0u});
            for (uint32_t s = 0; s < 2 * K; ++s) P.ppv_inw = std::max(P.ppv_inw, P.slots[s].words);
            P.ppv_outw = std::max(omax, P.ppg_umax + P.ppg_vmax + 1);
            // a block's four waves within one CU's LDS, else the MFMA form
            const size_t ww = 2 * K * (P.ppv_inw + 1) + P.ppv_tasks.size() * P.ppv_outw;
            if (ww * 4 * 4 > 160 * 1024) P.ppv = false, P.ppv_tasks.clear();
        }
    }
    std::vector<Item> prev;
    P.res_bound.assign(K, -1);
    for (uint32_t i = 0; i < K; ++i) {
        MulPlan::Col col{};
        reg[PP].used = 0;
        reg[PRE].used = 0;
        const int creg = (i & 1) ? CB : CA;
        reg[creg].used = 0;
        std::vector<Item> items;
        col.pp = (uint32_t)P.pp.size();
        col.ppm = (uint32_t)P.ppm.size();
        uint32_t ppm_omax = 0;
        for (uint32_t j = 0; j <= i; ++j) {
            const int64_t bnd = (int64_t)P.ab[j] + P.bb[i - j];
            if (bnd > kBoundLimit) return false;
            if (pp_slot[j][i - j] != ~0u) { // computed by the grouped launch
                items.push_back({pp_slot[j][i - j], bnd});
                continue;
            }
            const uint32_t s = new_slot(PP, bnd);
            const bool flip = pp_flip(P.is_signed, P.L, i, j);
            const uint32_t sa = j, sb = K + (i - j);
            const uint32_t wa = P.slots[sa].words, wb = P.slots[sb].words;
            // on the matrix cores unless a signed corner (+1) or a narrow operand
            if (P.mfma && !flip && std::min(wa, wb) >= kMfMinWords) {
                P.ppm.push_back(wa <= wb ? MulProdTask{sa, sb, s} : MulProdTask{sb, sa, s});
                col.ppl.vmax = std::max(col.ppl.vmax, std::max(wa, wb));
                col.ppl.umax = std::max(col.ppl.umax, std::min(wa, wb));
                ppm_omax = std::max(ppm_omax, P.slots[s].words);
            } else {
                P.pp.push_back({sa, sb, s, flip ? 1u : 0u});
            }
            items.push_back({s, bnd});
        }
        col.npp = (uint32_t)P.pp.size() - col.pp;
        // spans of the partial products: their whole (short) outputs, at most kMfSpan tiles
        col.ppl.span = std::min<uint32_t>(kMfSpan, (ppm_omax + 31) / 32);
        col.ppl.spans = (uint32_t)P.mspans.size();
        for (uint32_t t = 0; t < (uint32_t)P.ppm.size() - col.ppm; ++t)
            for (uint32_t base = 0; base < P.slots[P.ppm[col.ppm + t].out].words; base += 32 * col.ppl.span)
                P.mspans.push_back({t, base});
        col.ppl.nspans = (uint32_t)P.mspans.size() - col.ppl.spans;
        items.insert(items.end(), prev.begin(), prev.end());
        const bool push = i + 1 < K;
        std::vector<Item> cur;
        col.items = (uint32_t)P.lists.size();
        col.nitems = (uint32_t)items.size();
        for (auto &x : items) P.lists.push_back(x.slot);
        col.prefix = (uint32_t)P.lists.size();
        col.prod = (uint32_t)P.prod.size();
        int64_t pb = -1;          // bound of p_t (the running result before item t)
        uint32_t pslot = 0;       // slot of p_t (t >= 1)
        uint32_t maxw = 0;
        for (size_t t = 0; t < items.size(); ++t) {
            const Item &x = items[t];
            if (push && pb >= 0) { // carries.push(result & x_t) (common.rs:83-87, :93-96)
                const int64_t cbnd = pb + x.bound;
                if (cbnd > kBoundLimit) return false;
                const uint32_t cs = new_slot(creg, cbnd);
                const uint32_t wp = P.slots[pslot].words, wx = P.slots[x.slot].words;
                // the operand with fewer words is the uniform one (its bits are the decisions)
                if (wp <= wx) P.prod.push_back({pslot, x.slot, cs});
                else P.prod.push_back({x.slot, pslot, cs});
                P.work += (uint64_t)(pb / 32 + 1) * (uint64_t)(x.bound / 32 + 1);
                P.prod_pairs.push_back((double)(pb / 32 + 1) * (double)(x.bound / 32 + 1));
                cur.push_back({cs, cbnd});
            }
            pb = std::max(pb, x.bound); // result ^= x_t
            maxw = std::max(maxw, slot_words(pb));
            if (t + 1 < items.size()) {
                pslot = new_slot(PRE, pb);
                P.lists.push_back(pslot);
            }
        }
        col.maxwords = maxw;
        col.res = new_slot(PRE, -1); // degree-only slot (the output bit)
        P.res_slots.push_back(col.res);
        P.res_bound[i] = pb;
        // Karatsuba for the big products (their slots are final now: region offsets are fixed
        // when the regions are placed, so views are recorded relative and fixed up below)
        std::vector<bool> is_ka(P.prod.size() - col.prod, false);
        uint32_t nka = 0; // this column's Karatsuba products so far: they alternate lanes
        for (uint32_t k = col.prod; k < P.prod.size() && P.ka_min; ++k) {
            const MulProdTask &T = P.prod[k];
            const uint32_t nu = P.slots[T.u].words, nv = P.slots[T.v].words;
            if (std::min(nu, nv) < P.ka_min) continue;
            uint32_t lk = 0;
            while (((uint64_t)P.ka_leaf << lk) < std::max(nu, nv)) ++lk;
            if (lk == 0) continue;
            // leaf: the smallest multiple of 32 words with leaf * 2^lk >= max(nu, nv)
            const uint32_t mx = std::max(nu, nv);
            const uint32_t leaf = (((mx + (1u << lk) - 1) >> lk) + 31) & ~31u;
            // two lanes (kKaLanes): products alternate between two scratch regions, so that
            // mul_columns can run consecutive products on two streams
            const uint32_t lane = kKaLanes > 1 ? (nka++ & 1u) : 0u;
            const uint32_t region = lane ? KA2 : KA;
            auto view = [&](uint32_t slot) {
                return ((uint32_t)slot_reg[slot] << kRegShift) | P.slots[slot].off;
            };
            // one program from a builder rooted at size n: its sums by depth, its leaves, its
            // recombinations bottom-up (deg: the product's exact degree after them)
            auto push_prog = [&](const KaBuild &kb, uint32_t n, bool deg) {
                KaProg pg;
                pg.u = T.u, pg.v = T.v, pg.out = T.out;
                pg.lane = lane;
                pg.deg = deg;
                for (uint32_t l = 0; l < kb.sums.size(); ++l) {
                    if (kb.sums[l].empty()) continue;
                    pg.sums.push_back({(uint32_t)P.ka_sums.size(), (uint32_t)kb.sums[l].size(), n >> (l + 1)});
                    P.ka_sums.insert(P.ka_sums.end(), kb.sums[l].begin(), kb.sums[l].end());
                }
                pg.vtask = (uint32_t)P.ka_vtasks.size(), pg.nvtask = (uint32_t)kb.leaves.size();
                for (const MulVTask &t : kb.leaves) {
                    pg.leaf_umax = std::max(pg.leaf_umax, t.nu);
                    pg.leaf_vmax = std::max(pg.leaf_vmax, t.nv);
                    pg.leaf_omax = std::max(pg.leaf_omax, t.nout);
                }
                P.ka_vtasks.insert(P.ka_vtasks.end(), kb.leaves.begin(), kb.leaves.end());
                uint32_t wc = kNW - 1;
                for (uint32_t q = 0; q < kNW; ++q)
                    if (kMulTileW[q] * 64 >= 2 * leaf) {
                        wc = q;
                        break;
                    }
                pg.tiles[wc] = (uint32_t)P.ka_vtiles.size();
                for (uint32_t t = 0; t < pg.nvtask; ++t)
                    for (uint32_t b0 = 0; b0 < 2 * leaf; b0 += 64 * kMulTileW[wc])
                        P.ka_vtiles.push_back({t, b0});
                pg.ntiles[wc] = (uint32_t)P.ka_vtiles.size() - pg.tiles[wc];
                for (uint32_t l = (uint32_t)kb.combs.size(); l-- > 0;) {
                    if (kb.combs[l].empty()) continue;
                    pg.combs.push_back({(uint32_t)P.ka_combs.size(), (uint32_t)kb.combs[l].size(), n >> (l + 1)});
                    P.ka_combs.insert(P.ka_combs.end(), kb.combs[l].begin(), kb.combs[l].end());
                }
                reg[region].max = std::max(reg[region].max, kb.max);
                col.ka.push_back(std::move(pg));
            };
            // the scratch words KaBuild::node allocates for a (n, un, vn) node, without building it
            // (the same recursion, memoised: few distinct operand lengths per depth)
            const bool fuse = P.mfma && kFuseLeafSums;
            std::map<std::array<uint32_t, 3>, uint64_t> memo;
            std::function<uint64_t(uint32_t, uint32_t, uint32_t)> scratch = [&](uint32_t n, uint32_t un,
                                                                               uint32_t vn) -> uint64_t {
                if (n == leaf) return 0;
                const auto key = std::array<uint32_t, 3>{n, un, vn};
                if (auto it = memo.find(key); it != memo.end()) return it->second;
                const uint32_t h = n / 2;
                uint64_t s;
                if (un <= h && vn <= h) {
                    s = 2ull * h + scratch(h, un, vn);
                } else {
                    const uint32_t ulo = std::min(un, h), uhi = un > h ? un - h : 0u;
                    const uint32_t vlo = std::min(vn, h), vhi = vn > h ? vn - h : 0u;
                    const bool formed = !(fuse && h == leaf);
                    s = 4ull * h + (uhi && vhi ? 2ull * h : 0) + (formed && uhi ? h : 0) + (formed && vhi ? h : 0);
                    s += scratch(h, ulo, vlo) + (uhi && vhi ? scratch(h, uhi, vhi) : 0) +
                         scratch(h, uhi ? h : ulo, vhi ? h : vlo);
                }
                memo[key] = s;
                return s;
            };
            // u * v (views, logical size n) into r; scratch from `top` up (see kKaScratchWords)
            std::function<void(uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t,
                               uint64_t, bool)>
                plan_ka = [&](uint32_t uo, uint32_t un, uint32_t vo, uint32_t vn, uint32_t n,
                              uint32_t r, uint32_t rcap, uint64_t top, bool deg) {
                    if (scratch(n, std::min(un, n), std::min(vn, n)) <= P.ka_scratch || n <= 2 * leaf) {
                        KaBuild kb{region, leaf};
                        kb.fuse_leaf_sums = fuse;
                        kb.top = kb.max = top;
                        kb.node(0, uo, un, vo, vn, n, r, rcap);
                        return push_prog(kb, n, deg);
                    }
                    KaBuild rb{region, leaf};
                    rb.top = rb.max = top;
                    const std::vector<KaBuild::Child> ch = rb.split(uo, un, vo, vn, n, r, rcap);
                    KaBuild rs = rb; // the root's sums first (no leaves, no recombination)
                    rs.combs.clear();
                    push_prog(rs, n, false);
                    for (const KaBuild::Child &x : ch)
                        plan_ka(x.uo, x.un, x.vo, x.vn, n / 2, x.z, n, rb.top, false);
                    rb.sums.clear(); // ... and its recombination last
                    push_prog(rb, n, deg);
                };
            plan_ka(view(T.u), nu, view(T.v), nv, leaf << lk, view(T.out), P.slots[T.out].words, 0, true);
            is_ka[k - col.prod] = true;
        }
        // tiles of this column's schoolbook products: MFMA spans where the uniform operand has
        // at least kMfMinWords words (mfma plans), the rest grouped by per-lane VALU tile width
        std::vector<MulTile> byw[kNW];
        std::vector<uint32_t> mfk[3]; // MFMA schoolbook products by class
        uint32_t omax[3] = {0, 0, 0};
#ifndef HM_ROWS
#define HM_ROWS 1 // (A/B knob) 0: the small products stay in the MFMA tiny class
#endif
        col.rows = (uint32_t)P.row_tasks.size();
        auto rows_ok = [&](uint32_t k) {
            const uint32_t uw = P.slots[P.prod[k].u].words, vw = P.slots[P.prod[k].v].words;
            return HM_ROWS && P.mfma && !is_ka[k - col.prod] && uw >= kMfMinWords && uw <= kRowsU &&
                   vw <= kRowsV;
        };
        for (uint32_t k = col.prod; k < P.prod.size(); ++k)
            if (rows_ok(k)) {
                col.rows_uw = std::max(col.rows_uw, P.slots[P.prod[k].u].words);
                col.rows_qw = std::max(col.rows_qw, (uint32_t)(slot_bound(P.prod[k].u) / 32 + 1));
                col.rows_vw = std::max(col.rows_vw, P.slots[P.prod[k].v].words);
                col.rows_ow = std::max(col.rows_ow, P.slots[P.prod[k].out].words);
                ++col.nrows;
            }
        col.rows_ow = std::max(col.rows_ow, col.rows_uw + col.rows_vw + 1);
        // the column's small products on the VALU when a block's four waves' LDS fits one CU
        const bool use_rows =
            col.nrows && (size_t)col.nrows * (col.rows_uw + col.rows_vw + col.rows_ow + 8) * 4 * 4 <= 160 * 1024;
        if (!use_rows) col.nrows = 0;
        for (uint32_t k = col.prod; k < P.prod.size(); ++k) {
            if (is_ka[k - col.prod]) continue;
            const uint32_t uw = P.slots[P.prod[k].u].words;
            if (use_rows && rows_ok(k)) {
                P.row_tasks.push_back(P.prod[k]);
                continue;
            }
            if (P.mfma && uw >= kMfMinWords) {
                const int cl = uw <= kMfTinyWords ? 0 : uw <= kMfNarrowWords ? 1 : 2;
                mfk[cl].push_back(k);
                col.mfl[cl].vmax = std::max(col.mfl[cl].vmax, P.slots[P.prod[k].v].words);
                col.mfl[cl].umax = std::max(col.mfl[cl].umax, uw);
                omax[cl] = std::max(omax[cl], P.slots[P.prod[k].out].words);
                continue;
            }
            const uint32_t nout = P.slots[P.prod[k].out].words;
            const uint32_t need = (nout + 63) / 64;
            uint32_t wc = kNW - 1;
            for (uint32_t q = 0; q < kNW; ++q)
                if (kMulTileW[q] >= need) {
                    wc = q;
                    break;
                }
            const uint32_t span = 64 * kMulTileW[wc];
            for (uint32_t base = 0; base < nout; base += span) byw[wc].push_back({k - col.prod, base});
        }
        for (int cl = 0; cl < 3; ++cl) {
            MfLaunch &m = col.mfl[cl];
            m.lean = cl == 2 && kMfWideLean;
            m.span = std::min<uint32_t>(cl == 2 ? kMfWideSpan : kMfNarrowSpan,
                                        std::max<uint32_t>(1, (omax[cl] + 31) / 32));
            m.spans = (uint32_t)P.mspans.size();
            for (uint32_t k : mfk[cl])
                for (uint32_t base = 0; base < P.slots[P.prod[k].out].words; base += 32 * m.span)
                    P.mspans.push_back({k - col.prod, base});
            m.nspans = (uint32_t)P.mspans.size() - m.spans;
        }
        for (uint32_t q = 0; q < kNW; ++q) {
            col.tiles[q] = (uint32_t)P.tiles.size();
            col.ntiles[q] = (uint32_t)byw[q].size();
            P.tiles.insert(P.tiles.end(), byw[q].begin(), byw[q].end());
        }
        P.cols.push_back(col);
        prev.swap(cur);
    }
    // place the regions and make the offsets absolute
    for (int r = 0; r < NREG; ++r)
        if (reg[r].max >= (1ull << kRegShift)) return false; // planning views hold 28-bit offsets
    uint64_t base = 0;
    for (int r = 0; r < NREG; ++r) {
        reg[r].base = base;
        base += (reg[r].max + 3) & ~(uint64_t)3;
    }
    if (base >= (1ull << 32)) return false;
    for (size_t s = 0; s < P.slots.size(); ++s) P.slots[s].off += (uint32_t)reg[slot_reg[s]].base;
    // Karatsuba views: (region, relative offset) -> arena offset
    auto fix = [&](uint32_t o) -> uint32_t {
        return o == kKaNone ? o : (uint32_t)(reg[o >> kRegShift].base + (o & kRelMask));
    };
    for (auto &t : P.ka_sums) t.src = fix(t.src), t.dst = fix(t.dst);
    for (auto &t : P.ka_vtasks)
        t.u = fix(t.u), t.v = fix(t.v), t.out = fix(t.out), t.u2 = fix(t.u2), t.v2 = fix(t.v2);
    for (auto &t : P.ka_combs) t.z0 = fix(t.z0), t.z1 = fix(t.z1), t.z2 = fix(t.z2), t.r = fix(t.r);
    P.astride = std::max<uint64_t>(base, 4);
    // the MFMA spans resolved: every launch's span range of mspans, task indices relative to the
    // column's product list (ppm for the partial products' launch, prod for the carries)
    P.mrecs.assign(P.mspans.size(), MulSpanRec{});
    auto resolve = [&](const MfLaunch &m, const std::vector<MulProdTask> &tasks, uint32_t t0) {
        for (uint32_t i = m.spans; i < m.spans + m.nspans; ++i) {
            const MulProdTask &t = tasks[t0 + P.mspans[i].task];
            P.mrecs[i] = MulSpanRec{P.slots[t.u].off, P.slots[t.v].off, P.slots[t.out].off,
                                    P.slots[t.out].words, t.u, t.v, t.out, P.mspans[i].base};
        }
    };
    for (const auto &col : P.cols) {
        resolve(col.ppl, P.ppm, col.ppm);
        for (const MfLaunch &m : col.mfl) resolve(m, P.prod, col.prod);
    }
    // the row products resolved (base: the operands' slot capacities, u | v << 16)
    for (const MulProdTask &t : P.row_tasks)
        P.row_recs.push_back(MulSpanRec{P.slots[t.u].off, P.slots[t.v].off, P.slots[t.out].off,
                                        P.slots[t.out].words, t.u, t.v, t.out,
                                        P.slots[t.u].words | (P.slots[t.v].words << 16)});
    return true;
}

hm_status upload_plan(hm_ctx *c, MulPlan &P) {
    auto align = [](size_t v) { return (v + 15) & ~(size_t)15; };
    size_t o = 0;
    P.off_slots = o, o = align(o + P.slots.size() * sizeof(MulSlot));
    P.off_pp = o, o = align(o + P.pp.size() * sizeof(MulPPTask));
    P.off_lists = o, o = align(o + P.lists.size() * 4);
    P.off_prod = o, o = align(o + P.prod.size() * sizeof(MulProdTask));
    P.off_rows = o, o = align(o + P.row_recs.size() * sizeof(MulSpanRec));
    P.off_tiles = o, o = align(o + P.tiles.size() * sizeof(MulTile));
    P.off_res = o, o = align(o + P.res_slots.size() * 4);
    P.off_mspans = o, o = align(o + P.mspans.size() * sizeof(MulTile));
    P.off_mrecs = o, o = align(o + P.mrecs.size() * sizeof(MulSpanRec));
    P.off_ppm = o, o = align(o + P.ppm.size() * sizeof(MulProdTask));
    P.off_ppg_groups = o, o = align(o + P.ppg_groups.size() * sizeof(MulPPGroup));
    P.off_ppg_items = o, o = align(o + P.ppg_items.size() * sizeof(MulPPItem));
    P.off_ppv = o, o = align(o + P.ppv_tasks.size() * sizeof(MulPPTask));
    P.off_ka_sums = o, o = align(o + P.ka_sums.size() * sizeof(KaSum));
    P.off_ka_vtasks = o, o = align(o + P.ka_vtasks.size() * sizeof(MulVTask));
    P.off_ka_vtiles = o, o = align(o + P.ka_vtiles.size() * sizeof(MulVTile));
    P.off_ka_combs = o, o = align(o + P.ka_combs.size() * sizeof(KaComb));
    std::vector<uint8_t> h(std::max<size_t>(o, 16), 0);
    auto put = [&](size_t off, const void *src, size_t n) {
        if (n) std::memcpy(h.data() + off, src, n);
    };
    put(P.off_slots, P.slots.data(), P.slots.size() * sizeof(MulSlot));
    put(P.off_pp, P.pp.data(), P.pp.size() * sizeof(MulPPTask));
    put(P.off_lists, P.lists.data(), P.lists.size() * 4);
    put(P.off_prod, P.prod.data(), P.prod.size() * sizeof(MulProdTask));
    put(P.off_rows, P.row_recs.data(), P.row_recs.size() * sizeof(MulSpanRec));
    put(P.off_tiles, P.tiles.data(), P.tiles.size() * sizeof(MulTile));
    put(P.off_res, P.res_slots.data(), P.res_slots.size() * 4);
    put(P.off_mspans, P.mspans.data(), P.mspans.size() * sizeof(MulTile));
    put(P.off_mrecs, P.mrecs.data(), P.mrecs.size() * sizeof(MulSpanRec));
    put(P.off_ppm, P.ppm.data(), P.ppm.size() * sizeof(MulProdTask));
    put(P.off_ppg_groups, P.ppg_groups.data(), P.ppg_groups.size() * sizeof(MulPPGroup));
    put(P.off_ppg_items, P.ppg_items.data(), P.ppg_items.size() * sizeof(MulPPItem));
    put(P.off_ppv, P.ppv_tasks.data(), P.ppv_tasks.size() * sizeof(MulPPTask));
    put(P.off_ka_sums, P.ka_sums.data(), P.ka_sums.size() * sizeof(KaSum));
    put(P.off_ka_vtasks, P.ka_vtasks.data(), P.ka_vtasks.size() * sizeof(MulVTask));
    put(P.off_ka_vtiles, P.ka_vtiles.data(), P.ka_vtiles.size() * sizeof(MulVTile));
    put(P.off_ka_combs, P.ka_combs.data(), P.ka_combs.size() * sizeof(KaComb));
    DeviceGuard g(c->device);
    HM_HIP(c, hipStreamSynchronize(c->stream));
    HM_HIP(c, hipMalloc(&P.d_tab, h.size()));
    P.tab_bytes = h.size();
    HM_HIP(c, hipMemcpy(P.d_tab, h.data(), h.size(), hipMemcpyHostToDevice));
    return HM_OK;
}

constexpr size_t kMaxPlans = 8;

hm_status get_plan(hm_ctx *c, uint32_t L, uint32_t K, const uint32_t *ab, const uint32_t *bb,
                   bool is_signed, MulPlan *&out) {
    for (MulPlan *p : c->mul_plans)
        if (p->L == L && p->K == K && p->is_signed == is_signed && p->ka_min == c->ka_min &&
            p->ka_leaf == c->ka_leaf && p->ka_scratch == c->ka_scratch && p->mfma == mul_on_mfma(c) &&
            std::equal(p->ab.begin(), p->ab.end(), ab) && std::equal(p->bb.begin(), p->bb.end(), bb)) {
            out = p;
            return HM_OK;
        }
    auto P = std::make_unique<MulPlan>();
    P->L = L, P->K = K, P->is_signed = is_signed;
    P->ka_min = c->ka_min, P->ka_leaf = c->ka_leaf, P->ka_scratch = c->ka_scratch;
    P->mfma = mul_on_mfma(c);
    P->ab.assign(ab, ab + K), P->bb.assign(bb, bb + K);
    if (!build_plan(*P)) return HM_ERR_UNSUPPORTED;
    if (hm_status st = upload_plan(c, *P); st) {
        if (P->d_tab) (void)hipFree(P->d_tab);
        return st;
    }
    if (c->mul_plans.size() >= kMaxPlans) { // a captured graph may still hold the table: retire it
        MulPlan *old = c->mul_plans.front();
        retire(c, old->d_tab, old->tab_bytes, false);
        delete old;
        c->mul_plans.erase(c->mul_plans.begin());
    }
    out = P.release();
    c->mul_plans.push_back(out);
    return HM_OK;
}

} // namespace

bool mul_result_bounds(uint32_t nbits, uint32_t K, const uint32_t *a, const uint32_t *b,
                       bool is_signed, std::vector<int64_t> &res) {
    MulPlan P;
    P.L = nbits, P.K = K, P.is_signed = is_signed;
    P.ab.assign(a, a + K), P.bb.assign(b, b + K);
    if (!build_plan(P)) return false;
    res = P.res_bound;
    return true;
}

// The plan's recursion over bounds only (no slots, no limits): the cost model of hm_mul_cost.
void mul_cost_model(uint32_t nbits, uint32_t K, const uint32_t *a, const uint32_t *b,
                    double &pairs, double &out_bytes, double &maxdeg) {
    (void)nbits;
    std::vector<double> prev, cur;
    pairs = 0, out_bytes = 0, maxdeg = 0;
    for (uint32_t i = 0; i < K; ++i) {
        std::vector<double> items;
        for (uint32_t j = 0; j <= i; ++j) items.push_back((double)a[j] + (double)b[i - j]);
        items.insert(items.end(), prev.begin(), prev.end());
        const bool push = i + 1 < K;
        cur.clear();
        double pb = -1;
        for (double x : items) {
            if (push && pb >= 0) {
                pairs += (std::floor(pb / 32) + 1) * (std::floor(x / 32) + 1);
                cur.push_back(pb + x);
                maxdeg = std::max(maxdeg, pb + x);
            }
            pb = std::max(pb, x);
            maxdeg = std::max(maxdeg, pb);
        }
        out_bytes += 8 * (std::floor(std::max(pb, 0.0) / 64) + 1);
        prev.swap(cur);
    }
}

hm_status mul_plan_work(hm_ctx *c, uint32_t nbits, uint32_t K, const uint32_t *a, const uint32_t *b,
                        bool is_signed, double &executed) {
    MulPlan *P = nullptr;
    if (hm_status st = get_plan(c, nbits, K, a, b, is_signed, P); st) return st;
    // carries as the plan runs them: a schoolbook product's word pairs at its static bounds (as
    // hm_mul_cost counts them), a Karatsuba product's leaf products instead (a product's output
    // slot is its own, so it identifies the product)
    executed = 0;
    std::vector<bool> ka(P->slots.size(), false);
    for (const auto &col : P->cols)
        for (const KaProg &pg : col.ka) {
            ka[pg.out] = true;
            for (uint32_t t = pg.vtask; t < pg.vtask + pg.nvtask; ++t)
                executed += (double)P->ka_vtasks[t].nu * (double)P->ka_vtasks[t].nv;
        }
    for (size_t k = 0; k < P->prod.size(); ++k)
        if (!ka[P->prod[k].out]) executed += P->prod_pairs[k];
    return HM_OK;
}

void mul_plans_release(hm_ctx *c) {
    for (MulPlan *p : c->mul_plans) {
        if (p->d_tab) (void)hipFree(p->d_tab);
        delete p;
    }
    c->mul_plans.clear();
}

namespace {

// the launches of one Karatsuba product: sums by depth, leaf products, recombination bottom-up,
// and the exact output degree
hm_status run_ka(hm_ctx *c, const MulPlan &P, const KaProg &pg, const MulBase &B, hipStream_t st) {
    const uint8_t *T = P.d_tab;
    for (const auto &lv : pg.sums) {
        KaSumArgs a{};
        a.B = B, a.t = (const KaSum *)(T + P.off_ka_sums) + lv[0], a.nt = lv[1], a.h = lv[2];
        if (launch_ka_sum(a, st)) return hip_fail(c, hipGetLastError());
    }
    if (!pg.nvtask) {
        // (a split product's root sums or recombination: no leaves)
    } else if (P.mfma) {
        // the leaves on the matrix cores: one wave per (value, leaf)
        MulMfmaArgs a{};
        a.B = B, a.tasks = (const MulVTask *)(T + P.off_ka_vtasks) + pg.vtask;
        a.span = std::max(1u, (pg.leaf_omax + 31) / 32); // one span: the whole leaf output
        a.nspans = 1;
        a.nitems = pg.nvtask;
        a.vmax = pg.leaf_vmax, a.umax = pg.leaf_umax;
        a.wave_words = mul_mfma_wave_words(a.vmax, a.span, a.umax);
        // the lean instance for leaves up to kMfLeanLeafWords, when 16 waves' slices (4 blocks of 4)
        // fit a CU's 160 KB of LDS
        const uint32_t lw = mul_mfma_lean_leaf_wave_words(a.vmax, a.span, a.umax);
        if (a.umax <= kMfLeanLeafWords && a.umax >= kMfLeanLeafMin && (256 + 4 * (size_t)lw) * 4 * 4 <= 160 * 1024)
            a.lean = 1, a.wave_words = lw;
        if (launch_mul_mfma(a, true, st)) return hip_fail(c, hipGetLastError());
    } else {
        for (uint32_t q = 0; q < kNW; ++q) {
            if (!pg.ntiles[q]) continue;
            MulVProdArgs a{};
            a.B = B, a.tasks = (const MulVTask *)(T + P.off_ka_vtasks) + pg.vtask;
            a.tiles = (const MulVTile *)(T + P.off_ka_vtiles) + pg.tiles[q], a.ntiles = pg.ntiles[q];
            if (launch_mul_vprod(a, kMulTileW[q], st)) return hip_fail(c, hipGetLastError());
        }
    }
    for (const auto &lv : pg.combs) {
        KaCombArgs a{};
        a.B = B, a.t = (const KaComb *)(T + P.off_ka_combs) + lv[0], a.nt = lv[1], a.h = lv[2];
        if (launch_ka_comb(a, st)) return hip_fail(c, hipGetLastError());
    }
    if (!pg.deg) return HM_OK;
    MulDegArgs d{};
    d.B = B, d.u = pg.u, d.v = pg.v, d.out = pg.out;
    if (launch_mul_deg(d, st)) return hip_fail(c, hipGetLastError());
    return HM_OK;
}

} // namespace

hm_status mul_columns(hm_ctx *c, const hm_batch *a, const hm_batch *b, uint32_t K, bool is_signed,
                      hm_batch *out) {
    const uint32_t L = a->nbits;
    if (b->nbits != L || K == 0 || K > L || out->nbits != K) return HM_ERR_INVALID_ARGUMENT;
    const bool flip = is_signed && K == L; // the signed corners are in column L-1 only
    MulPlan *P = nullptr;
    if (hm_status st = get_plan(c, L, K, a->bound, b->bound, flip, P); st) return st;
    for (uint32_t i = 0; i < K; ++i)
        if (out->bound[i] < (uint32_t)std::max<int64_t>(P->res_bound[i], 0))
            return HM_ERR_INVALID_ARGUMENT;
    if (a->n == 0) return HM_OK;
    // workspace: arena + degree rows, chunked over values to a memory budget
    DeviceGuard g(c->device);
    const uint64_t nslots = P->slots.size();
    const uint64_t per_value = P->astride * 4 + nslots * 4;
    size_t freeb = 0, totalb = 0;
    HM_HIP(c, hipMemGetInfo(&freeb, &totalb));
    const uint64_t budget = std::max<uint64_t>((uint64_t)(freeb + c->mws_bytes) / 2, 1ull << 28);
    const uint64_t chunk = std::min<uint64_t>(a->n, budget / per_value);
    if (chunk == 0) return HM_ERR_UNSUPPORTED;
    const uint64_t arena_words = ((P->astride * chunk) + 63) & ~(uint64_t)63;
    HM_HIP(c, grow(c, c->d_mws, c->mws_bytes, (size_t)(arena_words + nslots * chunk) * 4));

    const uint8_t *T = P->d_tab;
    MulBase B{};
    B.arena = c->d_mws;
    B.astride = P->astride;
    B.deg1 = c->d_mws + arena_words;
    B.slots = (const MulSlot *)(T + P->off_slots);
    B.status = c->d_status;
    const BatchArg oa = batch_arg(out);
    std::vector<uint32_t> ooff(K);
    for (uint32_t i = 0, o = 0; i < K; ++i) ooff[i] = o, o += cap_of(out->bound[i]);
    for (uint64_t e0 = 0; e0 < a->n; e0 += chunk) {
        B.e0 = e0;
        B.nv = std::min<uint64_t>(chunk, a->n - e0);
        HM_HIP(c, hipMemsetAsync(B.deg1, 0, (size_t)nslots * B.nv * 4, c->stream));
        MulStageArgs S{};
        S.B = B, S.a = batch_arg(a), S.b = batch_arg(b), S.K = K;
        fill_bounds(S.ab, a), fill_bounds(S.bb, b);
        if (launch_mul_stage(S, c->stream)) return hip_fail(c, hipGetLastError());
        if (P->ppg && P->ppv && !P->ppv_tasks.empty()) {
            MulPPVArgs v{};
            v.B = B;
            v.tasks = (const MulPPTask *)(T + P->off_ppv);
            v.ntasks = (uint32_t)P->ppv_tasks.size();
            v.nin = 2 * K, v.inw = P->ppv_inw, v.qw = P->ppg_umax, v.outw = P->ppv_outw;
            v.wave_words = v.nin * (v.inw + 1) + v.ntasks * v.outw;
            if (launch_mul_ppv(v, c->stream)) return hip_fail(c, hipGetLastError());
        } else if (P->ppg && !P->ppg_groups.empty()) {
            MulPPGArgs g{};
            g.B = B;
            g.groups = (const MulPPGroup *)(T + P->off_ppg_groups);
            g.items = (const MulPPItem *)(T + P->off_ppg_items);
            g.ngroups = (uint32_t)P->ppg_groups.size();
            g.umax = P->ppg_umax, g.vmax = P->ppg_vmax, g.span = P->ppg_span;
            g.wave_words = mul_mfma_wave_words(g.vmax, g.span, g.umax) + 64 * kMfPPGBatch;
            if (launch_mul_ppg(g, c->stream)) return hip_fail(c, hipGetLastError());
        }
        for (uint32_t i = 0; i < K; ++i) {
            const MulPlan::Col &col = P->cols[i];
            MulPPArgs pp{};
            pp.B = B, pp.tasks = (const MulPPTask *)(T + P->off_pp) + col.pp, pp.ntasks = col.npp;
            if (launch_mul_pp(pp, c->stream)) return hip_fail(c, hipGetLastError());
            auto mf_launch = [&](const MfLaunch &m, size_t task_off, uint32_t task0) -> hm_status {
                if (!m.nspans) return HM_OK;
                MulMfmaArgs mf{};
                mf.B = B, mf.tasks = (const MulProdTask *)(T + task_off) + task0;
                mf.spans = (const MulTile *)(T + P->off_mspans) + m.spans;
                mf.recs = (const MulSpanRec *)(T + P->off_mrecs) + m.spans;
                mf.nitems = m.nspans, mf.span = m.span;
                mf.vmax = m.vmax, mf.umax = m.umax;
                mf.wave_words = mul_mfma_wave_words(mf.vmax, mf.span, mf.umax);
                if (m.lean) mf.lean = 1, mf.wave_words = mul_mfma_lean_leaf_wave_words(mf.vmax, mf.span, mf.umax);
                return launch_mul_mfma(mf, false, c->stream) ? hip_fail(c, hipGetLastError()) : HM_OK;
            };
            if (hm_status st = mf_launch(col.ppl, P->off_ppm, col.ppm); st) return st;
            MulScanArgs sc{};
            sc.B = B;
            sc.items = (const uint32_t *)(T + P->off_lists) + col.items;
            sc.prefix = (const uint32_t *)(T + P->off_lists) + col.prefix;
            sc.nitems = col.nitems;
            sc.res = col.res;
            sc.out = oa, sc.out_off = ooff[i], sc.out_cap = cap_of(out->bound[i]);
            sc.chunks = (std::max(col.maxwords, 2 * sc.out_cap) + 255) / 256;
            if (launch_mul_scan(sc, c->stream)) return hip_fail(c, hipGetLastError());
            if (col.nrows) {
                MulRowArgs ra{};
                ra.B = B, ra.recs = (const MulSpanRec *)(T + P->off_rows) + col.rows;
                ra.ntasks = col.nrows, ra.uw = col.rows_uw, ra.vw = col.rows_vw, ra.ow = col.rows_ow;
                ra.qw = std::min(col.rows_qw, col.rows_uw);
                ra.wave_words = col.nrows * (ra.uw + ra.vw + ra.ow + 2 + 6);
                if (launch_mul_rows(ra, c->stream)) return hip_fail(c, hipGetLastError());
            }
            for (const MfLaunch &m : col.mfl)
                if (hm_status st = mf_launch(m, P->off_prod, col.prod); st) return st;
            for (uint32_t q = 0; q < kNW; ++q) {
                if (!col.ntiles[q]) continue;
                MulProdArgs pr{};
                pr.B = B;
                pr.tasks = (const MulProdTask *)(T + P->off_prod) + col.prod;
                pr.tiles = (const MulTile *)(T + P->off_tiles) + col.tiles[q];
                pr.ntiles = col.ntiles[q];
                if (launch_mul_prod(pr, kMulTileW[q], c->stream)) return hip_fail(c, hipGetLastError());
            }
            // Karatsuba products: lane 0 on the context stream, lane 1 on the auxiliary stream
            // (each lane's products one at a time: they share the lane's scratch region); the
            // lanes fork after this column's scan and schoolbook launches (the products read its
            // prefixes) and join before the next column's scan (which reads their carries)
            const bool two = col.ka.size() > 1 && kKaLanes > 1;
            if (two) {
                if (hm_status st = ensure_aux_stream(c); st) return st;
                HM_HIP(c, hipEventRecord(c->ev_fork, c->stream));
                HM_HIP(c, hipStreamWaitEvent(c->aux_stream, c->ev_fork, 0));
            }
            hm_status kst = HM_OK;
            for (const KaProg &pg : col.ka)
                if ((kst = run_ka(c, *P, pg, B, two && pg.lane ? c->aux_stream : c->stream))) break;
            if (two) {
                // joined on every path, a failed lane's too: no unjoined fork under capture, and
                // no auxiliary-stream work left running behind a caller that syncs c->stream only
                const hipError_t e1 = hipEventRecord(c->ev_join, c->aux_stream);
                const hipError_t e2 = hipStreamWaitEvent(c->stream, c->ev_join, 0);
                if (kst == HM_OK && e1 != hipSuccess) return hip_fail(c, e1);
                if (kst == HM_OK && e2 != hipSuccess) return hip_fail(c, e2);
            }
            if (kst) return kst;
        }
        MulFinalArgs F{};
        F.B = B, F.res = (const uint32_t *)(T + P->off_res), F.K = K, F.out = oa;
        fill_bounds(F.ob, out);
        if (launch_mul_final(F, c->stream)) return hip_fail(c, hipGetLastError());
    }
    return HM_OK;
}

} // namespace hm
