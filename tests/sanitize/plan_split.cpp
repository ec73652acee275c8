// Host-only check of the multiplier planner's split Karatsuba plans (mul_host.cpp, round 6), under
// ASan/UBSan: the planner source is compiled into this driver (its planning functions are
// internal), no hm_ctx and no GPU.  Built and run by tests/test_sanitize.py.
//  - K = 16 with a 2^18-word scratch limit splits products into subtree programs, and the split
//    plan issues exactly the leaf products of the breadth-first plan (the same multiset of leaf
//    shapes), with every scratch region below the limit's bound;
//  - K = 21 plans with the default limit (its largest product needs 3.1e8 scratch words
//    breadth-first, past the 28-bit views), and K = 20's default plan is not split.
#include "../../homomorph-rust_amd/csrc/mul_host.cpp"

#include <cstdio>
#include <tuple>

static int fails = 0;
#define CHECK(c)                                                                                  \
    do {                                                                                          \
        if (!(c)) {                                                                               \
            std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c);                      \
            ++fails;                                                                              \
        }                                                                                         \
    } while (0)

static bool plan(uint32_t K, uint64_t scratch, hm::MulPlan &P) {
    P.L = 32, P.K = K, P.is_signed = false;
    P.ab.assign(K, 256), P.bb.assign(K, 256);
    P.ka_min = 256, P.ka_leaf = 256, P.mfma = true, P.ka_scratch = scratch;
    return hm::build_plan(P);
}

static size_t subprograms(const hm::MulPlan &P) {
    size_t n = 0;
    for (const auto &c : P.cols)
        for (const auto &g : c.ka) n += !g.deg;
    return n;
}

static std::vector<std::tuple<uint32_t, uint32_t, uint32_t>> leaf_shapes(const hm::MulPlan &P) {
    std::vector<std::tuple<uint32_t, uint32_t, uint32_t>> v;
    for (const auto &t : P.ka_vtasks) v.emplace_back(t.nu, t.nv, t.nout);
    std::sort(v.begin(), v.end());
    return v;
}

int main() {
    hm::MulPlan whole, split;
    CHECK(plan(16, hm::kKaScratchWords, whole));
    CHECK(plan(16, 1u << 18, split));
    CHECK(subprograms(whole) == 0);
    CHECK(subprograms(split) > 0);
    CHECK(whole.ka_vtasks.size() == split.ka_vtasks.size());
    CHECK(leaf_shapes(whole) == leaf_shapes(split));
    CHECK(split.astride < whole.astride); // less scratch per value
    hm::MulPlan k20, k21;
    CHECK(plan(20, hm::kKaScratchWords, k20));
    CHECK(subprograms(k20) == 0);
    CHECK(plan(21, hm::kKaScratchWords, k21));
    CHECK(subprograms(k21) > 0);
    if (fails) return 1;
    std::printf("ok (K = 16: %zu split programs, %zu leaves; K = 21: %zu split programs)\n",
                subprograms(split), split.ka_vtasks.size(), subprograms(k21));
    return 0;
}
