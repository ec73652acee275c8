// Exception safety of the C ABI (no C++ exception crosses the boundary).
// Replaces the global operator new of this executable so that the n-th allocation made inside the
// engine library's host code throws std::bad_alloc, for every n up to the entry point's last
// allocation, and checks that each host-only entry returns HM_ERR_OUT_OF_MEMORY (or HM_OK once no
// allocation fails) instead of unwinding into the caller.  hm_mul_out_bounds runs the
// multiplier's plan builder (mul_host.cpp build_plan) on the host, so a failure anywhere inside
// the plan is covered.  No hm_ctx is created, so no GPU is needed.  Built (unsanitised) and run
// by tests/test_sanitize.py.
#include <cstdio>
#include <cstdlib>
#include <new>
#include <string_view>
#include <vector>

#include "../../include/homomorph_gpu.h"

static long g_countdown = -1; // < 0: never fail; 0: the next allocation throws
static long g_allocs = 0;

void *operator new(std::size_t n) {
    ++g_allocs;
    if (g_countdown == 0) throw std::bad_alloc();
    if (g_countdown > 0) --g_countdown;
    void *p = std::malloc(n ? n : 1);
    if (!p) throw std::bad_alloc();
    return p;
}
void *operator new[](std::size_t n) { return operator new(n); }
void operator delete(void *p) noexcept { std::free(p); }
void operator delete[](void *p) noexcept { std::free(p); }
void operator delete(void *p, std::size_t) noexcept { std::free(p); }
void operator delete[](void *p, std::size_t) noexcept { std::free(p); }

static int fails = 0;
#define CHECK(c)                                                                                  \
    do {                                                                                          \
        if (!(c)) {                                                                               \
            std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c);                      \
            ++fails;                                                                              \
        }                                                                                         \
    } while (0)

// Calls f() with allocation k failing, for k = 0, 1, ... until f() runs without a failure; every
// failed run must return HM_ERR_OUT_OF_MEMORY and the clean run HM_OK.  Returns the number of
// allocation points exercised.
template <class F> static long sweep(const char *what, F f) {
    long k = 0;
    for (;; ++k) {
        g_countdown = k;
        const long before = g_allocs;
        const int st = f();
        const long used = g_allocs - before;
        g_countdown = -1;
        if (used <= k) { // no allocation failed: the call completed
            CHECK(st == HM_OK);
            break;
        }
        if (st != HM_ERR_OUT_OF_MEMORY) {
            std::fprintf(stderr, "%s: allocation %ld failed, status %d\n", what, k, st);
            ++fails;
        }
    }
    std::printf("%s: %ld allocation points, each one returned HM_ERR_OUT_OF_MEMORY\n", what, k);
    return k;
}

int main() {
    CHECK(hm_abi_version() == HM_ABI_VERSION);
    std::vector<uint32_t> b(32, 256), o(32);
    // the u8 multiplier plan, and the u32 plan's low 12 columns (build_plan's slots, products,
    // Karatsuba programs and task tables)
    long n1 = sweep("hm_mul_out_bounds u8", [&] {
        return (int)hm_mul_out_bounds(8, b.data(), b.data(), 0, o.data());
    });
    long n2 = sweep("hm_mul_out_bounds i8", [&] {
        return (int)hm_mul_out_bounds(8, b.data(), b.data(), 1, o.data());
    });
    long n3 = sweep("hm_mul_cost u32 k=20", [&] {
        double w, ob, md;
        return (int)hm_mul_cost(32, 20, b.data(), b.data(), 0, &w, &ob, &md);
    });
    CHECK(n1 > 10 && n2 > 10 && n3 > 2);
    // a failure that stops the plan part-way must leave nothing behind that breaks the next call
    CHECK(hm_mul_out_bounds(8, b.data(), b.data(), 0, o.data()) == HM_OK && o[7] == 14336);
    CHECK(std::string_view(hm_status_string(HM_ERR_OUT_OF_MEMORY)) != "unknown status");
    if (fails) return 1;
    std::printf("engine C ABI under forced allocation failures: ok\n");
    return 0;
}
