// ASan/UBSan driver for the engine library's HOST-ONLY entry points (include/homomorph_gpu.h):
// status strings, output bounds, the multiplier cost model, batch strides, the wire-format
// header parser (fed valid, truncated and randomly corrupted images) and NULL-context handling.
// No hm_ctx is created, so no GPU is needed.  Built and run by tests/test_sanitize.py, linked
// against the normally built kernel objects.
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/homomorph_gpu.h"

static int fails = 0;
#define CHECK(c)                                                                                  \
    do {                                                                                          \
        if (!(c)) {                                                                               \
            std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c);                      \
            ++fails;                                                                              \
        }                                                                                         \
    } while (0)

int main() {
    for (int s = -1; s < 16; ++s) CHECK(hm_status_string(s) != nullptr);
    CHECK(hm_abi_version() == HM_ABI_VERSION);
    std::vector<uint32_t> b(32, 256), o(32);
    CHECK(hm_add_out_bounds(32, b.data(), b.data(), o.data()) == HM_OK && o[31] == 92 * 256);
    CHECK(hm_add_out_bounds(0, b.data(), b.data(), o.data()) == HM_ERR_INVALID_ARGUMENT);
    CHECK(hm_mul_out_bounds(8, b.data(), b.data(), 0, o.data()) == HM_OK && o[7] == 14336);
    CHECK(hm_mul_out_bounds(32, b.data(), b.data(), 0, o.data()) == HM_ERR_UNSUPPORTED);
    double w = 0, ob = 0, md = 0;
    CHECK(hm_mul_cost(32, 32, b.data(), b.data(), 0, &w, &ob, &md) == HM_OK && w > 1e18);
    CHECK(hm_mul_cost(32, 33, b.data(), b.data(), 0, &w, &ob, &md) == HM_ERR_INVALID_ARGUMENT);
    for (int g = 0; g <= HM_OP_MUL_SIGNED; ++g) (void)hm_gate_out_bounds((hm_op)g, 32, b.data(), b.data(), o.data());
    CHECK(hm_gate_out_bounds(HM_OP_NOT, 32, b.data(), nullptr, o.data()) == HM_OK);
    CHECK(hm_batch_stride(32, b.data()) == 32 * 5);
    // wire header: a valid image, then truncations and random corruptions of it
    const uint32_t bd[3] = {128, 300, 0};
    const uint64_t n = 3;
    const uint64_t size = hm_wire_bytes(3, bd, n);
    CHECK(size > 0);
    std::vector<uint8_t> img(size, 0);
    std::memcpy(img.data(), "HMCB", 4);
    img[4] = 1, img[8] = 3, img[16] = (uint8_t)n;
    std::memcpy(img.data() + 24, bd, sizeof bd);
    uint32_t nb = 0, got[HM_MAX_BITS];
    uint64_t nv = 0;
    CHECK(hm_wire_peek(img.data(), img.size(), &nb, &nv, got) == HM_OK && nb == 3 && nv == n);
    for (size_t len = 0; len < img.size(); len += 7) (void)hm_wire_peek(img.data(), len, &nb, &nv, got);
    std::mt19937_64 rng(5);
    for (int t = 0; t < 20000; ++t) {
        std::vector<uint8_t> bad = img;
        const int flips = 1 + (int)(rng() % 4);
        for (int f = 0; f < flips; ++f) bad[rng() % 40] ^= (uint8_t)(1u << (rng() % 8));
        (void)hm_wire_peek(bad.data(), bad.size(), &nb, &nv, got);
    }
    CHECK(hm_wire_bytes(0, bd, 1) == 0 && hm_wire_bytes(3, nullptr, 1) == 0);
    // NULL contexts are rejected, never dereferenced
    uint16_t r = 0;
    CHECK(hm_validate_operation(nullptr, HM_OP_ADD, &r) != HM_OK);
    CHECK(hm_fresh_bound(nullptr) == 0 && hm_ctx_mask_bytes(nullptr) == 0);
    CHECK(hm_ctx_generation(nullptr) == 0 && hm_ctx_stream(nullptr) == nullptr);
    CHECK(hm_add_batch(nullptr, nullptr, nullptr, nullptr) != HM_OK);
    CHECK(hm_ctx_set_mul_scratch(nullptr, 1000) == HM_ERR_INVALID_ARGUMENT);
    CHECK(hm_ctx_clear_kernel_timing(nullptr) == HM_ERR_INVALID_ARGUMENT);
    CHECK(hm_wire_encode(nullptr, nullptr, nullptr, 0) != HM_OK);
    CHECK(hm_wire_decode(nullptr, img.data(), img.size(), nullptr) != HM_OK);
    hm_ctx_destroy(nullptr);
    if (fails) return 1;
    std::printf("engine host-only sanitizer run: ok\n");
    return 0;
}
