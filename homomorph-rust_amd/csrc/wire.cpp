// wire.cpp — the ciphertext batch wire format (include/homomorph_gpu.h, "wire format"): a
// self-describing little-endian image of an hm_batch for storage and host<->device transfer.
// The reference has no ciphertext serialisation; its key byte format (little-endian u64 limbs,
// src/polynomial.rs:99-122) is reused for the limbs.
#include <cstring>

#include "ctx.h"

namespace {

constexpr uint8_t kMagic[4] = {'H', 'M', 'C', 'B'};
constexpr uint32_t kVersion = 1;
constexpr size_t kHeader = 24;

struct Layout {
    uint64_t deg_off, limb_off, total, stride;
};

bool layout(uint32_t nbits, const uint32_t *bound, uint64_t n, Layout &L) {
    if (nbits == 0 || nbits > HM_MAX_BITS || !bound) return false;
    uint64_t stride = 0;
    for (uint32_t i = 0; i < nbits; ++i) {
        if (bound[i] > (1u << 30)) return false;
        stride += bound[i] / 64 + 1;
    }
    // n * stride limbs must not overflow (and stay addressable)
    if (n > ((uint64_t)1 << 40) || stride > ((uint64_t)1 << 30)) return false;
    L.stride = stride;
    L.deg_off = kHeader + 4ull * nbits;
    L.limb_off = (L.deg_off + 4ull * n * nbits + 7) & ~7ull;
    L.total = L.limb_off + 8ull * n * stride;
    return true;
}

inline uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
inline uint64_t rd64(const uint8_t *p) { return (uint64_t)rd32(p) | (uint64_t)rd32(p + 4) << 32; }
inline void wr32(uint8_t *p, uint32_t v) {
    for (int k = 0; k < 4; ++k) p[k] = (uint8_t)(v >> (8 * k));
}
inline void wr64(uint8_t *p, uint64_t v) { wr32(p, (uint32_t)v), wr32(p + 4, (uint32_t)(v >> 32)); }

// one polynomial of the image: degree within the bound, top coefficient set (or the null
// polynomial with degree 0), zeros above the degree -- the layout invariant the kernels assume
bool valid_poly(const uint8_t *limbs, uint32_t cap, uint32_t deg, uint32_t bound) {
    if (deg > bound) return false;
    const uint32_t top = deg / 64;
    for (uint32_t k = top + 1; k < cap; ++k)
        if (rd64(limbs + 8ull * k)) return false;
    const uint64_t w = rd64(limbs + 8ull * top);
    const uint32_t tb = deg % 64;
    if (tb < 63 && (w >> (tb + 1))) return false;
    return deg == 0 || ((w >> tb) & 1ull);
}

} // namespace

using hm::hip_fail;

extern "C" {

uint64_t hm_wire_bytes(uint32_t nbits, const uint32_t *bound, uint64_t n) {
    Layout L;
    return layout(nbits, bound, n, L) ? L.total : 0;
}

hm_status hm_wire_peek(const uint8_t *src, size_t len, uint32_t *nbits, uint64_t *n,
                       uint32_t *bound) try {
    if (!src || len < kHeader) return HM_ERR_INVALID_ARGUMENT;
    if (std::memcmp(src, kMagic, 4) || rd32(src + 4) != kVersion || rd32(src + 12) != 0)
        return HM_ERR_INVALID_ARGUMENT;
    const uint32_t nb = rd32(src + 8);
    const uint64_t nv = rd64(src + 16);
    if (nb == 0 || nb > HM_MAX_BITS || len < kHeader + 4ull * nb) return HM_ERR_INVALID_ARGUMENT;
    uint32_t bd[HM_MAX_BITS];
    for (uint32_t i = 0; i < nb; ++i) bd[i] = rd32(src + kHeader + 4ull * i);
    Layout L;
    if (!layout(nb, bd, nv, L) || L.total != len) return HM_ERR_INVALID_ARGUMENT;
    if (nbits) *nbits = nb;
    if (n) *n = nv;
    if (bound) std::memcpy(bound, bd, 4ull * nb);
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_wire_encode(hm_ctx *c, const hm_batch *in, uint8_t *dst, size_t cap) try {
    if (!c || !dst) return HM_ERR_INVALID_ARGUMENT;
    if (hm_status st = hm::check_batch(in); st) return st;
    Layout L;
    if (!layout(in->nbits, in->bound, in->n, L)) return HM_ERR_UNSUPPORTED;
    if (cap < L.total) return HM_ERR_INVALID_ARGUMENT;
    std::memset(dst, 0, L.limb_off);
    std::memcpy(dst, kMagic, 4);
    wr32(dst + 4, kVersion), wr32(dst + 8, in->nbits), wr32(dst + 12, 0), wr64(dst + 16, in->n);
    for (uint32_t i = 0; i < in->nbits; ++i) wr32(dst + kHeader + 4ull * i, in->bound[i]);
    if (in->n == 0) return HM_OK;
    hm::DeviceGuard g(c->device);
    HM_HIP(c, hipStreamSynchronize(c->stream));
    // the host is little-endian (x86-64), so the device words copy straight into the image
    HM_HIP(c, hipMemcpy(dst + L.deg_off, in->degree, 4ull * in->n * in->nbits,
                        hipMemcpyDeviceToHost));
    HM_HIP(c, hipMemcpy(dst + L.limb_off, in->limbs, 8ull * in->n * L.stride,
                        hipMemcpyDeviceToHost));
    return HM_OK;
} HM_ABI_CATCH

hm_status hm_wire_decode(hm_ctx *c, const uint8_t *src, size_t len, hm_batch *out) try {
    if (!c) return HM_ERR_INVALID_ARGUMENT;
    if (hm_status st = hm::check_batch(out); st) return st;
    uint32_t nb = 0;
    uint64_t nv = 0;
    uint32_t bd[HM_MAX_BITS];
    if (hm_status st = hm_wire_peek(src, len, &nb, &nv, bd); st) return st;
    if (nb != out->nbits || nv != out->n || std::memcmp(bd, out->bound, 4ull * nb))
        return HM_ERR_INVALID_ARGUMENT;
    Layout L;
    layout(nb, bd, nv, L);
    for (uint64_t e = 0; e < nv; ++e) {
        uint64_t off = 0;
        for (uint32_t i = 0; i < nb; ++i) {
            const uint32_t cap = bd[i] / 64 + 1;
            const uint32_t deg = rd32(src + L.deg_off + 4ull * (e * nb + i));
            if (!valid_poly(src + L.limb_off + 8ull * (e * L.stride + off), cap, deg, bd[i]))
                return HM_ERR_BAD_INPUT;
            off += cap;
        }
    }
    if (nv == 0) return HM_OK;
    hm::DeviceGuard g(c->device);
    HM_HIP(c, hipStreamSynchronize(c->stream));
    HM_HIP(c, hipMemcpy(out->degree, src + L.deg_off, 4ull * nv * nb, hipMemcpyHostToDevice));
    HM_HIP(c, hipMemcpy(out->limbs, src + L.limb_off, 8ull * nv * L.stride,
                        hipMemcpyHostToDevice));
    return HM_OK;
} HM_ABI_CATCH

} // extern "C"
