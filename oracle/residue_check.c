/*
 * residue_check.c — CPU CHECKER (test infrastructure only, like homomorph_oracle.c): residues of
 * ciphertext polynomials modulo a random degree-64 polynomial f = X^64 + g.
 *
 * P -> P mod f is a ring homomorphism GF(2)[X] -> GF(2)[X]/(f).  Every circuit of the reference
 * (src/impls/numbers/common.rs: add_internal :37-56, mul_unsigned_internal :66-105,
 * mul_signed_internal :115-155; the gates of src/cipher.rs:58-90) is a ring expression in its
 * input polynomials, so the residue of each output polynomial equals the same circuit evaluated
 * on the residues of the inputs.  Comparing the two checks EVERY output polynomial of a batch of
 * any size in O(size) time: a wrong output E != P passes only if f divides E - P, which for a
 * random f has probability about deg(E - P) / 2^64 (a CRC-64 with a secret polynomial).  This is
 * the size-independent parity check the tests use where the bit-serial oracle would take hours
 * (the full configs[4] batch, the u32 multiply's deep columns); the oracle itself still pins
 * sampled values bit for bit.
 *
 * The residue circuits below restate the reference's operation sequence over residues (XOR =
 * add, AND = product mod f, NOT = + 1) so that they read like the oracle's circuits.
 */
#include <immintrin.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int g_res_threads = 0; /* 0: OpenMP default */
void oracle_residue_threads(int n) { g_res_threads = n > 0 ? n : 0; }

typedef struct {
    uint64_t g;  /* f = X^64 + g */
    uint64_t mu; /* floor(X^128 / f) = X^64 + mu (Barrett) */
} modf;

static inline void clmul(uint64_t a, uint64_t b, uint64_t *lo, uint64_t *hi) {
    const __m128i p = _mm_clmulepi64_si128(_mm_cvtsi64_si128((long long)a),
                                           _mm_cvtsi64_si128((long long)b), 0);
    *lo = (uint64_t)_mm_cvtsi128_si64(p);
    *hi = (uint64_t)_mm_extract_epi64(p, 1);
}

/* (hi X^64 + lo) mod f, Barrett: q = floor((hi X^64 + lo) / f) = hi ^ floor(hi * mu / X^64);
 * r = lo ^ low64(q * g) (the X^64 part of q * f cancels hi exactly) */
static inline uint64_t reduce(const modf *m, uint64_t hi, uint64_t lo) {
    uint64_t l, h;
    clmul(hi, m->mu, &l, &h);
    const uint64_t q = hi ^ h;
    clmul(q, m->g, &l, &h);
    return lo ^ l;
}

static inline uint64_t mulmod(const modf *m, uint64_t a, uint64_t b) {
    uint64_t lo, hi;
    clmul(a, b, &lo, &hi);
    return reduce(m, hi, lo);
}

static modf make_modf(uint64_t g) {
    /* mu = floor(X^128 / (X^64 + g)) by long division over 129-bit values */
    modf m;
    m.g = g;
    uint64_t r[3] = {0, 0, 1}; /* X^128 */
    uint64_t q[2] = {0, 0};
    for (int k = 128; k >= 64; --k) {
        const int w = k / 64, b = k % 64;
        if ((r[w] >> b) & 1) {
            const int s = k - 64; /* subtract f * X^s */
            q[s / 64] |= 1ull << (s % 64);
            r[w] ^= 1ull << b;
            /* g * X^s */
            if (s % 64 == 0) {
                r[s / 64] ^= g;
            } else {
                r[s / 64] ^= g << (s % 64);
                r[s / 64 + 1] ^= g >> (64 - s % 64);
            }
        }
    }
    m.mu = q[0]; /* q = X^64 + mu */
    return m;
}

static inline uint64_t limbs_residue(const modf *m, const uint64_t *c, size_t len) {
    uint64_t acc = 0;
    for (size_t j = len; j-- > 0;) acc = reduce(m, acc, c[j]); /* acc * X^64 + c_j */
    return acc;
}

static inline uint32_t cap_of(uint32_t bound) { return bound / 64 + 1; }

/* Residue of every (value, bit) polynomial of a batch (layout of include/homomorph_gpu.h), and
 * the number of degree words that disagree with their limbs (the exact top bit; 0 for null). */
int oracle_residues(const uint64_t *limbs, const uint32_t *deg, const uint32_t *bound,
                    uint32_t nbits, size_t n, uint64_t g, uint64_t *out, size_t *bad_degrees) {
    const modf m = make_modf(g);
    size_t stride = 0;
    size_t *off = (size_t *)malloc(nbits * sizeof(size_t));
    if (!off) return 1;
    for (uint32_t i = 0; i < nbits; ++i) off[i] = stride, stride += cap_of(bound[i]);
    size_t bad = 0;
#pragma omp parallel for num_threads(g_res_threads ? g_res_threads : omp_get_max_threads()) \
    reduction(+ : bad) schedule(dynamic, 64) if (n > 1)
    for (size_t e = 0; e < n; ++e) {
        for (uint32_t i = 0; i < nbits; ++i) {
            const uint64_t *c = limbs + e * stride + off[i];
            const size_t len = cap_of(bound[i]);
            out[e * nbits + i] = limbs_residue(&m, c, len);
            size_t top = 0;
            for (size_t k = len; k-- > 0;)
                if (c[k]) {
                    top = 64 * k + 63 - (size_t)__builtin_clzll(c[k]);
                    break;
                }
            if (deg && top != deg[e * nbits + i]) ++bad;
        }
    }
    free(off);
    if (bad_degrees) *bad_degrees = bad;
    return 0;
}

/* add_internal (common.rs:37-56) over residues */
int oracle_residue_add(const uint64_t *ra, const uint64_t *rb, uint32_t nbits, size_t n,
                       uint64_t g, uint64_t *out) {
    const modf m = make_modf(g);
#pragma omp parallel for num_threads(g_res_threads ? g_res_threads : omp_get_max_threads()) \
    schedule(static) if (n > 1024)
    for (size_t e = 0; e < n; ++e) {
        const uint64_t *a = ra + e * nbits, *b = rb + e * nbits;
        uint64_t *o = out + e * nbits;
        uint64_t carry = 0; /* CipheredBit::zero */
        for (uint32_t i = 0; i < nbits; ++i) {
            o[i] = a[i] ^ b[i] ^ carry;
            if (i + 1 >= nbits) break;
            const uint64_t c = mulmod(&m, a[i] ^ b[i], carry);
            carry = c ^ mulmod(&m, mulmod(&m, a[i], b[i]), c ^ 1u);
        }
    }
    return 0;
}

/* mul_unsigned_internal / mul_signed_internal (common.rs:66-155) over residues: the k-bit
 * circuit on the first k residues of each value (k = nbits for the full product; the signed
 * corner terms only then).  ra/rb hold nbits residues per value, out k. */
int oracle_residue_mul(const uint64_t *ra, const uint64_t *rb, uint32_t nbits, uint32_t k,
                       int is_signed, size_t n, uint64_t g, uint64_t *out) {
    if (k == 0 || k > nbits) return 1;
    const modf m = make_modf(g);
    const size_t ncar = (size_t)k * k * (k + 1) / 2 + 1;
    int fail = 0;
#pragma omp parallel num_threads(g_res_threads ? g_res_threads : omp_get_max_threads()) if (n > 64)
    {
        uint64_t *pp = (uint64_t *)malloc((size_t)k * k * 8);
        uint64_t *carries = (uint64_t *)malloc(ncar * 8);
        if (!pp || !carries) {
#pragma omp atomic write
            fail = 1;
        }
#pragma omp for schedule(static)
        for (size_t e = 0; e < n; ++e) {
            if (!pp || !carries) continue;
            const uint64_t *a = ra + e * nbits, *b = rb + e * nbits;
            uint64_t *res = out + e * k;
            for (uint32_t i = 0; i < k; ++i) res[i] = 0;
            for (uint32_t i = 0; i < k; ++i)
                for (uint32_t j = 0; j < k; ++j) pp[i * k + j] = mulmod(&m, a[i], b[j]);
            if (is_signed && k == nbits) {
                pp[0 * k + (k - 1)] ^= 1u;
                pp[(k - 1) * k + 0] ^= 1u;
            }
            size_t nc = 0, offset = 0;
            for (uint32_t i = 0; i < k; ++i) {
                const size_t cur = (size_t)i * (i + 1) / 2;
                for (uint32_t j = 0; j <= i; ++j) {
                    const uint64_t p = pp[j * k + (i - j)];
                    if (i + 1 < k) carries[nc++] = mulmod(&m, p, res[i]);
                    res[i] ^= p;
                }
                for (size_t j = 0; j < cur; ++j) {
                    if (i + 1 < k) carries[nc++] = mulmod(&m, res[i], carries[offset + j]);
                    res[i] ^= carries[offset + j];
                }
                offset += cur;
            }
        }
        free(pp);
        free(carries);
    }
    return fail;
}

/* gates (cipher.rs:58-90): AND = a b, OR = a + b + a b, XOR = a + b, NOT = a + 1 */
int oracle_residue_gate(int op, const uint64_t *ra, const uint64_t *rb, size_t count, uint64_t g,
                        uint64_t *out) {
    const modf m = make_modf(g);
    for (size_t t = 0; t < count; ++t) {
        switch (op) {
        case 0: out[t] = mulmod(&m, ra[t], rb[t]); break;
        case 1: out[t] = ra[t] ^ rb[t] ^ mulmod(&m, ra[t], rb[t]); break;
        case 2: out[t] = ra[t] ^ rb[t]; break;
        case 3: out[t] = ra[t] ^ 1u; break;
        default: return 1;
        }
    }
    return 0;
}

/* residue of one polynomial and a product mod f (unit tests of the checker itself) */
uint64_t oracle_residue_of(const uint64_t *c, size_t len, uint64_t g) {
    const modf m = make_modf(g);
    return limbs_residue(&m, c, len);
}
uint64_t oracle_residue_mulmod(uint64_t a, uint64_t b, uint64_t g) {
    const modf m = make_modf(g);
    return mulmod(&m, a, b);
}
