/*
 * homomorph_oracle.c — CPU ORACLE (test infrastructure only; see homomorph_oracle.h).
 *
 * Operation-for-operation C restatement of the reference's hot path so that results AND the
 * reference's CPU cost profile are reproduced:
 *   src/polynomial.rs   degree bookkeeping, add / add_assign / add_bool_assign, bit-serial
 *                       carry-less mul, bitwise long-division rem, evaluate, equality;
 *   src/cipher.rs       CipheredBit gates, subset-sum cipher, rem-based decipher;
 *   src/impls/numbers/common.rs   ripple-carry add, carry-save unsigned / signed multiply.
 * Randomness (getrandom in the reference) is replaced by the SplitMix64 contract below.
 * Never linked into the product library; loaded by tests/, smoke() and bench.py's cpu leg.
 */
#include "homomorph_oracle.h"

#include <stdlib.h>
#include <string.h>

#define BPC 64 /* BITS_PER_COEFF, polynomial.rs:9 (usize = 64-bit) */

typedef struct {
    uint64_t *c;
    size_t len;
    size_t deg;
} poly;

static _Thread_local uint64_t g_limb_products = 0; /* calling thread only */
uint64_t oracle_limb_products(void) { return g_limb_products; }
void oracle_reset_counters(void) { g_limb_products = 0; }

static void *xcalloc(size_t n, size_t sz) {
    void *p = calloc(n ? n : 1, sz);
    if (!p) abort();
    return p;
}

/* polynomial.rs:35-42 — index of the highest set bit, 0 for the null polynomial */
size_t oracle_compute_degree(const uint64_t *c, size_t len) {
    for (size_t k = len; k-- > 0;) {
        if (c[k]) return (size_t)(BPC - 1 - __builtin_clzll(c[k])) + (size_t)BPC * k;
    }
    return 0;
}

static poly p_from(const uint64_t *src, size_t len) { /* Polynomial::new, :53-63 */
    poly p;
    p.len = len ? len : 1;
    p.c = (uint64_t *)xcalloc(p.len, 8);
    if (len) memcpy(p.c, src, len * 8);
    p.deg = oracle_compute_degree(p.c, p.len);
    return p;
}
static poly p_null(void) { /* :132-137 */
    poly p;
    p.len = 1;
    p.c = (uint64_t *)xcalloc(1, 8);
    p.deg = 0;
    return p;
}
static poly p_monomial(size_t d) { /* :142-150 */
    poly p;
    p.len = d / BPC + 1;
    p.c = (uint64_t *)xcalloc(p.len, 8);
    p.c[d / BPC] = 1ull << (d % BPC);
    p.deg = d;
    return p;
}
static void p_free(poly *p) {
    free(p->c);
    p->c = NULL;
    p->len = 0;
}
static int p_is_null(const poly *p) { return p->deg == 0 && (p->c[0] & 1) == 0; }

/* :190-213 — fresh buffer of max_deg/64+1 limbs; degree recomputed only on equal degrees */
static poly p_add(const poly *a, const poly *b) {
    size_t md = a->deg > b->deg ? a->deg : b->deg;
    poly r;
    r.len = md / BPC + 1;
    r.c = (uint64_t *)xcalloc(r.len, 8);
    for (size_t k = 0; k < r.len; k++) {
        uint64_t x = k < a->len ? a->c[k] : 0;
        uint64_t y = k < b->len ? b->c[k] : 0;
        r.c[k] = x ^ y;
    }
    r.deg = (a->deg == b->deg) ? oracle_compute_degree(r.c, r.len) : md;
    return r;
}

/* :216-235 — grow to the rhs's relevant length, XOR the overlapping limbs, rescan */
static void p_add_assign(poly *self, const poly *o) {
    size_t lhs = self->deg / BPC + 1, rhs = o->deg / BPC + 1;
    if (rhs > lhs) {
        uint64_t *nc = (uint64_t *)xcalloc(rhs, 8);
        memcpy(nc, self->c, lhs * 8);
        free(self->c);
        self->c = nc;
        self->len = rhs;
    }
    size_t m = self->len < o->len ? self->len : o->len;
    for (size_t k = 0; k < m; k++) self->c[k] ^= o->c[k];
    self->deg = oracle_compute_degree(self->c, self->len);
}

/* :238-243 */
static void p_add_bool_assign(poly *self, int x) {
    if (x) {
        self->c[0] ^= 1;
        self->deg = oracle_compute_degree(self->c, self->len);
    }
}

/* :252-310 — schoolbook over relevant limbs; inner loop walks the set bits of a's limb */
static poly p_mul(const poly *a, const poly *b) {
    if (p_is_null(a) || p_is_null(b)) return p_null();
    size_t rlen = (a->deg + b->deg) / BPC + 1;
    poly r;
    r.len = rlen;
    r.c = (uint64_t *)xcalloc(rlen, 8);
    size_t na = a->deg / BPC + 1, nb = b->deg / BPC + 1;
    g_limb_products += (uint64_t)na * nb;
    for (size_t i = 0; i < na; i++) {
        uint64_t ai = a->c[i];
        for (size_t j = 0; j < nb; j++) {
            uint64_t bj = b->c[j];
            uint64_t rest = ai;
            if (rest & 1) {
                r.c[i + j] ^= bj;
                rest ^= 1;
            }
            uint64_t hi = 0;
            while (rest) {
                unsigned k = (unsigned)__builtin_ctzll(rest);
                r.c[i + j] ^= bj << k;
                hi ^= bj >> (BPC - k); /* k >= 1 here */
                rest &= rest - 1;
            }
            if (i + j + 1 < rlen) r.c[i + j + 1] ^= hi;
        }
    }
    r.deg = a->deg + b->deg;
    return r;
}

/* :316-365 — bitwise long division keeping the dividend's buffer; returns status */
static int p_rem(const poly *a, const poly *s, poly *out) {
    if (!(s->deg > 0 || (s->c[0] & 1) == 1)) return OR_ERR_DIVIDE_BY_ZERO;
    if (s->deg == 0) return OR_ERR_DIVISOR_IS_ONE; /* the reference's loop never exits */
    poly r;
    r.len = a->len;
    r.c = (uint64_t *)xcalloc(r.len, 8);
    memcpy(r.c, a->c, a->len * 8);
    size_t rd = a->deg;
    size_t sl = s->deg / BPC + 1;
    while (rd >= s->deg) {
        size_t sh = rd - s->deg, ws = sh / BPC;
        unsigned bs = (unsigned)(sh % BPC);
        for (size_t k = 0; k < sl; k++) {
            r.c[ws + k] ^= s->c[k] << bs;
            if (bs != 0 && k < r.len - ws - 1) r.c[ws + k + 1] ^= s->c[k] >> (BPC - bs);
        }
        /* degree rescan (:347-358): walk down to the next set bit */
        while (rd > 0 && (r.c[rd / BPC] >> (rd % BPC)) == 0) {
            unsigned bp = (unsigned)(rd % BPC);
            uint64_t w = r.c[rd / BPC];
            uint64_t shifted = (BPC - bp) >= 64 ? w : (w << (BPC - bp)); /* wrapping_shl */
            size_t lz = shifted ? (size_t)__builtin_clzll(shifted) : 64;
            size_t step = (lz < bp ? lz : bp) + 1;
            rd = rd > step ? rd - step : 0;
        }
    }
    r.deg = rd;
    *out = r;
    return OR_OK;
}

/* ---- KAT-level wrappers ---- */
static int emit(const poly *p, uint64_t *out, size_t cap, size_t *deg, size_t *olen) {
    size_t rl = p->deg / BPC + 1;
    size_t n = p->len;
    if (rl > cap) return OR_ERR_CAPACITY;
    if (n > cap) n = cap; /* limbs above rl are zero */
    memset(out, 0, cap * 8);
    memcpy(out, p->c, (n < rl ? rl : n) * 8);
    if (deg) *deg = p->deg;
    if (olen) *olen = p->len;
    return OR_OK;
}

int oracle_poly_add(const uint64_t *a, size_t alen, const uint64_t *b, size_t blen,
                    uint64_t *out, size_t cap, size_t *deg, size_t *olen) {
    if (!alen || !blen) return OR_ERR_INVALID_ARGUMENT; /* :54-57 */
    poly pa = p_from(a, alen), pb = p_from(b, blen);
    poly r = p_add(&pa, &pb);
    int st = emit(&r, out, cap, deg, olen);
    p_free(&pa), p_free(&pb), p_free(&r);
    return st;
}

int oracle_poly_mul(const uint64_t *a, size_t alen, const uint64_t *b, size_t blen,
                    uint64_t *out, size_t cap, size_t *deg, size_t *olen) {
    if (!alen || !blen) return OR_ERR_INVALID_ARGUMENT;
    poly pa = p_from(a, alen), pb = p_from(b, blen);
    poly r = p_mul(&pa, &pb);
    int st = emit(&r, out, cap, deg, olen);
    p_free(&pa), p_free(&pb), p_free(&r);
    return st;
}

int oracle_poly_rem(const uint64_t *a, size_t alen, const uint64_t *b, size_t blen,
                    uint64_t *out, size_t cap, size_t *deg, size_t *olen) {
    if (!alen || !blen) return OR_ERR_INVALID_ARGUMENT;
    poly pa = p_from(a, alen), pb = p_from(b, blen), r;
    int st = p_rem(&pa, &pb, &r);
    if (st == OR_OK) {
        st = emit(&r, out, cap, deg, olen);
        p_free(&r);
    }
    p_free(&pa), p_free(&pb);
    return st;
}

int oracle_poly_evaluate(const uint64_t *a, size_t alen, int x) { /* :168-181 */
    if (!alen) return -1;
    if (!x) return (int)(a[0] & 1);
    unsigned ones = 0;
    for (size_t k = 0; k < alen; k++) ones += (unsigned)__builtin_popcountll(a[k]);
    return (int)(ones & 1);
}

int oracle_poly_eq(const uint64_t *a, size_t alen, const uint64_t *b, size_t blen) {
    size_t da = oracle_compute_degree(a, alen), db = oracle_compute_degree(b, blen);
    if (da != db) return 0;
    return memcmp(a, b, (da / BPC + 1) * 8) == 0;
}

/* ---- RNG contract ---- */
uint64_t oracle_splitmix64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* polynomial.rs:73-96: fill, mask above the degree bit, force the degree bit */
void oracle_poly_random(size_t degree, uint64_t *state, uint64_t *out) {
    size_t n = degree / BPC + 1;
    for (size_t k = 0; k < n; k++) out[k] = oracle_splitmix64(state);
    out[n - 1] &= (1ull << (degree % BPC)) - 1;
    out[n - 1] |= 1ull << (degree % BPC);
}

static poly p_random(size_t degree, uint64_t *state) {
    poly p;
    p.len = degree / BPC + 1;
    p.c = (uint64_t *)xcalloc(p.len, 8);
    oracle_poly_random(degree, state, p.c);
    p.deg = degree;
    return p;
}

int oracle_keygen(uint16_t d, uint16_t dp, uint16_t delta, uint16_t tau, uint64_t seed,
                  uint64_t *sk_out, uint64_t *pk_out, uint32_t *pk_deg) {
    /* Parameters::new asserts (context.rs:87-94) */
    if (!d || !dp || !delta || !tau || delta >= d) return OR_ERR_INVALID_ARGUMENT;
    uint64_t st = seed;
    poly s = p_random(d, &st); /* SecretKey::random, context.rs:160-162 */
    memcpy(sk_out, s.c, s.len * 8);
    size_t cap = ((size_t)d + dp) / BPC + 1;
    poly x1 = p_monomial(1);
    for (uint32_t i = 0; i < tau; i++) { /* PublicKey::random, context.rs:249-261 */
        poly q = p_random(dp, &st);
        poly sq = p_mul(&s, &q);
        poly r = p_random(delta, &st);
        poly rx = p_mul(&r, &x1);
        poly t = p_add(&sq, &rx);
        if (t.deg / BPC + 1 > cap) abort();
        memset(pk_out + (size_t)i * cap, 0, cap * 8);
        memcpy(pk_out + (size_t)i * cap, t.c, (t.deg / BPC + 1) * 8);
        pk_deg[i] = (uint32_t)t.deg;
        p_free(&q), p_free(&sq), p_free(&r), p_free(&rx), p_free(&t);
    }
    p_free(&x1);
    p_free(&s);
    return OR_OK;
}

/* ---- CipheredBit (cipher.rs:30-122) ---- */
static poly cb_and(const poly *a, const poly *b) { return p_mul(a, b); }  /* :58-60 */
static poly cb_xor(const poly *a, const poly *b) { return p_add(a, b); }  /* :67-69 */
static poly cb_or(const poly *a, const poly *b) {                         /* :79-81 */
    poly s = p_add(a, b), m = p_mul(a, b);
    poly r = p_add(&s, &m);
    p_free(&s), p_free(&m);
    return r;
}
static poly cb_not(const poly *a) { /* :88-90 */
    poly one = p_monomial(0);
    poly r = p_add(a, &one);
    p_free(&one);
    return r;
}

static poly cb_cipher(int x, const poly *pk, uint32_t tau, const uint8_t *mask) { /* :99-115 */
    poly sum = p_null();
    for (uint32_t i = 0; i < tau; i++) {
        if (mask[i / 8] & (1u << (i % 8))) p_add_assign(&sum, &pk[i]);
    }
    p_add_bool_assign(&sum, x);
    return sum;
}

static int cb_decipher(const poly *c, const poly *sk, int *bit) { /* :119-122 */
    poly r;
    int st = p_rem(c, sk, &r);
    if (st) return st;
    *bit = (int)(r.c[0] & 1); /* evaluate(false), polynomial.rs:169-173 */
    p_free(&r);
    return OR_OK;
}

/* ---- batch layout helpers ---- */
static size_t layout(const uint32_t *bound, uint32_t nbits, size_t *off) {
    size_t s = 0;
    for (uint32_t i = 0; i < nbits; i++) {
        off[i] = s;
        s += bound[i] / BPC + 1;
    }
    return s;
}

static int load_bits(const uint64_t *limbs, const uint32_t *deg, const uint32_t *bound,
                     uint32_t nbits, size_t e, const size_t *off, size_t stride, poly *bits) {
    for (uint32_t i = 0; i < nbits; i++) {
        size_t cap = bound[i] / BPC + 1;
        bits[i] = p_from(limbs + e * stride + off[i], cap);
        if (bits[i].deg != deg[e * nbits + i] || bits[i].deg > bound[i]) {
            for (uint32_t k = 0; k <= i; k++) p_free(&bits[k]);
            return OR_ERR_INVALID_ARGUMENT;
        }
    }
    return OR_OK;
}

static int store_bits(poly *bits, uint32_t nbits, size_t e, uint64_t *limbs, uint32_t *deg,
                      const uint32_t *bound, const size_t *off, size_t stride) {
    int st = OR_OK;
    for (uint32_t i = 0; i < nbits; i++) {
        size_t cap = bound[i] / BPC + 1;
        uint64_t *dst = limbs + e * stride + off[i];
        size_t rl = bits[i].deg / BPC + 1;
        if (rl > cap || bits[i].deg > bound[i]) {
            st = OR_ERR_CAPACITY;
            continue;
        }
        memset(dst, 0, cap * 8);
        memcpy(dst, bits[i].c, rl * 8);
        deg[e * nbits + i] = (uint32_t)bits[i].deg;
    }
    return st;
}

int oracle_encrypt_batch(const uint64_t *pk, uint32_t tau, uint32_t pk_cap,
                         const uint8_t *data, uint32_t nbytes, size_t n, const uint8_t *masks,
                         uint64_t *out_limbs, uint32_t *out_deg, const uint32_t *out_bound) {
    uint32_t nbits = 8 * nbytes, mb = (tau + 7) / 8;
    poly *pks = (poly *)xcalloc(tau, sizeof(poly));
    for (uint32_t i = 0; i < tau; i++) pks[i] = p_from(pk + (size_t)i * pk_cap, pk_cap);
    size_t *off = (size_t *)xcalloc(nbits, sizeof(size_t));
    size_t stride = layout(out_bound, nbits, off);
    poly *bits = (poly *)xcalloc(nbits, sizeof(poly));
    int st = OR_OK;
    for (size_t e = 0; e < n && st == OR_OK; e++) {
        for (uint32_t k = 0; k < nbits; k++) { /* cipher.rs:180-185: bytes LE, bits LSB-first */
            int x = (data[e * nbytes + k / 8] >> (k % 8)) & 1;
            bits[k] = cb_cipher(x, pks, tau, masks + (e * nbits + k) * mb);
        }
        st = store_bits(bits, nbits, e, out_limbs, out_deg, out_bound, off, stride);
        for (uint32_t k = 0; k < nbits; k++) p_free(&bits[k]);
    }
    for (uint32_t i = 0; i < tau; i++) p_free(&pks[i]);
    free(pks), free(off), free(bits);
    return st;
}

int oracle_decrypt_batch(const uint64_t *sk, uint32_t sk_len, const uint64_t *limbs,
                         const uint32_t *deg, const uint32_t *bound, uint32_t nbits, size_t n,
                         uint8_t *out_bytes) {
    if (nbits % 8) return OR_ERR_INVALID_ARGUMENT; /* cipher.rs:218-220 */
    poly s = p_from(sk, sk_len);
    size_t *off = (size_t *)xcalloc(nbits, sizeof(size_t));
    size_t stride = layout(bound, nbits, off);
    poly *bits = (poly *)xcalloc(nbits, sizeof(poly));
    int st = OR_OK;
    for (size_t e = 0; e < n && st == OR_OK; e++) {
        st = load_bits(limbs, deg, bound, nbits, e, off, stride, bits);
        if (st) break;
        for (uint32_t k = 0; k < nbits / 8; k++) out_bytes[e * (nbits / 8) + k] = 0;
        for (uint32_t k = 0; k < nbits && st == OR_OK; k++) { /* cipher.rs:227-237 */
            int b = 0;
            st = cb_decipher(&bits[k], &s, &b);
            out_bytes[e * (nbits / 8) + k / 8] |= (uint8_t)(b << (k % 8));
        }
        for (uint32_t k = 0; k < nbits; k++) p_free(&bits[k]);
    }
    p_free(&s);
    free(off), free(bits);
    return st;
}

/* common.rs:37-56 — ripple-carry adder; output length = a.len() (zip with b, same nbits) */
static void add_internal(const poly *a, const poly *b, uint32_t L, poly *res) {
    poly carry = p_null();
    poly one = p_monomial(0);
    for (uint32_t i = 0; i < L; i++) {
        poly ab = cb_xor(&a[i], &b[i]);
        res[i] = cb_xor(&ab, &carry);
        if (i + 1 >= L) {
            p_free(&ab);
            break;
        }
        poly cp = cb_and(&ab, &carry);        /* (a^b)&carry             :51 */
        poly a_b = cb_and(&a[i], &b[i]);      /* a&b                      :52 */
        poly cp1 = cb_xor(&cp, &one);         /* c_p1_p2 ^ 1              */
        poly t = cb_and(&a_b, &cp1);          /* (a&b)&(c_p1_p2^1)        */
        poly nc = cb_xor(&cp, &t);            /* carry'                   */
        p_free(&carry);
        carry = nc;
        p_free(&ab), p_free(&cp), p_free(&a_b), p_free(&cp1), p_free(&t);
    }
    p_free(&carry), p_free(&one);
}

/* common.rs:66-105 (unsigned) and :115-155 (signed: two partial products flipped) */
static void mul_internal(const poly *a, const poly *b, uint32_t L, int is_signed, poly *res) {
    poly *pp = (poly *)xcalloc((size_t)L * L, sizeof(poly));
    for (uint32_t i = 0; i < L; i++)
        for (uint32_t j = 0; j < L; j++) pp[(size_t)i * L + j] = cb_and(&a[i], &b[j]);
    if (is_signed) {
        poly one = p_monomial(0);
        poly t0 = cb_xor(&pp[L - 1], &one);
        p_free(&pp[L - 1]);
        pp[L - 1] = t0;
        poly t1 = cb_xor(&pp[(size_t)(L - 1) * L], &one);
        p_free(&pp[(size_t)(L - 1) * L]);
        pp[(size_t)(L - 1) * L] = t1;
        p_free(&one);
    }
    for (uint32_t i = 0; i < L; i++) res[i] = p_null();
    size_t maxc = (size_t)(L - 1) * L * (L + 1) / 6 + (size_t)L * L + 8;
    poly *carries = (poly *)xcalloc(maxc, sizeof(poly));
    size_t nc = 0, offset = 0;
    for (uint32_t i = 0; i < L; i++) {
        size_t cur = (size_t)i * (i + 1) / 2;
        for (uint32_t j = 0; j <= i; j++) { /* apply partial products */
            const poly *p = &pp[(size_t)j * L + (i - j)];
            if (i + 1 < L) carries[nc++] = cb_and(p, &res[i]);
            poly x = cb_xor(&res[i], p);
            p_free(&res[i]);
            res[i] = x;
        }
        for (size_t j = 0; j < cur; j++) { /* propagate carries of the previous column */
            if (i + 1 < L) carries[nc++] = cb_and(&res[i], &carries[offset + j]);
            poly x = cb_xor(&res[i], &carries[offset + j]);
            p_free(&res[i]);
            res[i] = x;
        }
        offset += cur;
    }
    for (size_t k = 0; k < nc; k++) p_free(&carries[k]);
    for (size_t k = 0; k < (size_t)L * L; k++) p_free(&pp[k]);
    free(carries), free(pp);
}

typedef enum { K_ADD, K_MUL, K_MULS, K_AND, K_OR, K_XOR, K_NOT } kind;

static int g_threads = 1; /* oracle_set_threads: batch-parallel CPU baseline (bench.py) */

void oracle_set_threads(int n) { g_threads = n > 0 ? n : 1; }

/* One value of a binary circuit (the reference runs one value per call, single-threaded). */
static int run_one(kind k, const uint64_t *a, const uint32_t *adeg, const uint32_t *abound,
                   const uint64_t *b, const uint32_t *bdeg, const uint32_t *bbound,
                   uint32_t nbits, size_t e, uint64_t *out, uint32_t *odeg,
                   const uint32_t *obound, const size_t *offa, size_t sa, const size_t *offb,
                   size_t sb, const size_t *offo, size_t so, poly *pa, poly *pb, poly *pr) {
    int st = load_bits(a, adeg, abound, nbits, e, offa, sa, pa);
    if (st) return st;
    st = load_bits(b, bdeg, bbound, nbits, e, offb, sb, pb);
    if (st) {
        for (uint32_t i = 0; i < nbits; i++) p_free(&pa[i]);
        return st;
    }
    switch (k) {
    case K_ADD: add_internal(pa, pb, nbits, pr); break;
    case K_MUL: mul_internal(pa, pb, nbits, 0, pr); break;
    case K_MULS: mul_internal(pa, pb, nbits, 1, pr); break;
    case K_AND: for (uint32_t i = 0; i < nbits; i++) pr[i] = cb_and(&pa[i], &pb[i]); break;
    case K_OR: for (uint32_t i = 0; i < nbits; i++) pr[i] = cb_or(&pa[i], &pb[i]); break;
    case K_XOR: for (uint32_t i = 0; i < nbits; i++) pr[i] = cb_xor(&pa[i], &pb[i]); break;
    case K_NOT: for (uint32_t i = 0; i < nbits; i++) pr[i] = cb_not(&pa[i]); break;
    }
    st = store_bits(pr, nbits, e, out, odeg, obound, offo, so);
    for (uint32_t i = 0; i < nbits; i++) p_free(&pa[i]), p_free(&pb[i]), p_free(&pr[i]);
    return st;
}

static int run_binary(kind k, const uint64_t *a, const uint32_t *adeg, const uint32_t *abound,
                      const uint64_t *b, const uint32_t *bdeg, const uint32_t *bbound,
                      uint32_t nbits, size_t n, uint64_t *out, uint32_t *odeg,
                      const uint32_t *obound) {
    size_t *offa = (size_t *)xcalloc(nbits, sizeof(size_t));
    size_t *offb = (size_t *)xcalloc(nbits, sizeof(size_t));
    size_t *offo = (size_t *)xcalloc(nbits, sizeof(size_t));
    size_t sa = layout(abound, nbits, offa), sb = layout(bbound, nbits, offb);
    size_t so = layout(obound, nbits, offo);
    int st = OR_OK;
    /* values are independent: the all-cores baseline splits the batch over threads */
#pragma omp parallel num_threads(g_threads) if (g_threads > 1 && n > 1)
    {
        poly *pa = (poly *)xcalloc(nbits, sizeof(poly));
        poly *pb = (poly *)xcalloc(nbits, sizeof(poly));
        poly *pr = (poly *)xcalloc(nbits, sizeof(poly));
#pragma omp for schedule(dynamic, 1)
        for (size_t e = 0; e < n; e++) {
            int r = run_one(k, a, adeg, abound, b, bdeg, bbound, nbits, e, out, odeg, obound,
                            offa, sa, offb, sb, offo, so, pa, pb, pr);
            if (r) {
#pragma omp critical
                if (!st) st = r;
            }
        }
        free(pa), free(pb), free(pr);
    }
    free(offa), free(offb), free(offo);
    return st;
}

int oracle_add_batch(const uint64_t *a, const uint32_t *adeg, const uint32_t *abound,
                     const uint64_t *b, const uint32_t *bdeg, const uint32_t *bbound,
                     uint32_t nbits, size_t n, uint64_t *out, uint32_t *odeg,
                     const uint32_t *obound) {
    return run_binary(K_ADD, a, adeg, abound, b, bdeg, bbound, nbits, n, out, odeg, obound);
}

int oracle_mul_batch(const uint64_t *a, const uint32_t *adeg, const uint32_t *abound,
                     const uint64_t *b, const uint32_t *bdeg, const uint32_t *bbound,
                     uint32_t nbits, size_t n, int is_signed, uint64_t *out, uint32_t *odeg,
                     const uint32_t *obound) {
    return run_binary(is_signed ? K_MULS : K_MUL, a, adeg, abound, b, bdeg, bbound, nbits, n,
                      out, odeg, obound);
}

int oracle_gate_batch(int op, const uint64_t *a, const uint32_t *adeg, const uint32_t *abound,
                      const uint64_t *b, const uint32_t *bdeg, const uint32_t *bbound,
                      uint32_t nbits, size_t n, uint64_t *out, uint32_t *odeg,
                      const uint32_t *obound) {
    static const kind map[4] = {K_AND, K_OR, K_XOR, K_NOT};
    if (op < 0 || op > 3) return OR_ERR_INVALID_ARGUMENT;
    if (op == 3) { b = a, bdeg = adeg, bbound = abound; }
    return run_binary(map[op], a, adeg, abound, b, bdeg, bbound, nbits, n, out, odeg, obound);
}
