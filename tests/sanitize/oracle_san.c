/* ASan/UBSan driver for the CPU oracle (test infrastructure, SURVEY.md s5 "race detection /
 * sanitizers"): the reference's polynomial KATs (src/polynomial.rs:522-590) and a small
 * encrypt -> add / mul / gates -> decrypt round trip (src/cipher.rs:275-304,
 * src/impls/numbers/uint.rs:176-293) run under -fsanitize=address,undefined; any report or
 * mismatch exits non-zero.  Built and run by tests/test_sanitize.py. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/homomorph_oracle.h"

static int fails = 0;
#define CHECK(c)                                                                                  \
    do {                                                                                          \
        if (!(c)) {                                                                               \
            fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c);                           \
            ++fails;                                                                              \
        }                                                                                         \
    } while (0)

static void kats(void) {
    uint64_t out[4];
    size_t deg, olen;
    uint64_t a1[] = {0x9}, b1[] = {0x3};
    CHECK(oracle_poly_add(a1, 1, b1, 1, out, 4, &deg, &olen) == OR_OK && out[0] == 0xA);
    uint64_t a2[] = {0x9, 1}, b2[] = {0x5, 1};
    CHECK(oracle_poly_add(a2, 2, b2, 2, out, 4, &deg, &olen) == OR_OK && out[0] == 0xC && deg == 3);
    uint64_t m1[] = {0x9}, m2[] = {0x3};
    CHECK(oracle_poly_mul(m1, 1, m2, 1, out, 4, &deg, &olen) == OR_OK && out[0] == 0x1B);
    uint64_t mx[] = {~0ull};
    CHECK(oracle_poly_mul(mx, 1, m2, 1, out, 4, &deg, &olen) == OR_OK && out[0] == 1 && out[1] == 1);
    uint64_t z[] = {0};
    CHECK(oracle_poly_mul(z, 1, m2, 1, out, 4, &deg, &olen) == OR_OK && out[0] == 0 && deg == 0);
    uint64_t r1[] = {0x2AD}, r2[] = {0x1B};
    CHECK(oracle_poly_rem(r1, 1, r2, 1, out, 4, &deg, &olen) == OR_OK && out[0] == 0xA);
    CHECK(oracle_poly_rem(r1, 1, z, 1, out, 4, &deg, &olen) == OR_ERR_DIVIDE_BY_ZERO);
    uint64_t one[] = {1};
    CHECK(oracle_poly_rem(r1, 1, one, 1, out, 4, &deg, &olen) == OR_ERR_DIVISOR_IS_ONE);
    CHECK(oracle_poly_mul(m1, 1, m2, 1, out, 0, &deg, &olen) == OR_ERR_CAPACITY);
}

static void circuits(void) {
    const uint16_t d = 64, dp = 64, delta = 1, tau = 64;
    const uint32_t D = d + dp, cap = D / 64 + 1, nbits = 8;
    const size_t n = 4;
    uint64_t sk[2], *pk = malloc(sizeof(uint64_t) * tau * cap);
    uint32_t pkdeg[64];
    uint64_t seed = 1;
    /* a key with S(0) = 0: decryption is then exact whatever the noise degree */
    for (;; ++seed) {
        CHECK(oracle_keygen(d, dp, delta, tau, seed, sk, pk, pkdeg) == OR_OK);
        if (!(sk[0] & 1)) break;
    }
    uint8_t x[4] = {22, 255, 7, 0}, y[4] = {20, 240, 9, 0};
    const size_t nm = n * nbits * (tau / 8); /* mask bytes per batch */
    uint8_t *masks = malloc(2 * nm);
    uint64_t st = 99;
    for (size_t i = 0; i < 2 * nm; ++i) masks[i] = (uint8_t)oracle_splitmix64(&st);
    uint32_t fb[8];
    for (int i = 0; i < 8; ++i) fb[i] = D;
    uint64_t *ea = calloc(n * nbits * cap, 8), *eb = calloc(n * nbits * cap, 8);
    uint32_t da[32], db[32];
    CHECK(oracle_encrypt_batch(pk, tau, cap, x, 1, n, masks, ea, da, fb) == OR_OK);
    CHECK(oracle_encrypt_batch(pk, tau, cap, y, 1, n, masks + nm, eb, db, fb) == OR_OK);
    uint8_t got[4];
    CHECK(oracle_decrypt_batch(sk, 2, ea, da, fb, nbits, n, got) == OR_OK && !memcmp(got, x, 4));
    /* add: output bounds of common.rs:37-56 (s_0 <= D, s_i <= (3i-1) D) */
    uint32_t ob[8], off = 0;
    ob[0] = D;
    for (int i = 1; i < 8; ++i) ob[i] = (3 * i - 1) * D;
    for (int i = 0; i < 8; ++i) off += ob[i] / 64 + 1;
    uint64_t *s = calloc(n * off, 8);
    uint32_t sd[32];
    CHECK(oracle_add_batch(ea, da, fb, eb, db, fb, nbits, n, s, sd, ob) == OR_OK);
    CHECK(oracle_decrypt_batch(sk, 2, s, sd, ob, nbits, n, got) == OR_OK);
    for (size_t e = 0; e < n; ++e) CHECK(got[e] == (uint8_t)(x[e] + y[e]));
    /* mul: generous bounds (the oracle reports OR_ERR_CAPACITY if they were short) */
    uint32_t mb[8], moff = 0;
    for (int i = 0; i < 8; ++i) mb[i] = 64 * D, moff += mb[i] / 64 + 1;
    uint64_t *m = calloc(n * moff, 8);
    uint32_t md[32];
    CHECK(oracle_mul_batch(ea, da, fb, eb, db, fb, nbits, n, 0, m, md, mb) == OR_OK);
    CHECK(oracle_decrypt_batch(sk, 2, m, md, mb, nbits, n, got) == OR_OK);
    for (size_t e = 0; e < n; ++e) CHECK(got[e] == (uint8_t)(x[e] * y[e]));
    /* gates */
    for (int op = 0; op < 4; ++op) {
        uint32_t gb[8];
        for (int i = 0; i < 8; ++i) gb[i] = 2 * D;
        uint64_t *g = calloc(n * nbits * (gb[0] / 64 + 1), 8);
        uint32_t gd[32];
        CHECK(oracle_gate_batch(op, ea, da, fb, eb, db, fb, nbits, n, g, gd, gb) == OR_OK);
        CHECK(oracle_decrypt_batch(sk, 2, g, gd, gb, nbits, n, got) == OR_OK);
        for (size_t e = 0; e < n; ++e) {
            const uint8_t w = op == 0 ? x[e] & y[e] : op == 1 ? x[e] | y[e] : op == 2 ? x[e] ^ y[e]
                                                                                    : (uint8_t)~x[e];
            CHECK(got[e] == w);
        }
        free(g);
    }
    free(pk), free(masks), free(ea), free(eb), free(s), free(m);
}

int main(void) {
    kats();
    circuits();
    if (fails) return 1;
    printf("oracle sanitizer run: ok\n");
    return 0;
}
