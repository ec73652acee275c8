/*
 * homomorph_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference crate's GF(2)[X] arithmetic, per-bit cipher and
 * integer circuits (mathisbot/homomorph-rust, read at /root/reference). It exists ONLY to
 * check the HIP engine: tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it; the product library (homomorph-rust_amd/csrc) never links or calls it.
 *
 * Parity pinning: the reference is Rust and no Rust toolchain exists here, so the reference
 * cannot be built or run.  This restatement is pinned by (1) every polynomial known-answer
 * test of src/polynomial.rs:433-612, (2) the reference's own encrypt->op->decrypt round-trip
 * tests (src/cipher.rs:275-304, src/impls/numbers/uint.rs:108-293), and (3) an independent
 * Python big-integer model (oracle/gf2_model.py) that restates the same mathematics in a
 * different form.  Circuit-level ciphertext bit patterns are not pinned by any reference
 * vector (none exist): see DESIGN.md "Oracle".
 *
 * Layout contract shared with the GPU engine ("batch layout"):
 *   element e, bit i occupies cap[i] = bound[i]/64 + 1 little-endian u64 limbs starting at
 *   limb e*stride + off[i], off = exclusive prefix sum of cap, stride = sum(cap);
 *   degree[e*nbits + i] is the exact degree (null polynomial -> 0, polynomial.rs:126-137);
 *   limbs above the degree are zero.
 */
#ifndef HOMOMORPH_ORACLE_H
#define HOMOMORPH_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    OR_OK = 0,
    OR_ERR_DIVIDE_BY_ZERO = 4,  /* polynomial.rs:319-322 panics */
    OR_ERR_DIVISOR_IS_ONE = 5,  /* polynomial.rs:330 would loop forever */
    OR_ERR_CAPACITY = 6,        /* output does not fit the caller's capacity */
    OR_ERR_INVALID_ARGUMENT = 9,
};

/* ---- single polynomials (KAT-level API), polynomial.rs ---- */
size_t oracle_compute_degree(const uint64_t *c, size_t len);                     /* :35-42 */
/* out must hold max(alen, blen) limbs; returns degree via *deg, used length via *olen */
int oracle_poly_add(const uint64_t *a, size_t alen, const uint64_t *b, size_t blen,
                    uint64_t *out, size_t cap, size_t *deg, size_t *olen);     /* :190-213 */
int oracle_poly_mul(const uint64_t *a, size_t alen, const uint64_t *b, size_t blen,
                    uint64_t *out, size_t cap, size_t *deg, size_t *olen);     /* :252-310 */
int oracle_poly_rem(const uint64_t *a, size_t alen, const uint64_t *b, size_t blen,
                    uint64_t *out, size_t cap, size_t *deg, size_t *olen);     /* :316-365 */
int oracle_poly_evaluate(const uint64_t *a, size_t alen, int x);               /* :168-181 */
int oracle_poly_eq(const uint64_t *a, size_t alen, const uint64_t *b, size_t blen); /* :417-426 */

/* ---- deterministic RNG contract replacing getrandom (polynomial.rs:87, cipher.rs:95) ---- */
uint64_t oracle_splitmix64(uint64_t *state);
/* Polynomial::random(degree) with limbs drawn from splitmix64 (polynomial.rs:73-96) */
void oracle_poly_random(size_t degree, uint64_t *state, uint64_t *out /* degree/64+1 */);

/* Key generation, context.rs:160-162 (sk) and :249-261 (pk): T_i = S*Q_i + X*R_i.
 * sk_out: d/64+1 limbs.  pk_out: tau * ((d+dp)/64+1) limbs, pk_deg: tau degrees. */
int oracle_keygen(uint16_t d, uint16_t dp, uint16_t delta, uint16_t tau, uint64_t seed,
                  uint64_t *sk_out, uint64_t *pk_out, uint32_t *pk_deg);

/* ---- batched cipher / circuits over the batch layout ---- */
/* Ciphered::try_cipher (cipher.rs:175-191) + CipheredBit::cipher (:99-115).
 * data: n * nbytes plaintext bytes (bincode fixint LE image of T), masks: n*(8*nbytes)*ceil(tau/8)
 * bytes, bit k of element e uses masks[(e*8*nbytes + k)*ceil(tau/8) ...] with mask bit
 * i = byte[i/8] >> (i%8) & 1 (cipher.rs:106). out_bound: per-bit degree bound (>= D). */
int oracle_encrypt_batch(const uint64_t *pk, uint32_t tau, uint32_t pk_cap,
                         const uint8_t *data, uint32_t nbytes, size_t n, const uint8_t *masks,
                         uint64_t *out_limbs, uint32_t *out_deg, const uint32_t *out_bound);
/* Ciphered::try_decipher (cipher.rs:217-250) with CipheredBit::decipher (:119-122) */
int oracle_decrypt_batch(const uint64_t *sk, uint32_t sk_len, const uint64_t *limbs,
                         const uint32_t *deg, const uint32_t *bound, uint32_t nbits, size_t n,
                         uint8_t *out_bytes);
/* common.rs:37-56 add_internal, :66-105 mul_unsigned_internal, :115-155 mul_signed_internal,
 * :5-35 gates (op: 0 and, 1 or, 2 xor, 3 not(a)). */
int oracle_add_batch(const uint64_t *a, const uint32_t *adeg, const uint32_t *abound,
                     const uint64_t *b, const uint32_t *bdeg, const uint32_t *bbound,
                     uint32_t nbits, size_t n,
                     uint64_t *out, uint32_t *odeg, const uint32_t *obound);
int oracle_mul_batch(const uint64_t *a, const uint32_t *adeg, const uint32_t *abound,
                     const uint64_t *b, const uint32_t *bdeg, const uint32_t *bbound,
                     uint32_t nbits, size_t n, int is_signed,
                     uint64_t *out, uint32_t *odeg, const uint32_t *obound);
int oracle_gate_batch(int op, const uint64_t *a, const uint32_t *adeg, const uint32_t *abound,
                      const uint64_t *b, const uint32_t *bdeg, const uint32_t *bbound,
                      uint32_t nbits, size_t n,
                      uint64_t *out, uint32_t *odeg, const uint32_t *obound);

/* Threads for the batch entry points (values split over threads; default 1, the reference is
 * single-threaded).  Used by bench.py's all-cores CPU baseline leg. */
void oracle_set_threads(int n);

/* Work counter: 64x64 limb products issued by oracle_poly_mul on the calling thread since the
 * last reset. */
uint64_t oracle_limb_products(void);
void oracle_reset_counters(void);

#ifdef __cplusplus
}
#endif
#endif
