/*
 * homomorph_gpu.h — C ABI of the MI355X (gfx950) GF(2)[X] homomorphic engine.
 *
 * This is the drop-in boundary for mathisbot/homomorph-rust's data-parallel hot path.  Each entry
 * point names the reference item it replaces (file:line, paths relative to the reference crate).
 * The reference has no batch API; every batch entry applies the reference's per-value operation
 * independently to n values (one `Ciphered<T>` = nbits ciphertext bits per value).
 *
 * Conventions
 *  - Plain C: pointers + sizes, no C++ types, no exceptions cross this boundary.  Every function
 *    returns hm_status; HM_OK == 0.
 *  - Device buffers are caller-owned device pointers (hipMalloc'd or a torch tensor's data_ptr);
 *    the library never frees caller memory.  Launches are asynchronous on the context's stream;
 *    no entry below synchronises unless its comment says so.
 *  - Polynomial layout (GF(2)[X], src/polynomial.rs:23-26): coefficient of X^k is bit k%64 of
 *    little-endian u64 limb k/64 (the code's layout, polynomial.rs:142-150, :168-173 — the doc
 *    comment at :16-21 describing reversed bits does not match the code).  Limbs above the degree
 *    are zero.  Degrees are exact; the null polynomial has degree 0 (polynomial.rs:126-137).
 *  - Batch layout (hm_batch): value e, bit i occupies cap[i] = bound[i]/64 + 1 limbs at limb offset
 *    e*stride + off[i] (off = exclusive prefix sum of cap, stride = sum(cap)); its exact degree is
 *    degree[e*nbits + i].  bound[i] is a static degree bound for bit position i (a fresh ciphertext
 *    has bound d+dp); outputs are sized with hm_*_out_bounds.  Bit i is bit i of the bincode fixint
 *    little-endian image of the value (src/cipher.rs:6-13, :175-191).
 *  - Thread-safety: calls on one context are serialised by the caller; contexts on different
 *    devices are independent (the reference's Context is a plain value, src/context.rs:300-306).
 */
#ifndef HOMOMORPH_GPU_H
#define HOMOMORPH_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HM_ABI_VERSION 5 /* 4: kernel timing by device stamps (HM_TIME_*), hm_ctx_last_hip_error;
                            5: hm_ctx_clear_kernel_timing, hm_ctx_set_mul_scratch */
#define HM_MAX_BITS 128 /* u128 is the widest type with impls (src/impls/numbers/uint.rs:58) */

typedef enum hm_status {
    HM_OK = 0,
    /* OperationError::InvalidParameters (src/operations.rs:11-18) */
    HM_ERR_INVALID_PARAMETERS = 1,
    /* ContextCryptoError::SecretKeyUnset / PublicKeyUnset (src/context.rs:41-46) */
    HM_ERR_SECRET_KEY_UNSET = 2,
    HM_ERR_PUBLIC_KEY_UNSET = 3,
    /* Polynomial::rem panics "attempt to divide by zero" (src/polynomial.rs:319-322) */
    HM_ERR_DIVIDE_BY_ZERO = 4,
    /* Polynomial::rem by the constant 1 never terminates in the reference (:330-343) */
    HM_ERR_DIVISOR_IS_ONE = 5,
    /* an output would exceed the capacity its bound gives (device-side check) */
    HM_ERR_CAPACITY = 6,
    /* sizes beyond what this build's kernels handle */
    HM_ERR_UNSUPPORTED = 7,
    HM_ERR_HIP = 8,
    HM_ERR_INVALID_ARGUMENT = 9,
    /* CipherError::InvalidCipheredLength (src/cipher.rs:18-24, :218-220) */
    HM_ERR_INVALID_CIPHERED_LENGTH = 10,
    /* an input polynomial's degree word disagrees with its limbs (device-side check) */
    HM_ERR_BAD_INPUT = 11,
    /* CipherError::Randomness (src/cipher.rs:18-24): the OS random source failed */
    HM_ERR_RANDOMNESS = 12,
    /* a host-side allocation failed (std::bad_alloc inside the library, caught at the entry) */
    HM_ERR_OUT_OF_MEMORY = 13,
    /* any other C++ exception raised inside the library, caught at the entry */
    HM_ERR_INTERNAL = 14,
} hm_status;

/* Operation marker types and their OperationRequirement::MIN_D_OVER_DELTA
 * (src/impls/numbers.rs:9-50). */
typedef enum hm_op {
    HM_OP_AND = 0,            /* HomomorphicAndGate,        min d/delta 2  */
    HM_OP_OR = 1,             /* HomomorphicOrGate,         min d/delta 2  */
    HM_OP_XOR = 2,            /* HomomorphicXorGate,        min d/delta 1  */
    HM_OP_NOT = 3,            /* HomomorphicNotGate,        min d/delta 1  */
    HM_OP_ADD = 4,            /* HomomorphicAddition,       min d/delta 21 */
    HM_OP_MUL = 5,            /* HomomorphicMultiplication, min d/delta 64 (unsigned types) */
    HM_OP_MUL_SIGNED = 6,     /* HomomorphicMultiplication on i8..i128 (common.rs:115-163) */
} hm_op;

typedef struct hm_ctx hm_ctx;

/* A batch of n values of nbits ciphertext bits each, in device memory (layout above). */
typedef struct hm_batch {
    uint64_t *limbs;        /* device, n*stride limbs */
    uint32_t *degree;       /* device, n*nbits exact degrees */
    const uint32_t *bound;  /* HOST, nbits per-bit-position degree bounds */
    uint32_t nbits;         /* 1..HM_MAX_BITS */
    uint64_t n;             /* number of values */
} hm_batch;

/* A batch of n independent polynomials, each with cap limbs, in device memory. */
typedef struct hm_polys {
    uint64_t *limbs;        /* device, n*cap limbs */
    uint32_t *degree;       /* device, n exact degrees */
    uint32_t cap;           /* limbs per polynomial */
    uint64_t n;
} hm_polys;

/* ---------------- library / context ---------------- */
/* Text of a status code; any int is accepted ("unknown status" outside hm_status). */
const char *hm_status_string(int s);
uint32_t hm_abi_version(void);

/* Context::new(Parameters::new(d, dp, delta, tau)) — src/context.rs:345-351 with the asserts of
 * Parameters::new (:87-94: all > 0, delta < d) reported as HM_ERR_INVALID_PARAMETERS.
 * device: HIP device ordinal; the context creates its own non-blocking stream. */
hm_status hm_ctx_create(uint16_t d, uint16_t dp, uint16_t delta, uint16_t tau, int device,
                        hm_ctx **out);
/* Drop: device copies of the secret key (and tables derived from it) are zeroed before release,
 * mirroring SecretKey's Drop (src/context.rs:197-206). */
void hm_ctx_destroy(hm_ctx *ctx);
/* Device buffers the kernels read (workspaces, key tables, decrypt tables, mask buffers) are
 * never freed while the context lives, because a HIP graph captured over the engine's launches
 * holds their raw pointers.  When one must be replaced (it grows, or a new key replaces its
 * contents) the old one is retired -- zeroed first if it holds secret-derived data -- and the
 * context generation advances.  A captured graph is valid only while the generation it was
 * captured at is current; hm_ctx_trim frees the retired buffers (no graph may use them after). */
uint64_t hm_ctx_generation(const hm_ctx *ctx);
hm_status hm_ctx_trim(hm_ctx *ctx);
/* Launch on a caller stream (hipStream_t passed as void*; NULL = the default null stream, as in
 * HIP) instead of the context's own non-blocking stream.  Use it to order the engine's launches
 * with the caller's copies, e.g. torch.cuda.current_stream().cuda_stream. */
hm_status hm_ctx_set_stream(hm_ctx *ctx, void *hip_stream);
void *hm_ctx_stream(const hm_ctx *ctx);
/* Parameters getters (src/context.rs:96-118). */
hm_status hm_ctx_parameters(const hm_ctx *ctx, uint16_t *d, uint16_t *dp, uint16_t *delta,
                            uint16_t *tau);

/* Context::set_secret_key(SecretKey::from_bytes) — src/context.rs:568-571 + :153-155.  limbs: host
 * little-endian u64 limbs of S (the bytes of SecretKey::to_bytes).  Clears the public key, as the
 * reference does. */
hm_status hm_ctx_set_secret_key(hm_ctx *ctx, const uint64_t *limbs, size_t nlimbs);
/* Context::set_public_key(PublicKey::from_bytes) — src/context.rs:593-595 + :239-245.  limbs: host,
 * tau polynomials of limbs_per_poly limbs each (row-major). */
hm_status hm_ctx_set_public_key(hm_ctx *ctx, const uint64_t *limbs, uint32_t tau,
                                uint32_t limbs_per_poly);
/* Context::generate_secret_key / generate_public_key — src/context.rs:421-454 (keygen shape
 * S = random(d), T_i = S*Q_i + X*R_i, :160-162 and :249-261).  As in the reference, every key
 * polynomial is drawn from getrandom(2) (src/polynomial.rs:73-96) and encryption masks from a
 * CSPRNG (a device ChaCha20 stream keyed with 32 getrandom bytes at context creation).
 * hm_ctx_seed_rng is a TEST hook: it switches key generation to a SplitMix64 stream and the mask
 * stream to a ChaCha20 key derived from the seed, so parity tests can reproduce both sides.
 * generate_secret_key clears the public key (:421-424); generate_public_key needs the secret key
 * (HM_ERR_SECRET_KEY_UNSET otherwise, :444-454).  Public-key rows are as wide as the widest
 * T_i (deg S + dp for a loaded secret key of any degree). */
hm_status hm_ctx_seed_rng(hm_ctx *ctx, uint64_t seed);
hm_status hm_ctx_generate_secret_key(hm_ctx *ctx);
hm_status hm_ctx_generate_public_key(hm_ctx *ctx);
/* Key export (SecretKey::to_bytes :192-194 / PublicKey::to_bytes :291-297) into host buffers. */
hm_status hm_ctx_get_secret_key(const hm_ctx *ctx, uint64_t *limbs, size_t cap, size_t *nlimbs);
hm_status hm_ctx_get_public_key(const hm_ctx *ctx, uint64_t *limbs, size_t cap, uint32_t *tau,
                                uint32_t *limbs_per_poly);

/* Multiplier strategy (no effect on results: every product is exact).  A carry product of the
 * carry-save circuit whose shorter operand has at least karatsuba_min_words 32-bit words runs as
 * a Karatsuba recursion down to leaves of at most karatsuba_leaf_words
 * words (rounded to a multiple of 32, at most 512); smaller products run as schoolbook tiles.
 * karatsuba_min_words = 0 disables it.  Defaults: 256 and 256 (measured best for the u32 multiply
 * prefixes at d = d' = 128 once the leaves run on the matrix cores; 192 and 192 at d = d' = 256). */
hm_status hm_ctx_set_mul_options(hm_ctx *ctx, uint32_t karatsuba_min_words,
                                 uint32_t karatsuba_leaf_words);
/* Karatsuba scratch (no effect on results).  A Karatsuba product's recursion runs breadth-first
 * (all its leaves in one launch, then the recombinations bottom-up), so every node's buffers are
 * alive at once and the scratch grows as n^1.585.  A product whose recursion needs more than
 * words_per_value 32-bit words of scratch per value is planned one subtree at a time instead: the
 * root's operand sums and child products first, then each child's own recursion (recursively,
 * reusing the scratch above the root's), then the root's recombination.  Default 2e8 words (every
 * product up to the u32 multiply's K = 20 prefix runs whole; K = 21..24 need the split).  At most
 * 2^27 + 2^26 words (the plan's views hold 28-bit offsets); at least 1. */
hm_status hm_ctx_set_mul_scratch(hm_ctx *ctx, uint64_t words_per_value);

/* Where the multiplier's products run (no effect on results: every product is exact): as {0,1}
 * Toeplitz GEMMs on the fp4 matrix cores (MFMA, reduced mod 2) or as VALU products.  The choice
 * covers every product kind of the carry-save plan: the Karatsuba leaf products, the schoolbook
 * carry products p_t * x_t, and the partial products a_j * b_k of fresh operands (products whose
 * shorter operand is below 4 words, and the signed circuit's flipped partial products, stay on
 * the VALU either way).  AUTO = MFMA on a device with the gfx950 fp4 MFMA, VALU elsewhere;
 * MFMA on a device without it is HM_ERR_UNSUPPORTED. */
#define HM_MUL_PRODUCTS_AUTO 0u
#define HM_MUL_PRODUCTS_MFMA 1u
#define HM_MUL_PRODUCTS_VALU 2u
hm_status hm_ctx_set_mul_products(hm_ctx *ctx, uint32_t products);

/* Adder strategy (no effect on results: both chains are exact).  The carry chain
 * carry' = ab_i ^ P_i * carry (src/impls/numbers/common.rs:37-56) runs its products either on the
 * matrix cores (a {0,1} Toeplitz product on fp4 MFMA, reduced mod 2; needs P_i within 49 words,
 * i.e. d + dp <= 512 for u32) or as scalar-decided VALU XORs.  AUTO picks the MFMA chain when it
 * applies (and the device has the gfx950 fp4 MFMA); MFMA on a plan or device it cannot run
 * returns HM_ERR_UNSUPPORTED at hm_add_batch. */
#define HM_ADD_CHAIN_AUTO 0u
#define HM_ADD_CHAIN_MFMA 1u
#define HM_ADD_CHAIN_VALU 2u
hm_status hm_ctx_set_add_options(hm_ctx *ctx, uint32_t chain);

/* Adder pipelining (no effect on results; off by default: measured no faster on configs[1],
 * DESIGN.md s4.1).  When enabled, an MFMA-chain add of at least 2048 values runs as two halves,
 * the second half's carry-independent prep on an auxiliary stream beside the first half's carry
 * chain, joined back into the context stream by events (a graph captured on the context stream
 * holds both branches).  Not used while kernel timing is on. */
hm_status hm_ctx_set_add_pipeline(hm_ctx *ctx, int enable);

/* Kernel timing (measurement only; no effect on results).  hm_ctx_set_kernel_timing(ctx, k)
 * times kernel k from now on (HM_TIME_OFF stops; setting resets the record and synchronizes the
 * stream): every launch of it made -- or captured into a graph -- while timing is on takes its
 * own record slot (up to 128), in which the kernel's waves stamp the device wall clock at their
 * start and end (a minimum over starts, a maximum over ends).  A captured launch keeps its slot
 * across replays and nothing clears it in between: the stamps are valid for ONE replay of the
 * graph (R replays make each slot span from the first replay's start to the last one's end).  So
 * enable, capture a K-step graph, replay it once, read: K launches (as the bench times it).
 * hm_ctx_clear_kernel_timing synchronizes the stream and clears the stamps of every slot while
 * keeping the slots (and the kernel timed): a graph captured earlier can then be replayed again
 * and read for that one replay.
 * hm_ctx_kernel_timing synchronizes the stream and returns the summed duration (earliest wave
 * start to latest wave end, per slot) of the launches recorded and their number.
 * HM_TIME_ADD_CHAIN = 1 (hm_add_batch's carry chain, the dominant kernel of the add),
 * HM_TIME_ENCRYPT: hm_encrypt_batch's encryption kernel (not the mask draw), HM_TIME_DECRYPT:
 * hm_decrypt_batch's kernel. */
enum { HM_TIME_OFF = 0, HM_TIME_ADD_CHAIN = 1, HM_TIME_ENCRYPT = 2, HM_TIME_DECRYPT = 3 };
hm_status hm_ctx_set_kernel_timing(hm_ctx *ctx, int kernel);
hm_status hm_ctx_clear_kernel_timing(hm_ctx *ctx);
hm_status hm_ctx_kernel_timing(hm_ctx *ctx, double *total_ms, uint32_t *launches);

/* Context::validate_operation (src/context.rs:310-323): HM_OK or HM_ERR_INVALID_PARAMETERS with
 * the OperationError payload written to *required_min_d_over_delta (may be NULL). */
hm_status hm_validate_operation(const hm_ctx *ctx, hm_op op, uint16_t *required_min_d_over_delta);

/* Static degree bounds (host only, no device work).  fresh bound = max(d + dp, max deg T_i):
 * a subset sum of public-key rows plus the plaintext bit (cipher.rs:99-115). */
uint32_t hm_fresh_bound(const hm_ctx *ctx);
/* Mask bytes per ciphertext bit: ceil(tau/8) with tau = the number of rows of the LOADED public
 * key (CipheredBit::cipher takes tau = pk.len(), cipher.rs:101-103; a loaded key may differ from
 * Parameters::tau, context.rs:585-593).  0 when no public key is set. */
uint32_t hm_ctx_mask_bytes(const hm_ctx *ctx);
/* Output bounds of the ripple-carry adder (common.rs:37-56) for input bounds a,b (nbits each). */
hm_status hm_add_out_bounds(uint32_t nbits, const uint32_t *a_bound, const uint32_t *b_bound,
                            uint32_t *out_bound);
/* Output bounds of the carry-save multiplier (common.rs:66-105 / :115-155). */
hm_status hm_mul_out_bounds(uint32_t nbits, const uint32_t *a_bound, const uint32_t *b_bound,
                            int is_signed, uint32_t *out_bound);
/* Cost model of the low k output bits of the nbits-bit carry-save multiplier (host only, no device
 * work): the symbolic run of common.rs:66-105 over static degree bounds, exactly as
 * hm_mul_low_batch plans it but without the engine's size limits, so the full u32 circuit (which
 * no engine can run: SURVEY.md s0.6) can be priced.  word_pairs: 32x32-bit carry-less word
 * products over all carries p_t * x_t; out_bytes: the k output bits at their capacities;
 * max_degree: the largest degree bound of any polynomial the circuit builds.  Outputs may be
 * NULL. */
hm_status hm_mul_cost(uint32_t nbits, uint32_t k, const uint32_t *a_bound, const uint32_t *b_bound,
                      int is_signed, double *word_pairs, double *out_bytes, double *max_degree);
/* The same carry products as the context's plan for hm_mul_low_batch / hm_mul_batch (k = nbits)
 * runs them, with the context's strategy options (hm_ctx_set_mul_options, _products): a schoolbook
 * product counts its word pairs at the static bounds (as hm_mul_cost does), a Karatsuba product its
 * leaf products' word pairs.  No kernel runs, but the plan is built and cached as the multiply
 * would: its task tables are allocated in device memory and copied (synchronously) on the
 * context's stream, so this call is not free and must not be made while that stream is being
 * captured into a graph; HM_ERR_UNSUPPORTED beyond the engine's limits.  The bench's
 * multiply rooflines use it as the issued work. */
hm_status hm_mul_plan_work(hm_ctx *ctx, uint32_t nbits, uint32_t k, const uint32_t *a_bound,
                           const uint32_t *b_bound, int is_signed, double *word_pairs);
/* Output bounds of a gate (common.rs:5-35). */
hm_status hm_gate_out_bounds(hm_op gate, uint32_t nbits, const uint32_t *a_bound,
                             const uint32_t *b_bound, uint32_t *out_bound);
/* stride (limbs per value) of a batch with these bounds */
uint64_t hm_batch_stride(uint32_t nbits, const uint32_t *bound);

/* ---------------- cipher (src/cipher.rs) ---------------- */
/* n bytes of the context's mask CSPRNG (device ChaCha20, see hm_ctx_seed_rng) into device
 * memory.  Every call -- and every replay of a graph that captured one -- draws fresh bytes. */
hm_status hm_random_bytes(hm_ctx *ctx, uint8_t *dev_dst, size_t nbytes);
/* Context::encrypt over a batch — Ciphered::try_cipher (cipher.rs:175-191) and
 * CipheredBit::cipher (:99-115).  data: device, n*nbytes plaintext bytes (the bincode fixint LE
 * image of each value).  masks: NULL = the engine draws them from its CSPRNG, as
 * CipheredBit::part (:92-97) draws from getrandom (the default); or device,
 * n*(8*nbytes)*M bytes with M = hm_ctx_mask_bytes(ctx): bit k of value e uses the M bytes at
 * ((e*8*nbytes)+k)*M, mask bit i = byte[i/8] >> (i%8) & 1 — exactly the bytes part() draws (the
 * test contract).  out: nbits = 8*nbytes, every bound >= hm_fresh_bound.  Requires the public
 * key. */
hm_status hm_encrypt_batch(hm_ctx *ctx, const uint8_t *data, uint32_t nbytes,
                           const uint8_t *masks, hm_batch *out);
/* Context::decrypt over a batch — Ciphered::try_decipher (cipher.rs:217-250): bit k =
 * (C_k mod S)(0) (CipheredBit::decipher :119-122), bytes assembled LSB-first.  out: device,
 * n*(nbits/8) bytes.  nbits % 8 != 0 -> HM_ERR_INVALID_CIPHERED_LENGTH.  Requires the secret key;
 * the first call for a given maximum bound builds a per-key table on the host (synchronous). */
hm_status hm_decrypt_batch(hm_ctx *ctx, const hm_batch *in, uint8_t *out);

/* ---------------- operations (HomomorphicOperation2 impls, src/impls/numbers/uint.rs) ------ */
/* Context::apply2::<HomomorphicAddition, uN>: validate (d >= 21*delta) then common::add
 * (common.rs:37-64) per value.  a, b, out: same nbits; out bounds from hm_add_out_bounds. */
hm_status hm_add_batch(hm_ctx *ctx, const hm_batch *a, const hm_batch *b, hm_batch *out);
/* Context::apply2::<HomomorphicMultiplication, uN / iN> (common.rs:66-163) per value.  Needs a
 * device workspace for the carry list; the context grows it on demand (synchronous allocation
 * on first use per size).  Sizes beyond the engine's limits return HM_ERR_UNSUPPORTED. */
hm_status hm_mul_batch(hm_ctx *ctx, const hm_batch *a, const hm_batch *b, int is_signed,
                       hm_batch *out);
/* The low k output bits of the nbits-bit multiplier ("u32-mul column
 * prefix").  Column i of the carry-save circuit (common.rs:66-105) reads input bits <= i and the
 * carries of columns < i only, so output bits 0..k-1 of the nbits-bit circuit equal the k-bit
 * circuit on the low k bits, bit for bit.  The signed circuit (:115-155) differs from the
 * unsigned one only in column nbits-1, so for k < nbits this is also the signed product's low
 * bits.  a, b: nbits-bit batches read in place; out: k bits, bounds from hm_mul_out_bounds over
 * the first k input bounds.  Same requirement as HM_OP_MUL (d >= 64 delta). */
hm_status hm_mul_low_batch(hm_ctx *ctx, const hm_batch *a, const hm_batch *b, uint32_t k,
                           hm_batch *out);
/* Context::apply2::<HomomorphicAnd/Or/XorGate> and apply1::<HomomorphicNotGate> (common.rs:5-35,
 * uint.rs:8-58).  For HM_OP_NOT, b is ignored (may be NULL). */
hm_status hm_gate_batch(hm_ctx *ctx, hm_op gate, const hm_batch *a, const hm_batch *b,
                        hm_batch *out);

/* ---------------- polynomial primitives (src/polynomial.rs), for unit parity ---------------- */
/* Polynomial::add (polynomial.rs:190-213) per pair: out = a ^ b, exact degree. */
hm_status hm_poly_add_batch(hm_ctx *ctx, const hm_polys *a, const hm_polys *b, hm_polys *out);
/* Polynomial::mul (polynomial.rs:252-310) per pair: carry-less product, null short-circuit. */
hm_status hm_poly_mul_batch(hm_ctx *ctx, const hm_polys *a, const hm_polys *b, hm_polys *out);
/* Polynomial::rem (polynomial.rs:316-365): remainder by ONE divisor s (host limbs) for every
 * polynomial of a; s = 0 -> HM_ERR_DIVIDE_BY_ZERO, s = 1 -> HM_ERR_DIVISOR_IS_ONE. */
hm_status hm_poly_rem_batch(hm_ctx *ctx, const hm_polys *a, const uint64_t *s_limbs,
                            size_t s_nlimbs, hm_polys *out);

/* ---------------- ciphertext batch wire format ---------------- */
/* The reference serialises no ciphertexts (only keys, src/context.rs:153-194, :239-297); this is
 * the engine's storage / transfer format for a batch, all fields little-endian:
 *   offset 0   magic "HMCB" (4 bytes)      offset 4   version (u32) = 1
 *   offset 8   nbits (u32)                 offset 12  flags (u32) = 0
 *   offset 16  n (u64)                     offset 24  bound[nbits] (u32)
 *   then       degree[n*nbits] (u32), zero padding to a multiple of 8 bytes,
 *   then       limbs[n*stride] (u64) in the batch layout above (stride = hm_batch_stride).
 * One Ciphered<T> is n = 1 with its Vec<CipheredBit> as the nbits polynomials, bit k of the
 * bincode image first-to-last (src/cipher.rs:127-130, :253-259).  Size in bytes of a batch: */
uint64_t hm_wire_bytes(uint32_t nbits, const uint32_t *bound, uint64_t n);
/* Parse a header (host buffer of len bytes): nbits, n and, when bound is non-NULL, the nbits
 * bounds.  HM_ERR_INVALID_ARGUMENT for a bad magic / version / flags or a length that disagrees
 * with the header. */
hm_status hm_wire_peek(const uint8_t *src, size_t len, uint32_t *nbits, uint64_t *n,
                       uint32_t *bound);
/* Device batch -> host wire image (synchronous: waits for the context's stream).  cap: bytes at
 * dst, at least hm_wire_bytes(in). */
hm_status hm_wire_encode(hm_ctx *ctx, const hm_batch *in, uint8_t *dst, size_t cap);
/* Host wire image -> device batch `out` (caller-allocated from hm_wire_peek: same nbits, n and
 * bounds).  Every polynomial is validated on the host first (degree within its bound, its top
 * coefficient set, zeros above it) -> HM_ERR_BAD_INPUT; synchronous. */
hm_status hm_wire_decode(hm_ctx *ctx, const uint8_t *src, size_t len, hm_batch *out);

/* ---------------- status / sync ---------------- */
/* Waits for the context's stream, then returns (and clears) the first device-side error raised by
 * any kernel since the last check (HM_ERR_CAPACITY, HM_ERR_BAD_INPUT) or a HIP error. */
hm_status hm_ctx_synchronize(hm_ctx *ctx);
/* The HIP runtime's error code (hipError_t) behind the context's most recent HM_ERR_HIP, or 0;
 * diagnostic only, not cleared by this call (hm_ctx_synchronize clears it). */
int32_t hm_ctx_last_hip_error(const hm_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* HOMOMORPH_GPU_H */
