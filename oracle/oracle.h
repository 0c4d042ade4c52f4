/*
 * oracle.h -- CPU restatement of the lcpc_proof_of_storage hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liblcpc_oracle.so, and only as the checker / the timed CPU baseline.
 *
 * This is a plain-C restatement of the reference Rust path (cited per function
 * in the .c files) plus the third-party semantics it depends on, restated from
 * their published specifications because the crates are absent here:
 *   ff 0.13 / ff_derive   (Montgomery limbs, to_repr, random, ROOT_OF_UNITY)
 *   fffft 0.4             (fft_io: natural in -> bit-reversed out, ifft_oi)
 *   blake3 1.5            (BLAKE3 hash, 32-byte output)
 *   merlin 2.0            (STROBE-128 over Keccak-f[1600])
 *   rand_chacha 0.3 / rand_core 0.6 / rand 0.8 (ChaCha20Rng, seed_from_u64,
 *                          Uniform<usize>)
 * Parity status: pinned by KATs for Keccak (SHA3 via hashlib),
 * ChaCha20 (RFC 7539 / rand_chacha test vectors), BLAKE3 (official test
 * vectors), and by the reference's own self-consistency invariants; the
 * Merlin/STROBE framing and fffft's root choice are restated from spec and are
 * "parity unpinned" against the Rust binary (no Rust toolchain here).
 *
 * Field elements everywhere are arrays of `nl` little-endian u64 limbs holding
 * the ff_derive internal Montgomery form (value * 2^(64 nl) mod p), which is
 * bit-identical to the reference's `[u64; N]` field structs.
 */
#ifndef LCPC_ORACLE_H
#define LCPC_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------- fields (lcpc-test-fields/src/lib.rs:13-70) ---------------- */
enum {
  OF_FT63 = 0,      /* lcpc-test-fields/src/lib.rs:18-22 (and PoS WriteableFt63) */
  OF_FT127 = 1,     /* lcpc-test-fields/src/lib.rs:41-45 */
  OF_FT191 = 2,     /* lcpc-test-fields/src/lib.rs:53-57 */
  OF_FT255 = 3,     /* lcpc-test-fields/src/lib.rs:65-69 */
  OF_FT253_192 = 4, /* proof-of-storage/src/fields/ft253_192.rs:6-10 (BE repr) */
  OF_NFIELDS = 5
};

int of_field_limbs(int fid);
int of_field_num_bits(int fid);
int of_field_s(int fid);
void of_field_modulus(int fid, uint64_t *out);
void of_field_root_of_unity(int fid, uint64_t *out_mont);

/* element-wise ops on arrays of n elements (Montgomery form) */
void of_from_canonical(int fid, const uint64_t *in, uint64_t *out, size_t n);
void of_to_canonical(int fid, const uint64_t *in, uint64_t *out, size_t n);
void of_add(int fid, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n);
void of_sub(int fid, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n);
void of_mul(int fid, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n);
void of_pow(int fid, const uint64_t *a, uint64_t e, uint64_t *out);
void of_inv(int fid, const uint64_t *a, uint64_t *out);
void of_to_repr(int fid, const uint64_t *in, uint8_t *out, size_t n);
int of_is_valid(int fid, const uint64_t *a);

/* ---------------- fffft semantics ---------------- */
/* 0 ok, 1 NotPowerOfTwo, 2 TooBig (log2 len > S) */
int of_fft_io(int fid, uint64_t *data, size_t len);
int of_ifft_oi(int fid, uint64_t *data, size_t len);
void of_ntt_omega(int fid, int log_len, uint64_t *out_mont);

/* ---------------- hashes ---------------- */
void of_blake3(const uint8_t *in, size_t len, uint8_t out[32]);
void of_keccak_f1600(uint64_t st[25]);
void of_sha3_256(const uint8_t *in, size_t len, uint8_t out[32]);

/* ---------------- merlin transcript ---------------- */
typedef struct of_transcript of_transcript;
of_transcript *of_transcript_new(const uint8_t *label, size_t label_len);
of_transcript *of_transcript_clone(const of_transcript *t);
void of_transcript_free(of_transcript *t);
void of_transcript_append_message(of_transcript *t, const uint8_t *label, size_t label_len,
                                  const uint8_t *msg, size_t msg_len);
void of_transcript_challenge_bytes(of_transcript *t, const uint8_t *label, size_t label_len,
                                   uint8_t *dest, size_t dest_len);

/* ---------------- rand_chacha / rand ---------------- */
typedef struct of_chacha of_chacha;
of_chacha *of_chacha_from_seed(const uint8_t seed[32], int rounds);
of_chacha *of_chacha_seed_from_u64(uint64_t state, int rounds);
void of_chacha_free(of_chacha *r);
uint32_t of_chacha_next_u32(of_chacha *r);
uint64_t of_chacha_next_u64(of_chacha *r);
void of_chacha_fill_bytes(of_chacha *r, uint8_t *dst, size_t n);
void of_chacha_set_stream(of_chacha *r, uint64_t stream);
uint64_t of_uniform_usize(of_chacha *r, uint64_t low, uint64_t high); /* Uniform::new(low,high) */
void of_field_random(int fid, of_chacha *r, uint64_t *out, size_t n);   /* F::random */
uint32_t of_gen_range_u32(of_chacha *r, uint32_t low, uint32_t high);  /* rng.gen_range(low..high) */

/* ---------------- lcpc-2d ---------------- */
size_t of_log2(size_t v);
size_t of_n_degree_tests(size_t lambda, size_t len, size_t flog2);
size_t of_ligero_n_col_opens(size_t rho_num, size_t rho_den);
int of_ligero_get_dims(int fid, size_t rho_num, size_t rho_den, size_t len, size_t *n_rows,
                       size_t *n_per_row, size_t *n_cols);

/* An encoding as lcpc-2d sees it through the LcEncoding trait. */
typedef struct of_enc {
  int fid;
  int kind; /* 0 = Ligero (fft_io), 1 = Brakedown (SDIG) */
  size_t n_per_row, n_cols, n_col_opens, n_degree_tests;
  void *bd; /* brakedown matrices (kind == 1) */
} of_enc;

of_enc *of_enc_ligero(int fid, size_t n_per_row, size_t n_cols, size_t n_col_opens,
                      size_t n_degree_tests);
void of_enc_free(of_enc *e);
int of_enc_encode(const of_enc *e, uint64_t *row); /* in place on n_cols elements */
/* rows r < n_rows: dst + r n_cols = encode(src + r src_stride's n_per_row elements, zero padded),
 * rows in parallel on of_set_threads threads (the row-parallel encode of commit,
 * lcpc-2d/src/lib.rs:677-682); 0 or the first error */
int of_enc_encode_rows(const of_enc *e, const uint64_t *src, size_t src_stride, size_t n_rows, uint64_t *dst);

typedef struct of_commit {
  int fid, nl;
  size_t n_rows, n_cols, n_per_row, n_hashes;
  uint64_t *comm;   /* n_rows * n_cols elements */
  uint64_t *coeffs; /* n_rows * n_per_row elements */
  uint8_t *hashes;  /* n_hashes * 32 */
} of_commit;

typedef struct of_proof {
  int fid, nl;
  size_t n_cols, n_per_row, n_rows, n_degree_tests, n_col_opens, path_len;
  uint64_t *p_eval;       /* n_per_row */
  uint64_t *p_random;     /* n_degree_tests * n_per_row */
  uint64_t *cols;         /* n_col_opens * n_rows */
  uint8_t *paths;         /* n_col_opens * path_len * 32 */
  uint64_t *col_idx;      /* indices the prover opened (informational) */
} of_proof;

void of_set_threads(int n);
of_commit *of_commit_new(const of_enc *e, const uint64_t *coeffs, size_t len);
void of_commit_free(of_commit *c);
of_proof *of_prove(const of_commit *c, const of_enc *e, const uint64_t *outer, of_transcript *tr,
                   int *err);
of_proof *of_proof_alloc(int fid, size_t n_cols, size_t n_per_row, size_t n_rows, size_t ndt,
                         size_t n_col_opens, size_t path_len);
void of_proof_free(of_proof *p);
/* returns 0 ok, else a VerifierError code (see of_lcpc.c); *out = evaluation */
int of_verify(const uint8_t root[32], const uint64_t *outer, size_t outer_len, const uint64_t *inner,
              size_t inner_len, const of_proof *p, const of_enc *e, of_transcript *tr,
              uint64_t *out);
void of_collapse_columns(int fid, const uint64_t *coeffs, const uint64_t *tensor, uint64_t *poly,
                         size_t n_rows, size_t n_per_row);
void of_hash_columns(int fid, const uint64_t *comm, size_t n_rows, size_t n_cols, uint8_t *out);
void of_merkle_tree(const uint8_t *ins, size_t n_ins, uint8_t *outs);
int of_open_column(const of_commit *c, size_t column, uint64_t *col_out, uint8_t *path_out);
int of_verify_column_path(int fid, const uint64_t *col, size_t n_rows, const uint8_t *path,
                          size_t path_len, size_t col_num, const uint8_t root[32]);
int of_verify_column_value(int fid, const uint64_t *col, const uint64_t *tensor, size_t n_rows,
                           const uint64_t *poly_eval);

/* ---------------- Brakedown / SDIG (lcpc-brakedown-pc) ---------------- */
of_enc *of_enc_sdig(int fid, size_t n_per_row, size_t n_cols_hint, uint64_t seed, int code_id,
                    size_t n_col_opens, size_t n_degree_tests);

/* BLAKE3 tree pieces: one chunk's chaining value; left-balanced merge of n chunk CVs (root) */
void of_blake3_chunk_cv(const uint8_t *in, size_t len, uint64_t counter, int is_root,
                        uint8_t out[32]);
void of_blake3_merge_cvs(const uint8_t *cvs, size_t n, uint8_t out[32]);

/* ---------------- proof-of-storage producers (proof-of-storage/src) ---------------- */
size_t of_pos_bytes_to_field(const uint8_t *bytes, size_t n_bytes, uint64_t *out);
void of_pos_field_to_bytes(const uint64_t *elems, size_t n, uint8_t *out, size_t expected_len);
void of_pos_default_dims(size_t field_len, size_t *n_per_row, size_t *n_cols, size_t *soundness);
size_t of_pos_column_indices(uint64_t seed, size_t amount, size_t max_index, uint64_t *out);
void of_pos_side_vectors(int fid, const uint64_t *x, size_t n_rows, size_t n_cols, uint64_t *left,
                         uint64_t *right);

#ifdef __cplusplus
}
#endif
#endif
