/*
 * lcpc_mi.h -- C ABI of liblcpc_mi.so, the MI355X-native lcpc-2d commit / prove / verify
 * row-encoding path.
 *
 * This is the drop-in boundary for the reference's LcEncoding trait and LcCommit /
 * LcEvalProof API (TrevorGKann/lcpc_proof_of_storage, lcpc-2d/src/lib.rs).  Each entry point
 * names the reference interface it replaces (file:line).  A Rust FFI shim (see
 * INTEGRATION.md) passes `&mut [F]` as `uint64_t*` after a size/alignment check: field
 * elements cross the boundary as `limbs(field)` little-endian u64 words holding ff_derive's
 * internal Montgomery form, bit-identical to the reference's `struct FtX([u64; N])`.
 *
 * Conventions
 *   - every function returns lcpc_status (0 = OK) unless it returns a size/bool; on error
 *     lcpc_last_error() returns a thread-local message;
 *   - "host" pointers are caller-owned CPU memory; "device" pointers are HIP device memory
 *     of the current device; handles own their device buffers;
 *   - handles may be used from several threads: each call leases a HIP stream from a
 *     per-device pool (commits / encodes, prove, and the latency-side calls each have their own
 *     pool; all streams run at one priority unless LCPC_PRIORITY_STREAMS=1), so independent
 *     calls, e.g. commitments of different objects, overlap on the device.
 * No torch / HIP types appear in the signatures; `void *stream` is an optional hipStream_t.
 */
#ifndef LCPC_MI_H
#define LCPC_MI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LCPC_ABI_VERSION 1

typedef enum lcpc_status {
  LCPC_OK = 0,
  /* ProverError (lcpc-2d/src/lib.rs:113-132) */
  LCPC_PROVER_TOO_BIG = 1,
  LCPC_PROVER_ENCODE = 2,
  LCPC_PROVER_COMMIT = 3,
  LCPC_PROVER_COLUMN_NUMBER = 4,
  LCPC_PROVER_OUTER_TENSOR = 5,
  /* VerifierError (lcpc-2d/src/lib.rs:139-167) */
  LCPC_VERIFIER_NUM_COL_OPENS = 10,
  LCPC_VERIFIER_COLUMN_PATH = 11,
  LCPC_VERIFIER_COLUMN_EVAL = 12,
  LCPC_VERIFIER_COLUMN_DEGREE = 13,
  LCPC_VERIFIER_OUTER_TENSOR = 14,
  LCPC_VERIFIER_INNER_TENSOR = 15,
  LCPC_VERIFIER_ENCODING_DIMS = 16,
  LCPC_VERIFIER_ENCODE = 17,
  /* fffft::FFTError (encode's Err type, lcpc-ligero-pc/src/lib.rs:159) */
  LCPC_FFT_NOT_POWER_OF_TWO = 20,
  LCPC_FFT_TOO_BIG = 21,
  LCPC_FFT_WRONG_SIZE_PRECOMP = 22,
  /* boundary-level failures (the Rust code panics / asserts here) */
  LCPC_ERR_INVALID_ARG = 30,
  LCPC_ERR_DEVICE = 31,
  LCPC_ERR_OUT_OF_MEMORY = 32,
  LCPC_ERR_NO_DEVICE = 33,
  LCPC_ERR_UNSUPPORTED = 34,
  /* a caller-owned transcript's callback (lcpc_transcript_ops) returned non-zero */
  LCPC_ERR_TRANSCRIPT = 35
} lcpc_status;

typedef enum lcpc_field {
  LCPC_FT63 = 0,      /* lcpc-test-fields/src/lib.rs:18-22; PoS WriteableFt63 (same p) */
  LCPC_FT127 = 1,     /* lcpc-test-fields/src/lib.rs:41-45 */
  LCPC_FT191 = 2,     /* lcpc-test-fields/src/lib.rs:53-57 (24-byte elements: row shards cut at chunks 2 mod 3) */
  LCPC_FT255 = 3,     /* lcpc-test-fields/src/lib.rs:65-69 */
  LCPC_FT253_192 = 4  /* proof-of-storage/src/fields/ft253_192.rs:6-10 (big-endian repr) */
} lcpc_field;

typedef struct lcpc_encoding lcpc_encoding;
typedef struct lcpc_commit lcpc_commit;
typedef struct lcpc_proof lcpc_proof;
typedef struct lcpc_transcript lcpc_transcript;

/* ------------------------------------------------------------------ library */
int lcpc_abi_version(void);
const char *lcpc_last_error(void);
/* Selects the HIP device used by handles created afterwards on this thread. */
lcpc_status lcpc_set_device(int device);
int lcpc_device_count(void);
/* u64 limbs per element (1, 2, 3, 4, 4); 0 for an unknown field */
int lcpc_field_limbs(lcpc_field f);
/* NUM_BITS of the field (SizedField::CLOG2, lcpc-2d/src/lib.rs:69-72) */
int lcpc_field_num_bits(lcpc_field f);
/* n draws of Field::random(&mut ChaCha20Rng::seed_from_u64(seed)) (ff_derive / rand_chacha):
 * the synthetic-input generator of the tests and benches (lcpc-test-fields random_coeffs,
 * lcpc-test-fields/src/lib.rs:86-108, with a seeded instead of a thread RNG). Host only. */
lcpc_status lcpc_field_random(lcpc_field f, uint64_t seed, uint64_t *out, size_t n);

/* ------------------------------------------------------------------ parameters
 * n_degree_tests (lcpc-2d/src/lib.rs:642-645), log2 (:857-859) */
size_t lcpc_n_degree_tests(size_t lambda, size_t len, size_t flog2);
size_t lcpc_log2(size_t v);
/* LigeroEncodingRho::_n_col_opens (lcpc-ligero-pc/src/lib.rs:61-64) */
size_t lcpc_ligero_n_col_opens(size_t rho_num, size_t rho_den);
/* LigeroEncodingRho::_get_dims (lcpc-ligero-pc/src/lib.rs:70-112); LCPC_PROVER_TOO_BIG when
 * the Rust function returns None */
lcpc_status lcpc_ligero_get_dims(lcpc_field f, size_t rho_num, size_t rho_den, size_t len,
                                 size_t *n_rows, size_t *n_per_row, size_t *n_cols);

/* ------------------------------------------------------------------ LcEncoding
 * Ligero: LigeroEncodingRho::{new, new_ml, new_from_dims} (lcpc-ligero-pc/src/lib.rs:121-148) */
lcpc_status lcpc_ligero_new(lcpc_field f, size_t rho_num, size_t rho_den, size_t len,
                            lcpc_encoding **out);
lcpc_status lcpc_ligero_new_ml(lcpc_field f, size_t rho_num, size_t rho_den, size_t n_vars,
                               lcpc_encoding **out);
lcpc_status lcpc_ligero_new_from_dims(lcpc_field f, size_t rho_num, size_t rho_den,
                                      size_t n_per_row, size_t n_cols, lcpc_encoding **out);
/* An R-S (fft_io) encoding with explicit soundness parameters, as the lcpc-2d test encoding
 * (lcpc-2d/src/tests.rs:23-121: N_COL_OPENS = 128, 2 degree tests). */
lcpc_status lcpc_rs_encoding_new(lcpc_field f, size_t n_per_row, size_t n_cols,
                                 size_t n_col_opens, size_t n_degree_tests, lcpc_encoding **out);
/* Brakedown: SdigEncodingS<F, SdigCodeK> (lcpc-brakedown-pc/src/lib.rs:40-176), code = K in
 * 1..6 (codespec.rs:169-232; the crate's default SdigEncoding is code 3).  The random expander
 * matrices are matgen::generate(n_per_row, seed) (matgen.rs:28-52), drawn bit-exactly. */
size_t lcpc_sdig_n_col_opens(int code);                       /* _n_col_opens :57-61 */
/* the n_per_row SdigEncodingS::new would choose for `len` coefficients (:103-110, :69-99) */
lcpc_status lcpc_sdig_get_n_per_row(lcpc_field f, int code, size_t len, size_t *n_per_row);
lcpc_status lcpc_sdig_new(lcpc_field f, int code, size_t len, uint64_t seed,
                          lcpc_encoding **out);                /* new :103-110 */
lcpc_status lcpc_sdig_new_ml(lcpc_field f, int code, size_t n_vars, uint64_t seed,
                             lcpc_encoding **out);             /* new_ml :114-123 */
lcpc_status lcpc_sdig_new_from_dims(lcpc_field f, int code, size_t n_per_row, size_t n_cols,
                                    uint64_t seed, lcpc_encoding **out); /* :126-137 */
/* 0 = Reed-Solomon / fft_io (Ligero), 1 = SDIG expander code (Brakedown) */
int lcpc_encoding_kind(const lcpc_encoding *e);
/* nonzeros of all SDIG precode + postcode matrices (0 for R-S encodings) */
size_t lcpc_encoding_matrix_nnz(const lcpc_encoding *e);
void lcpc_encoding_free(lcpc_encoding *e);
lcpc_field lcpc_encoding_field(const lcpc_encoding *e);
/* LcEncoding::get_dims / dims_ok / get_n_col_opens / get_n_degree_tests (lib.rs:94-104) */
void lcpc_encoding_get_dims(const lcpc_encoding *e, size_t len, size_t *n_rows, size_t *n_per_row,
                            size_t *n_cols);
int lcpc_encoding_dims_ok(const lcpc_encoding *e, size_t n_per_row, size_t n_cols);
size_t lcpc_encoding_n_col_opens(const lcpc_encoding *e);
size_t lcpc_encoding_n_degree_tests(const lcpc_encoding *e);
size_t lcpc_encoding_n_per_row(const lcpc_encoding *e);
size_t lcpc_encoding_n_cols(const lcpc_encoding *e);
/* Which kernel encodes rows of 2^15-point Ft63 rate-1/2 encodings (the proof-of-storage default
 * dims; no effect on any other encoding): AUTO (default) = the one-pass row kernel for file images
 * (lcpc_pos_commit_bytes_device) and the four-step pair for element rows, the measured choices
 * (DESIGN.md §4); FOURSTEP / ONEPASS force one kernel for both.  Results are identical either way.
 * No reference counterpart (fffft has one FFT).  Configuration, not a runtime switch: call it
 * right after creating the encoding, before any commit / encode / prove uses it (the setting is
 * read without synchronisation by concurrent calls on the encoding). */
#define LCPC_ROW_KERNEL_AUTO 0
#define LCPC_ROW_KERNEL_FOURSTEP 1
#define LCPC_ROW_KERNEL_ONEPASS 2
lcpc_status lcpc_encoding_set_row_kernel(lcpc_encoding *e, int kernel);
/* Pre-allocates the calling thread's page-locked staging for lcpc_prove on commitments of
 * n_rows rows under e (host only).  Optional: a thread's first prove otherwise pays the
 * hipHostMalloc.  No reference counterpart (rayon threads have no device staging). */
lcpc_status lcpc_prepare_thread(const lcpc_encoding *e, size_t n_rows);
/* Pre-allocates into the device pool the buffers and streams of `count` concurrent
 * commit + prove calls on `len` coefficients under e (otherwise the first calls at a new
 * concurrency pay hipMalloc / hipStreamCreate).  Optional. */
lcpc_status lcpc_reserve(const lcpc_encoding *e, size_t len, size_t count);
/* LcEncoding::encode (lcpc-2d/src/lib.rs:92; Ligero: fft_io_pc, lcpc-ligero-pc/src/lib.rs:
 * 162-164): in place on `len` elements (must equal n_cols) of host memory. */
lcpc_status lcpc_encode(const lcpc_encoding *e, uint64_t *inp, size_t len);
/* Batched encode of n_rows host rows (row r at rows + r * row_stride limbs-elements). */
lcpc_status lcpc_encode_rows(const lcpc_encoding *e, uint64_t *rows, size_t n_rows,
                             size_t row_stride);
/* Device batched encode: row r reads n_valid (<= n_cols) coefficients at
 * d_src + r * src_stride (elements), treats the rest of the row as zero, and writes n_cols
 * encoded elements at d_dst + r * dst_stride (>= n_cols).  Asynchronous on `stream`; with
 * stream == NULL it runs on a pooled stream and returns when the rows are written. */
lcpc_status lcpc_encode_rows_device(const lcpc_encoding *e, const void *d_src, size_t src_stride,
                                    size_t n_valid, void *d_dst, size_t dst_stride,
                                    size_t n_rows, void *stream);

/* ------------------------------------------------------------------ LcCommit
 * LcCommit::commit (lcpc-2d/src/lib.rs:314-316 -> commit :651-700).  The commitment (coeffs,
 * encoded matrix, Merkle hashes) stays resident in HBM; `len` elements of host memory.  The rows
 * cross PCIe in ~8 MiB blocks on a copy stream, each block encoded as soon as it has landed;
 * page-locked memory (hipHostMalloc / hipHostRegister) is read by the DMA engine directly,
 * pageable memory (a Rust Vec) through the HIP runtime's own pageable path, block by block. */
lcpc_status lcpc_commit_new(const lcpc_encoding *e, const uint64_t *coeffs, size_t len,
                            lcpc_commit **out);
/* 1 if the calling thread's last host-input commit read a page-locked source directly, 0 if it
 * took the pageable path (diagnostic) */
int lcpc_last_upload_pinned(void);
/* Same with the coefficients already in device memory (no PCIe transfer). */
lcpc_status lcpc_commit_new_device(const lcpc_encoding *e, const void *d_coeffs, size_t len,
                                   lcpc_commit **out);
void lcpc_commit_free(lcpc_commit *c);
/* LcCommit::get_root (:291-296) */
lcpc_status lcpc_commit_get_root(const lcpc_commit *c, uint8_t root[32]);
size_t lcpc_commit_n_rows(const lcpc_commit *c);      /* get_n_rows   :309-311 */
size_t lcpc_commit_n_cols(const lcpc_commit *c);      /* get_n_cols   :304-306 */
size_t lcpc_commit_n_per_row(const lcpc_commit *c);   /* get_n_per_row :299-301 */
size_t lcpc_commit_n_hashes(const lcpc_commit *c);
/* LcCommit's serde Deserialize (WrappedLcCommit, lib.rs:193-229): a commitment from its fields --
 * comm (n_rows x n_cols) and coeffs (n_rows x n_per_row) as row-major Montgomery limbs, the
 * n_hashes = 2 next_pow2(n_cols) - 1 digests in commit order (root last) -- loaded into HBM so
 * prove / open_column run on it.  Other sizes: LCPC_ERR_INVALID_ARG. */
lcpc_status lcpc_commit_from_parts(lcpc_field f, size_t n_rows, size_t n_cols, size_t n_per_row,
                                   const uint64_t *comm, const uint64_t *coeffs, const uint8_t *hashes,
                                   size_t n_hashes, lcpc_commit **out);
/* copies of the public fields comm / coeffs / hashes (:180-190) to host memory */
lcpc_status lcpc_commit_copy_comm(const lcpc_commit *c, uint64_t *out);
lcpc_status lcpc_commit_copy_coeffs(const lcpc_commit *c, uint64_t *out);
lcpc_status lcpc_commit_copy_hashes(const lcpc_commit *c, uint8_t *out);
/* device views (valid while the handle lives).  The encoded matrix is row-major [n_rows][n_cols]
 * for Ligero and element-major [n_cols][n_rows] for SDIG (lcpc_commit_col_major() == 1), where
 * every Merkle leaf is one contiguous column; copy_comm always returns the row-major layout. */
int lcpc_commit_col_major(const lcpc_commit *c);
/* 1 if the device codeword (lcpc_commit_device_comm) holds canonical values rather than
 * Montgomery words (R-S / Ligero commitments: the encode writes them so, and the Merkle leaves
 * hash canonical bytes); copy_comm and the opened columns are Montgomery either way. */
int lcpc_commit_comm_canonical(const lcpc_commit *c);
const void *lcpc_commit_device_comm(const lcpc_commit *c);
const void *lcpc_commit_device_coeffs(const lcpc_commit *c);
/* check_comm (:703-718) */
lcpc_status lcpc_check_comm(const lcpc_commit *c, const lcpc_encoding *e);
/* open_column (:818-855): n_rows elements + log2(n_cols) digests */
lcpc_status lcpc_open_column(const lcpc_commit *c, size_t column, uint64_t *col_out,
                             uint8_t *path_out);

/* ------------------------------------------------------------------ merlin::Transcript
 * (merlin 2.0; used by prove/verify at lcpc-2d/src/lib.rs:901,934,1057,1075-1077,1096-1104) */
lcpc_transcript *lcpc_transcript_new(const uint8_t *label, size_t label_len);
lcpc_transcript *lcpc_transcript_clone(const lcpc_transcript *t);
void lcpc_transcript_free(lcpc_transcript *t);
void lcpc_transcript_append_message(lcpc_transcript *t, const uint8_t *label, size_t label_len,
                                    const uint8_t *msg, size_t msg_len);
/* append_message(label, msgs + i * msg_len) for i < n_msgs (host bytes): the prover's per-element
 * absorption (lcpc-2d/src/lib.rs:1075-1077, 1096-1098) in one call */
void lcpc_transcript_append_messages(lcpc_transcript *t, const uint8_t *label, size_t label_len,
                                     const uint8_t *msgs, size_t msg_len, size_t n_msgs);
void lcpc_transcript_challenge_bytes(lcpc_transcript *t, const uint8_t *label, size_t label_len,
                                     uint8_t *dest, size_t dest_len);
/* A caller-owned transcript.  The reference's prove / verify take the CALLER's transcript,
 * `tr: &mut merlin::Transcript` (lcpc-2d/src/lib.rs:319-326, 547-556), and the caller keeps using
 * it afterwards (proof-of-storage/src/tests.rs:223-233, main.rs:47-57; lcpc-2d/src/tests.rs:318-413
 * continues one transcript over two proofs).  A handle made by lcpc_transcript_from_ops forwards
 * every absorb and squeeze of prove / verify -- in the reference's order, the only state being the
 * caller's -- to these functions:
 *   append_message(ctx, label, msg)          = Transcript::append_message   (merlin 2.0)
 *   append_messages(ctx, label, msgs, l, n)  = append_message(label, msgs + i * l) for i < n, the
 *       prover's per-coefficient absorption (:1075-1077, 1096-1098) in one call; may be NULL
 *       (then append_message is called n times)
 *   challenge_bytes(ctx, label, dest, n)     = Transcript::challenge_bytes
 * Labels are always one of "$l//DT", "$l//PR", "$l//PE", "$l//CO" (macros.rs:29-36), so a Rust
 * shim can map them back to its &'static [u8] constants.  Callbacks run on the calling thread,
 * inside the prove / verify call; 0 = success, anything else makes the call return
 * LCPC_ERR_TRANSCRIPT (a sharded prove still completes its exchanges first).  The handle holds no
 * transcript state of its own: lcpc_transcript_clone refuses it (NULL). */
typedef struct lcpc_transcript_ops {
  void *ctx;
  int (*append_message)(void *ctx, const uint8_t *label, size_t label_len, const uint8_t *msg,
                        size_t msg_len);
  int (*append_messages)(void *ctx, const uint8_t *label, size_t label_len, const uint8_t *msgs,
                         size_t msg_len, size_t n_msgs);
  int (*challenge_bytes)(void *ctx, const uint8_t *label, size_t label_len, uint8_t *dest,
                         size_t dest_len);
} lcpc_transcript_ops;
/* NULL (lcpc_last_error) if append_message or challenge_bytes is missing; ops is copied */
lcpc_transcript *lcpc_transcript_from_ops(const lcpc_transcript_ops *ops);
/* the first non-zero callback return seen by an ops transcript (0: none, or not an ops handle) */
int lcpc_transcript_status(const lcpc_transcript *t);

/* ------------------------------------------------------------------ LcEvalProof
 * LcCommit::prove (lcpc-2d/src/lib.rs:319-326 -> prove :1034-1123).  outer_tensor: host,
 * outer_len elements. */
lcpc_status lcpc_prove(const lcpc_commit *c, const uint64_t *outer_tensor, size_t outer_len,
                       const lcpc_encoding *e, lcpc_transcript *tr, lcpc_proof **out);
void lcpc_proof_free(lcpc_proof *p);
size_t lcpc_proof_n_cols(const lcpc_proof *p);          /* LcEvalProof::get_n_cols :537-539 */
size_t lcpc_proof_n_per_row(const lcpc_proof *p);       /* get_n_per_row :542-544 */
size_t lcpc_proof_n_rows(const lcpc_proof *p);
size_t lcpc_proof_n_degree_tests(const lcpc_proof *p);
size_t lcpc_proof_n_col_opens(const lcpc_proof *p);
size_t lcpc_proof_path_len(const lcpc_proof *p);
lcpc_field lcpc_proof_field(const lcpc_proof *p);
lcpc_status lcpc_proof_copy_p_eval(const lcpc_proof *p, uint64_t *out);
lcpc_status lcpc_proof_copy_p_random(const lcpc_proof *p, size_t i, uint64_t *out);
/* k-th opened column (LcColumn, :424-433): values (n_rows) and Merkle path (path_len x 32 B) */
lcpc_status lcpc_proof_copy_column(const lcpc_proof *p, size_t k, uint64_t *col, uint8_t *path);
/* Rebuild a proof from its public fields (e.g. after deserialisation, :591-610). */
lcpc_status lcpc_proof_from_parts(lcpc_field f, size_t n_cols, size_t n_per_row, size_t n_rows,
                                  size_t n_degree_tests, size_t n_col_opens, size_t path_len,
                                  const uint64_t *p_eval, const uint64_t *p_random,
                                  const uint64_t *cols, const uint8_t *paths, lcpc_proof **out);
/* LcEvalProof::verify (:547-556 -> verify :862-982); *eval_out = the evaluation (limbs). */
lcpc_status lcpc_verify(const uint8_t root[32], const uint64_t *outer_tensor, size_t outer_len,
                        const uint64_t *inner_tensor, size_t inner_len, const lcpc_proof *p,
                        const lcpc_encoding *e, lcpc_transcript *tr, uint64_t *eval_out);
/* lcpc_prove / lcpc_verify driving the caller's transcript through ops for this one call: the
 * drop-in for LcCommit::prove(&self, outer, enc, tr: &mut Transcript) (lib.rs:319-326) and
 * LcEvalProof::verify(.., tr: &mut Transcript) (:547-556) -- see lcpc_transcript_ops above */
lcpc_status lcpc_prove_ops(const lcpc_commit *c, const uint64_t *outer_tensor, size_t outer_len,
                           const lcpc_encoding *e, const lcpc_transcript_ops *ops, lcpc_proof **out);
lcpc_status lcpc_verify_ops(const uint8_t root[32], const uint64_t *outer_tensor, size_t outer_len,
                            const uint64_t *inner_tensor, size_t inner_len, const lcpc_proof *p,
                            const lcpc_encoding *e, const lcpc_transcript_ops *ops, uint64_t *eval_out);

/* ------------------------------------------------------------------ free functions */
/* collapse_columns (lcpc-2d/src/lib.rs:1126-1154) on host arrays: poly[c] += ... is computed
 * as poly = sum_r tensor[r] * coeffs[r][c] for c < n_per_row */
lcpc_status lcpc_collapse_columns(lcpc_field f, const uint64_t *coeffs, const uint64_t *tensor,
                                  uint64_t *poly, size_t n_rows, size_t n_per_row);
/* merkle_tree (lcpc-2d/src/lib.rs:777-790): ins has n_ins = 2^k digests, outs n_ins - 1 */
lcpc_status lcpc_merkle_tree(const uint8_t *ins, size_t n_ins, uint8_t *outs);
/* verify_column_path (:985-1012) and verify_column_value (:1015-1030): 1 = ok, 0 = fail */
int lcpc_verify_column_path(lcpc_field f, const uint64_t *col, size_t n_rows,
                            const uint8_t *path, size_t path_len, size_t col_num,
                            const uint8_t root[32]);
int lcpc_verify_column_value(lcpc_field f, const uint64_t *col, const uint64_t *tensor,
                             size_t n_rows, const uint64_t *poly_eval);
/* leaf digests of every column of a host matrix (hash_columns, :736-775) */
lcpc_status lcpc_hash_columns(lcpc_field f, const uint64_t *comm, size_t n_rows, size_t n_cols,
                              uint8_t *out);

/* ------------------------------------------------------------------ proof-of-storage producers
 * (proof-of-storage/src; the field is WriteableFt63 = LCPC_FT63's modulus and arithmetic) */
/* DataField::from_byte_vec for WriteableFt63 (fields/data_field.rs:38-46, writable_ft63.rs:
 * 35-40): each 7 little-endian data bytes (the last chunk zero padded) become one element whose
 * RAW u64 limb holds them (no Montgomery conversion).  *n_out = ceil(n_bytes / 7). */
lcpc_status lcpc_pos_bytes_to_field(const uint8_t *bytes, size_t n_bytes, uint64_t *out,
                                    size_t *n_out);
/* same on device buffers (8-byte aligned); asynchronous on `stream` (NULL: synchronous) */
lcpc_status lcpc_pos_bytes_to_field_device(const void *d_bytes, size_t n_bytes, void *d_out,
                                           void *stream);
/* The server's commitment to a file image in device memory: DataField::from_byte_vec then
 * LcCommit::commit (lcpc_online.rs:80-239, networking/server.rs:670-730), the same commitment as
 * lcpc_pos_bytes_to_field_device + lcpc_commit_new_device on ceil(n_bytes / 7) elements.  At the
 * default PoS dims (2^14 -> 2^15 Ft63 rows, 16-byte-aligned image) the bytes are unpacked inside
 * the one-pass encode (no element image in HBM); elsewhere they are packed first.  The image must
 * be 8-byte aligned; WriteableFt63 (LCPC_FT63) encodings only. */
lcpc_status lcpc_pos_commit_bytes_device(const lcpc_encoding *e, const void *d_bytes, size_t n_bytes,
                                         lcpc_commit **out);
/* The same commitment from a file image in HOST memory -- what the server has after reading the
 * file from disk on every proof request (networking/server.rs:670-679): the image crosses PCIe in
 * blocks of whole rows, and at the default dims each block is unpacked and encoded by the
 * one-pass kernel as soon as it has landed (page-locked or pageable, as lcpc_commit_new).  Any
 * alignment. */
lcpc_status lcpc_pos_commit_bytes(const lcpc_encoding *e, const uint8_t *bytes, size_t n_bytes,
                                  lcpc_commit **out);
/* DataField::field_vec_to_byte_vec truncated to expected_len (data_field.rs:57-62,
 * fields.rs:115-121) */
lcpc_status lcpc_pos_field_to_bytes(const uint64_t *elems, size_t n, uint8_t *out,
                                    size_t expected_len);
/* get_aspect_ratio_default_from_field_len + get_soundness_from_matrix_dims
 * (networking/server.rs:1139-1170) */
void lcpc_pos_default_dims(size_t field_len, size_t *n_per_row, size_t *n_cols,
                           size_t *soundness);
/* get_column_indicies_from_random_seed (networking/client.rs:443-456): ChaCha8Rng +
 * IteratorRandom::choose_multiple; *n_out = min(amount, max_index) */
lcpc_status lcpc_pos_column_indices(uint64_t seed, size_t amount, size_t max_index,
                                    uint64_t *out, size_t *n_out);
/* form_side_vectors_for_polynomial_evaluation_from_point (lcpc_online.rs:603-627):
 * right = [1, x, ..., x^(n_cols-1)], left = [1, x^n_cols, ..., x^((n_rows-1) n_cols)] */
lcpc_status lcpc_pos_side_vectors(lcpc_field f, const uint64_t *x, size_t n_rows, size_t n_cols,
                                  uint64_t *left, uint64_t *right);
/* verifiable_polynomial_evaluation (lcpc_online.rs:454-484): out[j] = sum_r left[r] comm[r][j]
 * over the ENCODED matrix (n_cols outputs; row-major commitments) */
lcpc_status lcpc_pos_eval_encoded(const lcpc_commit *c, const uint64_t *left, size_t n_rows,
                                  uint64_t *out);
/* One proof-of-storage request's GPU half in one call: lcpc_pos_commit_bytes_device on the
 * device file image, then verifiable_polynomial_evaluation with `left` (n_rows elements, the
 * commitment's row count) into eval_out (n_cols elements) -- the server's sequence
 * (networking/server.rs:670-730: convert_file_data_to_commit, then lcpc_online.rs:454-484).
 * The same commitment and the same values as the two calls.  The evaluation rides on the leaf
 * hashing's pass over the codeword (each thread sums its (chunk, column)'s rows) instead of a
 * second pass over it. */
lcpc_status lcpc_pos_commit_eval_bytes_device(const lcpc_encoding *e, const void *d_bytes, size_t n_bytes,
                                              const uint64_t *left, size_t n_rows, uint64_t *eval_out,
                                              lcpc_commit **out);
/* decode_row (lcpc_online.rs:568-574) = fffft ifft_oi on each of n_rows rows of len = 2^k
 * elements (in place); FFTError codes on bad lengths */
lcpc_status lcpc_ifft_oi_rows(lcpc_field f, uint64_t *rows, size_t n_rows, size_t len);
/* open_column (lcpc-2d/src/lib.rs:818-855) for n columns at once (server_retreive_columns,
 * lcpc_online.rs:241-247): cols_out n x n_rows elements, paths_out n x log2(n_cols) x 32 B */
lcpc_status lcpc_open_columns(const lcpc_commit *c, const uint64_t *idx, size_t n,
                              uint64_t *cols_out, uint8_t *paths_out);
/* CommitRequestType::ColumnsWithoutPath / Leaves (lcpc_online.rs:144-224): encode `len`
 * elements with e and return the requested columns (n x n_rows) and / or their BLAKE3 leaf
 * digests (n x 32 B) without building the Merkle tree; either output may be NULL */
/* PoS client verification (lcpc_online.rs:251-452):
 * hash_column_to_digest / hash_field_vec_to_digest for n_cols columns stored one after another
 * ([n_cols][n_rows] elements) -> n_cols x 32 B */
lcpc_status lcpc_hash_field_columns(lcpc_field f, const uint64_t *cols, size_t n_rows, size_t n_cols,
                                    uint8_t *out);
/* client_online_verify_column_paths_without_full_columns (:280-318): ok[k] = 1 iff leaf digest
 * k with its path (path_len x 32 B) hashes up to root at column idx[k] */
lcpc_status lcpc_verify_leaf_paths(const uint8_t *leaves, const uint8_t *paths, size_t n,
                                   size_t path_len, const uint64_t *idx, const uint8_t root[32],
                                   uint8_t *ok);
/* verify_column_value (lcpc-2d/src/lib.rs:1014-1030) batched, and the check of
 * verify_proper_partial_polynomial_evaluation (:487-516): ok[k] = 1 iff
 * sum_r tensor[r] cols[k][r] == values[idx[k]] (cols [n][n_rows]) */
lcpc_status lcpc_verify_column_values(lcpc_field f, const uint64_t *cols, size_t n, size_t n_rows,
                                      const uint64_t *tensor, const uint64_t *values,
                                      size_t n_values, const uint64_t *idx, uint8_t *ok);
lcpc_status lcpc_pos_columns(const lcpc_encoding *e, const uint64_t *elems, size_t len,
                             const uint64_t *idx, size_t n, uint64_t *cols_out,
                             uint8_t *leaves_out);

/* ------------------------------------------------------------------ PoS encoded files
 * (proof-of-storage/src/lcpc_online/encoded_file_{writer,reader}.rs, WriteableFt63).
 * A `.porenc` image is column-major: column c holds row_capacity elements starting at byte
 * c * row_capacity * 8, each the 8-byte little-endian canonical repr (F::WRITTEN_BYTES_WIDTH,
 * field_vec_to_raw_bytes, data_field.rs:24,62-70); rows past rows_written are not touched (zero in
 * a fresh set_len file).  A `.portree` image is MerkleTree::to_bytes: the 2 enc - 1 digests
 * leaves || parents, root last (merkle_tree.rs:14-27,61-63).  Callers pass mmaps of the files. */
/* EncodedFileWriter::convert_unencoded_file (encoded_file_writer.rs:134-231): the data's 7-byte
 * elements in rows of pre, each row zero padded and Ligero-encoded to enc elements, written to
 * porenc; tree = the Merkle tree of the column digests (ColumnDigestAccumulator,
 * column_digest_accumulator.rs:62-118).  *rows_written = ceil(ceil(n_bytes / 7) / pre) and
 * row_capacity must be >= it (the reference writer allocates 2 * rows, :77-80). */
lcpc_status lcpc_pos_encode_file(const uint8_t *data, size_t n_bytes, size_t pre, size_t enc,
                                 size_t row_capacity, uint8_t *porenc, uint8_t *tree,
                                 size_t *rows_written);
/* same, processing at most batch_rows rows per GPU pass (rounded to whole 1-KiB column-digest
 * chunks; 0 = automatic, about 4 GiB of device memory per pass) */
lcpc_status lcpc_pos_encode_file_batched(const uint8_t *data, size_t n_bytes, size_t pre, size_t enc,
                                         size_t row_capacity, uint8_t *porenc, uint8_t *tree,
                                         size_t *rows_written, size_t batch_rows);
/* The streaming writer itself: EncodedFileWriter::new (:40-105; porenc = the preallocated
 * image of row_capacity rows, batch_rows as above), push_bytes (:233-262), and
 * finalize_to_column_digest / _to_commit / _to_merkle_tree (:452-501): digests = the enc column
 * digests, tree = MerkleTree::to_bytes; either may be NULL.  Rows are encoded and written as
 * soon as the data is known to continue past them, the last ones at finalize.  When the file
 * must grow, the caller re-lays it out (EncodedFileReader::set_new_capacity, reader.rs:348-381)
 * and passes the new image with set_target.  porenc = NULL with row_capacity = 0 is a digest-only
 * writer: the rows are encoded and hashed into the column digests but written nowhere
 * (RowGeneratorIter::get_column_digests / convert_to_commit_root over a byte stream,
 * row_generator_iter.rs:29-41, 68-77; ColumnDigestAccumulator, column_digest_accumulator.rs:62-118). */
typedef struct lcpc_pos_writer lcpc_pos_writer;
lcpc_status lcpc_pos_writer_new(size_t pre, size_t enc, uint8_t *porenc, size_t row_capacity,
                                size_t batch_rows, lcpc_pos_writer **out);
void lcpc_pos_writer_free(lcpc_pos_writer *w);
lcpc_status lcpc_pos_writer_set_target(lcpc_pos_writer *w, uint8_t *porenc, size_t row_capacity);
size_t lcpc_pos_writer_rows_written(const lcpc_pos_writer *w);
lcpc_status lcpc_pos_writer_push_bytes(lcpc_pos_writer *w, const uint8_t *bytes, size_t n);
lcpc_status lcpc_pos_writer_finalize(lcpc_pos_writer *w, uint8_t *digests, uint8_t *tree,
                                     size_t *rows_written, size_t *bytes_of_data);
/* ColumnDigestAccumulator<Blake3, F> with ColumnsToCareAbout::All (column_digest_accumulator.rs:
 * 17-118; the server's upload path, server.rs:433, and RowGeneratorIter): column digests of a
 * matrix pushed a batch of encoded rows at a time (row-major, width elements each, Montgomery
 * limbs as everywhere else).  Each column's digest is BLAKE3(32 zero bytes || repr of its elements),
 * hashed on the GPU in 1-KiB chunks as they complete, so memory stays one batch of rows.  finalize
 * writes the width digests (get_column_digests) and / or the Merkle tree (finalize_to_merkle_tree:
 * 2 width - 1 digests, root last; width a power of two >= 2); either may be NULL.  Fields whose
 * elements tile a chunk (not Ft191).  ColumnsToCareAbout::Only is not offered: the reference's
 * update checks the row length against the tracked count and indexes the digests by column
 * number (:63-84), so it only works when it equals All, and no caller uses it. */
typedef struct lcpc_column_digests lcpc_column_digests;
/* batch_rows: rows buffered before a GPU pass hashes their complete chunks (0 = about 256 MiB) */
lcpc_status lcpc_column_digests_new(lcpc_field f, size_t width, size_t batch_rows,
                                    lcpc_column_digests **out);
void lcpc_column_digests_free(lcpc_column_digests *a);
size_t lcpc_column_digests_width(const lcpc_column_digests *a);      /* get_width :58-60 */
lcpc_status lcpc_column_digests_update(lcpc_column_digests *a, const uint64_t *rows, size_t n_rows);
lcpc_status lcpc_column_digests_finalize(lcpc_column_digests *a, uint8_t *digests, uint8_t *tree);
/* EncodedFileReader::process_file_to_merkle_tree (encoded_file_reader.rs:328-346).
 * LCPC_ERR_INVALID_ARG if an element is not canonical (from_repr(..).unwrap() panics there). */
lcpc_status lcpc_pos_porenc_tree(const uint8_t *porenc, size_t enc, size_t rows_written,
                                 size_t row_capacity, uint8_t *tree);
/* FileHandler::reencode_row (file_handler.rs:380-402) for a range of rows: bytes are the raw
 * data of rows [row_lo, row_lo + ceil(n_bytes / (7 pre))) (the last row may be short and is
 * zero-padded); each row is packed, encoded and written into the column-major .porenc image
 * (column stride row_capacity), as replace_encoded_row does (encoded_file_reader.rs:255-315).
 * edit_bytes / append_bytes (:279-366) re-encode the touched rows this way. */
lcpc_status lcpc_pos_reencode_rows(const uint8_t *bytes, size_t n_bytes, size_t pre, size_t enc,
                                   size_t row_lo, uint8_t *porenc, size_t row_capacity);
/* EncodedFileReader::get_unencoded_row_bytes / decode_to_target_file (encoded_file_reader.rs:
 * 59-91) for rows [row_lo, row_hi): (row_hi - row_lo) * pre * 7 bytes into out */
lcpc_status lcpc_pos_decode_porenc(const uint8_t *porenc, size_t pre, size_t enc,
                                   size_t row_capacity, size_t row_lo, size_t row_hi,
                                   uint8_t *out);

/* ------------------------------------------------------------------ row shards (multi-GPU)
 * One process per GPU holds rows [row0, row0 + n_shard_rows) of an n_rows x n_per_row Ligero
 * coefficient matrix.  With the exchanges done by the caller (lcpc_proof_of_storage_amd/
 * shard.py over RCCL: chaining values by column block, subtree roots, partial row sums,
 * challenge broadcasts) these reproduce commit (lcpc-2d/src/lib.rs:651-815) and prove
 * (:1034-1123) bit for bit.  Shard boundaries must fall on BLAKE3 chunk boundaries of the leaf
 * message (32 zero bytes || column): lcpc_leaf_chunk_first_row gives them. */
typedef struct lcpc_shard lcpc_shard;
size_t lcpc_leaf_n_chunks(lcpc_field f, size_t n_rows);          /* 1-KiB chunks per leaf */
size_t lcpc_leaf_chunk_first_row(lcpc_field f, size_t chunk);    /* first row of chunk */
lcpc_status lcpc_shard_new(const lcpc_encoding *e, const uint64_t *coeffs, size_t row0,
                           size_t n_shard_rows, size_t n_rows_total, lcpc_shard **out);
/* same with the shard's coefficient rows already in device memory */
lcpc_status lcpc_shard_new_device(const lcpc_encoding *e, const void *d_coeffs, size_t row0,
                                  size_t n_shard_rows, size_t n_rows_total, lcpc_shard **out);
void lcpc_shard_free(lcpc_shard *s);
/* chaining values of leaf chunks [chunk_lo, chunk_hi) of every column: out[chunk][col][32] */
lcpc_status lcpc_shard_chunk_cvs(const lcpc_shard *s, size_t chunk_lo, size_t chunk_hi,
                                 uint8_t *out);
/* leaf digests from all n_chunks chaining values of n_cols columns ([chunk][col][32]) */
lcpc_status lcpc_leaves_from_cvs(const uint8_t *cvs, size_t n_chunks, size_t n_cols,
                                 uint8_t *leaves);
/* partial collapse_columns over the shard's rows; tensors: n_tensors x n_shard_rows */
lcpc_status lcpc_shard_collapse(const lcpc_shard *s, const uint64_t *tensors, size_t n_tensors,
                                uint64_t *out);
/* the shard's rows of columns idx[]: out[k][r] (n x n_shard_rows elements) */
lcpc_status lcpc_shard_gather_columns(const lcpc_shard *s, const uint64_t *idx, size_t n,
                                      uint64_t *out);
/* out[i] = sum_k vecs[k][i] mod p */
lcpc_status lcpc_field_sum(lcpc_field f, const uint64_t *vecs, size_t n_vecs, size_t len,
                           uint64_t *out);
/* Device-resident variants for exchanges over RCCL (shard.py with the "nccl" backend): the
 * exchanged buffers are device pointers (torch tensors); host memory only for idx and the
 * folded row combination the transcript absorbs.  Same semantics as the host forms above. */
lcpc_status lcpc_shard_chunk_cvs_device(const lcpc_shard *s, size_t chunk_lo, size_t chunk_hi,
                                        void *d_out);
/* leaf digests of n_cols (a power of two) columns from d_cvs [chunk][col][32] (clobbered) and
 * their Merkle tree: d_hashes = leaves || level 1 || ... || root (2 n_cols - 1 digests) */
lcpc_status lcpc_leaves_tree_device(void *d_cvs, size_t n_chunks, size_t n_cols, void *d_hashes);
lcpc_status lcpc_shard_collapse_device(const lcpc_shard *s, const void *d_tensors,
                                       size_t n_tensors, void *d_out);
lcpc_status lcpc_shard_gather_columns_device(const lcpc_shard *s, const uint64_t *idx, size_t n,
                                             void *d_out);
lcpc_status lcpc_field_sum_device(lcpc_field f, const void *d_vecs, size_t n_vecs, size_t len,
                                  uint64_t *out);
/* the Fiat-Shamir steps of prove: degree-test tensor ("$l//DT" -> ChaCha20 -> Field::random,
 * lib.rs:1056-1062), absorbing field elements as their repr (lib.rs:1075-1077, 1096-1098) and
 * the column choice ("$l//CO" -> ChaCha20 -> Uniform(0, n_cols), lib.rs:1101-1110) */
lcpc_status lcpc_challenge_tensor(lcpc_transcript *tr, lcpc_field f, size_t n, uint64_t *out);
lcpc_status lcpc_transcript_append_field_elems(lcpc_transcript *tr, const uint8_t *label,
                                               size_t label_len, lcpc_field f,
                                               const uint64_t *elems, size_t n);
lcpc_status lcpc_challenge_columns(lcpc_transcript *tr, size_t n_cols, size_t n, uint64_t *out);

/* ------------------------------------------------------------------ communicators (multi-GPU)
 * One process per GPU.  A row-sharded commitment (below) moves its chaining values, subtree
 * digests, challenge vectors, partial row combinations and opened-column pieces through an
 * lcpc_comm: RCCL over xGMI (librccl.so.1, loaded at first use; every exchange is a device-side
 * send / recv on device buffers), or collectives the caller supplies (a host transport: the
 * tests, or several ranks sharing one GPU, which RCCL refuses).  All ranks must make the same
 * sequence of sharded calls on a comm, one at a time per comm.  Replaces the exchanges that
 * lcpc-2d's rayon row loop never needed (lcpc-2d/src/lib.rs:677-682 encodes rows in parallel on
 * one host; here the rows live on several GPUs). */
typedef struct lcpc_comm lcpc_comm;
#define LCPC_COMM_UNIQUE_ID_BYTES 128
/* ncclGetUniqueId: rank 0 makes the id and hands it to the other ranks out of band */
lcpc_status lcpc_comm_rccl_unique_id(uint8_t id[LCPC_COMM_UNIQUE_ID_BYTES]);
/* ncclCommInitRank on the calling thread's device (lcpc_set_device); collective */
lcpc_status lcpc_comm_rccl_new(const uint8_t id[LCPC_COMM_UNIQUE_ID_BYTES], int nranks, int rank,
                               lcpc_comm **out);
/* Caller-supplied collectives on DEVICE buffers of the current device.  The library drains the
 * work producing a buffer before the call and expects the data in place when it returns;
 * 0 = success.  all_gather: d_recv = the nranks ranks' `bytes`-byte buffers in rank order.
 * all_to_all_v: d_send holds send_bytes[k] bytes for rank k back to back, d_recv receives
 * recv_bytes[k] bytes from rank k back to back.  broadcast: root's d_buf to every rank. */
typedef struct lcpc_comm_ops {
  void *user;
  int (*all_gather)(void *user, const void *d_send, void *d_recv, size_t bytes);
  int (*all_to_all_v)(void *user, const void *d_send, const size_t *send_bytes, void *d_recv,
                      const size_t *recv_bytes);
  int (*broadcast)(void *user, void *d_buf, size_t bytes, int root);
} lcpc_comm_ops;
lcpc_status lcpc_comm_from_ops(const lcpc_comm_ops *ops, int nranks, int rank, lcpc_comm **out);
int lcpc_comm_nranks(const lcpc_comm *c);
int lcpc_comm_rank(const lcpc_comm *c);
int lcpc_comm_is_rccl(const lcpc_comm *c);
void lcpc_comm_free(lcpc_comm *c);

/* ------------------------------------------------------------------ row-sharded commitments
 * One Ligero or Brakedown commitment whose n_rows coefficient rows are split over the comm's ranks
 * (SURVEY.md §8e), reproducing commit (lcpc-2d/src/lib.rs:651-815) and prove (:1034-1123) bit
 * for bit.  Rank g encodes rows [row0_g, row0_g + n_g) -- cut on BLAKE3 chunk boundaries of the
 * leaf message -- and the chaining values of its chunks of every column; an all-to-all by column
 * block gives rank k the leaves and subtree of block k; an all-gather of the subtrees gives
 * every rank the whole Merkle tree (the bytes of lcpc_commit_copy_hashes).  prove runs the
 * Merlin transcript on one `root` rank: it broadcasts each challenge vector, gathers the ranks'
 * partial row combinations and folds them mod p (RCCL has no mod-p reduction), then gathers the
 * opened columns' row pieces.  Needs a power-of-two rank count of at most next_pow2(n_cols).
 * Rows are cut where a 1 KiB chunk starts on an element boundary (every chunk for 8/16/32-byte
 * elements, every third for Ft191).  Brakedown shards are element-major ([n_cols][rows], the
 * rows encoded independently, lcpc-brakedown-pc/src/encode.rs:36-94); the tree's leaves past
 * n_cols are zero digests, as in the single-GPU commit. */
/* the rows of rank `rank` */
lcpc_status lcpc_sharded_rows(lcpc_field f, size_t n_rows, int nranks, int rank, size_t *row0,
                              size_t *n_shard_rows);
typedef struct lcpc_sharded_commit lcpc_sharded_commit;
/* collective: d_rows = this rank's n_shard_rows zero-padded coefficient rows (n_per_row
 * elements each) in device memory; n_rows = the whole matrix's row count */
lcpc_status lcpc_sharded_commit_new_device(const lcpc_encoding *e, const void *d_rows, size_t n_rows,
                                           lcpc_comm *comm, lcpc_sharded_commit **out);
void lcpc_sharded_commit_free(lcpc_sharded_commit *c);
lcpc_status lcpc_sharded_commit_get_root(const lcpc_sharded_commit *c, uint8_t root[32]);
size_t lcpc_sharded_commit_n_hashes(const lcpc_sharded_commit *c);
lcpc_status lcpc_sharded_commit_copy_hashes(const lcpc_sharded_commit *c, uint8_t *out);
/* collective prove (:1034-1123): outer = the n_rows-element outer tensor (host, every rank);
 * on rank `root`, tr is the transcript and *out receives the proof; elsewhere tr is ignored
 * (may be NULL) and *out is set to NULL */
lcpc_status lcpc_sharded_prove(lcpc_sharded_commit *c, const uint64_t *outer, size_t outer_len,
                               const lcpc_encoding *e, lcpc_transcript *tr, int root,
                               lcpc_proof **out);
/* Collective proof-of-storage request on a row-sharded file commitment (networking/server.rs:
 * 652-737; the file's WriteableFt63 rows split over the ranks as above): on rank `root`,
 * eval_out (n_cols elements) = verifiable_polynomial_evaluation (proof-of-storage/src/
 * lcpc_online.rs:454-484), sum_r left[r] comm[r][j] over the ENCODED matrix -- the ranks'
 * partial sums over their rows gathered and folded mod p -- and cols_out / paths_out the n_open
 * requested columns (whole columns [k][n_rows], Montgomery, as lcpc_open_columns) with their
 * Merkle paths.  left (n_rows elements) and idx (n_open) are host inputs on every rank; outputs
 * are written on `root` only (NULL skips one).  Replaces lcpc_pos_eval_encoded +
 * lcpc_open_columns (lcpc_online.rs:454-484, 226-247) for one file committed over several GPUs. */
lcpc_status lcpc_sharded_pos_request(lcpc_sharded_commit *c, const uint64_t *left, size_t n_rows,
                                     const uint64_t *idx, size_t n_open, int root,
                                     uint64_t *eval_out, uint64_t *cols_out, uint8_t *paths_out);
/* Pipelined commit + prove of n_polys row-sharded polynomials (a proof-of-storage server's
 * objects, the bench's steps): polynomial i reads this rank's rows at d_rows[i] and is proved on
 * rank i % nranks, whose transcript is make_transcript(user, i, root_i) (the library frees it);
 * proofs[i] is set there and NULL elsewhere (proofs may be NULL: proofs are dropped), roots
 * (optional) gets every root on every rank.  Up to `depth` polynomials are in flight; the
 * exchanges of different polynomials go out in one fixed order on every rank (two RCCL groups per
 * pipeline tick: the stages with no host wait, then the tensor and column-index broadcasts that
 * wait on a transcript), `lag` ticks apart wherever the root rank absorbs a row combination into
 * its transcript (0: automatic). */
typedef lcpc_transcript *(*lcpc_make_transcript_fn)(void *user, size_t i, const uint8_t root[32]);
lcpc_status lcpc_sharded_commit_prove_many(const lcpc_encoding *e, const void *const *d_rows,
                                           size_t n_polys, size_t n_rows, const uint64_t *outer,
                                           lcpc_comm *comm, lcpc_make_transcript_fn make_transcript,
                                           void *user, size_t lag, lcpc_proof **proofs,
                                           uint8_t *roots);

/* Pre-populates this rank's device pool, page-locked staging and stream pool with what
 * lcpc_sharded_commit_prove_many(n_polys, lag) keeps in flight at once (every polynomial in
 * the pipeline holds its own rows, codeword, exchange and proof buffers), so the first call
 * at a new depth does not pay for hipMalloc / hipHostMalloc / stream creation inside it.  The
 * counterpart of lcpc_reserve for the sharded driver; no exchange. */
lcpc_status lcpc_sharded_reserve(const lcpc_encoding *e, size_t n_rows, lcpc_comm *comm,
                                 size_t n_polys, size_t lag);
/* Host-only (no device): the point-to-point transfers rank `rank` issues, in order, in every
 * exchange group of lcpc_sharded_commit_prove_many(n_polys, lag) -- the exact list run_group
 * hands RCCL as ncclSend / ncclRecv between ncclGroupStart / ncclGroupEnd.  Lets a single host
 * check that every rank's groups match (each send p -> q of n bytes meets a receive on q from p of
 * n bytes at the same position of the pair's sequence: no deadlock, right byte counts) for any
 * rank count without a GPU.  These exchanges replace nothing in the reference (its rows never
 * leave one host, lcpc-2d/src/lib.rs:677-682, 736-815); stage numbers: 0 chaining values,
 * 1 subtrees, 2 + 2r / 3 + 2r round r's tensor broadcast / partial gather, 2 + 2 rounds column
 * indices, 3 + 2 rounds opened columns (rounds = max(n_degree_tests, 1)).  A record's `tick` is
 * its exchange group: 2t + 0 / 2t + 1 for pipeline tick t's two groups.  *n_out = the record
 * count; LCPC_ERR_INVALID_ARG if it exceeds cap (out may be NULL with cap 0 to size). */
typedef struct lcpc_p2p_record {
  uint32_t tick, pos, poly, stage;
  int32_t is_send, peer;
  uint64_t bytes;
} lcpc_p2p_record;
lcpc_status lcpc_sharded_p2p_schedule(lcpc_field f, size_t n_rows, size_t n_per_row, size_t n_cols,
                                      size_t n_degree_tests, size_t n_col_opens, int nranks, int rank,
                                      size_t n_polys, size_t lag, lcpc_p2p_record *out, size_t cap,
                                      size_t *n_out);

/* ------------------------------------------------------------------ diagnostics
 * On-device check of the stream-ordered buffer pool the commit / prove / shard paths share
 * (no reference counterpart: its buffers are host Vecs).  Each round releases a 1 MiB block
 * while a writer that spins spin_us before storing still owns it, takes the same block on
 * another stream and overwrites it at once: *violations counts words the late writer clobbered
 * across the pool's fences (two fenced rounds per round: writer on the allocating stream, writer
 * on a second stream), *control_violations the same for one unfenced control round (expected
 * non-zero when the streams run concurrently), *reused the takes that returned the same block.
 * spin_us <= 100000. */
lcpc_status lcpc_selftest_pool_ordering(int rounds, uint32_t spin_us, uint64_t *violations,
                                        uint64_t *control_violations, uint64_t *reused);

/* ------------------------------------------------------------------ kernel timing
 * HIP-event timing of every kernel launch on the handle streams (off by default). */
void lcpc_prof_enable(int enable);
void lcpc_prof_reset(void);
/* accumulated milliseconds and launch count for a kernel name (0 if never launched) */
int lcpc_prof_get(const char *name, double *total_ms, uint64_t *count);
/* newline-separated kernel names seen so far; returns the full length */
size_t lcpc_prof_names(char *buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* LCPC_MI_H */
