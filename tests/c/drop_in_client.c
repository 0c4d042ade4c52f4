/* drop_in_client.c -- a plain C99 caller of liblcpc_mi.so, bound the way a Rust FFI crate binds
 * it (include/lcpc_mi.h only: plain pointers and sizes, no HIP or torch types).  It does what the
 * reference's callers do with lcpc-2d:
 *   LcEncoding::new, LcCommit::commit(&[F]) from host memory  (lcpc-2d/src/lib.rs:314-316, 651-700)
 *   LcCommit::prove(&outer, &enc, &mut tr) with the CALLER's transcript        (:319-326)
 *   LcEvalProof::verify(root, &outer, &inner, &enc, &mut tr)                   (:547-556)
 * The caller's transcript here is the library's Merlin restatement behind lcpc_transcript_ops,
 * standing in for merlin::Transcript behind a Rust shim ("level 2").  Checks:
 *   - prove through the ops table == prove with a library transcript (same p_eval, same columns);
 *   - the caller's transcript ends in the same state (the next challenge is equal);
 *   - verify through the ops table accepts, with the evaluation sum_c inner[c] p_eval[c];
 *   - a wrong root is rejected with a VerifierError status.
 * Usage: drop_in_client [log2 len]   (exit 0 and "drop-in client ok" on success)
 * Build: gcc -std=c99 -O2 drop_in_client.c -I../../include -L../../lcpc_proof_of_storage_amd -llcpc_mi
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lcpc_mi.h"

#define CHECK(x)                                                                          \
  do {                                                                                    \
    lcpc_status st__ = (x);                                                               \
    if (st__ != LCPC_OK) {                                                                \
      fprintf(stderr, "%s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #x, (int)st__,        \
              lcpc_last_error());                                                         \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

/* the ops table over a caller-side transcript object */
static int tr_append(void *ctx, const uint8_t *label, size_t ll, const uint8_t *msg, size_t ml) {
  lcpc_transcript_append_message((lcpc_transcript *)ctx, label, ll, msg, ml);
  return 0;
}
static int tr_append_many(void *ctx, const uint8_t *label, size_t ll, const uint8_t *msgs, size_t ml, size_t n) {
  lcpc_transcript_append_messages((lcpc_transcript *)ctx, label, ll, msgs, ml, n);
  return 0;
}
static int tr_challenge(void *ctx, const uint8_t *label, size_t ll, uint8_t *dest, size_t n) {
  lcpc_transcript_challenge_bytes((lcpc_transcript *)ctx, label, ll, dest, n);
  return 0;
}

/* the transcript prefix the reference's tests use: new(b"test transcript"), the root, n_col_opens */
static lcpc_transcript *fresh_transcript(const uint8_t root[32], size_t n_col_opens) {
  static const uint8_t name[] = "test transcript";
  lcpc_transcript *t = lcpc_transcript_new(name, sizeof(name) - 1);
  uint8_t nco[8];
  for (int i = 0; i < 8; i++) nco[i] = (uint8_t)(n_col_opens >> (56 - 8 * i));
  lcpc_transcript_append_message(t, (const uint8_t *)"polycommit", 10, root, 32);
  lcpc_transcript_append_message(t, (const uint8_t *)"ncols", 5, nco, 8);
  return t;
}

int main(int argc, char **argv) {
  const int log_len = argc > 1 ? atoi(argv[1]) : 16;
  const size_t len = (size_t)1 << log_len;
  const lcpc_field f = LCPC_FT127;
  const size_t nl = (size_t)lcpc_field_limbs(f);
  lcpc_encoding *e = NULL;
  CHECK(lcpc_ligero_new(f, 1, 2, len, &e));
  size_t n_rows, n_per_row, n_cols;
  lcpc_encoding_get_dims(e, len, &n_rows, &n_per_row, &n_cols);
  const size_t nco = lcpc_encoding_n_col_opens(e);

  uint64_t *coeffs = malloc(len * nl * 8), *outer = malloc(n_rows * nl * 8), *inner = malloc(n_per_row * nl * 8);
  if (!coeffs || !outer || !inner) return 1;
  CHECK(lcpc_field_random(f, 1, coeffs, len));
  CHECK(lcpc_field_random(f, 2, outer, n_rows));
  CHECK(lcpc_field_random(f, 3, inner, n_per_row));

  lcpc_commit *c = NULL;
  CHECK(lcpc_commit_new(e, coeffs, len, &c)); /* host memory: the caller's Vec<F> */
  uint8_t root[32];
  CHECK(lcpc_commit_get_root(c, root));

  /* prove: the library's transcript, then the caller's through the ops table */
  lcpc_transcript *t_lib = fresh_transcript(root, nco), *t_own = fresh_transcript(root, nco);
  lcpc_proof *p_lib = NULL, *p_ops = NULL;
  CHECK(lcpc_prove(c, outer, n_rows, e, t_lib, &p_lib));
  const lcpc_transcript_ops ops = {t_own, tr_append, tr_append_many, tr_challenge};
  CHECK(lcpc_prove_ops(c, outer, n_rows, e, &ops, &p_ops));

  uint64_t *ev_lib = malloc(n_per_row * nl * 8), *ev_ops = malloc(n_per_row * nl * 8);
  uint64_t *col_a = malloc(n_rows * nl * 8), *col_b = malloc(n_rows * nl * 8);
  const size_t pl = lcpc_proof_path_len(p_lib);
  uint8_t *path_a = malloc(pl * 32 + 1), *path_b = malloc(pl * 32 + 1);
  if (!ev_lib || !ev_ops || !col_a || !col_b || !path_a || !path_b) return 1;
  CHECK(lcpc_proof_copy_p_eval(p_lib, ev_lib));
  CHECK(lcpc_proof_copy_p_eval(p_ops, ev_ops));
  if (memcmp(ev_lib, ev_ops, n_per_row * nl * 8)) {
    fprintf(stderr, "p_eval differs between the library and the caller's transcript\n");
    return 1;
  }
  if (lcpc_proof_n_col_opens(p_ops) != nco) return 1;
  for (size_t k = 0; k < nco; k++) {
    CHECK(lcpc_proof_copy_column(p_lib, k, col_a, path_a));
    CHECK(lcpc_proof_copy_column(p_ops, k, col_b, path_b));
    if (memcmp(col_a, col_b, n_rows * nl * 8) || memcmp(path_a, path_b, pl * 32)) {
      fprintf(stderr, "opened column %zu differs\n", k);
      return 1;
    }
  }
  uint8_t ch_lib[32], ch_own[32];
  lcpc_transcript_challenge_bytes(t_lib, (const uint8_t *)"next", 4, ch_lib, 32);
  lcpc_transcript_challenge_bytes(t_own, (const uint8_t *)"next", 4, ch_own, 32);
  if (memcmp(ch_lib, ch_own, 32)) {
    fprintf(stderr, "the caller's transcript ended in another state\n");
    return 1;
  }

  /* verify through the ops table: accepted, and the evaluation is returned */
  lcpc_transcript *t_ver = fresh_transcript(root, nco);
  const lcpc_transcript_ops vops = {t_ver, tr_append, tr_append_many, tr_challenge};
  uint64_t eval[4] = {0, 0, 0, 0};
  CHECK(lcpc_verify_ops(root, outer, n_rows, inner, n_per_row, p_ops, e, &vops, eval));

  /* a wrong root: a VerifierError (the column paths no longer lead to it) */
  uint8_t bad_root[32];
  memcpy(bad_root, root, 32);
  bad_root[0] ^= 1;
  lcpc_transcript *t_bad = fresh_transcript(bad_root, nco);
  const lcpc_transcript_ops bops = {t_bad, tr_append, tr_append_many, tr_challenge};
  const lcpc_status st = lcpc_verify_ops(bad_root, outer, n_rows, inner, n_per_row, p_ops, e, &bops, eval);
  if (st == LCPC_OK || st < LCPC_VERIFIER_NUM_COL_OPENS || st > LCPC_VERIFIER_ENCODE) {
    fprintf(stderr, "a wrong root was not rejected as a VerifierError (status %d)\n", (int)st);
    return 1;
  }

  printf("drop-in client ok: 2^%d Ft127 coefficients, %zu x %zu -> %zu, %zu opened columns, root %02x%02x%02x%02x...\n",
         log_len, n_rows, n_per_row, n_cols, nco, root[0], root[1], root[2], root[3]);
  lcpc_transcript_free(t_lib);
  lcpc_transcript_free(t_own);
  lcpc_transcript_free(t_ver);
  lcpc_transcript_free(t_bad);
  lcpc_proof_free(p_lib);
  lcpc_proof_free(p_ops);
  lcpc_commit_free(c);
  lcpc_encoding_free(e);
  free(coeffs);
  free(outer);
  free(inner);
  free(ev_lib);
  free(ev_ops);
  free(col_a);
  free(col_b);
  free(path_a);
  free(path_b);
  return 0;
}
