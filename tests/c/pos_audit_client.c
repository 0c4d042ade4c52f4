/* pos_audit_client.c -- one proof-of-storage audit round in plain C99 over include/lcpc_mi.h,
 * bound the way the reference's Rust server and client would bind liblcpc_mi.so (host memory
 * only: plain pointers and sizes).  The sequence is the reference protocol's:
 *   server, on upload: EncodedFileWriter::convert_unencoded_file -> .porenc + .portree
 *                      (encoded_file_writer.rs:134-231)
 *   server, per request: convert_file_data_to_commit from the file bytes (server.rs:670-730)
 *   client: get_column_indicies_from_random_seed (client.rs:443-456), the challenge point's side
 *           vectors (lcpc_online.rs:603-627)
 *   server: server_retreive_columns (lcpc_online.rs:241-247), verifiable_polynomial_evaluation
 *           (:454-484)
 *   client: client_online_verify_column_paths_without_full_columns (:280-318) over
 *           hash_column_to_digest, verify_proper_partial_polynomial_evaluation (:487-516)
 *   server, on edit: reencode_row (file_handler.rs:380-402), process_file_to_merkle_tree
 *           (encoded_file_reader.rs:328-346); decode_to_target_file (:59-91)
 * Checks: the .portree root is the commitment root; every opened column's leaf and path lead to
 * it; every opened column agrees with the evaluation; a tampered evaluation fails exactly its
 * column; the commitment rebuilt from its fields (lcpc_commit_from_parts, LcCommit's serde
 * form) has the same root and opens the same columns; the encoded rows streamed through a
 * ColumnDigestAccumulator (lcpc_column_digests_*) give the .portree leaves; the .porenc image
 * decodes to the file; after a one-byte edit and a row re-encode the re-hashed .porenc tree is
 * the new commitment's root and differs from the old one.
 * Usage: pos_audit_client [n_bytes]   (exit 0 and "pos audit ok" on success)
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
#define EXPECT(c, msg)                          \
  do {                                          \
    if (!(c)) {                                 \
      fprintf(stderr, "FAILED: %s\n", msg);     \
      return 1;                                 \
    }                                           \
  } while (0)

static int commit_root(const lcpc_encoding *e, const uint8_t *data, size_t n, uint8_t root[32],
                       lcpc_commit **keep) {
  lcpc_commit *c = NULL;
  CHECK(lcpc_pos_commit_bytes(e, data, n, &c));
  CHECK(lcpc_commit_get_root(c, root));
  if (keep) *keep = c;
  else lcpc_commit_free(c);
  return 0;
}

int main(int argc, char **argv) {
  const size_t n_bytes = argc > 1 ? (size_t)strtoull(argv[1], NULL, 10) : (size_t)1 << 20;
  const lcpc_field f = LCPC_FT63;
  uint8_t *data = malloc(n_bytes ? n_bytes : 1);
  if (!data) return 1;
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (size_t i = 0; i < n_bytes; i++) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    data[i] = (uint8_t)(s >> 32);
  }

  /* the server's dims for this file (server.rs:1139-1170) */
  const size_t field_len = (n_bytes + 6) / 7;
  size_t pre, enc, soundness;
  lcpc_pos_default_dims(field_len, &pre, &enc, &soundness);
  const size_t rows = (field_len + pre - 1) / pre, cap = 2 * rows; /* the writer allocates 2x */
  size_t log_enc = 0;
  while (((size_t)1 << log_enc) < enc) log_enc++;

  /* upload: .porenc + .portree */
  uint8_t *porenc = calloc(enc * cap, 8), *tree = malloc((2 * enc - 1) * 32);
  EXPECT(porenc && tree, "allocation");
  size_t rows_written = 0;
  CHECK(lcpc_pos_encode_file(data, n_bytes, pre, enc, cap, porenc, tree, &rows_written));
  EXPECT(rows_written == rows, "rows_written");
  const uint8_t *file_root = tree + (2 * enc - 2) * 32;

  /* a request: commit to the file bytes; the root is the stored tree's */
  lcpc_encoding *e = NULL;
  CHECK(lcpc_ligero_new_from_dims(f, 1, 2, pre, enc, &e));
  lcpc_commit *c = NULL;
  uint8_t root[32];
  if (commit_root(e, data, n_bytes, root, &c)) return 1;
  EXPECT(!memcmp(root, file_root, 32), "the .portree root is not the commitment root");
  EXPECT(lcpc_commit_n_rows(c) == rows && lcpc_commit_n_cols(c) == enc, "commitment dims");

  /* the client's challenge: columns from a seed, a point x and its side vectors */
  uint64_t *idx = malloc(soundness * 8), x;
  size_t n_open = 0;
  EXPECT(idx, "allocation");
  CHECK(lcpc_pos_column_indices(1337, soundness, enc, idx, &n_open));
  EXPECT(n_open == (soundness < enc ? soundness : enc), "column count");
  CHECK(lcpc_field_random(f, 77, &x, 1));
  uint64_t *left = malloc(rows * 8), *right = malloc(pre * 8), *values = malloc(enc * 8);
  uint64_t *cols = malloc(n_open * rows * 8);
  uint8_t *paths = malloc(n_open * log_enc * 32 + 1), *leaves = malloc(n_open * 32), *ok = malloc(n_open);
  EXPECT(left && right && values && cols && paths && leaves && ok, "allocation");
  CHECK(lcpc_pos_side_vectors(f, &x, rows, pre, left, right));

  /* the server's answer: the opened columns and the encoded evaluation */
  CHECK(lcpc_open_columns(c, idx, n_open, cols, paths));
  CHECK(lcpc_pos_eval_encoded(c, left, rows, values));

  /* the client's checks */
  CHECK(lcpc_hash_field_columns(f, cols, rows, n_open, leaves));
  CHECK(lcpc_verify_leaf_paths(leaves, paths, n_open, log_enc, idx, root, ok));
  for (size_t k = 0; k < n_open; k++) EXPECT(ok[k] == 1, "an opened column's path does not lead to the root");
  CHECK(lcpc_verify_column_values(f, cols, n_open, rows, left, values, enc, idx, ok));
  for (size_t k = 0; k < n_open; k++) EXPECT(ok[k] == 1, "an opened column disagrees with the evaluation");
  values[idx[0]] ^= 1;
  CHECK(lcpc_verify_column_values(f, cols, n_open, rows, left, values, enc, idx, ok));
  for (size_t k = 0; k < n_open; k++)
    EXPECT(ok[k] == (idx[k] == idx[0] ? 0 : 1), "a tampered evaluation was not caught at its column only");
  leaves[0] ^= 1;
  CHECK(lcpc_verify_leaf_paths(leaves, paths, n_open, log_enc, idx, root, ok));
  EXPECT(ok[0] == 0, "a tampered leaf was accepted");

  /* the commitment's fields (serde Serialize) rebuild it (Deserialize: lcpc_commit_from_parts),
   * and the encoded rows streamed through a ColumnDigestAccumulator give the .portree leaves */
  {
    const size_t n_hashes = lcpc_commit_n_hashes(c);
    uint64_t *comm = malloc(rows * enc * 8), *coeffs = malloc(rows * pre * 8);
    uint8_t *hashes = malloc(n_hashes * 32), *digests = malloc(enc * 32), root3[32];
    EXPECT(comm && coeffs && hashes && digests, "allocation");
    CHECK(lcpc_commit_copy_comm(c, comm));
    CHECK(lcpc_commit_copy_coeffs(c, coeffs));
    CHECK(lcpc_commit_copy_hashes(c, hashes));
    lcpc_commit *c2 = NULL;
    CHECK(lcpc_commit_from_parts(f, rows, enc, pre, comm, coeffs, hashes, n_hashes, &c2));
    CHECK(lcpc_commit_get_root(c2, root3));
    EXPECT(!memcmp(root3, root, 32), "the rebuilt commitment has another root");
    uint64_t *cols2 = malloc(n_open * rows * 8);
    uint8_t *paths2 = malloc(n_open * log_enc * 32 + 1);
    EXPECT(cols2 && paths2, "allocation");
    CHECK(lcpc_open_columns(c2, idx, n_open, cols2, paths2));
    EXPECT(!memcmp(cols2, cols, n_open * rows * 8) && !memcmp(paths2, paths, n_open * log_enc * 32),
           "the rebuilt commitment opens other columns");
    lcpc_column_digests *acc = NULL;
    CHECK(lcpc_column_digests_new(f, enc, 64, &acc));
    for (size_t r = 0; r < rows; r += 100) /* ragged batches of encoded rows */
      CHECK(lcpc_column_digests_update(acc, comm + r * enc, rows - r < 100 ? rows - r : 100));
    CHECK(lcpc_column_digests_finalize(acc, digests, NULL));
    EXPECT(!memcmp(digests, tree, enc * 32), "the accumulator's digests are not the .portree leaves");
    lcpc_column_digests_free(acc);
    lcpc_commit_free(c2);
    free(comm); free(coeffs); free(hashes); free(digests); free(cols2); free(paths2);
  }

  /* the stored image decodes to the file */
  uint8_t *back = malloc(rows * pre * 7);
  EXPECT(back, "allocation");
  CHECK(lcpc_pos_decode_porenc(porenc, pre, enc, cap, 0, rows, back));
  EXPECT(!memcmp(back, data, n_bytes), "the .porenc image does not decode to the file");

  /* an edit: one byte in the middle row, that row re-encoded in place, the tree re-hashed */
  if (n_bytes) {
    const size_t row_bytes = 7 * pre, r = (rows - 1) / 2, lo = r * row_bytes;
    data[lo] ^= 0x5a;
    const size_t nb = n_bytes - lo < row_bytes ? n_bytes - lo : row_bytes;
    CHECK(lcpc_pos_reencode_rows(data + lo, nb, pre, enc, r, porenc, cap));
    uint8_t *tree2 = malloc((2 * enc - 1) * 32), root2[32];
    EXPECT(tree2, "allocation");
    CHECK(lcpc_pos_porenc_tree(porenc, enc, rows, cap, tree2));
    if (commit_root(e, data, n_bytes, root2, NULL)) return 1;
    EXPECT(!memcmp(root2, tree2 + (2 * enc - 2) * 32, 32), "the re-hashed tree is not the edited file's root");
    EXPECT(memcmp(root2, root, 32), "the edit did not change the root");
    free(tree2);
  }

  printf("pos audit ok: %zu bytes, %zu x %zu -> %zu Ft63, %zu columns opened, root %02x%02x%02x%02x...\n",
         n_bytes, rows, pre, enc, n_open, root[0], root[1], root[2], root[3]);
  lcpc_commit_free(c);
  lcpc_encoding_free(e);
  free(data); free(porenc); free(tree); free(idx); free(left); free(right); free(values);
  free(cols); free(paths); free(leaves); free(ok); free(back);
  return 0;
}
