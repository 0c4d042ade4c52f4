/*
 * of_pos.c -- proof-of-storage producers around the lcpc-2d path, restated (TEST ORACLE ONLY).
 *
 * Follows:
 *   DataField::from_byte_vec          proof-of-storage/src/fields/data_field.rs:38-46
 *   WriteableFt63::from_data_bytes     proof-of-storage/src/fields/writable_ft63.rs:35-40
 *     (7 little-endian data bytes, zero padded to a u64, taken as the RAW internal limb --
 *      i.e. the Montgomery representation, no conversion)
 *   DataField::field_vec_to_byte_vec   data_field.rs:57-62 (+ truncate, fields.rs:115-121)
 *   get_aspect_ratio_default_from_field_len / get_soundness_from_matrix_dims
 *                                      proof-of-storage/src/networking/server.rs:1139-1170
 *     ((field_len as f32).sqrt().ceil(), fields::is_power_of_two = x & (x - 1) == 0)
 *   get_column_indicies_from_random_seed
 *                                      proof-of-storage/src/networking/client.rs:443-456
 *     (ChaCha8Rng::seed_from_u64 + IteratorRandom::choose_multiple, rand 0.8: reservoir of the
 *      first `amount` indices, then element i+amount replaces slot gen_index(i + 1 + amount)
 *      when that is < amount; gen_index = gen_range(0..ubound as u32))
 *   form_side_vectors_for_polynomial_evaluation_from_point
 *                                      proof-of-storage/src/lcpc_online.rs:603-627
 * verifiable_polynomial_evaluation (lcpc_online.rs:454-484) is of_collapse_columns over the
 * encoded matrix, and decode_row (:568-574) is of_ifft_oi.
 */
#include <math.h>
#include <string.h>

#include "oracle.h"
#include "of_internal.h"

size_t of_pos_bytes_to_field(const uint8_t *bytes, size_t n_bytes, uint64_t *out) {
  const size_t n = (n_bytes + 6) / 7;
  for (size_t i = 0; i < n; i++) {
    uint64_t v = 0;
    for (size_t k = 0; k < 7 && 7 * i + k < n_bytes; k++) v |= (uint64_t)bytes[7 * i + k] << (8 * k);
    out[i] = v;
  }
  return n;
}

void of_pos_field_to_bytes(const uint64_t *elems, size_t n, uint8_t *out, size_t expected_len) {
  for (size_t b = 0; b < expected_len && b < 7 * n; b++) out[b] = (uint8_t)(elems[b / 7] >> (8 * (b % 7)));
}

static int is_pow2_ref(size_t x) { return (x & (x - 1)) == 0; }
static size_t np2(size_t x) {
  size_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

void of_pos_default_dims(size_t field_len, size_t *n_per_row, size_t *n_cols, size_t *soundness) {
  const size_t w = (size_t)ceilf(sqrtf((float)field_len));
  const size_t np = is_pow2_ref(w) ? w : np2(w);
  const size_t nc = np2(np + 1);
  const double den = log2((1.0 + (double)np / (double)nc) / 2.0);
  size_t th = (size_t)ceil(-128.0 / den);
  *n_per_row = np;
  *n_cols = nc;
  *soundness = th < nc ? th : nc;
}

size_t of_pos_column_indices(uint64_t seed, size_t amount, size_t max_index, uint64_t *out) {
  of_chacha *rng = of_chacha_seed_from_u64(seed, 8);
  size_t filled = 0;
  for (size_t i = 0; i < max_index && filled < amount; i++) out[filled++] = i;
  if (filled == amount) {
    for (size_t i = 0; amount + i < max_index; i++) {
      const size_t ub = i + 1 + amount;
      size_t k;
      if (ub <= 0xffffffffu) {
        k = of_gen_range_u32(rng, 0, (uint32_t)ub);
      } else { /* UniformInt<usize>::sample_single: u64 widening multiply, approximate zone */
        const uint64_t zone = ((uint64_t)ub << __builtin_clzll((uint64_t)ub)) - 1;
        for (;;) {
          const unsigned __int128 m = (unsigned __int128)of_chacha_next_u64(rng) * ub;
          if ((uint64_t)m <= zone) {
            k = (size_t)(m >> 64);
            break;
          }
        }
      }
      if (k < amount) out[k] = amount + i;
    }
  }
  of_chacha_free(rng);
  return filled;
}

void of_pos_side_vectors(int fid, const uint64_t *x, size_t n_rows, size_t n_cols, uint64_t *left,
                         uint64_t *right) {
  const of_field *f = of_get_field(fid);
  const int nl = f->nl;
  uint64_t acc[OF_MAXL];
  memcpy(acc, f->r, sizeof(acc)); /* ONE */
  for (size_t j = 0; j < n_cols; j++) {
    memcpy(right + j * nl, acc, sizeof(uint64_t) * nl);
    of_mont_mul(f, acc, x, acc);
  }
  uint64_t l[OF_MAXL];
  memcpy(l, f->r, sizeof(l));
  for (size_t i = 0; i < n_rows; i++) {
    memcpy(left + i * nl, l, sizeof(uint64_t) * nl);
    of_mont_mul(f, l, acc, l);
  }
}
