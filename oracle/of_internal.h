/* of_internal.h -- shared internals of the TEST ORACLE (not part of the product). */
#ifndef LCPC_ORACLE_INTERNAL_H
#define LCPC_ORACLE_INTERNAL_H
#include <stddef.h>
#include <stdint.h>

#define OF_MAXL 4

typedef struct of_field {
  const char *name;
  int nl;
  int big_endian_repr;
  uint32_t num_bits, s;
  uint64_t p[OF_MAXL];
  uint64_t inv; /* -p^-1 mod 2^64 */
  uint64_t r[OF_MAXL];
  uint64_t r2[OF_MAXL];
  uint64_t gen[OF_MAXL];  /* Montgomery */
  uint64_t root[OF_MAXL]; /* Montgomery ROOT_OF_UNITY */
} of_field;

const of_field *of_get_field(int fid);
void of_mont_mul(const of_field *f, const uint64_t *a, const uint64_t *b, uint64_t *out);
void of_mont_add(const of_field *f, const uint64_t *a, const uint64_t *b, uint64_t *out);
void of_mont_sub(const of_field *f, const uint64_t *a, const uint64_t *b, uint64_t *out);
void of_mont_pow_big(const of_field *f, const uint64_t *a, const uint64_t *e, int en, uint64_t *out);
void of_elem_to_repr(const of_field *f, const uint64_t *in, uint8_t *out);

/* BLAKE3 incremental hasher (enough state for one-shot and streaming use) */
typedef struct of_b3 {
  uint8_t *buf;
  size_t len, cap;
} of_b3;
void of_b3_init(of_b3 *h);
void of_b3_update(of_b3 *h, const uint8_t *d, size_t n);
void of_b3_finalize(of_b3 *h, uint8_t out[32]);
void of_b3_free(of_b3 *h);

/* parallel-for over [0, n) with the oracle's thread count */
typedef void (*of_range_fn)(void *ctx, size_t lo, size_t hi);
void of_parallel_for(size_t n, size_t min_chunk, of_range_fn fn, void *ctx);

/* brakedown encode (of_sdig.c) */
int of_sdig_encode(const void *bd, int fid, uint64_t *row);
void of_sdig_free(void *bd);

#endif
