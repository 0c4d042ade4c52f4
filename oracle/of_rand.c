/*
 * of_rand.c -- rand_chacha 0.3 / rand_core 0.6 / rand 0.8 semantics, restated
 * (TEST ORACLE ONLY).
 *
 * Reference uses (Cargo.toml:32-34):
 *   ChaCha20Rng::from_seed(key) after transcript challenges: lcpc-2d/src/lib.rs:900-906,
 *     933-940, 1056-1062, 1103-1110;
 *   F::random(&mut rng) (ff_derive; per limb next_u64, mask, reject >= p):
 *     lcpc-2d/src/lib.rs:904,1060, lcpc-brakedown-pc/src/matgen.rs:175-179;
 *   Uniform::new(0usize, n_cols).sample: lcpc-2d/src/lib.rs:937-938,1107-1108;
 *   ChaCha20Rng::seed_from_u64 + set_stream (Brakedown matgen): matgen.rs:43-44,119;
 *   ChaCha8Rng::seed_from_u64(1337) + choose_multiple (PoS column choice):
 *     proof-of-storage/src/networking/client.rs:443-456.
 * Restated:
 *   - ChaCha block: djb layout, 64-bit block counter in words 12-13, 64-bit stream id in
 *     words 14-15; key = seed as 8 LE u32 words; output = keystream as LE u32 words;
 *   - BlockRng buffer of 64 u32 (4 blocks); next_u32 takes one word; next_u64 takes two
 *     (low word first), straddling a refill as rand_core's BlockRng::next_u64 does;
 *   - fill_bytes: consumes whole u32 words (rand_core fill_via_u32_chunks), LE bytes;
 *   - seed_from_u64: PCG32 (MUL 6364136223846793005, INC 11634580027462260723) fills the
 *     32-byte seed, 4 bytes per step;
 *   - UniformInt<usize>::sample: widening multiply, zone = MAX - ((MAX - range + 1) % range);
 *   - gen_range(low..high) for u32: UniformInt<u32>::sample_single (zone from leading zeros).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "of_internal.h"

struct of_chacha {
  uint32_t key[8];
  uint64_t counter; /* next block counter */
  uint64_t stream;
  int rounds;
  uint32_t results[64];
  int index; /* 64 = empty */
};

static inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define QR(a, b, c, d)             \
  a += b; d ^= a; d = rotl32(d, 16); \
  c += d; b ^= c; b = rotl32(b, 12); \
  a += b; d ^= a; d = rotl32(d, 8);  \
  c += d; b ^= c; b = rotl32(b, 7);

static void chacha_block(const of_chacha *r, uint64_t ctr, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574};
  for (int i = 0; i < 8; i++) s[4 + i] = r->key[i];
  s[12] = (uint32_t)ctr;
  s[13] = (uint32_t)(ctr >> 32);
  s[14] = (uint32_t)r->stream;
  s[15] = (uint32_t)(r->stream >> 32);
  uint32_t x[16];
  memcpy(x, s, sizeof(x));
  for (int i = 0; i < r->rounds; i += 2) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

static void refill(of_chacha *r) {
  for (int b = 0; b < 4; b++) chacha_block(r, r->counter + (uint64_t)b, r->results + 16 * b);
  r->counter += 4;
}

of_chacha *of_chacha_from_seed(const uint8_t seed[32], int rounds) {
  of_chacha *r = (of_chacha *)calloc(1, sizeof(*r));
  for (int i = 0; i < 8; i++)
    r->key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) |
                ((uint32_t)seed[4 * i + 2] << 16) | ((uint32_t)seed[4 * i + 3] << 24);
  r->rounds = rounds;
  r->index = 64;
  return r;
}

of_chacha *of_chacha_seed_from_u64(uint64_t state, int rounds) {
  uint8_t seed[32];
  const uint64_t MUL = 6364136223846793005ULL, INC = 11634580027462260723ULL;
  for (int i = 0; i < 8; i++) {
    state = state * MUL + INC;
    uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
    uint32_t rot = (uint32_t)(state >> 59);
    uint32_t x = (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
    for (int k = 0; k < 4; k++) seed[4 * i + k] = (uint8_t)(x >> (8 * k));
  }
  return of_chacha_from_seed(seed, rounds);
}

void of_chacha_free(of_chacha *r) { free(r); }

/* rand_chacha set_stream: resets the buffer position to the current word position */
void of_chacha_set_stream(of_chacha *r, uint64_t stream) {
  /* word position = block counter of the buffered data + index */
  if (r->index < 64) {
    uint64_t wp_blocks = r->counter - 4; /* first block of the buffer */
    uint64_t word = wp_blocks * 16 + (uint64_t)r->index;
    r->stream = stream;
    r->counter = word / 16;
    r->index = 64;
    int rem = (int)(word % 16);
    if (rem) {
      refill(r);
      r->index = rem;
    }
  } else {
    r->stream = stream;
  }
}

uint32_t of_chacha_next_u32(of_chacha *r) {
  if (r->index >= 64) {
    refill(r);
    r->index = 0;
  }
  return r->results[r->index++];
}

uint64_t of_chacha_next_u64(of_chacha *r) {
  int len = 64, idx = r->index;
  if (idx < len - 1) {
    r->index += 2;
    return (uint64_t)r->results[idx] | ((uint64_t)r->results[idx + 1] << 32);
  } else if (idx >= len) {
    refill(r);
    r->index = 2;
    return (uint64_t)r->results[0] | ((uint64_t)r->results[1] << 32);
  } else {
    uint64_t x = r->results[len - 1];
    refill(r);
    r->index = 1;
    uint64_t y = r->results[0];
    return (y << 32) | x;
  }
}

void of_chacha_fill_bytes(of_chacha *r, uint8_t *dst, size_t n) {
  size_t done = 0;
  while (done < n) {
    if (r->index >= 64) {
      refill(r);
      r->index = 0;
    }
    /* consume whole words */
    size_t avail_words = (size_t)(64 - r->index);
    size_t need = n - done;
    size_t words = (need + 3) / 4;
    if (words > avail_words) words = avail_words;
    size_t bytes = words * 4 < need ? words * 4 : need;
    for (size_t b = 0; b < bytes; b++)
      dst[done + b] = (uint8_t)(r->results[r->index + b / 4] >> (8 * (b % 4)));
    r->index += (int)words;
    done += bytes;
  }
}

uint64_t of_uniform_usize(of_chacha *r, uint64_t low, uint64_t high) {
  /* Uniform::new(low, high) == new_inclusive(low, high - 1) */
  uint64_t range = high - 1 - low + 1;
  uint64_t ints_to_reject = range ? (UINT64_MAX - range + 1) % range : 0;
  if (range == 0) return of_chacha_next_u64(r);
  uint64_t zone = UINT64_MAX - ints_to_reject;
  for (;;) {
    uint64_t v = of_chacha_next_u64(r);
    unsigned __int128 m = (unsigned __int128)v * range;
    uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    if (lo <= zone) return low + hi;
  }
}

uint32_t of_gen_range_u32(of_chacha *r, uint32_t low, uint32_t high) {
  /* UniformInt<u32>::sample_single_inclusive(low, high - 1) (rand 0.8.5):
     range = high - low; zone = (range << range.leading_zeros()) - 1 (u32 arithmetic
     via $u_large = u32); v: u32 = rng.gen(); (hi, lo) = v.wmul(range); accept lo <= zone. */
  uint32_t range = high - 1 - low + 1;
  if (range == 0) return of_chacha_next_u32(r);
  uint32_t zone = (range << __builtin_clz(range)) - 1;
  for (;;) {
    uint32_t v = of_chacha_next_u32(r);
    uint64_t m = (uint64_t)v * range;
    uint32_t hi = (uint32_t)(m >> 32), lo = (uint32_t)m;
    if (lo <= zone) return low + hi;
  }
}

void of_field_random(int fid, of_chacha *r, uint64_t *out, size_t n) {
  const of_field *f = of_get_field(fid);
  const int shave = 64 * f->nl - (int)f->num_bits;
  const uint64_t mask = shave >= 64 ? 0 : (UINT64_MAX >> shave);
  for (size_t i = 0; i < n; i++) {
    uint64_t *e = out + i * f->nl;
    for (;;) {
      for (int k = 0; k < f->nl; k++) e[k] = of_chacha_next_u64(r);
      e[f->nl - 1] &= mask;
      if (of_is_valid(fid, e)) break;
    }
  }
}
