/*
 * of_hash.c -- BLAKE3, Keccak-f[1600]/SHA3-256, STROBE-128 + Merlin transcript,
 * restated from their public specifications (TEST ORACLE ONLY).
 *
 * Reference uses:
 *   BLAKE3 (blake3 1.5, Cargo.toml:8) as `D` for column leaves, Merkle nodes and paths:
 *     lcpc-2d/src/lib.rs:749-765 (leaf = H(32 zero bytes || repr(col))), :800-805 (node),
 *     :990-1009 (path check).
 *   Merlin (merlin 2.0, Cargo.toml:25) Transcript: append_message / challenge_bytes at
 *     lcpc-2d/src/lib.rs:901,921-923,926-929,934,1057,1075-1077,1096-1098,1104.
 * Merlin restated: Transcript::new(label) = STROBE-128("Merlin v1.0") then
 *   append_message(b"dom-sep", label); append_message(l, m) = meta_AD(l) ; meta_AD(LE32(|m|),
 *   more) ; AD(m); challenge_bytes(l, out) = meta_AD(l) ; meta_AD(LE32(|out|), more) ; PRF(out).
 * STROBE-128 (rate R = 166) as in merlin's strobe.rs: init state bytes
 *   [1, R+2, 1, 0, 1, 96] || "STROBEv1.0.2", keccak-f, then meta_AD(protocol label).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "of_internal.h"

/* ============================== BLAKE3 ============================== */
static const uint32_t B3_IV[8] = {0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
                                  0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19};
static const int B3_PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
enum { B3_CHUNK_START = 1, B3_CHUNK_END = 2, B3_PARENT = 4, B3_ROOT = 8 };

static inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

static void b3_g(uint32_t *s, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
  s[a] = s[a] + s[b] + mx;
  s[d] = rotr32(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];
  s[b] = rotr32(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + my;
  s[d] = rotr32(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];
  s[b] = rotr32(s[b] ^ s[c], 7);
}

/* compress: returns the 8-word chaining value (first half of the output) */
static void b3_compress(const uint32_t cv[8], const uint8_t block[64], uint64_t counter,
                        uint32_t block_len, uint32_t flags, uint32_t out[8]) {
  uint32_t m[16], s[16];
  for (int i = 0; i < 16; i++)
    m[i] = (uint32_t)block[4 * i] | ((uint32_t)block[4 * i + 1] << 8) |
           ((uint32_t)block[4 * i + 2] << 16) | ((uint32_t)block[4 * i + 3] << 24);
  for (int i = 0; i < 8; i++) s[i] = cv[i];
  s[8] = B3_IV[0];
  s[9] = B3_IV[1];
  s[10] = B3_IV[2];
  s[11] = B3_IV[3];
  s[12] = (uint32_t)counter;
  s[13] = (uint32_t)(counter >> 32);
  s[14] = block_len;
  s[15] = flags;
  for (int r = 0; r < 7; r++) {
    b3_g(s, 0, 4, 8, 12, m[0], m[1]);
    b3_g(s, 1, 5, 9, 13, m[2], m[3]);
    b3_g(s, 2, 6, 10, 14, m[4], m[5]);
    b3_g(s, 3, 7, 11, 15, m[6], m[7]);
    b3_g(s, 0, 5, 10, 15, m[8], m[9]);
    b3_g(s, 1, 6, 11, 12, m[10], m[11]);
    b3_g(s, 2, 7, 8, 13, m[12], m[13]);
    b3_g(s, 3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      uint32_t t[16];
      for (int i = 0; i < 16; i++) t[i] = m[B3_PERM[i]];
      memcpy(m, t, sizeof(m));
    }
  }
  for (int i = 0; i < 8; i++) out[i] = s[i] ^ s[i + 8];
}

/* chaining value of one chunk (len <= 1024) at chunk index `counter` */
static void b3_chunk_cv(const uint8_t *in, size_t len, uint64_t counter, int is_root,
                        uint32_t out[8]) {
  uint32_t cv[8];
  memcpy(cv, B3_IV, sizeof(cv));
  size_t nblocks = len == 0 ? 1 : (len + 63) / 64;
  for (size_t b = 0; b < nblocks; b++) {
    uint8_t block[64];
    memset(block, 0, 64);
    size_t off = b * 64, bl = len - off < 64 ? len - off : 64;
    if (len == 0) bl = 0;
    if (bl) memcpy(block, in + off, bl);
    uint32_t flags = 0;
    if (b == 0) flags |= B3_CHUNK_START;
    if (b == nblocks - 1) {
      flags |= B3_CHUNK_END;
      if (is_root) flags |= B3_ROOT;
    }
    b3_compress(cv, block, counter, (uint32_t)bl, flags, cv);
  }
  memcpy(out, cv, sizeof(cv));
}

static void b3_parent_cv(const uint32_t l[8], const uint32_t r[8], int is_root, uint32_t out[8]) {
  uint8_t block[64];
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) {
      block[4 * i + k] = (uint8_t)(l[i] >> (8 * k));
      block[32 + 4 * i + k] = (uint8_t)(r[i] >> (8 * k));
    }
  b3_compress(B3_IV, block, 0, 64, B3_PARENT | (is_root ? B3_ROOT : 0), out);
}

static void b3_subtree(const uint8_t *in, size_t len, uint64_t chunk0, int is_root,
                       uint32_t out[8]) {
  if (len <= 1024) {
    b3_chunk_cv(in, len, chunk0, is_root, out);
    return;
  }
  /* left subtree: largest power-of-two number of whole chunks leaving >= 1 byte */
  size_t full = (len - 1) / 1024, p2 = 1;
  while (p2 * 2 <= full) p2 *= 2;
  size_t left = p2 * 1024;
  uint32_t l[8], r[8];
  b3_subtree(in, left, chunk0, 0, l);
  b3_subtree(in + left, len - left, chunk0 + p2, 0, r);
  b3_parent_cv(l, r, is_root, out);
}

/* exported pieces of the tree (used by the row-shard protocol test): the chaining value of one
 * chunk, and the left-balanced merge of n chunk chaining values into the root */
static void cv_to_bytes(const uint32_t h[8], uint8_t *out) {
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (8 * k));
}
static void cv_from_bytes(const uint8_t *in, uint32_t h[8]) {
  for (int i = 0; i < 8; i++)
    h[i] = (uint32_t)in[4 * i] | ((uint32_t)in[4 * i + 1] << 8) | ((uint32_t)in[4 * i + 2] << 16) |
           ((uint32_t)in[4 * i + 3] << 24);
}
void of_blake3_chunk_cv(const uint8_t *in, size_t len, uint64_t counter, int is_root,
                        uint8_t out[32]) {
  uint32_t h[8];
  b3_chunk_cv(in, len, counter, is_root, h);
  cv_to_bytes(h, out);
}
static void merge_rec(const uint8_t *cvs, size_t n, int is_root, uint32_t out[8]) {
  if (n == 1) {
    cv_from_bytes(cvs, out);
    return;
  }
  size_t p2 = 1;
  while (p2 * 2 < n) p2 *= 2; /* left subtree: largest power of two < n */
  uint32_t l[8], r[8];
  merge_rec(cvs, p2, 0, l);
  merge_rec(cvs + 32 * p2, n - p2, 0, r);
  b3_parent_cv(l, r, is_root, out);
}
void of_blake3_merge_cvs(const uint8_t *cvs, size_t n, uint8_t out[32]) {
  uint32_t h[8];
  merge_rec(cvs, n, 1, h);
  cv_to_bytes(h, out);
}

void of_blake3(const uint8_t *in, size_t len, uint8_t out[32]) {
  uint32_t h[8];
  b3_subtree(in, len, 0, 1, h);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (8 * k));
}

void of_b3_init(of_b3 *h) {
  h->buf = NULL;
  h->len = h->cap = 0;
}
void of_b3_update(of_b3 *h, const uint8_t *d, size_t n) {
  if (h->len + n > h->cap) {
    size_t nc = h->cap ? h->cap : 256;
    while (nc < h->len + n) nc *= 2;
    h->buf = (uint8_t *)realloc(h->buf, nc);
    h->cap = nc;
  }
  memcpy(h->buf + h->len, d, n);
  h->len += n;
}
void of_b3_finalize(of_b3 *h, uint8_t out[32]) { of_blake3(h->buf, h->len, out); }
void of_b3_free(of_b3 *h) {
  free(h->buf);
  of_b3_init(h);
}

/* ============================== Keccak ============================== */
static const uint64_t KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
/* rotation offsets r[x][y], lane index x + 5y */
static const int KROT[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                             25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};

static inline uint64_t rotl64(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

void of_keccak_f1600(uint64_t a[25]) {
  for (int round = 0; round < 24; round++) {
    uint64_t c[5], d[5], b[25];
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; x++) d[x] = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
    for (int i = 0; i < 25; i++) a[i] ^= d[i % 5];
    /* rho + pi: B[y][2x+3y] = rot(A[x][y], r[x][y]) */
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(a[x + 5 * y], KROT[x + 5 * y]);
    for (int x = 0; x < 5; x++)
      for (int y = 0; y < 5; y++)
        a[x + 5 * y] = b[x + 5 * y] ^ ((~b[(x + 1) % 5 + 5 * y]) & b[(x + 2) % 5 + 5 * y]);
    a[0] ^= KRC[round];
  }
}

static void st_bytes_xor(uint64_t *st, size_t pos, uint8_t v) {
  st[pos / 8] ^= (uint64_t)v << (8 * (pos % 8));
}
static uint8_t st_byte(const uint64_t *st, size_t pos) { return (uint8_t)(st[pos / 8] >> (8 * (pos % 8))); }
static void st_set_byte(uint64_t *st, size_t pos, uint8_t v) {
  st[pos / 8] &= ~((uint64_t)0xff << (8 * (pos % 8)));
  st[pos / 8] |= (uint64_t)v << (8 * (pos % 8));
}

void of_sha3_256(const uint8_t *in, size_t len, uint8_t out[32]) {
  uint64_t st[25];
  memset(st, 0, sizeof(st));
  const size_t rate = 136;
  size_t pos = 0;
  for (size_t i = 0; i < len; i++) {
    st_bytes_xor(st, pos++, in[i]);
    if (pos == rate) {
      of_keccak_f1600(st);
      pos = 0;
    }
  }
  st_bytes_xor(st, pos, 0x06);
  st_bytes_xor(st, rate - 1, 0x80);
  of_keccak_f1600(st);
  for (int i = 0; i < 32; i++) out[i] = st_byte(st, i);
}

/* ============================== STROBE / Merlin ============================== */
#define STROBE_R 166
enum { FLAG_I = 1, FLAG_A = 2, FLAG_C = 4, FLAG_T = 8, FLAG_M = 16, FLAG_K = 32 };

struct of_transcript {
  uint64_t st[25];
  uint8_t pos, pos_begin, cur_flags;
};

static void strobe_run_f(of_transcript *s) {
  st_bytes_xor(s->st, s->pos, s->pos_begin);
  st_bytes_xor(s->st, s->pos + 1, 0x04);
  st_bytes_xor(s->st, STROBE_R + 1, 0x80);
  of_keccak_f1600(s->st);
  s->pos = 0;
  s->pos_begin = 0;
}
static void strobe_absorb(of_transcript *s, const uint8_t *d, size_t n) {
  for (size_t i = 0; i < n; i++) {
    st_bytes_xor(s->st, s->pos, d[i]);
    s->pos++;
    if (s->pos == STROBE_R) strobe_run_f(s);
  }
}
static void strobe_squeeze(of_transcript *s, uint8_t *d, size_t n) {
  for (size_t i = 0; i < n; i++) {
    d[i] = st_byte(s->st, s->pos);
    st_set_byte(s->st, s->pos, 0);
    s->pos++;
    if (s->pos == STROBE_R) strobe_run_f(s);
  }
}
static void strobe_begin_op(of_transcript *s, uint8_t flags, int more) {
  if (more) return; /* continuing op: flags must match (merlin asserts) */
  uint8_t old_begin = s->pos_begin;
  s->pos_begin = (uint8_t)(s->pos + 1);
  s->cur_flags = flags;
  uint8_t hdr[2] = {old_begin, flags};
  strobe_absorb(s, hdr, 2);
  if ((flags & (FLAG_C | FLAG_K)) && s->pos != 0) strobe_run_f(s);
}
static void strobe_meta_ad(of_transcript *s, const uint8_t *d, size_t n, int more) {
  strobe_begin_op(s, FLAG_M | FLAG_A, more);
  strobe_absorb(s, d, n);
}
static void strobe_ad(of_transcript *s, const uint8_t *d, size_t n, int more) {
  strobe_begin_op(s, FLAG_A, more);
  strobe_absorb(s, d, n);
}
static void strobe_prf(of_transcript *s, uint8_t *d, size_t n, int more) {
  strobe_begin_op(s, FLAG_I | FLAG_A | FLAG_C, more);
  strobe_squeeze(s, d, n);
}

of_transcript *of_transcript_new(const uint8_t *label, size_t label_len) {
  of_transcript *s = (of_transcript *)calloc(1, sizeof(*s));
  const uint8_t init[18] = {1, STROBE_R + 2, 1, 0, 1, 96, 'S', 'T', 'R', 'O', 'B', 'E', 'v', '1', '.', '0', '.', '2'};
  for (int i = 0; i < 18; i++) st_bytes_xor(s->st, i, init[i]);
  of_keccak_f1600(s->st);
  s->pos = s->pos_begin = s->cur_flags = 0;
  strobe_meta_ad(s, (const uint8_t *)"Merlin v1.0", 11, 0);
  of_transcript_append_message(s, (const uint8_t *)"dom-sep", 7, label, label_len);
  return s;
}
of_transcript *of_transcript_clone(const of_transcript *t) {
  of_transcript *s = (of_transcript *)malloc(sizeof(*s));
  memcpy(s, t, sizeof(*s));
  return s;
}
void of_transcript_free(of_transcript *t) { free(t); }

void of_transcript_append_message(of_transcript *t, const uint8_t *label, size_t label_len,
                                  const uint8_t *msg, size_t msg_len) {
  uint8_t l4[4] = {(uint8_t)msg_len, (uint8_t)(msg_len >> 8), (uint8_t)(msg_len >> 16),
                   (uint8_t)(msg_len >> 24)};
  strobe_meta_ad(t, label, label_len, 0);
  strobe_meta_ad(t, l4, 4, 1);
  strobe_ad(t, msg, msg_len, 0);
}

void of_transcript_challenge_bytes(of_transcript *t, const uint8_t *label, size_t label_len,
                                   uint8_t *dest, size_t dest_len) {
  uint8_t l4[4] = {(uint8_t)dest_len, (uint8_t)(dest_len >> 8), (uint8_t)(dest_len >> 16),
                   (uint8_t)(dest_len >> 24)};
  strobe_meta_ad(t, label, label_len, 0);
  strobe_meta_ad(t, l4, 4, 1);
  strobe_prf(t, dest, dest_len, 0);
}
