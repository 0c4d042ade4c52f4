/*
 * of_field.c -- ff_derive 0.13 PrimeField semantics, restated (TEST ORACLE ONLY).
 *
 * The reference declares its fields with #[derive(PrimeField)]:
 *   Ft63      lcpc-test-fields/src/lib.rs:18-22   p = 5102708120182849537,  g = 10, [u64;1]
 *   Ft127     lcpc-test-fields/src/lib.rs:41-45   p = 1468...4433,          g = 3,  [u64;2]
 *   Ft191     lcpc-test-fields/src/lib.rs:53-57                              g = 5,  [u64;3]
 *   Ft255     lcpc-test-fields/src/lib.rs:65-69                              g = 5,  [u64;4]
 *   Ft253_192 proof-of-storage/src/fields/ft253_192.rs:6-10 (repr big endian) g = 3, [u64;4]
 * ff_derive derives every constant from the decimal modulus at compile time; this file
 * does the same at load time (nothing is copied from a table), so the product's generated
 * constant header is cross-checked by construction.
 *
 * Semantics restated:
 *   - internal limbs are Montgomery form a*R mod p, R = 2^(64*limbs), always fully reduced;
 *   - INV = -p^-1 mod 2^64 computed by ff_derive's 63-step square-and-multiply;
 *   - ROOT_OF_UNITY = g^((p-1) >> S), S = 2-adicity of p-1;
 *   - random(): per limb next_u64(), top limb masked to NUM_BITS, accept iff < p,
 *     and the accepted limbs ARE the Montgomery representation (no conversion);
 *   - to_repr(): canonical value bytes, little endian (big endian for Ft253_192).
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "of_internal.h"

typedef unsigned __int128 u128;

static of_field g_fields[OF_NFIELDS];
static int g_init = 0;

static const struct {
  const char *name, *modulus, *gen;
  int nl, be;
} k_decl[OF_NFIELDS] = {
    {"Ft63", "5102708120182849537", "10", 1, 0},
    {"Ft127", "146823888364060453008360742206866194433", "3", 2, 0},
    {"Ft191", "1697146272512170708389931801544665676545308500647389167617", "5", 3, 0},
    {"Ft255", "46242760681095663677370860714659204618859642560429202607213929836750194081793", "5",
     4, 0},
    {"Ft253_192",
     "14474011154664524421669271390699307717822958659997404088829842556525106692097", "3", 4, 1},
};

/* ---- raw multi-limb helpers (nl <= OF_MAXL) ---- */
static int geq_n(const uint64_t *a, const uint64_t *b, int n) {
  for (int i = n - 1; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return 1;
}
static uint64_t sub_n(uint64_t *a, const uint64_t *b, int n) { /* a -= b, returns borrow */
  uint64_t br = 0;
  for (int i = 0; i < n; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) ? 1 : 0;
  }
  return br;
}
static uint64_t add_n(uint64_t *a, const uint64_t *b, int n) { /* a += b, returns carry */
  u128 c = 0;
  for (int i = 0; i < n; i++) {
    c += (u128)a[i] + b[i];
    a[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}

static void parse_decimal(const char *s, uint64_t *out, int n) {
  memset(out, 0, sizeof(uint64_t) * n);
  for (; *s; s++) {
    u128 c = (uint64_t)(*s - '0');
    for (int i = 0; i < n; i++) {
      c += (u128)out[i] * 10u;
      out[i] = (uint64_t)c;
      c >>= 64;
    }
  }
}

/* x = 2x mod p (x < p) */
static void dbl_mod(const of_field *f, uint64_t *x) {
  uint64_t c = add_n(x, x, f->nl);
  if (c || geq_n(x, f->p, f->nl)) sub_n(x, f->p, f->nl);
}

void of_mont_mul(const of_field *f, const uint64_t *a, const uint64_t *b, uint64_t *out) {
  /* CIOS Montgomery multiplication, 64-bit words */
  const int n = f->nl;
  uint64_t t[OF_MAXL + 2];
  memset(t, 0, sizeof(t));
  for (int i = 0; i < n; i++) {
    u128 c = 0;
    for (int j = 0; j < n; j++) {
      c += (u128)a[j] * b[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[n];
    t[n] = (uint64_t)c;
    t[n + 1] = (uint64_t)(c >> 64);
    uint64_t m = t[0] * f->inv;
    c = (u128)m * f->p[0] + t[0];
    c >>= 64;
    for (int j = 1; j < n; j++) {
      c += (u128)m * f->p[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[n];
    t[n - 1] = (uint64_t)c;
    t[n] = t[n + 1] + (uint64_t)(c >> 64);
  }
  if (t[n] || geq_n(t, f->p, n)) sub_n(t, f->p, n);
  memcpy(out, t, sizeof(uint64_t) * n);
}

void of_mont_add(const of_field *f, const uint64_t *a, const uint64_t *b, uint64_t *out) {
  uint64_t t[OF_MAXL];
  memcpy(t, a, sizeof(uint64_t) * f->nl);
  uint64_t c = add_n(t, b, f->nl);
  if (c || geq_n(t, f->p, f->nl)) sub_n(t, f->p, f->nl);
  memcpy(out, t, sizeof(uint64_t) * f->nl);
}

void of_mont_sub(const of_field *f, const uint64_t *a, const uint64_t *b, uint64_t *out) {
  uint64_t t[OF_MAXL];
  memcpy(t, a, sizeof(uint64_t) * f->nl);
  if (sub_n(t, b, f->nl)) add_n(t, f->p, f->nl);
  memcpy(out, t, sizeof(uint64_t) * f->nl);
}

void of_mont_pow_big(const of_field *f, const uint64_t *a, const uint64_t *e, int en,
                     uint64_t *out) {
  uint64_t acc[OF_MAXL], base[OF_MAXL];
  memcpy(acc, f->r, sizeof(acc));
  memcpy(base, a, sizeof(uint64_t) * f->nl);
  for (int i = en * 64 - 1; i >= 0; i--) {
    of_mont_mul(f, acc, acc, acc);
    if ((e[i / 64] >> (i % 64)) & 1) of_mont_mul(f, acc, base, acc);
  }
  memcpy(out, acc, sizeof(uint64_t) * f->nl);
}

static void field_init_one(of_field *f, int id) {
  memset(f, 0, sizeof(*f));
  f->name = k_decl[id].name;
  f->nl = k_decl[id].nl;
  f->big_endian_repr = k_decl[id].be;
  parse_decimal(k_decl[id].modulus, f->p, f->nl);
  /* NUM_BITS */
  int top = f->nl - 1;
  f->num_bits = 64 * top + (64 - __builtin_clzll(f->p[top]));
  /* INV = -p^-1 mod 2^64 (ff_derive: 63 x {square, mul by p0}, then negate) */
  uint64_t inv = 1;
  for (int i = 0; i < 63; i++) {
    inv *= inv;
    inv *= f->p[0];
  }
  f->inv = (uint64_t)0 - inv;
  /* R = 2^(64 nl) mod p, R2 = R^2 mod p, by doubling */
  uint64_t x[OF_MAXL] = {1, 0, 0, 0};
  for (int i = 0; i < 64 * f->nl; i++) dbl_mod(f, x);
  memcpy(f->r, x, sizeof(x));
  for (int i = 0; i < 64 * f->nl; i++) dbl_mod(f, x);
  memcpy(f->r2, x, sizeof(x));
  /* S, t = (p-1) >> S */
  uint64_t pm1[OF_MAXL];
  memcpy(pm1, f->p, sizeof(pm1));
  pm1[0] -= 1; /* p is odd */
  int s = 0;
  while (!((pm1[s / 64] >> (s % 64)) & 1)) s++;
  f->s = (uint32_t)s;
  uint64_t t[OF_MAXL] = {0, 0, 0, 0};
  for (int i = 0; i < f->nl; i++) {
    int src = i + s / 64, sh = s % 64;
    uint64_t lo = src < f->nl ? pm1[src] : 0, hi = src + 1 < f->nl ? pm1[src + 1] : 0;
    t[i] = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
  }
  /* generator in Montgomery form, ROOT_OF_UNITY = g^t */
  uint64_t g[OF_MAXL];
  parse_decimal(k_decl[id].gen, g, f->nl);
  of_mont_mul(f, g, f->r2, f->gen);
  of_mont_pow_big(f, f->gen, t, f->nl, f->root);
}

const of_field *of_get_field(int fid) {
  if (!g_init) {
    for (int i = 0; i < OF_NFIELDS; i++) field_init_one(&g_fields[i], i);
    g_init = 1;
  }
  if (fid < 0 || fid >= OF_NFIELDS) return NULL;
  return &g_fields[fid];
}

__attribute__((constructor)) static void of_field_ctor(void) { (void)of_get_field(0); }

int of_field_limbs(int fid) { return of_get_field(fid)->nl; }
int of_field_num_bits(int fid) { return (int)of_get_field(fid)->num_bits; }
int of_field_s(int fid) { return (int)of_get_field(fid)->s; }
void of_field_modulus(int fid, uint64_t *out) {
  const of_field *f = of_get_field(fid);
  memcpy(out, f->p, sizeof(uint64_t) * f->nl);
}
void of_field_root_of_unity(int fid, uint64_t *out) {
  const of_field *f = of_get_field(fid);
  memcpy(out, f->root, sizeof(uint64_t) * f->nl);
}

void of_from_canonical(int fid, const uint64_t *in, uint64_t *out, size_t n) {
  const of_field *f = of_get_field(fid);
  for (size_t i = 0; i < n; i++) of_mont_mul(f, in + i * f->nl, f->r2, out + i * f->nl);
}
void of_to_canonical(int fid, const uint64_t *in, uint64_t *out, size_t n) {
  const of_field *f = of_get_field(fid);
  const uint64_t one[OF_MAXL] = {1, 0, 0, 0};
  for (size_t i = 0; i < n; i++) of_mont_mul(f, in + i * f->nl, one, out + i * f->nl);
}
void of_add(int fid, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n) {
  const of_field *f = of_get_field(fid);
  for (size_t i = 0; i < n; i++) of_mont_add(f, a + i * f->nl, b + i * f->nl, out + i * f->nl);
}
void of_sub(int fid, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n) {
  const of_field *f = of_get_field(fid);
  for (size_t i = 0; i < n; i++) of_mont_sub(f, a + i * f->nl, b + i * f->nl, out + i * f->nl);
}
void of_mul(int fid, const uint64_t *a, const uint64_t *b, uint64_t *out, size_t n) {
  const of_field *f = of_get_field(fid);
  for (size_t i = 0; i < n; i++) of_mont_mul(f, a + i * f->nl, b + i * f->nl, out + i * f->nl);
}
void of_pow(int fid, const uint64_t *a, uint64_t e, uint64_t *out) {
  const of_field *f = of_get_field(fid);
  uint64_t ee[1] = {e};
  of_mont_pow_big(f, a, ee, 1, out);
}
void of_inv(int fid, const uint64_t *a, uint64_t *out) {
  const of_field *f = of_get_field(fid);
  uint64_t e[OF_MAXL];
  memcpy(e, f->p, sizeof(e));
  /* p - 2 with borrow: Ft253_192's low limb is exactly 1 */
  uint64_t borrow = 2;
  for (int i = 0; i < f->nl && borrow; i++) {
    const uint64_t prev = e[i];
    e[i] = prev - borrow;
    borrow = prev < borrow ? 1 : 0;
  }
  of_mont_pow_big(f, a, e, f->nl, out);
}

int of_is_valid(int fid, const uint64_t *a) {
  const of_field *f = of_get_field(fid);
  return !geq_n(a, f->p, f->nl);
}

void of_elem_to_repr(const of_field *f, const uint64_t *in, uint8_t *out) {
  const uint64_t one[OF_MAXL] = {1, 0, 0, 0};
  uint64_t c[OF_MAXL];
  of_mont_mul(f, in, one, c);
  const int nb = 8 * f->nl;
  for (int i = 0; i < nb; i++) {
    uint8_t byte = (uint8_t)(c[i / 8] >> (8 * (i % 8)));
    if (f->big_endian_repr)
      out[nb - 1 - i] = byte;
    else
      out[i] = byte;
  }
}

void of_to_repr(int fid, const uint64_t *in, uint8_t *out, size_t n) {
  const of_field *f = of_get_field(fid);
  for (size_t i = 0; i < n; i++) of_elem_to_repr(f, in + i * f->nl, out + i * 8 * f->nl);
}
