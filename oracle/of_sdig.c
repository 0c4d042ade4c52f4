/*
 * of_sdig.c -- Brakedown / SDIG expander-code encoding, restated (TEST ORACLE ONLY).
 *
 * Follows:
 *   SdigEncodingS::_n_col_opens / _n_degree_tests / new / _new_from_np1 / new_from_dims
 *                                         lcpc-brakedown-pc/src/lib.rs:54-137
 *   encode::codeword_length               lcpc-brakedown-pc/src/encode.rs:18-33
 *   encode::encode                        encode.rs:36-94
 *   encode::reed_solomon                  encode.rs:97-110
 *   matgen::generate                      matgen.rs:28-52 (per level i: ChaCha20Rng::
 *                                         seed_from_u64(seed) + set_stream(i), precode then
 *                                         postcode drawn from the same stream)
 *   matgen::get_dims                      matgen.rs:56-111
 *   matgen::gen_code                      matgen.rs:114-188 (CSC, shape (m, n); per column:
 *                                         distinct Uniform(0,m) rows until d, sorted; one
 *                                         nonzero F::random per row index)
 *   codespec SdigCode1..6                 codespec.rs:169-232 (default SdigCode3, lib.rs:19)
 * sprs' CSC `dot` is an exact field sum, so its summation order can not change a bit.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "of_internal.h"

typedef struct {
  size_t an, ad, bn, bd, rn, rd, blen;
} sdig_spec;

static const sdig_spec k_specs[7] = {
    {0, 0, 0, 0, 0, 0, 0},
    {239, 2000, 71, 2500, 71, 50, 20},     /* SdigCode1 codespec.rs:169-177 */
    {69, 500, 111, 2500, 147, 100, 20},    /* SdigCode2 :180-188 */
    {89, 500, 61, 1000, 1521, 1000, 20},   /* SdigCode3 :191-199 (default) */
    {1, 5, 41, 500, 41, 25, 20},           /* SdigCode4 :202-210 */
    {211, 1000, 97, 1000, 202, 125, 20},   /* SdigCode5 :213-221 */
    {119, 500, 241, 2000, 43, 25, 20},     /* SdigCode6 :224-232 */
};

typedef struct {
  size_t rows, cols, nnz;
  size_t *ptr;  /* cols + 1 */
  size_t *idx;  /* nnz row indices */
  uint64_t *val; /* nnz elements */
} csc;

typedef struct {
  int nlev;
  csc *pre, *post;
  size_t n_per_row, n_cols;
} sdig;

static double ent(double z) {
  double m = 1.0 - z;
  return -z * log2(z) - m * log2(m);
}
static double sp_alpha(const sdig_spec *s) { return (double)s->an / (double)s->ad; }
static double sp_beta(const sdig_spec *s) { return (double)s->bn / (double)s->bd; }
static double sp_r(const sdig_spec *s) { return (double)s->rn / (double)s->rd; }
static double sp_mu(const sdig_spec *s) { return sp_r(s) - 1.0 - sp_r(s) * sp_alpha(s); }
static double sp_nu(const sdig_spec *s) { return sp_beta(s) + sp_alpha(s) * sp_beta(s) + 0.03; }
static double cn1(const sdig_spec *s) {
  return ent(sp_beta(s)) + sp_alpha(s) * ent(1.28 * sp_beta(s) / sp_alpha(s));
}
static double cn2(const sdig_spec *s) { return sp_beta(s) * log2(sp_alpha(s) / (1.28 * sp_beta(s))); }
static double dn1(const sdig_spec *s) {
  return sp_r(s) * sp_alpha(s) * ent(sp_beta(s) / sp_r(s)) + sp_mu(s) * ent(sp_nu(s) / sp_mu(s));
}
static double dn2(const sdig_spec *s) { return sp_alpha(s) * sp_beta(s) * log2(sp_mu(s) / sp_nu(s)); }
static size_t ceil_muldiv(size_t n, size_t num, size_t den) { return (n * num + den - 1) / den; }
static size_t zmin(size_t a, size_t b) { return a < b ? a : b; }
static size_t zmax(size_t a, size_t b) { return a > b ? a : b; }

size_t of_sdig_n_col_opens(int code_id) {
  const sdig_spec *s = &k_specs[code_id];
  double dist = (double)(s->bn * s->rd) / (double)(s->bd * s->rn);
  double den = log2(1.0 - dist / 3.0);
  return (size_t)ceil(-128.0 / den);
}

/* matgen::get_dims -> number of levels; fills pre[i] = (n, m, cn), post[i] = (n', m', dn) */
static int sdig_get_dims(const sdig_spec *s, size_t n, double log2p, size_t pre[][3],
                         size_t post[][3]) {
  size_t chain[64];
  int k = 0;
  if (!(n > s->blen)) return -1;
  for (size_t ni = n; ni > s->blen; ni = ceil_muldiv(ni, s->an, s->ad)) chain[k++] = ni;
  chain[k] = ceil_muldiv(chain[k - 1], s->an, s->ad);
  k++;
  int nlev = k - 1;
  for (int i = 0; i < nlev; i++) {
    size_t ni = chain[i], mi = chain[i + 1];
    size_t a = ceil_muldiv(ni, 32 * s->bn, 25 * s->bd);
    size_t b = 4 + ceil_muldiv(ni, s->bn, s->bd);
    size_t c = (size_t)ceil((110.0 / (double)ni + cn1(s)) / cn2(s));
    size_t cn = zmin(zmax(a, b), c);
    cn = zmin(cn, mi);
    pre[i][0] = ni;
    pre[i][1] = mi;
    pre[i][2] = cn;
    size_t nip = ceil_muldiv(mi, s->rn, s->rd);
    size_t mip = ceil_muldiv(ni, s->rn, s->rd) - ni - nip;
    size_t t1 = ceil_muldiv(ni, 2 * s->bn, s->bd);
    size_t t2 = ceil_muldiv(ni, s->rn, s->rd) - ni + 110;
    size_t dn = zmin(t1 + (size_t)ceil((double)t2 / log2p),
                     (size_t)ceil((110.0 / (double)ni + dn1(s)) / dn2(s)));
    dn = zmin(dn, mip);
    post[i][0] = nip;
    post[i][1] = mip;
    post[i][2] = dn;
  }
  return nlev;
}

static int cmp_sz(const void *a, const void *b) {
  size_t x = *(const size_t *)a, y = *(const size_t *)b;
  return x < y ? -1 : x > y;
}

static void gen_code(int fid, size_t n, size_t m, size_t d, of_chacha *rng, csc *out) {
  const int nl = of_field_limbs(fid);
  out->rows = m;
  out->cols = n;
  out->ptr = (size_t *)malloc(sizeof(size_t) * (n + 1));
  out->idx = (size_t *)malloc(sizeof(size_t) * (d * n + 1));
  out->val = (uint64_t *)malloc(sizeof(uint64_t) * nl * (d * n + 1));
  size_t *tmp = (size_t *)malloc(sizeof(size_t) * (d + 1));
  size_t nnz = 0;
  out->ptr[0] = 0;
  for (size_t c = 0; c < n; c++) {
    size_t cnt = 0;
    while (cnt < d) {
      size_t x = (size_t)of_uniform_usize(rng, 0, m);
      int dup = 0;
      for (size_t k = 0; k < cnt; k++)
        if (tmp[k] == x) {
          dup = 1;
          break;
        }
      if (!dup) tmp[cnt++] = x;
    }
    qsort(tmp, cnt, sizeof(size_t), cmp_sz);
    size_t last = m + 1;
    for (size_t k = 0; k < cnt; k++) {
      if (tmp[k] == last) continue;
      last = tmp[k];
      uint64_t *v = out->val + nnz * nl;
      for (;;) {
        of_field_random(fid, rng, v, 1);
        int z = 1;
        for (int l = 0; l < nl; l++) z &= v[l] == 0;
        if (!z) break;
      }
      out->idx[nnz++] = tmp[k];
    }
    out->ptr[c + 1] = nnz;
  }
  out->nnz = nnz;
  free(tmp);
}

static size_t codeword_length(const sdig *s) {
  size_t len = s->pre[0].cols + s->post[s->nlev - 1].cols;
  for (int i = 0; i < s->nlev - 1; i++) len += s->pre[i].rows;
  for (int i = 0; i < s->nlev; i++) len += s->post[i].rows;
  return len;
}

/* y (m) = M x (n), CSC */
static void csc_dot(const of_field *f, const csc *M, const uint64_t *x, uint64_t *y) {
  const int nl = f->nl;
  uint64_t t[OF_MAXL];
  memset(y, 0, sizeof(uint64_t) * nl * M->rows);
  for (size_t c = 0; c < M->cols; c++)
    for (size_t k = M->ptr[c]; k < M->ptr[c + 1]; k++) {
      of_mont_mul(f, M->val + k * nl, x + c * nl, t);
      of_mont_add(f, y + M->idx[k] * nl, t, y + M->idx[k] * nl);
    }
}

static void reed_solomon(const of_field *f, const uint64_t *xi, size_t nin, uint64_t *xo,
                         size_t nout) {
  const int nl = f->nl;
  uint64_t x[OF_MAXL], r[OF_MAXL];
  memcpy(x, f->r, sizeof(x)); /* ONE */
  for (size_t k = 0; k < nout; k++) {
    memset(r, 0, sizeof(r));
    for (size_t j = nin; j-- > 0;) {
      of_mont_mul(f, r, x, r);
      of_mont_add(f, r, xi + j * nl, r);
    }
    memcpy(xo + k * nl, r, sizeof(uint64_t) * nl);
    of_mont_add(f, x, f->r, x);
  }
}

int of_sdig_encode(const void *bdv, int fid, uint64_t *xi) {
  const sdig *s = (const sdig *)bdv;
  const of_field *f = of_get_field(fid);
  const int nl = f->nl;
  size_t in_start = 0;
  for (int i = 0; i < s->nlev - 1; i++) {
    const csc *P = &s->pre[i];
    size_t in_end = in_start + P->cols;
    csc_dot(f, P, xi + in_start * nl, xi + in_end * nl);
    in_start = in_end;
  }
  const csc *PL = &s->pre[s->nlev - 1];
  size_t in_end = in_start + PL->cols;
  uint64_t *tmp = (uint64_t *)malloc(sizeof(uint64_t) * nl * (PL->rows + 1));
  csc_dot(f, PL, xi + in_start * nl, tmp);
  size_t out_end = in_end + s->post[s->nlev - 1].cols;
  reed_solomon(f, tmp, PL->rows, xi + in_end * nl, out_end - in_end);
  free(tmp);
  in_start = in_end + PL->rows;
  size_t out_start = out_end;
  for (int i = s->nlev - 1; i >= 0; i--) {
    in_start -= s->pre[i].rows;
    const csc *Q = &s->post[i];
    if (out_start - in_start != Q->cols) return 3;
    /* output region starts at out_start, input region [in_start, out_start) -- disjoint */
    csc_dot(f, Q, xi + in_start * nl, xi + out_start * nl);
    out_start += Q->rows;
  }
  if (in_start != s->pre[0].cols || out_start != s->n_cols) return 3;
  return 0;
}

void of_sdig_free(void *bdv) {
  sdig *s = (sdig *)bdv;
  if (!s) return;
  for (int i = 0; i < s->nlev; i++) {
    free(s->pre[i].ptr); free(s->pre[i].idx); free(s->pre[i].val);
    free(s->post[i].ptr); free(s->post[i].idx); free(s->post[i].val);
  }
  free(s->pre);
  free(s->post);
  free(s);
}

static sdig *sdig_generate(int fid, int code_id, size_t n, uint64_t seed) {
  const sdig_spec *sp = &k_specs[code_id];
  size_t pre[64][3], post[64][3];
  int nlev = sdig_get_dims(sp, n, (double)(of_field_num_bits(fid) - 1), pre, post);
  if (nlev < 1) return NULL;
  sdig *s = (sdig *)calloc(1, sizeof(*s));
  s->nlev = nlev;
  s->pre = (csc *)calloc(nlev, sizeof(csc));
  s->post = (csc *)calloc(nlev, sizeof(csc));
  for (int i = 0; i < nlev; i++) {
    of_chacha *rng = of_chacha_seed_from_u64(seed, 20);
    of_chacha_set_stream(rng, (uint64_t)i);
    gen_code(fid, pre[i][0], pre[i][1], pre[i][2], rng, &s->pre[i]);
    gen_code(fid, post[i][0], post[i][1], post[i][2], rng, &s->post[i]);
    of_chacha_free(rng);
  }
  s->n_per_row = n;
  s->n_cols = codeword_length(s);
  return s;
}

/* SdigEncodingS::_new_from_np1 (lib.rs:69-99) -> n_per_row choice */
size_t of_sdig_choose_np(int fid, int code_id, size_t len, size_t np1) {
  if (np1 > len) np1 = len;
  size_t nco = of_sdig_n_col_opens(code_id);
  size_t flog2 = (size_t)of_field_num_bits(fid) - 1;
  size_t nr1 = (len + np1 - 1) / np1;
  size_t nd1 = of_n_degree_tests(128, np1 * 2, flog2);
  size_t np2 = np1 / 2;
  size_t nr2 = (len + np2 - 1) / np2;
  size_t nd2 = of_n_degree_tests(128, np2 * 2, flog2);
  size_t sz1 = nco * nr1 + (1 + nd1) * np1;
  size_t sz2 = nco * nr2 + (1 + nd2) * np2;
  return sz1 < sz2 ? np1 : np2;
}

/* SdigEncodingS::new (lib.rs:103-110) -> n_per_row */
size_t of_sdig_new_np(int fid, int code_id, size_t len) {
  size_t nco = of_sdig_n_col_opens(code_id);
  size_t flog2 = (size_t)of_field_num_bits(fid) - 1;
  double lncf = (double)(nco * len);
  double ndt = (double)of_n_degree_tests(128, (size_t)ceil(sqrt(lncf)) * 2, flog2);
  size_t np1 = (size_t)ceil(sqrt(lncf / ndt));
  return of_sdig_choose_np(fid, code_id, len, np1);
}

/* n_cols_hint: 0 = take the generated length; otherwise it must match (new_from_dims) */
of_enc *of_enc_sdig(int fid, size_t n_per_row, size_t n_cols_hint, uint64_t seed, int code_id,
                    size_t n_col_opens, size_t n_degree_tests) {
  if (code_id < 1 || code_id > 6) return NULL;
  sdig *s = sdig_generate(fid, code_id, n_per_row, seed);
  if (!s) return NULL;
  if (n_cols_hint && n_cols_hint != s->n_cols) {
    of_sdig_free(s);
    return NULL;
  }
  of_enc *e = (of_enc *)calloc(1, sizeof(*e));
  e->fid = fid;
  e->kind = 1;
  e->bd = s;
  e->n_per_row = n_per_row;
  e->n_cols = s->n_cols;
  e->n_col_opens = n_col_opens ? n_col_opens : of_sdig_n_col_opens(code_id);
  e->n_degree_tests = n_degree_tests
                          ? n_degree_tests
                          : of_n_degree_tests(128, s->n_cols, (size_t)of_field_num_bits(fid) - 1);
  return e;
}

/* matrix export for tests: level, which (0 pre / 1 post), returns nnz; copies if buffers */
size_t of_sdig_matrix(const of_enc *e, int level, int which, size_t *rows, size_t *cols,
                      size_t *ptr, size_t *idx, uint64_t *val) {
  const sdig *s = (const sdig *)e->bd;
  if (level < 0 || level >= s->nlev) return 0;
  const csc *M = which ? &s->post[level] : &s->pre[level];
  const int nl = of_field_limbs(e->fid);
  *rows = M->rows;
  *cols = M->cols;
  if (ptr) memcpy(ptr, M->ptr, sizeof(size_t) * (M->cols + 1));
  if (idx) memcpy(idx, M->idx, sizeof(size_t) * M->nnz);
  if (val) memcpy(val, M->val, sizeof(uint64_t) * nl * M->nnz);
  return M->nnz;
}
int of_sdig_levels(const of_enc *e) { return ((const sdig *)e->bd)->nlev; }
