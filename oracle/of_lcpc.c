/*
 * of_lcpc.c -- lcpc-2d commit / Merkle / prove / verify and the Ligero encoding,
 * restated in C (TEST ORACLE ONLY; also the timed CPU baseline of bench.py).
 *
 * Follows, function by function:
 *   n_degree_tests     lcpc-2d/src/lib.rs:642-645     log2           :857-859
 *   commit             :651-700                        check_comm     :703-718
 *   merkleize          :720-734                        hash_columns   :736-775
 *   merkle_tree/layer  :777-815                        open_column    :818-855
 *   verify             :862-982                        verify_column_path  :985-1012
 *   verify_column_value :1015-1030                     prove          :1034-1123
 *   collapse_columns   :1126-1154
 *   Ligero dims/params lcpc-ligero-pc/src/lib.rs:45-118, encode :162-164
 *   labels             lcpc-2d/src/macros.rs:29-36 -- `b"$l//DT"` is a byte-string literal,
 *                      which macro_rules! does not substitute into, so every encoding's
 *                      labels are literally "$l//DT", "$l//PR", "$l//PE", "$l//CO".
 * rayon's parallel loops become a pthread parallel-for (of_set_threads); all arithmetic is
 * exact, so the thread count can not change any output bit.
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "of_internal.h"

static const uint8_t LABEL_DT[] = "$l//DT";
static const uint8_t LABEL_PR[] = "$l//PR";
static const uint8_t LABEL_PE[] = "$l//PE";
static const uint8_t LABEL_CO[] = "$l//CO";
#define LABEL_LEN 6

/* ---------------- thread pool-less parallel for ---------------- */
static int g_threads = 1;
void of_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
int of_get_threads(void) { return g_threads; }

typedef struct {
  of_range_fn fn;
  void *ctx;
  size_t lo, hi;
} pf_arg;
static void *pf_tramp(void *p) {
  pf_arg *a = (pf_arg *)p;
  a->fn(a->ctx, a->lo, a->hi);
  return NULL;
}
void of_parallel_for(size_t n, size_t min_chunk, of_range_fn fn, void *ctx) {
  int nt = g_threads;
  if (min_chunk < 1) min_chunk = 1;
  if ((size_t)nt > n / min_chunk) nt = (int)(n / min_chunk);
  if (nt <= 1) {
    fn(ctx, 0, n);
    return;
  }
  pthread_t th[256];
  pf_arg args[256];
  if (nt > 256) nt = 256;
  int started[256];
  for (int t = 0; t < nt; t++) {
    args[t].fn = fn;
    args[t].ctx = ctx;
    args[t].lo = n * (size_t)t / (size_t)nt;
    args[t].hi = n * (size_t)(t + 1) / (size_t)nt;
    started[t] = t > 0 && pthread_create(&th[t], NULL, pf_tramp, &args[t]) == 0;
  }
  fn(ctx, args[0].lo, args[0].hi); /* the calling thread takes the first range */
  for (int t = 1; t < nt; t++) {
    if (started[t])
      pthread_join(th[t], NULL);
    else
      fn(ctx, args[t].lo, args[t].hi); /* could not spawn: run inline */
  }
}

/* ---------------- parameters ---------------- */
size_t of_log2(size_t v) { /* (63 - v.next_power_of_two().leading_zeros()) */
  size_t p = 1;
  while (p < v) p <<= 1;
  size_t l = 0;
  while (((size_t)1 << l) < p) l++;
  return l;
}

size_t of_n_degree_tests(size_t lambda, size_t len, size_t flog2) {
  size_t den = flog2 - of_log2(len);
  return (lambda + den - 1) / den;
}

static double ligero_rho(size_t num, size_t den) { return (double)num / (double)den; }

size_t of_ligero_n_col_opens(size_t rho_num, size_t rho_den) {
  double den = log2((1.0 + ligero_rho(rho_num, rho_den)) / 2.0);
  return (size_t)ceil(-128.0 / den);
}

static size_t next_pow2(size_t v) {
  size_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

/* LigeroEncodingRho::_get_dims (lcpc-ligero-pc/src/lib.rs:70-112); returns 0 on None */
int of_ligero_get_dims(int fid, size_t rho_num, size_t rho_den, size_t len, size_t *nr,
                       size_t *np, size_t *nc) {
  const of_field *f = of_get_field(fid);
  const size_t flog2 = f->num_bits - 1;
  const double rho = ligero_rho(rho_num, rho_den);
  size_t n_col_opens = of_ligero_n_col_opens(rho_num, rho_den);
  double lncf = (double)(n_col_opens * len);
  size_t ndt_len = (size_t)ceil(sqrt(lncf) / rho);
  double ndt = (double)of_n_degree_tests(128, ndt_len, flog2);
  size_t nc1 = next_pow2((size_t)ceil(sqrt(lncf / ndt) / rho));
  if (f->s < 63 && nc1 > ((size_t)1 << f->s)) return 0;
  size_t np1 = nc1 * rho_num / rho_den;
  size_t nr1 = (len + np1 - 1) / np1;
  size_t nd1 = of_n_degree_tests(128, nc1, flog2);
  size_t nc2 = nc1 / 2, np2 = np1 / 2;
  size_t nr2 = (len + np2 - 1) / np2;
  size_t nd2 = of_n_degree_tests(128, nc2, flog2);
  size_t sz1 = n_col_opens * nr1 + (1 + nd1) * np1;
  size_t sz2 = n_col_opens * nr2 + (1 + nd2) * np2;
  if (sz1 < sz2) {
    *nr = nr1; *np = np1; *nc = nc1;
  } else {
    *nr = nr2; *np = np2; *nc = nc2;
  }
  return 1;
}

/* ---------------- encodings ---------------- */
of_enc *of_enc_ligero(int fid, size_t n_per_row, size_t n_cols, size_t n_col_opens,
                      size_t n_degree_tests) {
  of_enc *e = (of_enc *)calloc(1, sizeof(*e));
  e->fid = fid;
  e->kind = 0;
  e->n_per_row = n_per_row;
  e->n_cols = n_cols;
  e->n_col_opens = n_col_opens;
  e->n_degree_tests = n_degree_tests;
  return e;
}
void of_enc_free(of_enc *e) {
  if (!e) return;
  if (e->kind == 1) of_sdig_free(e->bd);
  free(e);
}
int of_enc_encode(const of_enc *e, uint64_t *row) {
  if (e->kind == 0) return of_fft_io(e->fid, row, e->n_cols);
  return of_sdig_encode(e->bd, e->fid, row);
}
static int enc_dims_ok(const of_enc *e, size_t n_per_row, size_t n_cols) {
  if (e->kind == 0) {
    int pow = n_cols && !(n_cols & (n_cols - 1));
    return n_per_row < n_cols && pow && n_per_row == e->n_per_row && n_cols == e->n_cols;
  }
  return n_per_row == e->n_per_row && n_cols == e->n_cols;
}

/* ---------------- commit ---------------- */
typedef struct {
  const of_enc *e;
  uint64_t *comm;
  const uint64_t *coeffs;
  int err;
  size_t src_stride; /* elements between rows of coeffs (n_per_row for a commitment) */
} enc_ctx;
static void enc_rows(void *p, size_t lo, size_t hi) {
  enc_ctx *c = (enc_ctx *)p;
  const int nl = of_field_limbs(c->e->fid);
  const size_t np = c->e->n_per_row, nc = c->e->n_cols;
  for (size_t r = lo; r < hi; r++) {
    uint64_t *row = c->comm + r * nc * nl;
    memcpy(row, c->coeffs + r * c->src_stride * nl, sizeof(uint64_t) * nl * np);
    memset(row + np * nl, 0, sizeof(uint64_t) * nl * (nc - np));
    if (of_enc_encode(c->e, row)) c->err = 1;
  }
}
int of_enc_encode_rows(const of_enc *e, const uint64_t *src, size_t src_stride, size_t n_rows, uint64_t *dst) {
  enc_ctx ec = {e, dst, src, 0, src_stride};
  of_parallel_for(n_rows, 1, enc_rows, &ec);
  return ec.err ? 8 : 0;
}

typedef struct {
  const of_field *f;
  const uint64_t *comm;
  size_t n_rows, n_cols;
  uint8_t *out;
} hash_ctx;
static void hash_cols(void *p, size_t lo, size_t hi) {
  hash_ctx *c = (hash_ctx *)p;
  const int nl = c->f->nl, eb = 8 * nl;
  size_t len = 32 + c->n_rows * (size_t)eb;
  uint8_t *buf = (uint8_t *)malloc(len);
  memset(buf, 0, 32);
  for (size_t col = lo; col < hi; col++) {
    for (size_t r = 0; r < c->n_rows; r++)
      of_elem_to_repr(c->f, c->comm + (r * c->n_cols + col) * nl, buf + 32 + r * eb);
    of_blake3(buf, len, c->out + 32 * col);
  }
  free(buf);
}

void of_hash_columns(int fid, const uint64_t *comm, size_t n_rows, size_t n_cols, uint8_t *out) {
  hash_ctx hc = {of_get_field(fid), comm, n_rows, n_cols, out};
  of_parallel_for(n_cols, 32, hash_cols, &hc);
}

/* merkle_tree: ins.len() == outs.len() + 1, layer by layer */
void of_merkle_tree(const uint8_t *ins, size_t n_ins, uint8_t *outs) {
  size_t n_outs = n_ins - 1;
  while (n_outs > 0) {
    size_t layer = (n_outs + 1) / 2;
    for (size_t i = 0; i < layer; i++) of_blake3(ins + 64 * i, 64, outs + 32 * i);
    ins = outs;
    outs += 32 * layer;
    n_outs -= layer;
  }
}

of_commit *of_commit_new(const of_enc *e, const uint64_t *coeffs_in, size_t len) {
  const int nl = of_field_limbs(e->fid);
  size_t n_per_row = e->n_per_row, n_cols = e->n_cols;
  size_t n_rows = (len + n_per_row - 1) / n_per_row; /* get_dims */
  if (n_rows == 0 || !(n_rows * n_per_row >= len) || !((n_rows - 1) * n_per_row < len) ||
      !enc_dims_ok(e, n_per_row, n_cols))
    return NULL; /* commit asserts (panics) on these, lib.rs:659-661 */
  of_commit *c = (of_commit *)calloc(1, sizeof(*c));
  c->fid = e->fid;
  c->nl = nl;
  c->n_rows = n_rows;
  c->n_cols = n_cols;
  c->n_per_row = n_per_row;
  c->coeffs = (uint64_t *)calloc(n_rows * n_per_row * nl, sizeof(uint64_t));
  c->comm = (uint64_t *)calloc(n_rows * n_cols * nl, sizeof(uint64_t));
  memcpy(c->coeffs, coeffs_in, sizeof(uint64_t) * nl * len);
  enc_ctx ec = {e, c->comm, c->coeffs, 0, n_per_row};
  of_parallel_for(n_rows, 1, enc_rows, &ec);
  if (ec.err) {
    of_commit_free(c);
    return NULL;
  }
  size_t np2 = next_pow2(n_cols);
  c->n_hashes = 2 * np2 - 1;
  c->hashes = (uint8_t *)calloc(c->n_hashes, 32); /* Output::default() = zeros */
  of_hash_columns(e->fid, c->comm, n_rows, n_cols, c->hashes);
  of_merkle_tree(c->hashes, np2, c->hashes + 32 * np2);
  return c;
}

void of_commit_free(of_commit *c) {
  if (!c) return;
  free(c->comm);
  free(c->coeffs);
  free(c->hashes);
  free(c);
}

/* ---------------- prove ---------------- */
typedef struct {
  const of_field *f;
  const uint64_t *coeffs, *tensor;
  uint64_t *poly;
  size_t n_rows, n_per_row;
} col_ctx;
static void collapse_range(void *p, size_t lo, size_t hi) {
  col_ctx *c = (col_ctx *)p;
  const int nl = c->f->nl;
  uint64_t t[OF_MAXL];
  for (size_t col = lo; col < hi; col++) memset(c->poly + col * nl, 0, sizeof(uint64_t) * nl);
  for (size_t r = 0; r < c->n_rows; r++)
    for (size_t col = lo; col < hi; col++) {
      of_mont_mul(c->f, c->coeffs + (r * c->n_per_row + col) * nl, c->tensor + r * nl, t);
      of_mont_add(c->f, c->poly + col * nl, t, c->poly + col * nl);
    }
}
void of_collapse_columns(int fid, const uint64_t *coeffs, const uint64_t *tensor, uint64_t *poly,
                         size_t n_rows, size_t n_per_row) {
  col_ctx cc = {of_get_field(fid), coeffs, tensor, poly, n_rows, n_per_row};
  of_parallel_for(n_per_row, 32, collapse_range, &cc);
}

int of_open_column(const of_commit *c, size_t column, uint64_t *col_out, uint8_t *path_out) {
  if (column >= c->n_cols) return 4; /* ProverError::ColumnNumber */
  for (size_t r = 0; r < c->n_rows; r++)
    memcpy(col_out + r * c->nl, c->comm + (r * c->n_cols + column) * c->nl, 8 * c->nl);
  const uint8_t *hashes = c->hashes;
  size_t hlen = c->n_hashes;
  size_t path_len = of_log2(c->n_cols);
  for (size_t i = 0; i < path_len; i++) {
    size_t other = (column & ~(size_t)1) | (~column & 1);
    memcpy(path_out + 32 * i, hashes + 32 * other, 32);
    size_t skip = (hlen + 1) / 2;
    hashes += 32 * skip;
    hlen -= skip;
    column >>= 1;
  }
  return 0;
}

of_proof *of_proof_alloc(int fid, size_t n_cols, size_t n_per_row, size_t n_rows, size_t ndt,
                         size_t n_col_opens, size_t path_len) {
  const int nl = of_field_limbs(fid);
  of_proof *p = (of_proof *)calloc(1, sizeof(*p));
  p->fid = fid;
  p->nl = nl;
  p->n_cols = n_cols;
  p->n_per_row = n_per_row;
  p->n_rows = n_rows;
  p->n_degree_tests = ndt;
  p->n_col_opens = n_col_opens;
  p->path_len = path_len;
  p->p_eval = (uint64_t *)calloc(n_per_row * nl, 8);
  p->p_random = (uint64_t *)calloc(ndt * n_per_row * nl + 1, 8);
  p->cols = (uint64_t *)calloc(n_col_opens * n_rows * nl + 1, 8);
  p->paths = (uint8_t *)calloc(n_col_opens * path_len * 32 + 1, 1);
  p->col_idx = (uint64_t *)calloc(n_col_opens + 1, 8);
  return p;
}
void of_proof_free(of_proof *p) {
  if (!p) return;
  free(p->p_eval);
  free(p->p_random);
  free(p->cols);
  free(p->paths);
  free(p->col_idx);
  free(p);
}

static void transcript_update_vec(const of_field *f, of_transcript *tr, const uint8_t *label,
                                  const uint64_t *v, size_t n) {
  uint8_t repr[8 * OF_MAXL];
  for (size_t i = 0; i < n; i++) {
    of_elem_to_repr(f, v + i * f->nl, repr);
    of_transcript_append_message(tr, label, LABEL_LEN, repr, 8 * f->nl);
  }
}

static void challenge_tensor(int fid, of_transcript *tr, size_t n, uint64_t *out) {
  uint8_t key[32];
  of_transcript_challenge_bytes(tr, LABEL_DT, LABEL_LEN, key, 32);
  of_chacha *rng = of_chacha_from_seed(key, 20);
  of_field_random(fid, rng, out, n);
  of_chacha_free(rng);
}

static void challenge_columns(of_transcript *tr, size_t n_cols, size_t n_opens, uint64_t *idx) {
  uint8_t key[32];
  of_transcript_challenge_bytes(tr, LABEL_CO, LABEL_LEN, key, 32);
  of_chacha *rng = of_chacha_from_seed(key, 20);
  for (size_t i = 0; i < n_opens; i++) idx[i] = of_uniform_usize(rng, 0, n_cols);
  of_chacha_free(rng);
}

of_proof *of_prove(const of_commit *c, const of_enc *e, const uint64_t *outer, of_transcript *tr,
                   int *err) {
  const of_field *f = of_get_field(c->fid);
  const int nl = f->nl;
  *err = 0;
  /* check_comm */
  if (c->n_hashes != 2 * next_pow2(c->n_cols) - 1 || !enc_dims_ok(e, c->n_per_row, c->n_cols)) {
    *err = 3; /* ProverError::Commit */
    return NULL;
  }
  size_t ndt = e->n_degree_tests, nco = e->n_col_opens, path_len = of_log2(c->n_cols);
  of_proof *p = of_proof_alloc(c->fid, c->n_cols, c->n_per_row, c->n_rows, ndt, nco, path_len);
  uint64_t *tensor = (uint64_t *)malloc(sizeof(uint64_t) * nl * c->n_rows);
  for (size_t i = 0; i < ndt; i++) {
    challenge_tensor(c->fid, tr, c->n_rows, tensor);
    uint64_t *pr = p->p_random + i * c->n_per_row * nl;
    of_collapse_columns(c->fid, c->coeffs, tensor, pr, c->n_rows, c->n_per_row);
    transcript_update_vec(f, tr, LABEL_PR, pr, c->n_per_row);
  }
  of_collapse_columns(c->fid, c->coeffs, outer, p->p_eval, c->n_rows, c->n_per_row);
  transcript_update_vec(f, tr, LABEL_PE, p->p_eval, c->n_per_row);
  challenge_columns(tr, c->n_cols, nco, p->col_idx);
  for (size_t k = 0; k < nco; k++)
    of_open_column(c, (size_t)p->col_idx[k], p->cols + k * c->n_rows * nl,
                   p->paths + k * path_len * 32);
  free(tensor);
  return p;
}

/* ---------------- verify ---------------- */
int of_verify_column_path(int fid, const uint64_t *col, size_t n_rows, const uint8_t *path,
                          size_t path_len, size_t col_num, const uint8_t root[32]) {
  const of_field *f = of_get_field(fid);
  const int eb = 8 * f->nl;
  size_t len = 32 + n_rows * eb;
  uint8_t *buf = (uint8_t *)calloc(len, 1);
  for (size_t r = 0; r < n_rows; r++) of_elem_to_repr(f, col + r * f->nl, buf + 32 + r * eb);
  uint8_t hash[32], blk[64];
  of_blake3(buf, len, hash);
  free(buf);
  for (size_t i = 0; i < path_len; i++) {
    if (col_num % 2 == 0) {
      memcpy(blk, hash, 32);
      memcpy(blk + 32, path + 32 * i, 32);
    } else {
      memcpy(blk, path + 32 * i, 32);
      memcpy(blk + 32, hash, 32);
    }
    of_blake3(blk, 64, hash);
    col_num >>= 1;
  }
  return memcmp(hash, root, 32) == 0;
}

int of_verify_column_value(int fid, const uint64_t *col, const uint64_t *tensor, size_t n_rows,
                           const uint64_t *poly_eval) {
  const of_field *f = of_get_field(fid);
  uint64_t acc[OF_MAXL] = {0, 0, 0, 0}, t[OF_MAXL];
  for (size_t r = 0; r < n_rows; r++) {
    of_mont_mul(f, tensor + r * f->nl, col + r * f->nl, t);
    of_mont_add(f, acc, t, acc);
  }
  return memcmp(acc, poly_eval, 8 * f->nl) == 0;
}

/* VerifierError codes: 1 NumColOpens, 2 ColumnPath, 3 ColumnEval, 4 ColumnDegree,
   5 OuterTensor, 6 InnerTensor, 7 EncodingDims, 8 Encode */
int of_verify(const uint8_t root[32], const uint64_t *outer, size_t outer_len, const uint64_t *inner,
              size_t inner_len, const of_proof *p, const of_enc *e, of_transcript *tr,
              uint64_t *out) {
  const of_field *f = of_get_field(e->fid);
  const int nl = f->nl;
  size_t nco = e->n_col_opens;
  if (nco != p->n_col_opens || nco == 0) return 1;
  size_t n_rows = p->n_rows, n_cols = p->n_cols, n_per_row = p->n_per_row;
  if (inner_len != n_per_row) return 6;
  if (outer_len != n_rows) return 5;
  if (!enc_dims_ok(e, n_per_row, n_cols)) return 7;
  size_t ndt = e->n_degree_tests;
  if (p->n_degree_tests != ndt) return 7; /* (the Rust code would index out of bounds) */
  uint64_t *tensors = (uint64_t *)malloc(sizeof(uint64_t) * nl * n_rows * (ndt + 1));
  uint64_t *encs = (uint64_t *)calloc(nl * n_cols * (ndt + 1), 8);
  int rc = 0;
  for (size_t i = 0; i < ndt; i++) {
    challenge_tensor(e->fid, tr, n_rows, tensors + i * n_rows * nl);
    uint64_t *tmp = encs + i * n_cols * nl;
    memcpy(tmp, p->p_random + i * n_per_row * nl, sizeof(uint64_t) * nl * n_per_row);
    if (of_enc_encode(e, tmp)) {
      rc = 8;
      goto done;
    }
    transcript_update_vec(f, tr, LABEL_PR, p->p_random + i * n_per_row * nl, n_per_row);
  }
  transcript_update_vec(f, tr, LABEL_PE, p->p_eval, n_per_row);
  uint64_t *idx = (uint64_t *)malloc(sizeof(uint64_t) * nco);
  challenge_columns(tr, n_cols, nco, idx);
  {
    uint64_t *tmp = encs + ndt * n_cols * nl;
    memcpy(tmp, p->p_eval, sizeof(uint64_t) * nl * n_per_row);
    if (of_enc_encode(e, tmp)) {
      free(idx);
      rc = 8;
      goto done;
    }
  }
  /* rayon try_for_each: the first failing column (in index order) decides, as the
     sequential order the Rust code reports when a single column is bad. */
  for (size_t k = 0; k < nco && !rc; k++) {
    const uint64_t *col = p->cols + k * n_rows * nl;
    size_t cn = (size_t)idx[k];
    int rnd = 1;
    for (size_t i = 0; i < ndt; i++)
      rnd &= of_verify_column_value(e->fid, col, tensors + i * n_rows * nl, n_rows,
                                    encs + (i * n_cols + cn) * nl);
    int ev = of_verify_column_value(e->fid, col, outer, n_rows, encs + (ndt * n_cols + cn) * nl);
    int pa = of_verify_column_path(e->fid, col, n_rows, p->paths + k * p->path_len * 32,
                                   p->path_len, cn, root);
    if (!rnd)
      rc = 4;
    else if (!ev)
      rc = 3;
    else if (!pa)
      rc = 2;
  }
  free(idx);
  if (!rc) {
    uint64_t acc[OF_MAXL] = {0, 0, 0, 0}, t[OF_MAXL];
    for (size_t c = 0; c < n_per_row; c++) {
      of_mont_mul(f, inner + c * nl, p->p_eval + c * nl, t);
      of_mont_add(f, acc, t, acc);
    }
    memcpy(out, acc, 8 * nl);
  }
done:
  free(tensors);
  free(encs);
  return rc;
}
