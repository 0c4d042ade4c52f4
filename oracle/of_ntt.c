/*
 * of_ntt.c -- fffft radix-2 NTT semantics, restated (TEST ORACLE ONLY).
 *
 * Reference call sites: LigeroEncodingRho::encode -> FieldFFT::fft_io_pc
 * (lcpc-ligero-pc/src/lib.rs:162-164) with the precomputation from
 * precomp_fft(n_cols) (lcpc-ligero-pc/src/lib.rs:138-148); the inverse ifft_oi is used by
 * lcpc-2d/src/tests.rs:224 and proof-of-storage/src/lcpc_online.rs:568-574 (decode_row).
 *
 * fffft is a path dependency absent from /root/reference (Cargo.toml:17; the 2021 logs name
 * fffft v0.4.0).  Its published algorithm, restated:
 *   - len must be a power of two (FFTError::NotPowerOfTwo) with log2(len) <= S (TooBig);
 *   - omega = ROOT_OF_UNITY squared (S - log2 len) times (a primitive len-th root of unity);
 *   - roots[i] = omega^i for i < len/2;
 *   - fft_io: decimation in frequency, gap = len/2 .. 1, butterfly
 *       (a, b) -> (a + b, (a - b) * roots[nchunks * i]),  nchunks = len / (2 gap)
 *     natural-order input, bit-reversed output:  out[bitrev(j)] = sum_i in[i] omega^(i j);
 *   - ifft_oi: decimation in time with omega^-1 roots, bit-reversed input, natural output,
 *     then every element multiplied by len^-1.
 * The butterfly order cannot change any output bit (field arithmetic is exact); the two
 * choices that can -- which root and which output order -- are NOT pinned by the reference's
 * own invariant tests (lcpc-2d/src/tests.rs:193-234 commit test: ifft_oi inverts encode and
 * the encoded rows are R-S evaluations, ported by tests/test_oracle_invariants.py), which hold
 * under either.  They are the switches of include/lcpc_fft_convention.h, shared with the
 * product's NTT plans; the defaults are the restatement above.
 */
#include <stdlib.h>
#include <string.h>

#include "../include/lcpc_fft_convention.h"
#include "oracle.h"
#include "of_internal.h"

#if !LCPC_FFT_OUTPUT_BITREV
/* x[j] <-> x[bitrev_lg(j)] (the LCPC_FFT_OUTPUT_BITREV = 0 convention's reordering) */
static void bitrev_permute(uint64_t *x, int lg, int nl) {
  const size_t n = (size_t)1 << lg;
  for (size_t j = 0; j < n; j++) {
    size_t r = 0;
    for (int b = 0; b < lg; b++) r |= ((j >> b) & 1) << (lg - 1 - b);
    if (j < r)
      for (int k = 0; k < nl; k++) {
        const uint64_t t = x[j * nl + k];
        x[j * nl + k] = x[r * nl + k];
        x[r * nl + k] = t;
      }
  }
}
#endif

static int log2_exact(size_t len, int *lg) {
  if (len == 0 || (len & (len - 1))) return 0;
  int l = 0;
  while (((size_t)1 << l) < len) l++;
  *lg = l;
  return 1;
}

void of_ntt_omega(int fid, int log_len, uint64_t *out) {
  const of_field *f = of_get_field(fid);
  uint64_t w[OF_MAXL];
  memcpy(w, f->root, sizeof(w));
  for (uint32_t i = 0; i < f->s - (uint32_t)log_len; i++) of_mont_mul(f, w, w, w);
#if LCPC_FFT_OMEGA_INVERSE
  uint64_t wi[OF_MAXL];
  of_inv(fid, w, wi);
  memcpy(w, wi, sizeof(w));
#endif
  memcpy(out, w, sizeof(uint64_t) * f->nl);
}

static uint64_t *roots_table(const of_field *f, int lg, const uint64_t *w) {
  size_t half = ((size_t)1 << lg) / 2;
  if (half == 0) half = 1;
  uint64_t *r = (uint64_t *)malloc(sizeof(uint64_t) * f->nl * half);
  memcpy(r, f->r, sizeof(uint64_t) * f->nl);
  for (size_t i = 1; i < half; i++) of_mont_mul(f, r + (i - 1) * f->nl, w, r + i * f->nl);
  return r;
}

int of_fft_io(int fid, uint64_t *x, size_t len) {
  const of_field *f = of_get_field(fid);
  int lg;
  if (!log2_exact(len, &lg)) return 1;
  if ((uint32_t)lg > f->s) return 2;
  if (len == 1) return 0;
  const int nl = f->nl;
  uint64_t w[OF_MAXL];
  of_ntt_omega(fid, lg, w);
  uint64_t *roots = roots_table(f, lg, w);
  uint64_t a[OF_MAXL], b[OF_MAXL], d[OF_MAXL];
  for (size_t gap = len / 2; gap > 0; gap /= 2) {
    size_t nchunks = len / (2 * gap);
    for (size_t c = 0; c < nchunks; c++) {
      uint64_t *base = x + c * 2 * gap * nl;
      for (size_t i = 0; i < gap; i++) {
        memcpy(a, base + i * nl, sizeof(uint64_t) * nl);
        memcpy(b, base + (i + gap) * nl, sizeof(uint64_t) * nl);
        of_mont_add(f, a, b, base + i * nl);
        of_mont_sub(f, a, b, d);
        of_mont_mul(f, d, roots + nchunks * i * nl, base + (i + gap) * nl);
      }
    }
  }
  free(roots);
#if !LCPC_FFT_OUTPUT_BITREV
  bitrev_permute(x, lg, nl);
#endif
  return 0;
}

int of_ifft_oi(int fid, uint64_t *x, size_t len) {
  const of_field *f = of_get_field(fid);
  int lg;
  if (!log2_exact(len, &lg)) return 1;
  if ((uint32_t)lg > f->s) return 2;
  if (len == 1) return 0;
  const int nl = f->nl;
  uint64_t w[OF_MAXL], wi[OF_MAXL];
  of_ntt_omega(fid, lg, w);
  of_inv(fid, w, wi);
  uint64_t *roots = roots_table(f, lg, wi);
  uint64_t a[OF_MAXL], b[OF_MAXL];
#if !LCPC_FFT_OUTPUT_BITREV
  bitrev_permute(x, lg, nl);  /* natural-order evaluations in: the DIT below reads bit-reversed */
#endif
  for (size_t gap = 1; gap < len; gap *= 2) {
    size_t nchunks = len / (2 * gap);
    for (size_t c = 0; c < nchunks; c++) {
      uint64_t *base = x + c * 2 * gap * nl;
      for (size_t i = 0; i < gap; i++) {
        memcpy(a, base + i * nl, sizeof(uint64_t) * nl);
        of_mont_mul(f, base + (i + gap) * nl, roots + nchunks * i * nl, b);
        of_mont_add(f, a, b, base + i * nl);
        of_mont_sub(f, a, b, base + (i + gap) * nl);
      }
    }
  }
  /* multiply by len^-1 */
  uint64_t n_m[OF_MAXL] = {0, 0, 0, 0}, n_c[OF_MAXL] = {(uint64_t)len, 0, 0, 0}, ninv[OF_MAXL];
  of_mont_mul(f, n_c, f->r2, n_m);
  of_inv(fid, n_m, ninv);
  for (size_t i = 0; i < len; i++) of_mont_mul(f, x + i * nl, ninv, x + i * nl);
  free(roots);
  return 0;
}
