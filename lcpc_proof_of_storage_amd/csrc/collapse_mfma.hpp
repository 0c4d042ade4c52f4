// collapse_mfma.hpp -- the row combinations of prove (collapse_columns, lcpc-2d/src/lib.rs:
// 1126-1154) for Ft127 on the gfx950 int8 matrix cores.
//
//     out[t][c] = sum_r tensor_t[r] * coeffs[r][c]            (Montgomery words in and out)
//
// The contraction over rows is a (T x n_rows) x (n_rows x n_per_row) matrix product over F_p
// whose left operand (the challenge tensors) is tiny and shared by every column, which is what a
// limb contraction on MFMA needs.  Write each coefficient word C (raw Montgomery value < p) in
// 16 balanced base-256 digits, C = sum_a d_a 2^(8a), d_a in [-128, 128), and precompute for
// every tensor entry the 16 residues H[r][a] = T_r 2^(8a) mod p, again in balanced digits
// H[r][a] = sum_u h[r][a][u] 2^(8u).  Then
//
//     Y[u][c] = sum_(r, a) h[r][a][u] d_a(coeffs[r][c])          (an exact int32 GEMM)
//     sum_u Y[u][c] 2^(8u) = sum_r T_r C_rc   (mod p)
//
// and one Montgomery reduction per output turns that into sum_r T_r C_rc R^-1 = the field sum
// of Montgomery products, bit-identical to the VALU path.  The GEMM is
// v_mfma_i32_16x16x64_i8: M = the 16 digit positions u, K = 4 rows x 16 coefficient digits,
// N = 16 columns.  |h d| <= 2^14, so a K = 64 step adds < 2^20; a split of at most 512 rows
// keeps every accumulator below 2^27.
//
// Work per coefficient: 16 x 16 int8 products per tensor on the matrix cores (a 16-B element
// is one lane's B fragment, loaded straight from the row-major matrix) plus 8 VALU ops for the
// balanced-digit conversion; the kernel is bound by the HBM read of the coefficient matrix,
// not by 64-bit multiply-adds (the VALU path: 44 v_mad_u64_u32 per product pair).
#pragma once
#include "field.hpp"

namespace lcpc {
namespace cmfma {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int COLS_PER_WAVE = 64;  // 4 MFMA column tiles of 16
constexpr int TILES = COLS_PER_WAVE / 16;
constexpr size_t MAX_SPLIT_ROWS = 512;  // bounds |Y| below the offset added before the reduction

// 16 balanced base-256 digits of a 128-bit value x < 2^127 - 2^120 (true for every x < p of
// Ft127): V = x + 0x80..80 has no carry out, and digit a = byte_a(V) - 128 = byte_a(V) ^ 0x80
// read as int8.
__device__ __forceinline__ v4i balanced_digits(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3) {
  uint32_t c = 0;
  const uint32_t v0 = __builtin_addc(x0, 0x80808080u, c, &c);
  const uint32_t v1 = __builtin_addc(x1, 0x80808080u, c, &c);
  const uint32_t v2 = __builtin_addc(x2, 0x80808080u, c, &c);
  const uint32_t v3 = __builtin_addc(x3, 0x80808080u, c, &c);
  v4i d;
  d.x = (int)(v0 ^ 0x80808080u);
  d.y = (int)(v1 ^ 0x80808080u);
  d.z = (int)(v2 ^ 0x80808080u);
  d.w = (int)(v3 ^ 0x80808080u);
  return d;
}

// hdig[(t n_rows + r) 16 + u] = the 16 bytes h[r][a = 0..15][u] of tensor t.  One thread per
// (t, r, a): H = T_r 2^(8a) mod p = fe_mul(T_r, 2^(8a) R mod p).
template <class F>
__global__ __launch_bounds__(256) void k_tensor_digits(const uint32_t *__restrict__ tensors, size_t n_rows,
                                                       int n_tensors, uint8_t *__restrict__ hdig) {
  static_assert(F::N == 4, "Ft127 layout");
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (size_t)n_tensors * n_rows * 16) return;
  const int a = (int)(g & 15);
  const size_t tr = g >> 4;  // t * n_rows + r
  const Fe<F> x = fe_load<F>(tensors, tr);
  Fe<F> pw = fe_zero<F>();  // 2^(8a) as an integer (< p), then to Montgomery form
  pw.v[a >> 2] = 1u << (8 * (a & 3));
  const Fe<F> h = fe_mul<F>(x, fe_to_mont<F>(pw));
  const v4i d = balanced_digits(h.v[0], h.v[1], h.v[2], h.v[3]);
  const uint32_t w[4] = {(uint32_t)d.x, (uint32_t)d.y, (uint32_t)d.z, (uint32_t)d.w};
#pragma unroll
  for (int u = 0; u < 16; u++) hdig[(tr * 16 + u) * 16 + a] = (uint8_t)(w[u >> 2] >> (8 * (u & 3)));
}

// out = (x + top 2^128) R^-1 mod p for a 128-bit x and 0 <= top < 2^23 (Ft127, R = 2^128):
// REDC(x) lies in [0, p], so REDC(x) + top needs at most one subtraction of p.
template <class F>
__device__ __forceinline__ Fe<F> redc_plus(const uint32_t x[4], uint32_t top) {
  Fe<F> a;
#pragma unroll
  for (int i = 0; i < 4; i++) a.v[i] = x[i];
  const Fe<F> r = fe_from_mont_generic<F>(a);
  uint32_t s[4], c = 0;
  s[0] = __builtin_addc(r.v[0], top, c, &c);
#pragma unroll
  for (int i = 1; i < 4; i++) s[i] = __builtin_addc(r.v[i], 0u, c, &c);
  // s < p + 2^23 < 2p < 2^128: subtract p if s >= p
  uint32_t u[4], br = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) u[i] = __builtin_subc(s[i], F::P[i], br, &br);
  Fe<F> o;
#pragma unroll
  for (int i = 0; i < 4; i++) o.v[i] = br ? s[i] : u[i];
  return o;
}

// The field element of a digit-position accumulator column: sum_u Y[u] 2^(8u) R^-1 mod p, for
// |Y[u]| < 2^27 (at most 512 x 16 products of balanced digits per accumulator).
template <class F>
__device__ __forceinline__ Fe<F> recombine_redc(const int (&Y)[16]) {
  // Y = sum_u Y_u 2^(8u) as S_w = sum_j Y_(4w+j) 2^(8j) (int64), then signed carries
  int64_t S[4];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    int64_t sum = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) sum += (int64_t)Y[4 * w + j] * ((int64_t)1 << (8 * j));
    S[w] = sum;
  }
  uint32_t y[4];
  int64_t carry = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const int64_t v = S[w] + carry;
    y[w] = (uint32_t)v;
    carry = v >> 32;  // arithmetic
  }
  // Y = y + carry 2^128 with |Y| < 512 2^18 2^120.01 < 2^147.01; add OFF = p 2^22 (a multiple
  // of p, > 2^148.8 > |Y|) so that Y + OFF is nonnegative
  constexpr uint32_t O0 = F::P[0] << 22;
  constexpr uint32_t O1 = (F::P[1] << 22) | (F::P[0] >> 10);
  constexpr uint32_t O2 = (F::P[2] << 22) | (F::P[1] >> 10);
  constexpr uint32_t O3 = (F::P[3] << 22) | (F::P[2] >> 10);
  constexpr uint32_t O4 = F::P[3] >> 10;
  uint32_t cc = 0;
  y[0] = __builtin_addc(y[0], O0, cc, &cc);
  y[1] = __builtin_addc(y[1], O1, cc, &cc);
  y[2] = __builtin_addc(y[2], O2, cc, &cc);
  y[3] = __builtin_addc(y[3], O3, cc, &cc);
  const uint32_t top = (uint32_t)(carry + (int64_t)O4 + (int64_t)cc);
  return redc_plus<F>(y, top);
}

// One wave = 64 columns x the split's rows; 4 waves per block on adjacent column ranges.
// partial[(split T + t) n_per_row + c] = sum over the split's rows (a field element).
template <class F, int T>
__global__ __launch_bounds__(256) void k_collapse_mfma(const uint32_t *__restrict__ coeffs, size_t n_rows,
                                                       size_t n_per_row, const uint8_t *__restrict__ hdig,
                                                       uint32_t *__restrict__ partial, size_t rows_per_split) {
  static_assert(F::N == 4, "Ft127 layout");
  __shared__ int red[4][TILES][16][17];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane >> 4, n = lane & 15;
  const size_t col0 = ((size_t)blockIdx.x * 4 + wave) * COLS_PER_WAVE;
  const size_t split = blockIdx.y;
  const size_t r0 = split * rows_per_split;
  const size_t r1 = r0 + rows_per_split < n_rows ? r0 + rows_per_split : n_rows;
  const uint4 *cm = reinterpret_cast<const uint4 *>(coeffs);
  const uint4 *hd = reinterpret_cast<const uint4 *>(hdig);
  bool colok[TILES];
#pragma unroll
  for (int k = 0; k < TILES; k++) colok[k] = col0 + 16 * k + n < n_per_row;

  v4i acc[T][TILES];
#pragma unroll
  for (int t = 0; t < T; t++)
#pragma unroll
    for (int k = 0; k < TILES; k++) acc[t][k] = v4i{0, 0, 0, 0};

  auto load = [&](size_t rg, uint4 *x, uint4 *a) {
    const size_t r = rg + grp;
    const bool ok = r < r1;
#pragma unroll
    for (int k = 0; k < TILES; k++)
      x[k] = ok && colok[k] ? cm[r * n_per_row + col0 + 16 * k + n] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int t = 0; t < T; t++)
      a[t] = ok ? hd[((size_t)t * n_rows + r) * 16 + n] : make_uint4(0, 0, 0, 0);
  };
  uint4 xc[TILES], ac[T], xn[TILES], an[T];
  if (r0 < r1) load(r0, xc, ac);
  for (size_t rg = r0; rg < r1; rg += 4) {
    const bool more = rg + 4 < r1;
    if (more) load(rg + 4, xn, an);
#pragma unroll
    for (int k = 0; k < TILES; k++) {
      const v4i d = balanced_digits(xc[k].x, xc[k].y, xc[k].z, xc[k].w);
#pragma unroll
      for (int t = 0; t < T; t++) {
        const v4i av = v4i{(int)ac[t].x, (int)ac[t].y, (int)ac[t].z, (int)ac[t].w};
        acc[t][k] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, d, acc[t][k], 0, 0, 0);
      }
    }
    if (more) {
#pragma unroll
      for (int k = 0; k < TILES; k++) xc[k] = xn[k];
#pragma unroll
      for (int t = 0; t < T; t++) ac[t] = an[t];
    }
  }
  // C/D layout (16x16): lane holds rows (digit positions) u = 4 grp + j of column n.  Each wave
  // turns its own accumulators into field elements through its own LDS slice, one tensor at a
  // time: one output (t, column col0 + lane) per lane.
  const int k = lane >> 4;
  const size_t c = col0 + lane;
  int(*rw)[16][17] = red[wave];
#pragma unroll
  for (int t = 0; t < T; t++) {
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < TILES; q++) {
      rw[q][4 * grp + 0][n] = acc[t][q].x;
      rw[q][4 * grp + 1][n] = acc[t][q].y;
      rw[q][4 * grp + 2][n] = acc[t][q].z;
      rw[q][4 * grp + 3][n] = acc[t][q].w;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int Y[16];
#pragma unroll
    for (int u = 0; u < 16; u++) Y[u] = rw[k][u][n];
    if (c < n_per_row) fe_store<F>(partial, (split * T + t) * n_per_row + c, recombine_redc<F>(Y));
  }
}

}  // namespace cmfma
}  // namespace lcpc
