// collapse.hip -- random linear combinations of matrix rows on gfx950.
//
// Replaces collapse_columns (lcpc-2d/src/lib.rs:1126-1154), called by prove for every degree-
// test tensor and for the evaluation tensor (:1064-1071, :1085-1092):
//     out[t][c] = sum_r tensor_t[r] * coeffs[r][c]
// and the verifier's per-column dot products verify_column_value (:1015-1030, used at
// :956-966) and final inner product (:977-981).  Field sums are exact, so the reduction order
// (split over row blocks, then folded) cannot change a bit.
//
// Layout: one thread per column c (lanes = adjacent columns -> 1-KiB coalesced row segments),
// all tensors accumulated from ONE read of each coefficient; the tensor entries of a row are
// wave-uniform (scalar loads).  Rows are split over blockIdx.y so the grid fills 256 CUs; the
// per-split partials are folded by a second kernel.
//
// Ft127 with up to 3 tensors (every prove launch of the Ligero / Brakedown commitments over
// Ft127) runs the contraction on the int8 matrix cores instead (collapse_mfma.hpp): there the
// kernel streams the coefficient matrix at the HBM rate instead of being bound by 64-bit
// multiply-adds.
#include "collapse_mfma.hpp"
#include "field.hpp"
#include "kernels.hpp"
#include "prof.hpp"

#include <algorithm>
#include <cstdlib>

namespace lcpc {

namespace {

constexpr int MAXT = 4;

template <class F, int T>
__global__ __launch_bounds__(256) void k_collapse_partial(const uint32_t *__restrict__ coeffs,
                                                          size_t n_rows, size_t n_per_row,
                                                          const uint32_t *__restrict__ tensors,
                                                          uint32_t *__restrict__ partial,
                                                          size_t rows_per_split) {
  const size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t split = blockIdx.y;
  if (c >= n_per_row) return;
  const size_t r0 = split * rows_per_split;
  const size_t r1 = r0 + rows_per_split < n_rows ? r0 + rows_per_split : n_rows;
  Fe<F> acc[T];
#pragma unroll
  for (int t = 0; t < T; t++) acc[t] = fe_zero<F>();
  // K rows per step, one Montgomery reduction per K products (fe_dot, lazy reduction)
  constexpr int K = fe_dot_kmax<F>() < 4 ? fe_dot_kmax<F>() : 4;
  size_t r = r0;
  for (; r + K <= r1; r += K) {
    Fe<F> x[K];
#pragma unroll
    for (int q = 0; q < K; q++) x[q] = fe_load<F>(coeffs, (r + q) * n_per_row + c);
#pragma unroll
    for (int t = 0; t < T; t++) {
      Fe<F> w[K];
#pragma unroll
      for (int q = 0; q < K; q++) w[q] = fe_load<F>(tensors, t * n_rows + r + q);
      acc[t] = fe_add<F>(acc[t], fe_dot<F, K>(x, w));
    }
  }
  for (; r < r1; r++) {
    const Fe<F> x = fe_load<F>(coeffs, r * n_per_row + c);
#pragma unroll
    for (int t = 0; t < T; t++) acc[t] = fe_add<F>(acc[t], fe_mul<F>(x, fe_load<F>(tensors, t * n_rows + r)));
  }
#pragma unroll
  for (int t = 0; t < T; t++) fe_store<F>(partial, (split * T + t) * n_per_row + c, acc[t]);
}

template <class F, int T>
__global__ __launch_bounds__(256) void k_collapse_fold(const uint32_t *__restrict__ partial,
                                                       size_t n_splits, size_t n_per_row,
                                                       uint32_t *__restrict__ out) {
  const size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n_per_row) return;
#pragma unroll
  for (int t = 0; t < T; t++) {
    Fe<F> acc = fe_zero<F>();
    for (size_t s = 0; s < n_splits; s++)
      acc = fe_add<F>(acc, fe_load<F>(partial, (s * T + t) * n_per_row + c));
    fe_store<F>(out, t * n_per_row + c, acc);
  }
}

size_t n_splits_for(size_t n_rows, size_t n_per_row) {
  // aim for >= 8192 waves of work in flight, at least 16 rows per split
  const size_t col_waves = (n_per_row + 63) / 64;
  size_t splits = (8192 + col_waves - 1) / col_waves;
  size_t max_splits = (n_rows + 15) / 16;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  return splits;
}

// dots for the verifier: one thread per (opened column k, tensor t)
template <class F>
__global__ void k_column_checks(const uint32_t *__restrict__ cols, size_t n_open, size_t n_rows,
                                const uint32_t *__restrict__ tensors, int n_tensors,
                                const uint32_t *__restrict__ encs, size_t enc_len,
                                const uint64_t *__restrict__ idx, uint32_t *__restrict__ flags) {
  const size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_open * (size_t)n_tensors) return;
  const size_t k = g / n_tensors;
  const int t = (int)(g % n_tensors);
  Fe<F> acc = fe_zero<F>();
  for (size_t r = 0; r < n_rows; r++)
    acc = fe_add<F>(acc, fe_mul<F>(fe_load<F>(tensors, t * n_rows + r), fe_load<F>(cols, k * n_rows + r)));
  const Fe<F> want = fe_load<F>(encs, t * enc_len + idx[k]);
  flags[g] = fe_eq<F>(acc, want) ? 1u : 0u;
}

template <class F>
__global__ __launch_bounds__(1024) void k_dot(const uint32_t *__restrict__ a,
                                              const uint32_t *__restrict__ b, size_t n,
                                              uint32_t *__restrict__ out) {
  __shared__ Fe<F> red[1024];
  Fe<F> acc = fe_zero<F>();
  for (size_t i = threadIdx.x; i < n; i += 1024)
    acc = fe_add<F>(acc, fe_mul<F>(fe_load<F>(a, i), fe_load<F>(b, i)));
  red[threadIdx.x] = acc;
  for (int w = 512; w > 0; w >>= 1) {
    __syncthreads();
    if ((int)threadIdx.x < w) red[threadIdx.x] = fe_add<F>(red[threadIdx.x], red[threadIdx.x + w]);
  }
  if (threadIdx.x == 0) fe_store<F>(out, 0, red[0]);
}

template <class F>
__global__ void k_convert(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, size_t n,
                          int to_mont, uint32_t *__restrict__ bad) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fe<F> x = fe_load<F>(in, i);
  // canonical input that is not < p: flagged (PrimeField::from_repr would refuse it)
  if (bad && to_mont && !fe_is_canonical<F>(x)) atomicOr(bad, 1u);
  fe_store<F>(out, i, to_mont ? fe_to_mont<F>(x) : fe_from_mont<F>(x));
}

template <class F>
__global__ void k_mul(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b,
                      uint32_t *__restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe_store<F>(out, i, fe_mul<F>(fe_load<F>(a, i), fe_load<F>(b, i)));
}

template <class F, int T>
hipError_t collapse_t(const uint32_t *coeffs, size_t n_rows, size_t n_per_row,
                      const uint32_t *tensors, uint32_t *out, void *scratch, hipStream_t s) {
  const size_t splits = n_splits_for(n_rows, n_per_row);
  const size_t rps = (n_rows + splits - 1) / splits;
  dim3 grid((unsigned)((n_per_row + 255) / 256), (unsigned)splits);
  prof::Scope ps("collapse_partial", s);
  hipLaunchKernelGGL((k_collapse_partial<F, T>), grid, dim3(256), 0, s, coeffs, n_rows, n_per_row,
                     tensors, (uint32_t *)scratch, rps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  prof::Scope ps2("collapse_fold", s);
  hipLaunchKernelGGL((k_collapse_fold<F, T>), dim3((unsigned)((n_per_row + 255) / 256)), dim3(256),
                     0, s, (const uint32_t *)scratch, splits, n_per_row, out);
  return hipGetLastError();
}

// MFMA path (Ft127, T <= 3): row splits of at most MAX_SPLIT_ROWS rows, about 512 blocks
size_t mfma_splits_for(size_t n_rows, size_t n_per_row) {
  const size_t blocks_x = (n_per_row + 4 * cmfma::COLS_PER_WAVE - 1) / (4 * cmfma::COLS_PER_WAVE);
  size_t splits = (512 + blocks_x - 1) / blocks_x;
  const size_t max_splits = (n_rows + 15) / 16;
  if (splits > max_splits) splits = max_splits;
  const size_t min_splits = (n_rows + cmfma::MAX_SPLIT_ROWS - 1) / cmfma::MAX_SPLIT_ROWS;
  if (splits < min_splits) splits = min_splits;
  return splits < 1 ? 1 : splits;
}

bool use_mfma(int fid, int n_tensors) {
  return !no_mfma() && fid == Ft127::ID && n_tensors >= 1 && n_tensors <= 3;
}

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

template <int T>
hipError_t collapse_mfma_t(const uint32_t *coeffs, size_t n_rows, size_t n_per_row, const uint32_t *tensors,
                           uint32_t *out, void *scratch, hipStream_t s) {
  using F = Ft127;
  const size_t splits = mfma_splits_for(n_rows, n_per_row);
  const size_t rps = (n_rows + splits - 1) / splits;
  uint32_t *partial = (uint32_t *)scratch;
  uint8_t *hdig = (uint8_t *)scratch + round_up(splits * T * n_per_row * 16, 256);
  const size_t nd = (size_t)T * n_rows * 16;
  prof::Scope ps("collapse_partial", s);
  hipLaunchKernelGGL((cmfma::k_tensor_digits<F>), dim3((unsigned)((nd + 255) / 256)), dim3(256), 0, s, tensors,
                     n_rows, T, hdig);
  // (one-wave blocks, whose 4.3 KiB of LDS fit beside four encode blocks on a CU, measured the
  // same at K = 20: profiles/r05_k20_collapse_waves_ab.json)
  dim3 grid((unsigned)((n_per_row + 4 * cmfma::COLS_PER_WAVE - 1) / (4 * cmfma::COLS_PER_WAVE)), (unsigned)splits);
  hipLaunchKernelGGL((cmfma::k_collapse_mfma<F, T>), grid, dim3(256), 0, s, coeffs, n_rows, n_per_row,
                     (const uint8_t *)hdig, partial, rps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  prof::Scope ps2("collapse_fold", s);
  hipLaunchKernelGGL((k_collapse_fold<F, T>), dim3((unsigned)((n_per_row + 255) / 256)), dim3(256), 0, s,
                     (const uint32_t *)partial, splits, n_per_row, out);
  return hipGetLastError();
}

// dst[i] = src[i] in 16- or 8-byte words (either side may be page-locked host memory: the
// prover's results go to host memory by these stores, not by a copy-engine transfer)
// A few workgroups with a grid-stride loop: a transfer to / from host memory is bound by the
// link, and a full-size grid would only hold wave slots that the concurrent encodes could use.
template <class W>
__global__ __launch_bounds__(256) void k_copy_words(W *__restrict__ dst, const W *__restrict__ src, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}
constexpr size_t COPY_MAX_BLOCKS = 64;  // (measured: a full grid cost K = 256 0.5 G/s)

}  // namespace

// LCPC_NO_MFMA=1: the VALU kernels instead of the int8 matrix-core ones (row combinations, SDIG
// levels) for A/B measurements; the results are identical
bool no_mfma() {
  static const bool v = [] {
    const char *e = getenv("LCPC_NO_MFMA");
    return e && *e && *e != '0';
  }();
  return v;
}

hipError_t copy_words(void *dst, const void *src, size_t bytes, hipStream_t s, bool over_link) {
  if (!bytes) return hipSuccess;
  // device-to-device copies are HBM-bound: a full grid; copies over the host link: a few groups
  const size_t cap = over_link ? COPY_MAX_BLOCKS : (size_t)1 << 20;
  if (((uintptr_t)dst | (uintptr_t)src | bytes) & 7) return hipErrorInvalidValue;
  if (!(((uintptr_t)dst | (uintptr_t)src | bytes) & 15)) {
    const size_t n = bytes / 16;
    hipLaunchKernelGGL((k_copy_words<uint4>), dim3((unsigned)std::min((n + 255) / 256, cap)), dim3(256),
                       0, s, (uint4 *)dst, (const uint4 *)src, n);
  } else {
    const size_t n = bytes / 8;
    hipLaunchKernelGGL((k_copy_words<uint2>), dim3((unsigned)std::min((n + 255) / 256, cap)), dim3(256),
                       0, s, (uint2 *)dst, (const uint2 *)src, n);
  }
  return hipGetLastError();
}

hipError_t collapse_fold_rows(int fid, const uint32_t *vecs, size_t n_vecs, size_t len, uint32_t *out,
                              hipStream_t s) {
  return dispatch_field(fid, [&]<class F>() {
    hipLaunchKernelGGL((k_collapse_fold<F, 1>), dim3((unsigned)((len + 255) / 256)), dim3(256), 0, s,
                       vecs, n_vecs, len, out);
    return hipGetLastError();
  });
}

size_t collapse_scratch_bytes(int fid, size_t n_rows, size_t n_per_row, int n_tensors) {
  const size_t valu = n_splits_for(n_rows, n_per_row) * (size_t)n_tensors * n_per_row * field_bytes(fid);
  if (!use_mfma(fid, n_tensors)) return valu;
  const size_t mfma = round_up(mfma_splits_for(n_rows, n_per_row) * n_tensors * n_per_row * 16, 256) +
                      (size_t)n_tensors * n_rows * 256;
  return mfma > valu ? mfma : valu;
}

hipError_t collapse_rows(int fid, const uint32_t *coeffs, size_t n_rows, size_t n_per_row,
                         const uint32_t *tensors, int n_tensors, uint32_t *out, void *scratch,
                         hipStream_t s) {
  if (n_tensors < 1 || n_tensors > MAXT) return hipErrorInvalidValue;
  if (n_per_row == 0) return hipSuccess;
  if (n_rows == 0) return hipMemsetAsync(out, 0, (size_t)n_tensors * n_per_row * field_bytes(fid), s);
  if (use_mfma(fid, n_tensors)) {
    switch (n_tensors) {
      case 1: return collapse_mfma_t<1>(coeffs, n_rows, n_per_row, tensors, out, scratch, s);
      case 2: return collapse_mfma_t<2>(coeffs, n_rows, n_per_row, tensors, out, scratch, s);
      default: return collapse_mfma_t<3>(coeffs, n_rows, n_per_row, tensors, out, scratch, s);
    }
  }
  return dispatch_field(fid, [&]<class F>() {
    switch (n_tensors) {
      case 1: return collapse_t<F, 1>(coeffs, n_rows, n_per_row, tensors, out, scratch, s);
      case 2: return collapse_t<F, 2>(coeffs, n_rows, n_per_row, tensors, out, scratch, s);
      case 3: return collapse_t<F, 3>(coeffs, n_rows, n_per_row, tensors, out, scratch, s);
      default: return collapse_t<F, 4>(coeffs, n_rows, n_per_row, tensors, out, scratch, s);
    }
  });
}

hipError_t column_checks(int fid, const uint32_t *cols, size_t n_open, size_t n_rows,
                         const uint32_t *tensors, int n_tensors, const uint32_t *encs,
                         size_t enc_len, const uint64_t *idx, uint32_t *flags, hipStream_t s) {
  const size_t n = n_open * (size_t)n_tensors;
  if (!n) return hipSuccess;
  return dispatch_field(fid, [&]<class F>() {
    hipLaunchKernelGGL((k_column_checks<F>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, cols,
                       n_open, n_rows, tensors, n_tensors, encs, enc_len, idx, flags);
    return hipGetLastError();
  });
}

hipError_t dot(int fid, const uint32_t *a, const uint32_t *b, size_t n, uint32_t *out,
               void *scratch, hipStream_t s) {
  (void)scratch;
  return dispatch_field(fid, [&]<class F>() {
    hipLaunchKernelGGL((k_dot<F>), dim3(1), dim3(1024), 0, s, a, b, n, out);
    return hipGetLastError();
  });
}

hipError_t convert(int fid, const uint32_t *in, uint32_t *out, size_t n, bool to_mont,
                   hipStream_t s, uint32_t *bad) {
  if (!n) return hipSuccess;
  return dispatch_field(fid, [&]<class F>() {
    hipLaunchKernelGGL((k_convert<F>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out,
                       n, to_mont ? 1 : 0, bad);
    return hipGetLastError();
  });
}

hipError_t mul_elementwise(int fid, const uint32_t *a, const uint32_t *b, uint32_t *out, size_t n,
                           hipStream_t s) {
  if (!n) return hipSuccess;
  return dispatch_field(fid, [&]<class F>() {
    hipLaunchKernelGGL((k_mul<F>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a, b, out, n);
    return hipGetLastError();
  });
}

}  // namespace lcpc
