// sdig.hip -- Brakedown / SDIG encode on gfx950 (see sdig.hpp).
//
// Layout: the codeword of R rows is element-major, cw[j][b] = element j of row b.  A sparse
// level y = M x becomes, for every output j and row b, y[j][b] = sum_k val[k] * x[idx[k]][b]
// over the nonzeros k of output row j (CSR).  Threads are (j, b) pairs with b fastest: the R
// threads of one output read the same nonzero (one broadcast load) and R adjacent elements of
// one input (a coalesced R * B-byte run), so no gather is scattered even though the matrix is.
// Field sums are exact, so the CSR order (vs sprs' CSC dot) cannot change a bit.
#include "field.hpp"
#include "kernels.hpp"
#include "prof.hpp"
#include "sdig.hpp"

namespace lcpc {

namespace {

template <class F>
__global__ __launch_bounds__(256) void k_spmm(const uint32_t *__restrict__ ptr,
                                              const uint32_t *__restrict__ idx,
                                              const uint32_t *__restrict__ val,
                                              const uint32_t *__restrict__ x,
                                              uint32_t *__restrict__ y, size_t m, uint32_t R) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= m * R) return;
  const size_t j = t / R;
  const uint32_t b = (uint32_t)(t - j * R);
  Fe<F> acc = fe_zero<F>();
  const uint32_t k1 = ptr[j + 1];
  uint32_t k = ptr[j];
  // K nonzeros per step, one Montgomery reduction per K products (fe_dot, lazy reduction)
  constexpr int K = fe_dot_kmax<F>() < 4 ? fe_dot_kmax<F>() : 4;
  for (; k + K <= k1; k += K) {
    Fe<F> v[K], xs[K];
#pragma unroll
    for (int q = 0; q < K; q++) {
      v[q] = fe_load<F>(val, k + q);
      xs[q] = fe_load<F>(x, (size_t)idx[k + q] * R + b);
    }
    acc = fe_add<F>(acc, fe_dot<F, K>(v, xs));
  }
  for (; k < k1; k++)
    acc = fe_add<F>(acc, fe_mul<F>(fe_load<F>(val, k), fe_load<F>(x, (size_t)idx[k] * R + b)));
  fe_store<F>(y, t, acc);
}

// encode::reed_solomon (encode.rs:97-110): out[k] = sum_j in[j] (k+1)^j by Horner, per row b
template <class F>
__global__ __launch_bounds__(256) void k_reed_solomon(const uint32_t *__restrict__ in, size_t m,
                                                      uint32_t *__restrict__ out, size_t n_out,
                                                      uint32_t R) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_out * R) return;
  const size_t k = t / R;
  const uint32_t b = (uint32_t)(t - k * R);
  const Fe<F> one = fe_one<F>();
  Fe<F> x = one;
  for (size_t i = 0; i < k; i++) x = fe_add<F>(x, one);
  Fe<F> r = fe_zero<F>();
  for (size_t jj = m; jj-- > 0;) r = fe_add<F>(fe_mul<F>(r, x), fe_load<F>(in, jj * R + b));
  fe_store<F>(out, t, r);
}

// 32 x 32 element tiles through LDS (padded row: no repeated bank pattern down a column).
// MODE: TR_PLAIN copies elements; TR_FROM_MONT writes canonical values (the PoS on-disk repr);
// TR_TO_MONT reads canonical values, flags any that is not < p in *bad (from_repr's check).
template <class F, int MODE>
__global__ __launch_bounds__(256) void k_transpose(const uint32_t *__restrict__ src, size_t rows,
                                                   size_t cols, size_t ss, size_t nv,
                                                   uint32_t *__restrict__ dst, size_t ds,
                                                   uint32_t *__restrict__ bad) {
  __shared__ Fe<F> tile[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const size_t c0 = (size_t)blockIdx.x * 32, r0 = (size_t)blockIdx.y * 32;
  bool ok = true;
  for (int i = ty; i < 32; i += 8) {
    const size_t r = r0 + i, c = c0 + tx;
    Fe<F> x = (r < rows && c < cols && c < nv) ? fe_load<F>(src, r * ss + c) : fe_zero<F>();
    if constexpr (MODE == TR_TO_MONT) {
      ok &= fe_is_canonical<F>(x);
      x = fe_to_mont<F>(x);
    }
    tile[i][tx] = x;
  }
  if constexpr (MODE == TR_TO_MONT) {
    if (!ok) atomicOr(bad, 1u);
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const size_t c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) {
      if constexpr (MODE == TR_FROM_MONT)
        fe_store<F>(dst, c * ds + r, fe_from_mont<F>(tile[tx][i]));
      else
        fe_store<F>(dst, c * ds + r, tile[tx][i]);
    }
  }
}

template <class F>
hipError_t spmm(const CsrDev &M, const uint32_t *x, uint32_t *y, size_t R, hipStream_t s) {
  const size_t n = M.rows * R;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL((k_spmm<F>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, M.ptr, M.idx,
                     M.val, x, y, M.rows, (uint32_t)R);
  return hipGetLastError();
}

template <class F>
hipError_t encode_cm(const SdigPlan &p, uint32_t *cw, size_t R, uint32_t *tmp, hipStream_t s) {
  constexpr int N = F::N;
  const int L = (int)p.pre.size();
  prof::Scope ps("sdig_encode", s);
  hipError_t e;
  // precodes all the way down (encode.rs:46-59): input [in_start, in_end), output right after
  size_t in_start = 0;
  for (int i = 0; i + 1 < L; i++) {
    const CsrDev &M = p.pre[i];
    const size_t in_end = in_start + M.cols;
    if ((e = spmm<F>(M, cw + in_start * R * N, cw + in_end * R * N, R, s)) != hipSuccess) return e;
    in_start = in_end;
  }
  // last precode into scratch, then Reed-Solomon into the codeword (:61-74)
  const CsrDev &ML = p.pre[L - 1];
  const size_t in_end = in_start + ML.cols;
  if ((e = spmm<F>(ML, cw + in_start * R * N, tmp, R, s)) != hipSuccess) return e;
  const size_t n_rs = p.post[L - 1].cols;
  if (n_rs * R) {
    hipLaunchKernelGGL((k_reed_solomon<F>), dim3((unsigned)((n_rs * R + 255) / 256)), dim3(256), 0,
                       s, tmp, ML.rows, cw + in_end * R * N, n_rs, (uint32_t)R);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  // postcodes in reverse (:76-90): input [in_start, out_start), output at out_start
  size_t in_pos = in_end + ML.rows, out_pos = in_end + n_rs;
  for (int i = L - 1; i >= 0; i--) {
    in_pos -= p.pre[i].rows;
    const CsrDev &Q = p.post[i];
    if (out_pos - in_pos != Q.cols) return hipErrorInvalidValue;
    if ((e = spmm<F>(Q, cw + in_pos * R * N, cw + out_pos * R * N, R, s)) != hipSuccess) return e;
    out_pos += Q.rows;
  }
  if (in_pos != p.pre[0].cols || out_pos != p.n_cols) return hipErrorInvalidValue;
  return hipSuccess;
}

}  // namespace

hipError_t sdig_plan_upload(SdigPlan &plan, int fid, const std::vector<CsrHost> &pre,
                            const std::vector<CsrHost> &post, hipStream_t s) {
  const int N = field_words(fid);
  auto bytes_of = [&](const CsrHost &h) {
    const size_t a = ((h.rows + 1) * 4 + 255) & ~(size_t)255;
    const size_t b = (h.idx.size() * 4 + 255) & ~(size_t)255;
    const size_t c = (h.idx.size() * N * 4 + 255) & ~(size_t)255;
    return a + b + c;
  };
  size_t total = 0;
  for (const auto &h : pre) total += bytes_of(h);
  for (const auto &h : post) total += bytes_of(h);
  hipError_t e = hipMalloc(&plan.d_buf, total ? total : 256);
  if (e != hipSuccess) return e;
  plan.fid = fid;
  plan.n_per_row = pre[0].cols;
  plan.n_cols = sdig_codeword_length(pre, post);
  plan.tmp_elems = pre.back().rows;
  uint8_t *cur = (uint8_t *)plan.d_buf;
  auto put = [&](const CsrHost &h, CsrDev &d) -> hipError_t {
    d.rows = h.rows;
    d.cols = h.cols;
    d.nnz = h.idx.size();
    const size_t a = ((h.rows + 1) * 4 + 255) & ~(size_t)255;
    const size_t b = (h.idx.size() * 4 + 255) & ~(size_t)255;
    const size_t c = (h.idx.size() * N * 4 + 255) & ~(size_t)255;
    d.ptr = (const uint32_t *)cur;
    d.idx = (const uint32_t *)(cur + a);
    d.val = (const uint32_t *)(cur + a + b);
    hipError_t r = hipMemcpyAsync(cur, h.ptr.data(), (h.rows + 1) * 4, hipMemcpyHostToDevice, s);
    if (r == hipSuccess && d.nnz)
      r = hipMemcpyAsync(cur + a, h.idx.data(), d.nnz * 4, hipMemcpyHostToDevice, s);
    if (r == hipSuccess && d.nnz)  // u64 limbs == little-endian u32 words
      r = hipMemcpyAsync(cur + a + b, h.val.data(), d.nnz * N * 4, hipMemcpyHostToDevice, s);
    cur += a + b + c;
    return r;
  };
  plan.pre.assign(pre.size(), CsrDev{});
  plan.post.assign(post.size(), CsrDev{});
  for (size_t i = 0; i < pre.size(); i++)
    if ((e = put(pre[i], plan.pre[i])) != hipSuccess) return e;
  for (size_t i = 0; i < post.size(); i++)
    if ((e = put(post[i], plan.post[i])) != hipSuccess) return e;
  return hipStreamSynchronize(s);  // host vectors may be freed after return
}

void sdig_plan_free(SdigPlan &plan) {
  if (plan.d_buf) (void)hipFree(plan.d_buf);
  plan.d_buf = nullptr;
  plan.pre.clear();
  plan.post.clear();
}

hipError_t sdig_encode_cm(const SdigPlan &plan, uint32_t *cw, size_t R, uint32_t *tmp,
                          hipStream_t s) {
  if (R == 0) return hipSuccess;
  return dispatch_field(plan.fid, [&]<class F>() { return encode_cm<F>(plan, cw, R, tmp, s); });
}

hipError_t transpose_elems(int fid, const uint32_t *src, size_t rows, size_t cols,
                           size_t src_stride, size_t n_valid, uint32_t *dst, size_t dst_stride,
                           hipStream_t s, int mode, uint32_t *bad) {
  if (!rows || !cols) return hipSuccess;
  if (mode == TR_TO_MONT && !bad) return hipErrorInvalidValue;
  return dispatch_field(fid, [&]<class F>() {
    prof::Scope ps("transpose", s);
    dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32));
    if (mode == TR_FROM_MONT)
      hipLaunchKernelGGL((k_transpose<F, TR_FROM_MONT>), grid, dim3(256), 0, s, src, rows, cols,
                         src_stride, n_valid, dst, dst_stride, bad);
    else if (mode == TR_TO_MONT)
      hipLaunchKernelGGL((k_transpose<F, TR_TO_MONT>), grid, dim3(256), 0, s, src, rows, cols,
                         src_stride, n_valid, dst, dst_stride, bad);
    else
      hipLaunchKernelGGL((k_transpose<F, TR_PLAIN>), grid, dim3(256), 0, s, src, rows, cols,
                         src_stride, n_valid, dst, dst_stride, bad);
    return hipGetLastError();
  });
}

}  // namespace lcpc
