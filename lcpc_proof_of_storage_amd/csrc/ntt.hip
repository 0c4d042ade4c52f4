// ntt.hip -- Ligero encode plan / dispatch (kernels: ntt_impl.hpp, one TU per field).
#include "kernels.hpp"
#include "field.hpp"

namespace lcpc {

#define DECL(n)                                                                                   \
  hipError_t ntt_rows_##n(const NttPlan &, const uint32_t *, size_t, size_t, uint32_t *, size_t, \
                          size_t, hipStream_t, uint32_t *, size_t, bool);                         \
  hipError_t ntt_tw_table_##n(uint32_t *, int, bool, hipStream_t);
DECL(ft63)
DECL(ft127)
DECL(ft191)
DECL(ft255)
DECL(ft253)
#undef DECL

namespace {
// out[(t << l2) + c] = tw[c * bitrev_l1(t)]: an element copy of `words` u32 words
__global__ __launch_bounds__(256) void k_tw2(const uint32_t *__restrict__ tw, uint32_t *__restrict__ out, int l1,
                                             int l2, int words) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ((size_t)1 << (l1 + l2))) return;
  const size_t t = i >> l2, c = i & (((size_t)1 << l2) - 1);
  const size_t bt = l1 ? (size_t)(__builtin_bitreverse32((uint32_t)t) >> (32 - l1)) : 0;
  const size_t e = c * bt;
  for (int w = 0; w < words; w++) out[i * words + w] = tw[e * words + w];
}
}  // namespace

hipError_t ntt_tw2_table(int fid, const uint32_t *tw, int log_n, int l1, uint32_t *out, hipStream_t s) {
  const size_t n = (size_t)1 << log_n;
  hipLaunchKernelGGL(k_tw2, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tw, out, l1, log_n - l1,
                     field_words(fid));
  return hipGetLastError();
}

int field_words(int fid) {
  return dispatch_field(fid, []<class F>() { return F::N; });
}

bool field_gpu_supported(int fid) { return fid >= 0 && fid <= 4; }

int ntt_max_log_n(int fid) { return fid >= 2 ? 22 : 24; }

hipError_t ntt_plan_init(NttPlan &p, int fid, int log_n, bool inverse, hipStream_t s) {
  if (!field_gpu_supported(fid) || log_n < 0 || log_n > ntt_max_log_n(fid))
    return hipErrorInvalidValue;
  p.fid = fid;
  p.log_n = log_n;
  p.inverse = inverse;
  // include/lcpc_fft_convention.h: the forward transform's root is omega or omega^-1, the
  // inverse's the other one
  const bool inv_root = inverse != (LCPC_FFT_OMEGA_INVERSE != 0);
  // Ft63 at 2^15 (the PoS default n_cols): the l1 = 8 split measured 5 % faster than l1 = 7
  // (tools/microbench/nttbench.hip mode 5, 9363 rows); every other shape splits evenly.
  p.l1 = fid == 0 && log_n == 15 ? 8 : log_n / 2;
  p.l2 = log_n - p.l1;
  const size_t n = (size_t)1 << log_n;
  hipError_t e = hipMalloc(&p.d_tw, n * field_bytes(fid));
  if (e != hipSuccess) return e;
  switch (fid) {
    case 0: e = ntt_tw_table_ft63(p.d_tw, log_n, inv_root, s); break;
    case 1: e = ntt_tw_table_ft127(p.d_tw, log_n, inv_root, s); break;
    case 2: e = ntt_tw_table_ft191(p.d_tw, log_n, inv_root, s); break;
    case 3: e = ntt_tw_table_ft255(p.d_tw, log_n, inv_root, s); break;
    default: e = ntt_tw_table_ft253(p.d_tw, log_n, inv_root, s); break;
  }
  if (e != hipSuccess) return e;
  if (log_n > 12) {  // the pass-A kernels' [t][c] inter-pass twiddles
    if ((e = hipMalloc(&p.d_tw2, n * field_bytes(fid))) != hipSuccess) return e;
    if ((e = ntt_tw2_table(fid, p.d_tw, log_n, p.l1, p.d_tw2, s)) != hipSuccess) return e;
  }
  if (inverse) return hipSuccess;
  // canonical words of w^e = Montgomery words of w^e R^-1 (canon_out encodes)
  e = hipMalloc(&p.d_tw_canon, n * field_bytes(fid));
  if (e != hipSuccess) return e;
  if ((e = convert(fid, p.d_tw, p.d_tw_canon, n, false, s)) != hipSuccess) return e;
  if (log_n > 12) {
    if ((e = hipMalloc(&p.d_tw2_canon, n * field_bytes(fid))) != hipSuccess) return e;
    if ((e = ntt_tw2_table(fid, p.d_tw_canon, log_n, p.l1, p.d_tw2_canon, s)) != hipSuccess) return e;
  }
  return hipSuccess;
}

void ntt_plan_free(NttPlan &p) {
  if (p.d_tw) (void)hipFree(p.d_tw);
  if (p.d_tw_canon) (void)hipFree(p.d_tw_canon);
  if (p.d_tw2) (void)hipFree(p.d_tw2);
  if (p.d_tw2_canon) (void)hipFree(p.d_tw2_canon);
  p.d_tw = nullptr;
  p.d_tw_canon = nullptr;
  p.d_tw2 = nullptr;
  p.d_tw2_canon = nullptr;
}

hipError_t ntt_rows(const NttPlan &p, const uint32_t *src, size_t src_stride, size_t n_valid,
                    uint32_t *dst, size_t dst_stride, size_t n_rows, hipStream_t s, uint32_t *copy,
                    size_t copy_stride, bool canon) {
  hipError_t e;
  switch (p.fid) {
    case 0: e = ntt_rows_ft63(p, src, src_stride, n_valid, dst, dst_stride, n_rows, s, copy, copy_stride, canon); break;
    case 1: e = ntt_rows_ft127(p, src, src_stride, n_valid, dst, dst_stride, n_rows, s, copy, copy_stride, canon); break;
    case 2: e = ntt_rows_ft191(p, src, src_stride, n_valid, dst, dst_stride, n_rows, s, copy, copy_stride, canon); break;
    case 3: e = ntt_rows_ft255(p, src, src_stride, n_valid, dst, dst_stride, n_rows, s, copy, copy_stride, canon); break;
    case 4: e = ntt_rows_ft253(p, src, src_stride, n_valid, dst, dst_stride, n_rows, s, copy, copy_stride, canon); break;
    default: return hipErrorInvalidValue;
  }
#if !LCPC_FFT_OUTPUT_BITREV
  if (e == hipSuccess && !p.inverse) e = bitrev_rows_inplace(p.fid, dst, dst_stride, p.log_n, n_rows, s);
#endif
  return e;
}

}  // namespace lcpc
