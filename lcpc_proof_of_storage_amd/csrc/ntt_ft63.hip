// ntt_ft63.hip -- instantiation of the Ligero encode kernels for Ft63 (see ntt_impl.hpp).
#include "ntt_impl.hpp"

namespace lcpc {
hipError_t ntt_rows_ft63(const NttPlan &p, const uint32_t *src, size_t ss, size_t nv, uint32_t *dst,
                      size_t ds, size_t n_rows, hipStream_t s, uint32_t *cp, size_t cs, bool canon) {
  return ntt_detail::ntt_rows_t<Ft63>(p, src, ss, nv, dst, ds, n_rows, s, cp, cs, canon);
}
bool ntt_row1_bytes(const NttPlan &p) { return p.row_kernel != 1; }  // (LCPC_ROW_KERNEL_FOURSTEP: pack first)
bool ntt_rows_pos_bytes_ok(const NttPlan &p, size_t n_per_row) {
  return p.fid == 0 && p.log_n == ntt_row1::LOG_N && n_per_row == ((size_t)1 << (ntt_row1::LOG_N - 1)) &&
         p.d_tw_canon;
}
hipError_t ntt_rows_pos_bytes(const NttPlan &p, const uint8_t *bytes, size_t n_bytes, uint32_t *dst,
                              size_t dst_stride, size_t n_rows, hipStream_t s, uint32_t *copy, size_t copy_stride) {
  if (!ntt_rows_pos_bytes_ok(p, (size_t)1 << (ntt_row1::LOG_N - 1)) || ((uintptr_t)bytes & 15) || !copy)
    return hipErrorInvalidValue;
  if (n_rows == 0) return hipSuccess;
  hipError_t e = ntt_row1::launch_bytes<Ft63>(p, bytes, n_bytes, dst, dst_stride, n_rows, s, copy, copy_stride);
#if !LCPC_FFT_OUTPUT_BITREV
  if (e == hipSuccess) e = bitrev_rows_inplace(p.fid, dst, dst_stride, p.log_n, n_rows, s);
#endif
  return e;
}
hipError_t ntt_tw_table_ft63(uint32_t *tw, int log_n, bool inverse, hipStream_t s) {
  const size_t n = (size_t)1 << log_n;
  hipLaunchKernelGGL((ntt_detail::k_tw_table<Ft63>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     s, tw, log_n, inverse ? 1 : 0);
  return hipGetLastError();
}
}  // namespace lcpc
