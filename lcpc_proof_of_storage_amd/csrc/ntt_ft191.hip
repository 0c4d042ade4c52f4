// ntt_ft191.hip -- instantiation of the Ligero encode kernels for Ft191 (see ntt_impl.hpp).
#include "ntt_impl.hpp"

namespace lcpc {
hipError_t ntt_rows_ft191(const NttPlan &p, const uint32_t *src, size_t ss, size_t nv, uint32_t *dst,
                      size_t ds, size_t n_rows, hipStream_t s, uint32_t *cp, size_t cs, bool canon) {
  return ntt_detail::ntt_rows_t<Ft191>(p, src, ss, nv, dst, ds, n_rows, s, cp, cs, canon);
}
hipError_t ntt_tw_table_ft191(uint32_t *tw, int log_n, bool inverse, hipStream_t s) {
  const size_t n = (size_t)1 << log_n;
  hipLaunchKernelGGL((ntt_detail::k_tw_table<Ft191>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     s, tw, log_n, inverse ? 1 : 0);
  return hipGetLastError();
}
}  // namespace lcpc
