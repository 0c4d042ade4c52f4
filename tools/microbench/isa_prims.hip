// isa_prims.hip -- the Ligero encode's field primitives as stand-alone kernels, compiled to
// gfx950 assembly only (tools/isa_attribution.py counts their VALU instructions; never run).
#include "field.hpp"
using namespace lcpc;
using F = Ft127;
extern "C" __global__ void k_mul_lazy(uint32_t *io, const uint32_t *tw) {
  const int i = threadIdx.x;
  Fe<F> a = fe_load<F>(io, i), w = fe_load<F>(tw, i);
  fe_store<F>(io, i, fe_mul_lazy<F>(a, w));
}
extern "C" __global__ void k_add2p(uint32_t *io, const uint32_t *tw) {
  const int i = threadIdx.x;
  Fe<F> a = fe_load<F>(io, i), w = fe_load<F>(tw, i);
  fe_store<F>(io, i, fe_add_2p<F>(a, w));
}
extern "C" __global__ void k_sub2p(uint32_t *io, const uint32_t *tw) {
  const int i = threadIdx.x;
  Fe<F> a = fe_load<F>(io, i), w = fe_load<F>(tw, i);
  fe_store<F>(io, i, fe_sub_2p<F>(a, w));
}
extern "C" __global__ void k_bfly(uint32_t *io, const uint32_t *tw) {
  const int i = threadIdx.x;
  Fe<F> a = fe_load<F>(io, i), c = fe_load<F>(io, i + 64), w = fe_load<F>(tw, i);
  fe_store<F>(io, i, fe_add_2p<F>(a, c));
  fe_store<F>(io, i + 64, fe_mul_lazy<F>(fe_sub_2p<F>(a, c), w));
}
extern "C" __global__ void k_load_store(uint32_t *io, const uint32_t *tw) {
  const int i = threadIdx.x;
  Fe<F> a = fe_load<F>(io, i), c = fe_load<F>(io, i + 64), w = fe_load<F>(tw, i);
  fe_store<F>(io, i, a);
  fe_store<F>(io, i + 64, c);
  fe_store<F>(io, i + 128, w);
}
