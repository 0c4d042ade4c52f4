// femul_free.hip -- the carry-free mads of fe_mul_fips (field.hpp, fips_free_mask) checked and
// timed on gfx950.
//   check: for every field the library builds, 2^24 products of biased-random operands (each
//     low limb 0xffffffff with probability 1/2, the top limb near its bound) and the extremes
//     (p - 1, 2p - 1, ...): fe_mul_fips (full and lazy: a < 2p, b < p) against the generic CIOS
//     product, which has no such mads.  Any carry the mask wrongly dropped shows as a mismatch.
//   time: a dependent chain of lazy products per thread (Ft127), as femul2's loop.
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 femul_free.hip -o femul_free
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../../lcpc_proof_of_storage_amd/csrc/field.hpp"

using namespace lcpc;

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return (uint32_t)x;
}

// x mod p for x < 2p
template <class F>
__device__ Fe<F> red(Fe<F> x) {
  return fe_is_canonical<F>(x) ? x : fe_reduce_2p<F>(x);
}

// a biased-random value < lim * p (lim 1 or 2); extremes for the first few indices
template <class F>
__device__ Fe<F> draw(uint64_t id, uint32_t salt, int lim) {
  constexpr int N = F::N;
  Fe<F> x;
  const uint32_t kind = (uint32_t)(id & 15);
  if (kind < 3) {  // p - 1, 2p - 1 (lim 2), p - 2^32 ...: all borrowed from p's own limbs
    uint32_t br = 0;
    for (int i = 0; i < N; i++) {
      const uint32_t pi = lim == 2 ? TwoP<F>::limb(i) : F::P[i];
      x.v[i] = __builtin_subc(pi, i == 0 ? 1u + kind : 0u, br, &br);
    }
    return x;
  }
  for (int i = 0; i < N; i++) {
    const uint32_t r = mix(id * 0x9E3779B97F4A7C15ull + salt * 1315423911u + i);
    x.v[i] = (mix(r + 77) & 1u) ? 0xffffffffu : r;
  }
  const uint32_t top = lim == 2 ? TwoP<F>::limb(N - 1) : F::P[N - 1];
  x.v[N - 1] = top - (mix(id + salt) & 7u);
  // reduce into range: x < lim * p (subtract p while not)
  for (int k = 0; k < 3; k++) {
    Fe<F> lp;
    for (int i = 0; i < N; i++) lp.v[i] = lim == 2 ? TwoP<F>::limb(i) : F::P[i];
    // x >= lim p ?
    bool ge = true;
    for (int i = N - 1; i >= 0; i--)
      if (x.v[i] != lp.v[i]) {
        ge = x.v[i] > lp.v[i];
        break;
      }
    if (!ge) break;
    uint32_t br = 0;
    for (int i = 0; i < N; i++) x.v[i] = __builtin_subc(x.v[i], F::P[i], br, &br);
  }
  return x;
}

template <class F>
__global__ void k_check(size_t n, unsigned long long *bad) {
  const size_t id = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= n) return;
  const Fe<F> a2 = draw<F>(id, 1, 2), a1 = draw<F>(id, 3, 1), b = draw<F>(id >> 4, 2, 1);
  const Fe<F> want_l = fe_mul_cios<F>(a2, b), want_f = fe_mul_cios<F>(a1, b);
  const Fe<F> got_l = red<F>(fe_mul_fips<F, true>(a2, b)), got_f = fe_mul_fips<F, false>(a1, b);
  if (!fe_eq<F>(want_l, got_l) || !fe_eq<F>(want_f, got_f)) atomicAdd(bad, 1ull);
}

template <class F>
__global__ void k_chain(uint32_t *out, int iters) {
  const size_t id = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  Fe<F> x = draw<F>(id + 5, 9, 2), w = draw<F>(id + 7, 8, 1);
  for (int i = 0; i < iters; i++) x = fe_mul_lazy<F>(x, w);
  uint32_t s = 0;
  for (int i = 0; i < F::N; i++) s ^= x.v[i];
  out[id] = s;
}

template <class F>
static unsigned long long check(const char *name) {
  const size_t n = (size_t)1 << 24;
  unsigned long long *d, h = 0;
  CK(hipMalloc(&d, 8));
  CK(hipMemset(d, 0, 8));
  hipLaunchKernelGGL(k_check<F>, dim3((unsigned)(n / 256)), dim3(256), 0, 0, n, d);
  CK(hipGetLastError());
  CK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost));
  CK(hipFree(d));
  printf("%-10s %zu lazy + %zu full products against CIOS: %llu mismatches\n", name, n, n, h);
  return h;
}

int main() {
  unsigned long long bad = 0;
  bad += check<Ft63>("Ft63");
  bad += check<Ft127>("Ft127");
  bad += check<Ft191>("Ft191");
  bad += check<Ft255>("Ft255");
  bad += check<Ft253_192>("Ft253_192");
  // throughput: 1M threads x 256 dependent lazy products
  const int blocks = 4096, iters = 256;
  uint32_t *o;
  CK(hipMalloc(&o, (size_t)blocks * 256 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; rep++) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_chain<Ft127>, dim3(blocks), dim3(256), 0, 0, o, iters);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (rep == 2)
      printf("Ft127 lazy product chain: %.3f ms, %.1f G mul/s\n", ms, (double)blocks * 256 * iters / (ms * 1e6));
  }
  CK(hipFree(o));
  return bad ? 1 : 0;
}
