// femul2.hip -- A/B of the product-scanning Montgomery multiply's column transition.
// Library (field.hpp fe_mul_fips): acc = (hi | r2 << 32) + (lo != 0) through cndmask + 64-bit add.
// Variant: m = 0 - lo sets the borrow (lo != 0); hi + borrow and r2 + carry are two v_addc, each
// written straight into the next column's 64-bit addend halves.
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 femul2.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

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

// m = -lo (borrow = lo != 0); nlo = hi + borrow; nhi = r2 + carry
__device__ __forceinline__ void col_step(uint32_t lo, uint32_t hi, uint32_t r2, uint32_t &m, uint32_t &nlo,
                                         uint32_t &nhi) {
  uint64_t c0, c1, c2;
  asm(
      "v_sub_co_u32_e64 %0, %3, 0, %6\n\t"
      "v_addc_co_u32_e64 %1, %4, %7, 0, %3\n\t"
      "v_addc_co_u32_e64 %2, %5, %8, 0, %4"
      : "=&v"(m), "=&v"(nlo), "=&v"(nhi), "=&s"(c0), "=&s"(c1), "=&s"(c2)
      : "v"(lo), "v"(hi), "v"(r2));
}

template <class F>
__device__ __forceinline__ Fe<F> fe_mul_v2(const Fe<F> &a, const Fe<F> &b) {
  constexpr int N = F::N;
  uint32_t m[N], out[N];
  uint64_t acc = 0;
  uint32_t r2 = 0;
#pragma unroll
  for (int k = 0; k < 2 * N; k++) {
    uint64_t cprev = 0, ccur;
    bool have = false;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j < 0 || j >= N) continue;
      acc = mad_co_vv(a.v[i], b.v[j], acc, ccur);
      if (have) r2 = add_carry(r2, cprev);
      cprev = ccur;
      have = true;
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i >= k || j < 1 || j >= N) continue;
      acc = mad_co_vs(m[i], F::P[j], acc, ccur);
      if (have) r2 = add_carry(r2, cprev);
      cprev = ccur;
      have = true;
    }
    if (have) r2 = add_carry(r2, cprev);
    if (k < N) {
      uint32_t nlo, nhi;
      col_step((uint32_t)acc, (uint32_t)(acc >> 32), r2, m[k], nlo, nhi);
      acc = ((uint64_t)nhi << 32) | nlo;
    } else {
      out[k - N] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)r2 << 32);
    }
    r2 = 0;
  }
  Fe<F> u, r;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; i++) u.v[i] = __builtin_subc(out[i], F::P[i], br, &br);
  const bool take_u = ((uint32_t)acc != 0u) | (br ^ 1u);
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = take_u ? u.v[i] : out[i];
  return r;
}

#define ITERS 4096
template <class F, int V>
__global__ void k_femul(uint32_t *out, uint32_t seed) {
  Fe<F> a, b, c, d;
  for (int i = 0; i < F::N; i++) {
    a.v[i] = F::ONE[i] ^ (threadIdx.x * 3 + seed);
    b.v[i] = F::R2[i];
    c.v[i] = F::ROOT[i];
    d.v[i] = F::ONE[i];
  }
  a.v[F::N - 1] &= 0x0fffffff;
  c.v[F::N - 1] &= 0x0fffffff;
  for (int i = 0; i < ITERS / 8; i++) {
    if constexpr (V == 0) {
      a = fe_mul<F>(a, b); c = fe_mul<F>(c, b); d = fe_mul<F>(d, b); b = fe_mul<F>(b, a);
    } else {
      a = fe_mul_v2<F>(a, b); c = fe_mul_v2<F>(c, b); d = fe_mul_v2<F>(d, b); b = fe_mul_v2<F>(b, a);
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < F::N; i++) x ^= a.v[i] ^ b.v[i] ^ c.v[i] ^ d.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// equality on random operands < p
template <class F>
__global__ void k_check(const uint32_t *in, uint32_t *bad, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  Fe<F> a, b;
  for (int i = 0; i < F::N; i++) {
    a.v[i] = in[(2 * t) * F::N + i];
    b.v[i] = in[(2 * t + 1) * F::N + i];
  }
  const Fe<F> x = fe_mul<F>(a, b), y = fe_mul_v2<F>(a, b);
  for (int i = 0; i < F::N; i++)
    if (x.v[i] != y.v[i]) atomicAdd(bad, 1u);
}

template <class F>
void run(const char *name) {
  uint32_t *buf, *bad;
  const int blocks = 256 * 64, threads = 256;
  CK(hipMalloc(&buf, (size_t)blocks * threads * 4));
  CK(hipMalloc(&bad, 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int n = 1 << 20;
  std::vector<uint32_t> h((size_t)2 * n * F::N);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < h.size(); i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h[i] = (uint32_t)x;
    if (i % F::N == F::N - 1) h[i] &= 0x3fffffffu;  // < p (top limb below p's)
  }
  uint32_t *din;
  CK(hipMalloc(&din, h.size() * 4));
  CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL((k_check<F>), dim3(n / 256), dim3(256), 0, 0, din, bad, n);
  uint32_t nb = 0;
  CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
  for (int v = 0; v < 2; v++) {
    for (int rep = 0; rep < 3; rep++) {
      CK(hipEventRecord(e0));
      if (v == 0)
        hipLaunchKernelGGL((k_femul<F, 0>), dim3(blocks), dim3(threads), 0, 0, buf, 7u);
      else
        hipLaunchKernelGGL((k_femul<F, 1>), dim3(blocks), dim3(threads), 0, 0, buf, 7u);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep == 2)
        printf("%s %s  %8.3f ms  %8.2f G mul/s  %s\n", name, v ? "v2 (asm column step)" : "library           ", ms,
               (double)blocks * threads * (ITERS / 2) / (ms * 1e-3) / 1e9, nb ? "MISMATCH" : "equal on 2^20 random pairs");
    }
  }
  CK(hipFree(buf));
  CK(hipFree(bad));
  CK(hipFree(din));
}

int main() {
  run<Ft127>("Ft127");
  run<Ft63>("Ft63 ");
  run<Ft255>("Ft255");
  return 0;
}
