// mulbench.hip -- throughput of the integer / fp64 multiply primitives and of Fe<F> Montgomery
// multiplication on gfx950 (informs the NTT arithmetic design).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <chrono>
#include "../../lcpc_proof_of_storage_amd/csrc/field.hpp"
using namespace lcpc;

#define ITERS 4096
__global__ void k_mad64(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed, b = blockIdx.x * 77 + seed;
  uint64_t c0 = a, c1 = b, c2 = a ^ b, c3 = a + b, c4 = 3, c5 = 5, c6 = 7, c7 = 9;
  for (int i = 0; i < ITERS; i++) {
    c0 = (uint64_t)a * b + c0; c1 = (uint64_t)a * (b + 1) + c1; c2 = (uint64_t)(a + 1) * b + c2; c3 = (uint64_t)(a + 2) * b + c3;
    c4 = (uint64_t)a * (b + 2) + c4; c5 = (uint64_t)(a + 3) * b + c5; c6 = (uint64_t)a * (b + 3) + c6; c7 = (uint64_t)(a + 4) * b + c7;
    a ^= (uint32_t)c0;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}
__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed, b = blockIdx.x * 77 + seed;
  uint32_t c0 = a, c1 = b, c2 = 3, c3 = 5, c4 = 7, c5 = 9, c6 = 11, c7 = 13;
  for (int i = 0; i < ITERS; i++) {
    c0 = c0 * b + a; c1 = c1 * b + a; c2 = c2 * b + a; c3 = c3 * b + a; c4 = c4 * b + a; c5 = c5 * b + a; c6 = c6 * b + a; c7 = c7 * b + a;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}
__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed, b = blockIdx.x * 77 + seed;
  uint32_t c0 = a, c1 = b, c2 = 3, c3 = 5, c4 = 7, c5 = 9, c6 = 11, c7 = 13;
  for (int i = 0; i < ITERS; i++) {
    c0 = __umulhi(c0, b) ^ a; c1 = __umulhi(c1, b) ^ a; c2 = __umulhi(c2, b) ^ a; c3 = __umulhi(c3, b) ^ a;
    c4 = __umulhi(c4, b) ^ a; c5 = __umulhi(c5, b) ^ a; c6 = __umulhi(c6, b) ^ a; c7 = __umulhi(c7, b) ^ a;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}
__global__ void k_fma64(double* out, double seed) {
  double a = threadIdx.x + seed, b = blockIdx.x * 0.5 + seed;
  double c0 = a, c1 = b, c2 = 3, c3 = 5, c4 = 7, c5 = 9, c6 = 11, c7 = 13;
  for (int i = 0; i < ITERS; i++) {
    c0 = fma(c0, b, a); c1 = fma(c1, b, a); c2 = fma(c2, b, a); c3 = fma(c3, b, a);
    c4 = fma(c4, b, a); c5 = fma(c5, b, a); c6 = fma(c6, b, a); c7 = fma(c7, b, a);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
}
__global__ void k_add32(uint32_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x + seed, b = blockIdx.x * 77 + seed;
  uint32_t c0 = a, c1 = b, c2 = 3, c3 = 5, c4 = 7, c5 = 9, c6 = 11, c7 = 13;
  for (int i = 0; i < ITERS; i++) {
    c0 = (c0 ^ b) + a; c1 = (c1 ^ b) + a; c2 = (c2 ^ b) + a; c3 = (c3 ^ b) + a;
    c4 = (c4 ^ b) + a; c5 = (c5 ^ b) + a; c6 = (c6 ^ b) + a; c7 = (c7 ^ b) + a;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
}
template <class F>
__global__ void k_femul(uint32_t* out, uint32_t seed) {
  Fe<F> a, b, c, d;
  for (int i = 0; i < F::N; i++) { a.v[i] = F::ONE[i] ^ (threadIdx.x * 3 + seed); b.v[i] = F::R2[i]; c.v[i] = F::ROOT[i]; d.v[i] = F::ONE[i]; }
  a.v[F::N - 1] &= 0x0fffffff; c.v[F::N-1] &= 0x0fffffff;
  for (int i = 0; i < ITERS / 8; i++) {
    a = fe_mul<F>(a, b); c = fe_mul<F>(c, b); d = fe_mul<F>(d, b); b = fe_mul<F>(b, a);
  }
  uint32_t x = 0;
  for (int i = 0; i < F::N; i++) x ^= a.v[i] ^ b.v[i] ^ c.v[i] ^ d.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
template <class F>
__global__ void k_feadd(uint32_t* out, uint32_t seed) {
  Fe<F> a, b, c, d;
  for (int i = 0; i < F::N; i++) { a.v[i] = F::ONE[i] ^ (threadIdx.x * 3 + seed); b.v[i] = F::R2[i]; c.v[i] = F::ROOT[i]; d.v[i] = F::ONE[i]; }
  a.v[F::N - 1] &= 0x0fffffff; c.v[F::N-1] &= 0x0fffffff;
  for (int i = 0; i < ITERS / 8; i++) {
    a = fe_add<F>(a, b); c = fe_sub<F>(c, b); d = fe_add<F>(d, a); b = fe_sub<F>(b, c);
  }
  uint32_t x = 0;
  for (int i = 0; i < F::N; i++) x ^= a.v[i] ^ b.v[i] ^ c.v[i] ^ d.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <class K, class T>
void run(const char* name, K kern, T* buf, double ops_per_thread_iter, int iters) {
  const int blocks = 256 * 16, threads = 256;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, (T)1);
  hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  for (int r = 0; r < 5; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, (T)1);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double ops = 5.0 * blocks * threads * ops_per_thread_iter * iters;
  printf("%-12s %8.3f ms  %10.2f Gop/s (lane ops)\n", name, ms, ops / (ms * 1e-3) / 1e9);
}
int main() {
  void* buf; hipMalloc(&buf, 256 * 16 * 256 * 8);
  run("mad_u64_u32", k_mad64, (uint64_t*)buf, 8, ITERS);
  run("mul_lo_u32", k_mullo, (uint32_t*)buf, 8, ITERS);
  run("mul_hi_u32", k_mulhi, (uint32_t*)buf, 8, ITERS);
  run("fma_f64", k_fma64, (double*)buf, 8, ITERS);
  run("add+xor", k_add32, (uint32_t*)buf, 16, ITERS);
  run("Ft127 mul", k_femul<Ft127>, (uint32_t*)buf, 4, ITERS / 8);
  run("Ft63 mul", k_femul<Ft63>, (uint32_t*)buf, 4, ITERS / 8);
  run("Ft255 mul", k_femul<Ft255>, (uint32_t*)buf, 4, ITERS / 8);
  run("Ft127 add", k_feadd<Ft127>, (uint32_t*)buf, 4, ITERS / 8);
  return 0;
}
