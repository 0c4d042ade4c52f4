#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>
#include "../../lcpc_proof_of_storage_amd/csrc/field.hpp"
using namespace lcpc;
#define ITERS 4096
template <class F, int V>
__global__ void k_femul(uint32_t* out, uint32_t seed) {
  Fe<F> a, b, c, d;
  for (int i = 0; i < F::N; i++) { a.v[i] = F::ONE[i] ^ (threadIdx.x * 3 + seed); b.v[i] = F::R2[i]; c.v[i] = F::ROOT[i]; d.v[i] = F::ONE[i]; }
  a.v[F::N - 1] &= 0x0fffffff; c.v[F::N-1] &= 0x0fffffff;
  for (int i = 0; i < ITERS / 8; i++) {
    if (V == 0) { a = fe_mul_cios<F>(a, b); c = fe_mul_cios<F>(c, b); d = fe_mul_cios<F>(d, b); b = fe_mul_cios<F>(b, a); }
    else { a = fe_mul_fips<F>(a, b); c = fe_mul_fips<F>(c, b); d = fe_mul_fips<F>(d, b); b = fe_mul_fips<F>(b, a); }
  }
  uint32_t x = 0;
  for (int i = 0; i < F::N; i++) x ^= a.v[i] ^ b.v[i] ^ c.v[i] ^ d.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
template <class F>
__global__ void k_check(const uint32_t* A, const uint32_t* B, size_t n, uint32_t* bad) {
  size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= n) return;
  Fe<F> a = fe_load<F>(A, t), b = fe_load<F>(B, t);
  Fe<F> x = fe_mul_cios<F>(a, b), y = fe_mul_fips<F>(a, b);
  if (!fe_eq<F>(x, y)) atomicAdd(bad, 1u);
  if (!fe_eq<F>(fe_from_mont_generic<F>(a), fe_from_mont_fips<F>(a))) atomicAdd(bad, 1u);
}
// fe_dot<F, K> == sum of fe_mul (K = 2 and kmax), on random inputs
template <class F, int K>
__global__ void k_check_dot(const uint32_t* A, const uint32_t* B, size_t n, uint32_t* bad) {
  size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t * K + K > n) return;
  Fe<F> a[K], b[K];
  Fe<F> want = fe_zero<F>();
  for (int q = 0; q < K; q++) {
    a[q] = fe_load<F>(A, t * K + q); b[q] = fe_load<F>(B, t * K + q);
    want = fe_add<F>(want, fe_mul_cios<F>(a[q], b[q]));
  }
  if (!fe_eq<F>(want, fe_dot<F, K>(a, b))) atomicAdd(bad, 1u);
}

template <class F>
void run(const char* name) {
  const size_t n = 1 << 22;
  std::vector<uint32_t> h(n * F::N);
  std::mt19937_64 rng(42);
  // random values < p: take random words, clear top bits so < p (top word < P[N-1])
  for (size_t i = 0; i < n; i++) {
    for (int k = 0; k < F::N; k++) h[i * F::N + k] = (uint32_t)rng();
    h[i * F::N + F::N - 1] %= F::P[F::N - 1];
    if (i < 16) { for (int k = 0; k < F::N; k++) h[i*F::N+k] = (i & 1) ? F::P[k] - (k==0) : 0; }  // p-1 and 0
  }
  uint32_t *dA, *dB, *dbad, *dout;
  hipMalloc(&dA, h.size() * 4); hipMalloc(&dB, h.size() * 4); hipMalloc(&dbad, 4); hipMalloc(&dout, 1 << 24);
  hipMemcpy(dA, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  std::reverse(h.begin(), h.end());
  for (size_t i = 0; i < n; i++) { h[i * F::N + F::N - 1] %= F::P[F::N - 1]; }
  hipMemcpy(dB, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipMemset(dbad, 0, 4);
  hipLaunchKernelGGL(k_check<F>, dim3(n / 256), dim3(256), 0, 0, dA, dB, n, dbad);
  uint32_t bad = 0; hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
  hipMemset(dbad, 0, 4);
  hipLaunchKernelGGL((k_check_dot<F, 2>), dim3(n / 256), dim3(256), 0, 0, dA, dB, n, dbad);
  hipLaunchKernelGGL((k_check_dot<F, fe_dot_kmax<F>() < 8 ? fe_dot_kmax<F>() : 8>), dim3(n / 256), dim3(256), 0, 0, dA, dB, n, dbad);
  uint32_t bad_dot = 0; hipMemcpy(&bad_dot, dbad, 4, hipMemcpyDeviceToHost);
  printf("%s: fe_dot mismatches %u (kmax %d)\n", name, bad_dot, fe_dot_kmax<F>());
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms[2];
  for (int v = 0; v < 2; v++) {
    auto launch = [&]() { if (v == 0) hipLaunchKernelGGL((k_femul<F, 0>), dim3(2048), dim3(256), 0, 0, dout, 1u); else hipLaunchKernelGGL((k_femul<F, 1>), dim3(2048), dim3(256), 0, 0, dout, 1u); };
    launch(); hipDeviceSynchronize();
    hipEventRecord(e0); for (int r = 0; r < 5; r++) launch(); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms[v], e0, e1);
  }
  const double muls = 5.0 * 2048 * 256 * (ITERS / 8) * 4;
  printf("%s: mismatches %u; cios %.1f G/s  fips %.1f G/s\n", name, bad, muls / ms[0] / 1e6, muls / ms[1] / 1e6);
}
int main() { run<Ft63>("Ft63"); run<Ft127>("Ft127"); run<Ft255>("Ft255"); run<Ft253_192>("Ft253"); return 0; }
