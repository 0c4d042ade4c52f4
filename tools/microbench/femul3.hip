// femul3.hip -- A/B: one Montgomery product at a time (field.hpp fe_mul_fips: every v_mad_u64_u32
// accumulates into the previous one's result, and gfx950 needs a wait state between such a pair,
// so the compiler puts an s_nop 0 between them) against two independent products interleaved
// instruction by instruction (fe_mul_pair below: each dependent pair has the other product's
// instruction between them, no s_nop).  Result on MI355X (profiles/r02_femul3.txt): no
// difference (Ft127 500.6 vs 502.5 G mul/s) -- with several waves per SIMD the wait states cost
// nothing, the issue rate is the bound; the same pairing inside the NTT butterflies left the
// passes unchanged (Ft127 0.456 / 0.362 ms, Ft63 at the PoS dims 1.06 / 0.58 ms), so the
// library keeps one product at a time.
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 femul3.hip -o femul3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../lcpc_proof_of_storage_amd/csrc/field.hpp"

using namespace lcpc;

// Two independent Montgomery products, r = a b R^-1 and s = c d R^-1, computed in lock step:
// fe_mul_fips's schedule for each, one instruction of the one and one of the other in turn.  A
// v_mad_u64_u32 that accumulates into the previous one's result needs a wait state on gfx950
// (the compiler puts an s_nop 0 between them: ~1 per product term); interleaved, the other
// product's instruction fills it.  Bit-identical to two fe_mul calls (r, s may alias a..d).
template <class F>
__device__ __forceinline__ void fe_mul_pair(const Fe<F>& a, const Fe<F>& b, const Fe<F>& c, const Fe<F>& d,
                                            Fe<F>& r, Fe<F>& s) {
  constexpr int N = F::N;
  static_assert(F::NP == 0xffffffffu && F::P[0] == 1u, "p = 1 mod 2^32");
  uint32_t m0[N], m1[N], o0[N], o1[N];
  uint64_t acc0 = 0, acc1 = 0;
  uint32_t r20 = 0, r21 = 0;
#pragma unroll
  for (int k = 0; k < 2 * N; k++) {
    uint64_t cp0 = 0, cp1 = 0, cc0, cc1;
    bool have = false;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j < 0 || j >= N) continue;
      acc0 = mad_co_vv(a.v[i], b.v[j], acc0, cc0);
      acc1 = mad_co_vv(c.v[i], d.v[j], acc1, cc1);
      if (have) {
        r20 = add_carry(r20, cp0);
        r21 = add_carry(r21, cp1);
      }
      cp0 = cc0;
      cp1 = cc1;
      have = true;
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i >= k || j < 1 || j >= N) continue;
      acc0 = mad_co_vs(m0[i], F::P[j], acc0, cc0);
      acc1 = mad_co_vs(m1[i], F::P[j], acc1, cc1);
      if (have) {
        r20 = add_carry(r20, cp0);
        r21 = add_carry(r21, cp1);
      }
      cp0 = cc0;
      cp1 = cc1;
      have = true;
    }
    if (have) {
      r20 = add_carry(r20, cp0);
      r21 = add_carry(r21, cp1);
    }
    if (k < N) {
      uint32_t l0, h0, l1, h1;
      fips_col_step((uint32_t)acc0, (uint32_t)(acc0 >> 32), r20, m0[k], l0, h0);
      fips_col_step((uint32_t)acc1, (uint32_t)(acc1 >> 32), r21, m1[k], l1, h1);
      acc0 = ((uint64_t)h0 << 32) | l0;
      acc1 = ((uint64_t)h1 << 32) | l1;
    } else {
      o0[k - N] = (uint32_t)acc0;
      o1[k - N] = (uint32_t)acc1;
      acc0 = (acc0 >> 32) | ((uint64_t)r20 << 32);
      acc1 = (acc1 >> 32) | ((uint64_t)r21 << 32);
    }
    r20 = 0;
    r21 = 0;
  }
  Fe<F> u0, u1;
  uint32_t b0 = 0, b1 = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    u0.v[i] = __builtin_subc(o0[i], F::P[i], b0, &b0);
    u1.v[i] = __builtin_subc(o1[i], F::P[i], b1, &b1);
  }
  const bool t0 = ((uint32_t)acc0 != 0u) | (b0 ^ 1u), t1 = ((uint32_t)acc1 != 0u) | (b1 ^ 1u);
#pragma unroll
  for (int i = 0; i < N; i++) {
    r.v[i] = t0 ? u0.v[i] : o0[i];
    s.v[i] = t1 ? u1.v[i] : o1[i];
  }
}


#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

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
      fe_mul_pair<F>(a, b, c, b, a, c);  // a = a b, c = c b
      fe_mul_pair<F>(d, b, b, a, d, b);  // d = d b, b = b a (both read the old b)
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
  if (2 * t + 1 >= n) return;
  Fe<F> a, b, c, d;
  for (int i = 0; i < F::N; i++) {
    a.v[i] = in[(2 * t) * F::N + i];
    b.v[i] = in[(2 * t + 1) * F::N + i];
    c.v[i] = in[(2 * t + 1) * F::N + i] ^ 0x5a5a5a5au;
    d.v[i] = in[(2 * t) * F::N + i] ^ 0x13579bdfu;
  }
  c.v[F::N - 1] &= 0x0fffffff;
  d.v[F::N - 1] &= 0x0fffffff;
  const Fe<F> x = fe_mul<F>(a, b), y = fe_mul<F>(c, d);
  Fe<F> u, v;
  fe_mul_pair<F>(a, b, c, d, u, v);
  for (int i = 0; i < F::N; i++)
    if (x.v[i] != u.v[i] || y.v[i] != v.v[i]) atomicAdd(bad, 1u);
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
        printf("%s %s  %8.3f ms  %8.2f G mul/s  %s\n", name, v ? "pair (interleaved)" : "single (library)  ", ms,
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
