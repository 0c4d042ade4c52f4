// femul_f64.hip -- study: can FP64 FMA limb products beat the library's integer Ft127 multiply?
//
// MI355X issues fma_f64 at 36.6 T lane-ops/s against 20.6 T for v_mad_u64_u32
// (profiles/r01_mulbench.txt), so an f64-limb product is the obvious candidate (Emmart, Zheng and
// Weems' exact FMA splitting).  An Ft127 element as three 52-bit limbs in doubles; one 52 x 52-bit
// partial product a b, exactly, as two integers:
//     hi  = fma(a, b, 2^104)           the mantissa holds round(a b / 2^52)  (ulp 2^52 at 2^104)
//     lo  = fma(a, b, -(hi - 2^104))   a b - round(a b / 2^52) 2^52, exact, |lo| <= 2^51
//     lo' = lo + 3 2^51                the mantissa holds lo + 2^51 (ulp 1)
// and the bit patterns of hi and lo' are accumulated as int64 column sums (the constant biases
// are subtracted once per column).  That is 4 FP ops + 2 int64 adds per partial product, 9
// partial products for the 254-bit product -- BEFORE any Montgomery reduction, which needs 9
// more partial products plus the quotient digits (52-bit low products: 2 FMAs each).
//
// This kernel times only the UNREDUCED f64 product (operand conversion included) against the
// library's COMPLETE Montgomery product (fe_mul, field.hpp) and checks the f64 product exactly
// against a 32-bit-limb schoolbook product.  If the unreduced half alone is not faster than the
// whole integer multiply, the f64 route cannot win.  Result on MI355X: profiles/r03_femul_f64.txt.
// Build: make -C tools/microbench femul_f64
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

constexpr double C104 = 20282409603651670423947251286016.0;  // 2^104
constexpr double C3_51 = 6755399441055744.0;                  // 3 * 2^51

// 4 x 32-bit words (< 2^128) -> three 52-bit limbs (the top one 24 bits) as exact doubles
__device__ __forceinline__ void to_limbs(const uint32_t w[4], double d[3]) {
  const uint64_t lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32), hi = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  const uint64_t M = (1ull << 52) - 1;
  d[0] = (double)(lo & M);
  d[1] = (double)(((lo >> 52) | (hi << 12)) & M);
  d[2] = (double)(hi >> 40);
}

// the 254-bit product as 6 column sums c[k] = sum_{i+j=k} a_i b_j split into (hi, lo) parts:
// value = sum_k (H[k] 2^52 + L[k]) 2^(52 k), returned as raw int64 sums with the biases removed
__device__ __forceinline__ void mul_f64(const double a[3], const double b[3], int64_t H[5], int64_t L[5]) {
  const int64_t BH = (int64_t)__double_as_longlong(C104), BL = (int64_t)__double_as_longlong(C3_51);
#pragma unroll
  for (int k = 0; k < 5; k++) H[k] = L[k] = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const double hi = __fma_rn(a[i], b[j], C104);
      const double lo = __fma_rn(a[i], b[j], -(hi - C104));
      const double lb = lo + C3_51;
      H[i + j] += (int64_t)__double_as_longlong(hi) - BH;
      L[i + j] += (int64_t)__double_as_longlong(lb) - BL;
    }
  }
}

#define ITERS 1024
// V = 0: library Montgomery product (complete, reduced); V = 1: the f64 unreduced product
template <int V>
__global__ void k_rate(uint32_t *out, uint32_t seed) {
  using F = Ft127;
  Fe<F> a, b;
  for (int i = 0; i < 4; i++) {
    a.v[i] = F::ONE[i] ^ (threadIdx.x * 3 + seed);
    b.v[i] = F::R2[i];
  }
  a.v[3] &= 0x0fffffff;
  uint32_t x = 0;
  if constexpr (V == 0) {
    for (int i = 0; i < ITERS; i++) a = fe_mul<F>(a, b);
    for (int i = 0; i < 4; i++) x ^= a.v[i];
  } else {
    for (int i = 0; i < ITERS; i++) {
      double da[3], db[3];
      to_limbs(a.v, da);
      to_limbs(b.v, db);
      int64_t H[5], L[5];
      mul_f64(da, db, H, L);
      // feed the result back as the next operand (keeps the chain dependent, like V = 0)
      a.v[0] ^= (uint32_t)(H[0] ^ L[1]);
      a.v[1] ^= (uint32_t)(H[1] ^ L[2]);
      a.v[2] ^= (uint32_t)(H[2] ^ L[3] ^ H[4]);
      a.v[3] = (a.v[3] ^ (uint32_t)(H[3] ^ L[4] ^ L[0])) & 0x0fffffff;
    }
    for (int i = 0; i < 4; i++) x ^= a.v[i];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

// exactness: the f64 column sums recombined equal the schoolbook product (8 words)
__global__ void k_check(const uint32_t *in, uint32_t *bad, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint32_t a[4], b[4];
  for (int i = 0; i < 4; i++) a[i] = in[8 * t + i], b[i] = in[8 * t + 4 + i];
  // schoolbook on 32-bit words
  uint32_t ref[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 4; j++) {
      const uint64_t s = (uint64_t)a[i] * b[j] + ref[i + j] + c;
      ref[i + j] = (uint32_t)s;
      c = s >> 32;
    }
    ref[i + 4] = (uint32_t)c;
  }
  double da[3], db[3];
  to_limbs(a, da);
  to_limbs(b, db);
  int64_t H[5], L[5];
  mul_f64(da, db, H, L);
  // value = sum_k L[k] 2^(52k) + H[k] 2^(52(k+1)), signed terms: accumulate into 9 words
  int64_t acc[12] = {0};
  auto add_at = [&](int64_t v, int bit) {
    // add signed v * 2^bit into 32-bit words (acc holds signed partial sums per word)
    const int w = bit / 32, s = bit % 32;
    const __int128 x = (__int128)v << s;
    acc[w] += (int64_t)(uint32_t)(uint64_t)x;
    acc[w + 1] += (int64_t)(uint32_t)(uint64_t)(x >> 32);
    acc[w + 2] += (int64_t)(x >> 64);
  };
  for (int k = 0; k < 5; k++) {
    add_at(L[k], 52 * k);
    add_at(H[k], 52 * (k + 1));
  }
  int64_t c = 0;
  uint32_t got[8];
  for (int w = 0; w < 8; w++) {
    const int64_t s = acc[w] + c;
    got[w] = (uint32_t)s;
    c = s >> 32;  // arithmetic shift: signed carry
  }
  for (int w = 0; w < 8; w++)
    if (got[w] != ref[w]) {
      atomicAdd(bad, 1u);
      break;
    }
}

int main() {
  uint32_t *buf, *bad;
  const int blocks = 256 * 64, threads = 256;
  CK(hipMalloc(&buf, (size_t)blocks * threads * 4));
  CK(hipMalloc(&bad, 4));
  const int n = 1 << 20;
  std::vector<uint32_t> h((size_t)8 * n);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < h.size(); i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h[i] = (uint32_t)x;
    if (i % 4 == 3) h[i] &= 0x7fffffffu;  // < 2^127
  }
  uint32_t *din;
  CK(hipMalloc(&din, h.size() * 4));
  CK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(bad, 0, 4));
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, din, bad, n);
  uint32_t nb = 0;
  CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
  printf("f64 limb product exact on 2^20 random 127-bit pairs: %s (%u mismatches)\n", nb ? "NO" : "yes", nb);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char *names[2] = {"Ft127 Montgomery product, integer (library fe_mul, reduced)",
                          "Ft127 254-bit product, f64 limbs (UNREDUCED, conversions incl.)"};
  for (int v = 0; v < 2; v++) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
      CK(hipEventRecord(e0));
      if (v == 0)
        hipLaunchKernelGGL(k_rate<0>, dim3(blocks), dim3(threads), 0, 0, buf, 7u);
      else
        hipLaunchKernelGGL(k_rate<1>, dim3(blocks), dim3(threads), 0, 0, buf, 7u);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("%-66s %8.3f ms  %8.2f G products/s\n", names[v], best,
           (double)blocks * threads * ITERS / (best * 1e-3) / 1e9);
  }
  return 0;
}
