// nttmfma.hip -- one radix-16 DFT stage over Ft127 on the int8 matrix cores, with the
// recombination of each output in its own lane (the round-3 review's "digit-GEMM DFT" lever).
//
// y_j = sum_i W[j][i] x_i (W = the 16-point DFT matrix over F_p) for many vectors x, exactly:
//   * every x_i (canonical, < 2^127 - 2^120) as 16 balanced base-256 digits d_a(x_i) (int8);
//   * for every (j, i, a) the balanced digits h_u of H = W[j][i] 2^(8a) 2^32 mod p;
//   * v_mfma_i32_32x32x32_i8: C[(j, u)][vector] += sum_(i, a) h_u(H_jia) d_a(x_i): M = 32 rows =
//     2 outputs j x 16 digit positions u, K = 32 = 2 inputs x 16 digits, N = 32 vectors.  The
//     rows are placed so that lane (vector r, half h) holds all 16 Y_u of ONE output in its 16
//     accumulator registers (C row = (reg & 3) + 8 (reg >> 2) + 4 h): no cross-lane movement;
//   * per output: V = sum_u Y_u 2^(8u) (|V| < 2^142.01) + p 2^16, ONE Montgomery word step
//     ((V + m p) / 2^32, m = -V mod 2^32: the 2^32 folded into H cancels it): a value < p + 2^112,
//     whose balanced digits feed the next stage straight from the lane (output j = 2p + h is the
//     next stage's input i = 2 ks + h of the same lane).
// The bench applies the stage `reps` times to each wave's 32 vectors in registers (load once,
// store once) and reports SIMD-cycles per element per stage; the host checks W^reps x exactly
// on a sample of vectors.
// Build: hipcc -O3 --offload-arch=gfx950 nttmfma.hip -o nttmfma
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "f127_host.hpp"

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

namespace {
constexpr uint32_t P0 = 0x00000001u, P1 = 0x7f2bd900u, P2 = 0xba20e0bfu, P3 = 0x6e754097u;

__device__ __forceinline__ v4i digits(const uint32_t x[4]) {
  uint32_t c = 0;
  const uint32_t v0 = __builtin_addc(x[0], 0x80808080u, c, &c);
  const uint32_t v1 = __builtin_addc(x[1], 0x80808080u, c, &c);
  const uint32_t v2 = __builtin_addc(x[2], 0x80808080u, c, &c);
  const uint32_t v3 = __builtin_addc(x[3], 0x80808080u, c, &c);
  return v4i{(int)(v0 ^ 0x80808080u), (int)(v1 ^ 0x80808080u), (int)(v2 ^ 0x80808080u), (int)(v3 ^ 0x80808080u)};
}

// V = sum_u Y_u 2^(8u), |Y_u| < 2^22, then ONE Montgomery word step on V + OFF:
// out = (V + OFF + m p) / 2^32 with m = -(V + OFF) mod 2^32, a value < p + 2^114 congruent to
// V 2^-32 (mod p).  32-bit operations only:
//   P_q = Y_2q + Y_(2q+1) 2^8 (|P_q| < 2^31), V = sum_w (P_2w + P_(2w+1) 2^16) 2^(32w);
//   P_2w + (P_(2w+1) << 16 mod 2^32) = lo_w + 2^32 hi_w with hi_w = carry - [P_2w < 0];
//   V = sum_w lo_w 2^(32w) + sum_w K_(w+1) 2^(32(w+1)), K_(w+1) = hi_w + (P_(2w+1) >>a 16);
//   K + 2^16 >= 0, and OFF = p 2^18 - 2^16 sum_(w=1..4) 2^(32w) (positive, a multiple of p
//   minus the bias) keeps every limb sum nonnegative: V + OFF < 2^146.
__device__ __forceinline__ void recombine(const v16i &Y, uint32_t out[4]) {
  int32_t Pq[8];
#pragma unroll
  for (int q = 0; q < 8; q++) Pq[q] = Y[2 * q] + (Y[2 * q + 1] << 8);
  uint32_t lo[4], K[5];
  K[0] = 0;
#pragma unroll
  for (int w = 0; w < 4; w++) {
    uint32_t c;
    lo[w] = __builtin_addc((uint32_t)Pq[2 * w], (uint32_t)Pq[2 * w + 1] << 16, 0u, &c);
    K[w + 1] = (uint32_t)((Pq[2 * w] >> 31) + (Pq[2 * w + 1] >> 16) + 0x10000) + c;
  }
  // OFF = p 2^18 - 2^16 (2^32 + 2^64 + 2^96 + 2^128), limbs
  constexpr uint32_t OFF0 = 0x00040000u, OFF1 = 0x63ff0000u, OFF2 = 0x82fcfcafu, OFF3 = 0x025de883u,
                     OFF4 = 0x0000b9d5u;
  uint32_t L[5], c = 0;
  L[0] = __builtin_addc(lo[0], OFF0, 0u, &c);
  L[1] = __builtin_addc(lo[1], OFF1, c, &c);
  L[2] = __builtin_addc(lo[2], OFF2, c, &c);
  L[3] = __builtin_addc(lo[3], OFF3, c, &c);
  L[4] = OFF4 + c;
  c = 0;
  L[1] = __builtin_addc(L[1], K[1], 0u, &c);
  L[2] = __builtin_addc(L[2], K[2], c, &c);
  L[3] = __builtin_addc(L[3], K[3], c, &c);
  L[4] = L[4] + K[4] + c;
  // one Montgomery word step (p = 1 mod 2^32: m p0 + L0 = 2^32 [L0 != 0])
  const uint32_t m = 0u - L[0];
  uint64_t t = (uint64_t)m * P1 + ((uint64_t)L[1] + (L[0] != 0u));
  out[0] = (uint32_t)t;
  t = (uint64_t)m * P2 + ((t >> 32) + L[2]);
  out[1] = (uint32_t)t;
  t = (uint64_t)m * P3 + ((t >> 32) + L[3]);
  out[2] = (uint32_t)t;
  out[3] = (uint32_t)(t >> 32) + L[4];
}

__device__ __forceinline__ void reduce_p(uint32_t x[4]) {  // x < 2p -> x mod p
  uint32_t u[4], br = 0;
  u[0] = __builtin_subc(x[0], P0, br, &br);
  u[1] = __builtin_subc(x[1], P1, br, &br);
  u[2] = __builtin_subc(x[2], P2, br, &br);
  u[3] = __builtin_subc(x[3], P3, br, &br);
  if (!br)
    for (int i = 0; i < 4; i++) x[i] = u[i];
}

// one wave = 32 vectors of 16 elements ([vec][i] canonical 16-byte elements); reps stages
// MODE 0: the stage; 1: the matrix-core part alone (the next digits are a cheap mix of the
// accumulators); 2: the VALU part alone (the accumulators are a cheap mix of the digits)
template <int MODE>
__global__ __launch_bounds__(256) void k_stage(const uint4 *__restrict__ in, uint4 *__restrict__ out,
                                               const uint4 *__restrict__ ht, int reps, size_t nvec) {
  __shared__ uint4 sh[64 * 64];  // the 64 A fragments (64 KB)
  for (int i = threadIdx.x; i < 64 * 64; i += 256) sh[i] = ht[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const size_t vec = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 + r;
  if (vec >= nvec) return;
  v4i B[8];
#pragma unroll
  for (int ks = 0; ks < 8; ks++) {
    const uint4 q = in[vec * 16 + 2 * ks + h];
    const uint32_t x[4] = {q.x, q.y, q.z, q.w};
    B[ks] = digits(x);
  }
  for (int rep = 0; rep + 1 < reps; rep++) {
    v4i Bn[8];
#pragma unroll
    for (int p = 0; p < 8; p++) {
      v16i acc = {0};
      if constexpr (MODE == 3) {
        // two output pairs per pass: two independent accumulation chains interleaved
        if (p & 1) continue;
        v16i acc2 = {0};
#pragma unroll
        for (int ks = 0; ks < 8; ks++) {
          const uint4 a = sh[(p * 8 + ks) * 64 + lane];
          const uint4 a2 = sh[((p + 1) * 8 + ks) * 64 + lane];
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(v4i{(int)a.x, (int)a.y, (int)a.z, (int)a.w}, B[ks], acc, 0, 0, 0);
          acc2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(v4i{(int)a2.x, (int)a2.y, (int)a2.z, (int)a2.w}, B[ks], acc2, 0, 0, 0);
        }
        uint32_t y[4], y2[4];
        recombine(acc, y);
        recombine(acc2, y2);
        Bn[p] = digits(y);
        Bn[p + 1] = digits(y2);
        __builtin_amdgcn_sched_barrier(0);
        continue;
      }
      if constexpr (MODE == 2) {
#pragma unroll
        for (int u = 0; u < 16; u++) acc[u] = B[u & 7][u >> 3] ^ (p * 0x1010101 + u);
      } else {
#pragma unroll
        for (int ks = 0; ks < 8; ks++) {
          const uint4 a = sh[(p * 8 + ks) * 64 + lane];
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(v4i{(int)a.x, (int)a.y, (int)a.z, (int)a.w}, B[ks], acc, 0, 0, 0);
        }
      }
      if constexpr (MODE == 1) {
        Bn[p] = v4i{acc[0] ^ acc[4], acc[1] ^ acc[8], acc[2] ^ acc[12], acc[3] ^ acc[15]};
        __builtin_amdgcn_sched_barrier(0);
        continue;
      }
      uint32_t y[4];
      recombine(acc, y);
      Bn[p] = digits(y);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int ks = 0; ks < 8; ks++) B[ks] = Bn[ks];
  }
#pragma unroll
  for (int p = 0; p < 8; p++) {
    v16i acc = {0};
#pragma unroll
    for (int ks = 0; ks < 8; ks++) {
      const uint4 a = sh[(p * 8 + ks) * 64 + lane];
      acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(v4i{(int)a.x, (int)a.y, (int)a.z, (int)a.w}, B[ks], acc, 0, 0, 0);
    }
    uint32_t y[4];
    recombine(acc, y);
    reduce_p(y);
    out[vec * 16 + 2 * p + h] = make_uint4(y[0], y[1], y[2], y[3]);
    __builtin_amdgcn_sched_barrier(0);
  }
}
}  // namespace

int main(int argc, char **argv) {
  using namespace f127h;
  const size_t nvec = argc > 1 ? (size_t)atol(argv[1]) : (size_t)1 << 17;  // 2M elements
  const int reps = argc > 2 ? atoi(argv[2]) : 8;
  // W[j][i] = w16^(i j), natural order
  const u128 w16 = root_of_order(4);
  u128 W[16][16];
  for (int j = 0; j < 16; j++)
    for (int i = 0; i < 16; i++) W[j][i] = pow(w16, (u128)(i * j));
  // the A fragments: frag (p, ks), lane l = m + 32 h': 16 bytes, byte a = h_u(W[j][i] 2^(8a) 2^32)
  std::vector<int8_t> ht(64 * 64 * 16);
  u128 s2a[16];
  for (int a = 0; a < 16; a++) s2a[a] = two_pow(8 * a + 32);
  for (int p = 0; p < 8; p++)
    for (int ks = 0; ks < 8; ks++)
      for (int l = 0; l < 64; l++) {
        const int m = l & 31, hp = l >> 5;
        const int j = 2 * p + ((m >> 2) & 1), u = (m & 3) + 4 * (m >> 3), i = 2 * ks + hp;
        for (int a = 0; a < 16; a++) {
          int8_t d[16];
          balanced(mul(W[j][i], s2a[a]), d);
          ht[((p * 8 + ks) * 64 + l) * 16 + a] = d[u];
        }
      }
  // inputs: canonical pseudo-random values < p
  std::vector<uint32_t> hin(nvec * 16 * 4);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  auto rnd = [&]() {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    return s;
  };
  for (size_t e = 0; e < nvec * 16; e++) {
    u128 x = (((u128)rnd() << 64) | rnd()) % P;
    to_words(x, &hin[e * 4]);
  }
  uint4 *din, *dout, *dht;
  CK(hipMalloc(&din, nvec * 16 * 16));
  CK(hipMalloc(&dout, nvec * 16 * 16));
  CK(hipMalloc(&dht, ht.size()));
  CK(hipMemcpy(din, hin.data(), nvec * 256, hipMemcpyHostToDevice));
  CK(hipMemcpy(dht, ht.data(), ht.size(), hipMemcpyHostToDevice));
  const unsigned blocks = (unsigned)((nvec + 127) / 128);
  hipLaunchKernelGGL(k_stage<0>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, reps, nvec);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 10;
  CK(hipEventRecord(e0));
  for (int it = 0; it < iters; it++)
    hipLaunchKernelGGL(k_stage<0>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, reps, nvec);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  // the same launch with reps = 0 (load + digits + store only) to subtract the memory part
  CK(hipEventRecord(e0));
  for (int it = 0; it < iters; it++)
    hipLaunchKernelGGL(k_stage<0>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, 1, nvec);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms1 = 0;
  CK(hipEventElapsedTime(&ms1, e0, e1));
  ms1 /= iters;
  float msm[3] = {ms, 0, 0};
  float ms3 = 0;
  for (int md = 1; md <= 3; md++) {
    CK(hipEventRecord(e0));
    for (int it = 0; it < iters; it++) {
      if (md == 1) hipLaunchKernelGGL(k_stage<1>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, reps, nvec);
      else if (md == 2) hipLaunchKernelGGL(k_stage<2>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, reps, nvec);
      else hipLaunchKernelGGL(k_stage<3>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, reps, nvec);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float& dst = md == 3 ? ms3 : msm[md];
    CK(hipEventElapsedTime(&dst, e0, e1));
    dst /= iters;
  }
  {
    const double el = (double)nvec * 16;
    auto cyc = [&](float m) { return (m - ms1) * 1e-3 / (reps - 1) / el * 2.4e9 * 1024; };
    printf("nttmfma split: whole stage %.2f, matrix cores alone %.2f, VALU alone %.2f, two interleaved chains %.2f "
           "SIMD-cycles per element (nominal)\n",
           cyc(msm[0]), cyc(msm[1]), cyc(msm[2]), cyc(ms3));
  }
  hipLaunchKernelGGL(k_stage<0>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, reps, nvec);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> hout(nvec * 16 * 4);
  CK(hipMemcpy(hout.data(), dout, nvec * 256, hipMemcpyDeviceToHost));
  // exact check on a sample
  size_t bad = 0, checked = 0;
  for (size_t v = 0; v < nvec; v += nvec / 64 + 1) {
    u128 x[16], y[16];
    for (int i = 0; i < 16; i++) x[i] = from_words(&hin[(v * 16 + i) * 4]);
    for (int r = 0; r < reps; r++) {
      for (int j = 0; j < 16; j++) {
        u128 acc = 0;
        for (int i = 0; i < 16; i++) acc = add(acc, mul(W[j][i], x[i]));
        y[j] = acc;
      }
      for (int j = 0; j < 16; j++) x[j] = y[j];
    }
    for (int j = 0; j < 16; j++) {
      checked++;
      if (from_words(&hout[(v * 16 + j) * 4]) != x[j]) bad++;
    }
  }
  const double elems = (double)nvec * 16;
  const double clk = 2.4e9, simds = 1024;  // nominal: cycles at 2.4 GHz over 1024 SIMDs
  const double per = (ms - ms1) * 1e-3 / (reps - 1) / elems * clk * simds;
  printf("nttmfma: %zu vectors x 16, reps %d: %.3f ms (1 rep: %.3f ms); %.2f SIMD-cycles per element per stage "
         "(nominal 2.4 GHz); check %zu/%zu %s\n",
         nvec, reps, ms, ms1, per, checked - bad, checked, bad ? "MISMATCH" : "exact");
  return bad ? 1 : 0;
}
