// nttmfma63.hip -- nttmfma.hip's radix-16 DFT stage for Ft63 (the proof-of-storage field,
// p = 0x46d0760000000001, lcpc-test-fields/src/lib.rs:18-22): 8 balanced digits per element, so a
// 16-point DFT is a (16 x 8) x (16 x 8) int8 product per vector -- 1024 MACs per element, a quarter
// of Ft127's.
//   v_mfma_i32_32x32x32_i8: M = 32 = 4 outputs x 8 digit positions, K = 32 = 4 inputs x 8 digits,
//   N = 32 vectors.  A row m = (reg & 3) + 8 (reg >> 2) + 4 h of the C layout is output
//   o = 2 h + (reg >> 3), digit u = reg & 7: lane (vector r, half h) holds all 8 partials of two
//   outputs, 4 q + 2 h and 4 q + 2 h + 1 -- the two elements its B fragment of k-step q holds in the
//   next stage (16 bytes = two 8-byte elements' digits).
//   Per output: V = sum_u Y_u 2^(8u) (|V| < 2^77) + OFF, one Montgomery word step: < p + 2^46.
// Reports SIMD-cycles per element per stage (stage applied `reps` times in registers) and checks
// W^reps x exactly against host 128-bit arithmetic.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm --amdgpu-mfma-vgpr-form nttmfma63.hip -o nttmfma63
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

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
typedef unsigned __int128 u128;

namespace {
constexpr uint64_t P64 = 0x46d0760000000001ull;
constexpr uint32_t P1 = 0x46d07600u;

// 8 balanced digits of x < 2^63 - 2^56, as two dwords
__device__ __forceinline__ int2 digits2(uint32_t lo, uint32_t hi) {
  uint32_t c = 0;
  const uint32_t v0 = __builtin_addc(lo, 0x80808080u, c, &c);
  const uint32_t v1 = __builtin_addc(hi, 0x80808080u, c, &c);
  return make_int2((int)(v0 ^ 0x80808080u), (int)(v1 ^ 0x80808080u));
}

// V = sum_(u < 8) Y[u0 + u] 2^(8u), |Y| < 2^21; out = (V + OFF + m p) / 2^32 < p + 2^46
//   P_q = Y_2q + Y_(2q+1) 2^8; V = sum_w (P_2w + P_(2w+1) 2^16) 2^(32w), w = 0, 1;
//   lo_w, K_(w+1) = hi_w + (P_(2w+1) >>a 16) + 2^16 as in nttmfma.hip;
//   OFF = p 2^18 - 2^16 (2^32 + 2^64) (positive), V + OFF < 2^81: three limbs
__device__ __forceinline__ void recombine63(const v16i &Y, int u0, uint32_t &o0, uint32_t &o1) {
  int32_t Pq[4];
#pragma unroll
  for (int q = 0; q < 4; q++) Pq[q] = Y[u0 + 2 * q] + (Y[u0 + 2 * q + 1] << 8);
  uint32_t lo[2], K[3];
  K[0] = 0;
#pragma unroll
  for (int w = 0; w < 2; w++) {
    uint32_t c;
    lo[w] = __builtin_addc((uint32_t)Pq[2 * w], (uint32_t)Pq[2 * w + 1] << 16, 0u, &c);
    K[w + 1] = (uint32_t)((Pq[2 * w] >> 31) + (Pq[2 * w + 1] >> 16) + 0x10000) + c;
  }
  // OFF limbs: p 2^18 = {0x00040000, 0xd8000000, 0x00011b41}; minus 2^16 at limbs 1 and 2
  constexpr uint32_t OFF0 = 0x00040000u, OFF1 = 0xd7ff0000u, OFF2 = 0x00001b41u;
  uint32_t L0, L1, L2, c = 0;
  L0 = __builtin_addc(lo[0], OFF0, 0u, &c);
  L1 = __builtin_addc(lo[1], OFF1, c, &c);
  L2 = OFF2 + c;
  c = 0;
  L1 = __builtin_addc(L1, K[1], 0u, &c);
  L2 = L2 + K[2] + c;
  const uint32_t m = 0u - L0;
  const uint64_t t = (uint64_t)m * P1 + ((uint64_t)L1 + (L0 != 0u));
  o0 = (uint32_t)t;
  o1 = (uint32_t)(t >> 32) + L2;
}

template <int MODE>  // 0: the stage; 1: matrix cores alone; 2: VALU alone
__global__ __launch_bounds__(256) void k_stage63(const uint2 *__restrict__ in, uint2 *__restrict__ out,
                                                 const uint4 *__restrict__ ht, int reps, size_t nvec) {
  __shared__ uint4 sh[16 * 64];  // 16 A fragments (q, ks), 16 KB
  for (int i = threadIdx.x; i < 16 * 64; i += 256) sh[i] = ht[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
  const size_t vec = ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 32 + r;
  if (vec >= nvec) return;
  v4i B[4];  // k-step ks: elements 4 ks + 2 h, +1
#pragma unroll
  for (int ks = 0; ks < 4; ks++) {
    const uint2 a = in[vec * 16 + 4 * ks + 2 * h], b = in[vec * 16 + 4 * ks + 2 * h + 1];
    const int2 da = digits2(a.x, a.y), db = digits2(b.x, b.y);
    B[ks] = v4i{da.x, da.y, db.x, db.y};
  }
  for (int rep = 0; rep < reps; rep++) {
    const bool last = rep + 1 == reps;
    v4i Bn[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      v16i acc = {0};
      if constexpr (MODE == 2) {
#pragma unroll
        for (int u = 0; u < 16; u++) acc[u] = B[u & 3][u >> 2] ^ (q * 0x1010101 + u);
      } else {
#pragma unroll
        for (int ks = 0; ks < 4; ks++) {
          const uint4 a = sh[(q * 4 + ks) * 64 + lane];
          acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(v4i{(int)a.x, (int)a.y, (int)a.z, (int)a.w}, B[ks], acc, 0, 0, 0);
        }
      }
      if constexpr (MODE == 1) {
        Bn[q] = v4i{acc[0] ^ acc[5], acc[1] ^ acc[9], acc[2] ^ acc[13], acc[3] ^ acc[15]};
      } else {
        uint32_t a0, a1, b0, b1;
        recombine63(acc, 0, a0, a1);
        recombine63(acc, 8, b0, b1);
        if (last) {
          // < p + 2^46: one conditional subtraction
          uint64_t x = ((uint64_t)a1 << 32) | a0, y = ((uint64_t)b1 << 32) | b0;
          if (x >= P64) x -= P64;
          if (y >= P64) y -= P64;
          out[vec * 16 + 4 * q + 2 * h] = make_uint2((uint32_t)x, (uint32_t)(x >> 32));
          out[vec * 16 + 4 * q + 2 * h + 1] = make_uint2((uint32_t)y, (uint32_t)(y >> 32));
        } else {
          const int2 da = digits2(a0, a1), db = digits2(b0, b1);
          Bn[q] = v4i{da.x, da.y, db.x, db.y};
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int ks = 0; ks < 4; ks++) B[ks] = Bn[ks];
  }
  if constexpr (MODE != 0) {  // keep the timed work live
    const v4i t = B[0] ^ B[1] ^ B[2] ^ B[3];
    out[vec * 16 + h] = make_uint2((uint32_t)(t.x ^ t.y), (uint32_t)(t.z ^ t.w));
  }
}

u128 mulm(u128 a, u128 b) { return (a * b) % P64; }
u128 powm(u128 a, uint64_t e) {
  u128 r = 1;
  while (e) {
    if (e & 1) r = mulm(r, a);
    a = mulm(a, a);
    e >>= 1;
  }
  return r;
}
}  // namespace

int main(int argc, char **argv) {
  const size_t nvec = argc > 1 ? (size_t)atol(argv[1]) : (size_t)1 << 20;
  const int reps = argc > 2 ? atoi(argv[2]) : 8;
  // ROOT_OF_UNITY of Ft63: g^((p-1)/2^41), g = 10 (lcpc-test-fields/src/lib.rs:18-22); w16 = its 2^37th power
  u128 w = powm(10, (P64 - 1) >> 41);
  for (int i = 0; i < 37; i++) w = mulm(w, w);
  if (powm(w, 16) != 1 || powm(w, 8) == 1) {
    printf("bad w16\n");
    return 2;
  }
  u128 W[16][16];
  for (int j = 0; j < 16; j++)
    for (int i = 0; i < 16; i++) W[j][i] = powm(w, (uint64_t)(i * j));
  std::vector<int8_t> ht(16 * 64 * 16);
  for (int q = 0; q < 4; q++)
    for (int ks = 0; ks < 4; ks++)
      for (int l = 0; l < 64; l++) {
        const int m = l & 31, hp = l >> 5;
        const int hm = (m >> 2) & 1, rg = (m & 3) + 4 * (m >> 3);
        const int o = 2 * hm + (rg >> 3), u = rg & 7, j = 4 * q + o;
        for (int d = 0; d < 16; d++) {
          const int i = 4 * ks + 2 * hp + (d >> 3), a = d & 7;
          const u128 H = mulm(W[j][i], powm(2, 8 * a + 32));
          // balanced digit u of H
          u128 c = 0;
          for (int k = 0; k < 8; k++) c |= (u128)0x80 << (8 * k);
          const u128 v = H + c;
          ht[((q * 4 + ks) * 64 + l) * 16 + d] = (int8_t)(uint8_t)(((v >> (8 * u)) & 0xff) ^ 0x80);
        }
      }
  std::vector<uint64_t> hin(nvec * 16);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  for (auto &x : hin) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    x = s % P64;
  }
  uint2 *din, *dout;
  uint4 *dht;
  CK(hipMalloc(&din, nvec * 128));
  CK(hipMalloc(&dout, nvec * 128));
  CK(hipMalloc(&dht, ht.size()));
  CK(hipMemcpy(din, hin.data(), nvec * 128, hipMemcpyHostToDevice));
  CK(hipMemcpy(dht, ht.data(), ht.size(), hipMemcpyHostToDevice));
  const unsigned blocks = (unsigned)((nvec + 127) / 128);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](int mode, int rp) {
    const int iters = 10;
    if (mode == 0) hipLaunchKernelGGL(k_stage63<0>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, rp, nvec);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int it = 0; it < iters; it++) {
      if (mode == 0) hipLaunchKernelGGL(k_stage63<0>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, rp, nvec);
      if (mode == 1) hipLaunchKernelGGL(k_stage63<1>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, rp, nvec);
      if (mode == 2) hipLaunchKernelGGL(k_stage63<2>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, rp, nvec);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
  };
  const float m1 = timeit(0, 1), m0 = timeit(0, reps), mm = timeit(1, reps), mv = timeit(2, reps);
  const double el = (double)nvec * 16;
  auto cyc = [&](float m) { return (m - m1) * 1e-3 / (reps - 1) / el * 2.4e9 * 1024; };
  hipLaunchKernelGGL(k_stage63<0>, dim3(blocks), dim3(256), 0, 0, din, dout, dht, reps, nvec);
  CK(hipDeviceSynchronize());
  std::vector<uint64_t> hout(nvec * 16);
  CK(hipMemcpy(hout.data(), dout, nvec * 128, hipMemcpyDeviceToHost));
  size_t bad = 0, checked = 0;
  for (size_t v = 0; v < nvec; v += nvec / 256 + 1) {
    u128 x[16], y[16];
    for (int i = 0; i < 16; i++) x[i] = hin[v * 16 + i];
    for (int rp = 0; rp < reps; rp++) {
      for (int j = 0; j < 16; j++) {
        u128 acc = 0;
        for (int i = 0; i < 16; i++) acc = (acc + mulm(W[j][i], x[i])) % P64;
        y[j] = acc;
      }
      for (int j = 0; j < 16; j++) x[j] = y[j];
    }
    for (int j = 0; j < 16; j++) {
      checked++;
      bad += (u128)hout[v * 16 + j] != x[j];
    }
  }
  printf("nttmfma63: %zu vectors x 16 Ft63, %d stages: whole stage %.2f, matrix cores alone %.2f, VALU alone %.2f "
         "SIMD-cycles per element per stage (nominal 2.4 GHz); check %zu/%zu %s\n",
         nvec, reps, cyc(m0), cyc(mm), cyc(mv), checked - bad, checked, bad ? "MISMATCH" : "exact");
  return bad ? 1 : 0;
}
