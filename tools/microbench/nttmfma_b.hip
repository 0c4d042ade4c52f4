// nttmfma_b.hip -- the Ligero encode's pass B (k_pass_b: the 256-point DIF of every contiguous
// block, bit-reversed output) on the int8 matrix cores, against a host big-int reference.
//
// Block x[c], c = c0 + 16 c1 (integers < p):
//   stage 1: u_c0[k1] = sum_c1 x[c0 + 16 c1] w16^(c1 k1)          (MFMA, W16, shared)
//   twiddle: u_c0[k1] *= w256^(c0 k1)                               (VALU Montgomery product)
//   stage 2: v_k1[k2] = sum_c0 u_c0[k1] w16^(c0 k2)                 (MFMA, W16)
//   out[bitrev4(k2) + 16 bitrev4(k1)] = v_k1[k2]                    (= fft_io's bitrev8(k1 + 16 k2))
// Each MFMA stage: v_mfma_i32_32x32x32_i8 with A = the digit table of W16 2^(8a) 2^32 (rows = 2
// outputs x 16 digit positions, so a lane holds all 16 partials of one output), B = 32 vectors'
// balanced digits; per output one recombination + one Montgomery word step (nttmfma.hip).
// Workgroup: 8 waves, a tile of 8 blocks (2048 elements) in LDS; wave w computes output pair w
// (outputs 2w, 2w + 1) of every vector of the tile in both stages, its 8 A fragments (32 VGPRs)
// loaded once.  The tile: HBM -> digits in LDS -> stage 1 -> twiddle -> digits in LDS -> stage 2
// -> canonical values in LDS (bit-reversed positions) -> HBM, contiguous.
// Build: hipcc -O3 --offload-arch=gfx950 -mllvm --amdgpu-mfma-vgpr-form -I../../lcpc_proof_of_storage_amd/csrc
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "f127_host.hpp"
#include "field.hpp"

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
using lcpc::Fe;
using lcpc::Ft127;

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

// (sum_u Y_u 2^(8u) + OFF + m p) / 2^32, < p + 2^114 (nttmfma.hip)
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
#pragma unroll
    for (int i = 0; i < 4; i++) x[i] = u[i];
}

constexpr int BLK = 8;                 // blocks per tile
constexpr int NV = BLK * 16;           // vectors per stage
constexpr int VPITCH = 17;             // 16-byte slots per vector row in LDS (one pad slot)

// ht: W16 digit fragments [p][ks][lane] (uint4); tw: w256^(c0 k1) R mod p at [c0][k1] (Montgomery).
// PP output pairs per wave (8 / PP waves): every B fragment read from LDS feeds PP matrix-core ops.
template <int PP>
__global__ __launch_bounds__(64 * 8 / PP) void k_pass_b_mfma(uint4 *__restrict__ data, const uint4 *__restrict__ ht,
                                                             const uint4 *__restrict__ tw, size_t n_blocks) {
  constexpr int NT = 64 * 8 / PP;
  __shared__ uint4 s_in[NV * VPITCH];   // digits, [vector][element]
  __shared__ uint4 s_mid[NV * VPITCH];  // stage-2 digits, then the output values
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const size_t blk0 = (size_t)blockIdx.x * BLK;
  uint4 *io = data + blk0 * 256;
  v4i A[PP][8];
#pragma unroll
  for (int pp = 0; pp < PP; pp++)
#pragma unroll
    for (int ks = 0; ks < 8; ks++) {
      const uint4 a = ht[((wave * PP + pp) * 8 + ks) * 64 + lane];
      A[pp][ks] = v4i{(int)a.x, (int)a.y, (int)a.z, (int)a.w};
    }
  for (int e = tid; e < BLK * 256; e += NT) {
    const int b = e >> 8, c = e & 255;
    const uint4 q = io[e];
    const uint32_t x[4] = {q.x, q.y, q.z, q.w};
    const v4i d = digits(x);
    s_in[((b << 4) + (c & 15)) * VPITCH + (c >> 4)] = make_uint4(d.x, d.y, d.z, d.w);
  }
  __syncthreads();
#pragma unroll 1
  for (int q = 0; q < NV / 32; q++) {
    const int v = q * 32 + r, c0 = v & 15, b = v >> 4;
    v16i acc[PP];
#pragma unroll
    for (int pp = 0; pp < PP; pp++) acc[pp] = v16i{0};
#pragma unroll
    for (int ks = 0; ks < 8; ks++) {
      const uint4 d = s_in[v * VPITCH + 2 * ks + h];
      const v4i dv = v4i{(int)d.x, (int)d.y, (int)d.z, (int)d.w};
#pragma unroll
      for (int pp = 0; pp < PP; pp++) acc[pp] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[pp][ks], dv, acc[pp], 0, 0, 0);
    }
#pragma unroll
    for (int pp = 0; pp < PP; pp++) {
      const int k1 = 2 * (wave * PP + pp) + h;
      uint32_t y[4];
      recombine(acc[pp], y);
      Fe<Ft127> u, t;
#pragma unroll
      for (int i = 0; i < 4; i++) u.v[i] = y[i];
      const uint4 tq = tw[c0 * 16 + k1];
      t.v[0] = tq.x, t.v[1] = tq.y, t.v[2] = tq.z, t.v[3] = tq.w;
      const Fe<Ft127> z = lcpc::fe_mul<Ft127>(u, t);
      const uint32_t zz[4] = {z.v[0], z.v[1], z.v[2], z.v[3]};
      const v4i dz = digits(zz);
      s_mid[((b << 4) + k1) * VPITCH + c0] = make_uint4(dz.x, dz.y, dz.z, dz.w);
    }
  }
  __syncthreads();
  uint4 res[NV / 32][PP];
#pragma unroll 1
  for (int q = 0; q < NV / 32; q++) {
    const int v = q * 32 + r;
    v16i acc[PP];
#pragma unroll
    for (int pp = 0; pp < PP; pp++) acc[pp] = v16i{0};
#pragma unroll
    for (int ks = 0; ks < 8; ks++) {
      const uint4 d = s_mid[v * VPITCH + 2 * ks + h];
      const v4i dv = v4i{(int)d.x, (int)d.y, (int)d.z, (int)d.w};
#pragma unroll
      for (int pp = 0; pp < PP; pp++) acc[pp] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[pp][ks], dv, acc[pp], 0, 0, 0);
    }
#pragma unroll
    for (int pp = 0; pp < PP; pp++) {
      uint32_t y[4];
      recombine(acc[pp], y);
      reduce_p(y);
      res[q][pp] = make_uint4(y[0], y[1], y[2], y[3]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NV / 32; q++)
#pragma unroll
    for (int pp = 0; pp < PP; pp++) {
      const int v = q * 32 + r, b = v >> 4, kk1 = v & 15, k2 = 2 * (wave * PP + pp) + h;
      const int pos = (__builtin_bitreverse32((uint32_t)k2) >> 28) + 16 * (__builtin_bitreverse32((uint32_t)kk1) >> 28);
      s_mid[b * 256 + pos] = res[q][pp];
    }
  __syncthreads();
  for (int e = tid; e < BLK * 256; e += NT) io[e] = s_mid[e];
}
}  // namespace

int main(int argc, char **argv) {
  using namespace f127h;
  const size_t n_blocks = argc > 1 ? (size_t)atol(argv[1]) : (size_t)512 * 256;  // cfg3: 512 rows x 256 blocks
  const u128 w256 = root_of_order(8), w16 = mul(mul(pow(w256, 4), pow(w256, 4)), mul(pow(w256, 4), pow(w256, 4)));
  // W16 fragments: frag (p, ks), lane l = m + 32 h': byte a = h_u(W[j][i] 2^(8a) 2^32), j = 2p + ((m>>2)&1),
  // u = (m&3) + 4(m>>3), i = 2ks + h'
  std::vector<int8_t> ht(64 * 64 * 16);
  u128 s2a[16];
  for (int a = 0; a < 16; a++) s2a[a] = two_pow(8 * a + 32);
  for (int p = 0; p < 8; p++)
    for (int ks = 0; ks < 8; ks++)
      for (int l = 0; l < 64; l++) {
        const int m = l & 31, hp = l >> 5;
        const int j = 2 * p + ((m >> 2) & 1), u = (m & 3) + 4 * (m >> 3), i = 2 * ks + hp;
        const u128 wji = pow(w16, (u128)(i * j));
        for (int a = 0; a < 16; a++) {
          int8_t d[16];
          balanced(mul(wji, s2a[a]), d);
          ht[((p * 8 + ks) * 64 + l) * 16 + a] = d[u];
        }
      }
  // twiddles w256^(c0 k1), Montgomery form (x R mod p, R = 2^128)
  const u128 R = add(two_pow(127), two_pow(127));
  std::vector<uint32_t> htw(256 * 4);
  for (int c0 = 0; c0 < 16; c0++)
    for (int k1 = 0; k1 < 16; k1++) to_words(mul(pow(w256, (u128)(c0 * k1)), R), &htw[(c0 * 16 + k1) * 4]);
  std::vector<u128> wpow(256);
  for (int e = 0; e < 256; e++) wpow[e] = pow(w256, (u128)e);
  std::vector<uint32_t> hin(n_blocks * 256 * 4);
  uint64_t s = 0x9e3779b97f4a7c15ull;
  auto rnd = [&]() {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    return s;
  };
  for (size_t e = 0; e < n_blocks * 256; e++) to_words((((u128)rnd() << 64) | rnd()) % P, &hin[e * 4]);
  uint4 *d, *dht, *dtw;
  CK(hipMalloc(&d, hin.size() * 4));
  CK(hipMalloc(&dht, ht.size()));
  CK(hipMalloc(&dtw, htw.size() * 4));
  CK(hipMemcpy(dht, ht.data(), ht.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dtw, htw.data(), htw.size() * 4, hipMemcpyHostToDevice));
  const unsigned grid = (unsigned)(n_blocks / BLK);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  size_t bad = 0, checked = 0;
  const double el = (double)n_blocks * 256;
  for (int pp : {1, 2, 4}) {
    float best = 1e9;
    for (int it = 0; it < 5; it++) {
      CK(hipMemcpy(d, hin.data(), hin.size() * 4, hipMemcpyHostToDevice));
      CK(hipEventRecord(e0));
      if (pp == 1) hipLaunchKernelGGL(k_pass_b_mfma<1>, dim3(grid), dim3(512), 0, 0, d, dht, dtw, n_blocks);
      if (pp == 2) hipLaunchKernelGGL(k_pass_b_mfma<2>, dim3(grid), dim3(256), 0, 0, d, dht, dtw, n_blocks);
      if (pp == 4) hipLaunchKernelGGL(k_pass_b_mfma<4>, dim3(grid), dim3(128), 0, 0, d, dht, dtw, n_blocks);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    std::vector<uint32_t> hout(hin.size());
    CK(hipMemcpy(hout.data(), d, hout.size() * 4, hipMemcpyDeviceToHost));
    size_t b0 = bad;
    for (size_t b = 0; b < n_blocks; b += n_blocks / 2 + 1) {
      u128 x[256];
      for (int c = 0; c < 256; c++) x[c] = from_words(&hin[(b * 256 + c) * 4]);
      for (int k = 0; k < 256; k += 5) {
        u128 acc = 0;
        for (int c = 0; c < 256; c++) acc = add(acc, mul(x[c], wpow[(c * k) & 255]));
        const int pos = (int)(__builtin_bitreverse32((uint32_t)k) >> 24);
        checked++;
        if (from_words(&hout[(b * 256 + pos) * 4]) != acc) bad++;
      }
    }
    printf("pass B (MFMA, %d output pairs per wave): %zu blocks of 256: %.3f ms, %.1f G elements/s, %.2f SIMD-cycles "
           "per element (nominal 2.4 GHz); check %s\n",
           pp, n_blocks, best, el / best / 1e6, best * 1e-3 / el * 2.4e9 * 1024, bad == b0 ? "exact" : "MISMATCH");
    fflush(stdout);
  }
  printf("checked %zu outputs, %zu wrong\n", checked, bad);
  return bad ? 1 : 0;
}
