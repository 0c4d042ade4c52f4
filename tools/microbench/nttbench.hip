// nttbench.hip -- A/B harness for NTT pass variants on gfx950 (one process, interleaved
// rounds; outputs checked bit-for-bit against the product kernels, which the GPU parity tests
// pin to the CPU oracle).  Usage: ./nttbench [log_n] [rows]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "../../lcpc_proof_of_storage_amd/csrc/ntt_impl.hpp"

using namespace lcpc;

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <class F>
__global__ void k_fill(uint32_t *p, size_t n, uint32_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)i * 0x9E3779B9u ^ seed;
  x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
  p[i] = ((i % F::N) == F::N - 1) ? (x & 0x0fffffffu) : x;  // < p for every field
}

struct Variant {
  std::string name;
  std::function<void(const uint32_t *, uint32_t *, hipStream_t)> run;
};

template <class F>
void bench(const char *fname, int log_n, size_t rows, bool with_copy = false) {
  const size_t n = (size_t)1 << log_n, np = n / 2;
  const size_t W = F::N;
  uint32_t *coeffs, *ref, *out, *tw;
  CK(hipMalloc(&coeffs, rows * np * W * 4));
  CK(hipMalloc(&ref, rows * n * W * 4));
  CK(hipMalloc(&out, rows * n * W * 4));
  CK(hipMalloc(&tw, n * W * 4));
  uint32_t *cpy = nullptr;
  if (with_copy) CK(hipMalloc(&cpy, rows * np * W * 4));
  hipLaunchKernelGGL(k_fill<F>, dim3((rows * np * W + 255) / 256), dim3(256), 0, 0, coeffs, rows * np * W, 12345u);
  hipLaunchKernelGGL((ntt_detail::k_tw_table<F>), dim3((n + 255) / 256), dim3(256), 0, 0, tw, log_n, 0);
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreate(&s));
  // pass A's [t][c] inter-pass twiddles, one table per pass-A split
  std::map<int, uint32_t *> tw2s;
  auto tw2_for = [&](int l1) {
    uint32_t *&t2 = tw2s[l1];
    if (!t2) {
      // (the same permutation as ntt.hip's ntt_tw2_table, done on the host here)
      std::vector<uint32_t> h(n * W), h2(n * W);
      CK(hipMemcpy(h.data(), tw, n * W * 4, hipMemcpyDeviceToHost));
      const int l2 = log_n - l1;
      for (size_t t = 0; t < ((size_t)1 << l1); t++) {
        size_t bt = 0;
        for (int b = 0; b < l1; b++) bt |= ((t >> b) & 1) << (l1 - 1 - b);
        for (size_t c = 0; c < ((size_t)1 << l2); c++)
          std::memcpy(&h2[((t << l2) + c) * W], &h[c * bt * W], W * 4);
      }
      CK(hipMalloc(&t2, n * W * 4));
      CK(hipMemcpy(t2, h2.data(), n * W * 4, hipMemcpyHostToDevice));
    }
    return t2;
  };
  NttPlan plan;
  plan.fid = F::ID; plan.log_n = log_n; plan.l1 = log_n / 2; plan.l2 = log_n - plan.l1; plan.d_tw = tw;
  plan.d_tw2 = tw2_for(plan.l1);
  CK(ntt_detail::ntt_rows_t<F>(plan, coeffs, np, np, ref, n, rows, s, nullptr, 0, false));
  CK(hipStreamSynchronize(s));

  std::vector<Variant> vs;
  vs.push_back({"product (ntt_rows_t)", [&](const uint32_t *c, uint32_t *o, hipStream_t st) {
                  CK(ntt_detail::ntt_rows_t<F>(plan, c, np, np, o, n, rows, st, nullptr, 0, false));
                }});
#define V2(LA, CWA, TA, LB, CWB, TB)                                                           \
  vs.push_back({"v2 A(S=2^" #LA ",CW=2^" #CWA ",T=2^" #TA ") B(S=2^" #LB ",CW=2^" #CWB ",T=2^" #TB ")", \
                [&](const uint32_t *c, uint32_t *o, hipStream_t st) {                          \
                  CK((ntt_v2::launch_a<F, LA, CWA, TA, true>(c, np, np, o, n, tw, log_n, rows, st, cpy, np,  \
                                                             tw2_for(LA))));                    \
                  CK((ntt_v2::launch_b<F, LB, CWB, TB>(o, n, tw, log_n, rows, st)));           \
                }});
  if constexpr (F::ID == 1) {
    if (log_n == 16) {
      V2(8, 3, 8, 8, 3, 8)
      V2(8, 2, 7, 8, 2, 7)
      V2(8, 2, 8, 8, 2, 8)
      V2(8, 3, 9, 8, 3, 9)
      V2(8, 1, 7, 8, 1, 7)
      V2(8, 4, 9, 8, 3, 8)
      V2(8, 3, 8, 8, 4, 9)
      V2(7, 3, 7, 9, 2, 8)
      V2(7, 4, 8, 9, 2, 8)
      V2(6, 4, 7, 10, 1, 8)
    } else if (log_n == 14) {  // cfg2 (128 rows): the product shape first, then occupancy / tile sweeps
      V2(7, 4, 8, 7, 4, 8)
      V2(7, 3, 7, 7, 3, 7)
      V2(7, 2, 6, 7, 2, 6)
      V2(7, 4, 9, 7, 4, 9)
      V2(7, 3, 8, 7, 3, 8)
      V2(7, 2, 7, 7, 2, 7)
      V2(7, 5, 9, 7, 5, 9)
      V2(7, 5, 10, 7, 5, 10)
      V2(7, 3, 7, 7, 4, 8)
      V2(7, 4, 8, 7, 3, 7)
      V2(7, 2, 6, 7, 3, 7)
    }
  } else if constexpr (F::ID == 0) {
    if (log_n == 15) {  // PoS default dims: l1 = 7, l2 = 8; pass-A shapes at a fixed pass B, then B
      V2(7, 5, 9, 8, 4, 9)
      V2(7, 3, 7, 8, 4, 9)
      V2(7, 3, 8, 8, 4, 9)
      V2(7, 4, 8, 8, 4, 9)
      V2(7, 4, 9, 8, 4, 9)
      V2(7, 5, 10, 8, 4, 9)
      V2(7, 6, 10, 8, 4, 9)
      V2(7, 2, 7, 8, 4, 9)
      V2(7, 5, 9, 8, 3, 8)
      V2(7, 5, 9, 8, 2, 7)
      V2(7, 5, 9, 8, 3, 9)
      V2(7, 5, 9, 8, 2, 8)
      V2(7, 5, 9, 8, 1, 7)
      // the other split, l1 = 8 (pass A over 256-point columns, pass B over 128-point blocks)
      V2(8, 4, 9, 7, 5, 9)
      V2(8, 4, 8, 7, 5, 9)
      V2(8, 3, 8, 7, 5, 9)
      V2(8, 5, 10, 7, 5, 9)
      V2(8, 4, 9, 7, 4, 9)
      V2(8, 4, 9, 7, 6, 10)
    } else if (log_n == 17) {  // PoS bench dims 65536 -> 131072: product l1 = 8 first, then l1 = 9
      V2(8, 4, 9, 9, 3, 9)
      V2(8, 5, 10, 9, 3, 9)
      V2(8, 4, 9, 9, 2, 8)
      V2(9, 3, 9, 8, 4, 9)
      V2(9, 3, 9, 8, 5, 10)
      V2(9, 2, 8, 8, 4, 9)
      V2(9, 4, 10, 8, 4, 9)
      V2(9, 3, 9, 8, 3, 8)
    } else {
      V2(8, 4, 8, 8, 4, 8)
      V2(8, 3, 8, 8, 3, 8)
      V2(8, 4, 9, 8, 4, 9)
      V2(8, 5, 9, 8, 5, 9)
      V2(8, 3, 7, 8, 3, 7)
    }
  } else {
    V2(8, 2, 8, 9, 1, 8)
    V2(8, 3, 8, 9, 2, 8)
    V2(8, 2, 7, 9, 1, 7)
    V2(8, 1, 7, 9, 1, 8)
    V2(8, 3, 9, 9, 2, 9)
  }
  std::vector<uint32_t> h_ref(rows * n * W), h_out(rows * n * W);
  CK(hipMemcpy(h_ref.data(), ref, h_ref.size() * 4, hipMemcpyDeviceToHost));
  std::vector<std::vector<float>> times(vs.size());
  std::vector<bool> ok(vs.size(), true);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (size_t i = 0; i < vs.size(); i++) {  // correctness
    CK(hipMemset(out, 0, rows * n * W * 4));
    vs[i].run(coeffs, out, s);
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h_out.data(), out, h_out.size() * 4, hipMemcpyDeviceToHost));
    ok[i] = h_out == h_ref;
  }
  for (int round = 0; round < 7; round++)
    for (size_t i = 0; i < vs.size(); i++) {
      CK(hipEventRecord(a, s));
      vs[i].run(coeffs, out, s);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (round > 0) times[i].push_back(ms);
    }
  const double bytes = (double)rows * (np + n) * W * 4;
  printf("%s log_n=%d rows=%zu  algorithmic bytes %.1f MiB\n", fname, log_n, rows, bytes / 1048576);
  for (size_t i = 0; i < vs.size(); i++) {
    auto t = times[i];
    std::sort(t.begin(), t.end());
    printf("%-52s %s  median %.3f ms  min %.3f ms  (%.0f GB/s algorithmic)\n", vs[i].name.c_str(),
           ok[i] ? "OK " : "BAD", t[t.size() / 2], t[0], bytes / (t[t.size() / 2] * 1e-3) / 1e9);
  }
}

int main(int argc, char **argv) {
  const int which = argc > 1 ? atoi(argv[1]) : 1;
  if (which == 1) { bench<Ft127>("Ft127", 16, 512); bench<Ft127>("Ft127", 14, 128); }
  if (which == 2) bench<Ft127>("Ft127 cfg2", 14, 128);
  if (which == 0) bench<Ft63>("Ft63", 16, 512);
  if (which == 5) bench<Ft63>("Ft63 PoS 1 GiB (copy)", 15, 9363, true);
  if (which == 7) bench<Ft63>("Ft63 PoS bench dims (copy)", 17, 2341, true);
  if (which == 3) bench<Ft255>("Ft255", 17, 256);
  return 0;
}
