// leafbench.hip -- where the column-leaf BLAKE3 kernel's time goes, at the PoS dims (Ft63,
// 9363 x 32768) and cfg3 (Ft127, 512 x 65536): the library kernel, a loads-only twin (same
// grid, same addresses, XOR instead of compress), a compute-only twin (same grid, messages from
// registers), and a two-columns-per-lane variant (16-B loads for Ft63, two interleaved
// compressions), whose chaining values are compared with the library's.
// Build: hipcc -O3 -std=c++20 --offload-arch=gfx950 leafbench.hip ../../lcpc_proof_of_storage_amd/csrc/prof.cpp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <functional>
#include <vector>

#include "../../lcpc_proof_of_storage_amd/csrc/blake3.hip"

using namespace lcpc;
namespace lcpc {
int field_words(int fid) { return fid == 0 ? 2 : fid == 1 ? 4 : fid == 2 ? 6 : 8; }
}  // namespace lcpc

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

namespace lcpc {
namespace {

// interior chunks only (chunk >= 1 and full), as the library's fast path
template <class F>
__global__ __launch_bounds__(256) void v_loads_only(const uint32_t *__restrict__ m, size_t n_rows, size_t n_cols,
                                                    uint32_t *__restrict__ cvs, int n_full) {
  constexpr int N = F::N, EPB = 16 / N;
  const size_t col = (size_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int chunk = 1 + blockIdx.y * 4 + (threadIdx.x >> 6);
  if (col >= n_cols || chunk > n_full) return;
  const size_t r_first = ((size_t)chunk * 256 - 8) / N;
  const uint32_t *colp = m + col * N;
  size_t e = r_first * n_cols;
  uint32_t acc[8] = {};
  for (int b = 0; b < 16; b++) {
    Fe<F> el[EPB];
#pragma unroll
    for (int k = 0; k < EPB; k++) el[k] = fe_load<F>(colp, e + k * n_cols);
    e += EPB * n_cols;
#pragma unroll
    for (int k = 0; k < EPB; k++)
#pragma unroll
      for (int i = 0; i < N; i++) acc[(k * N + i) & 7] ^= el[k].v[i];
  }
  store8(cvs + ((size_t)chunk * n_cols + col) * 8, acc);
}

template <class F>
__global__ __launch_bounds__(256) void v_compute_only(size_t n_cols, uint32_t *__restrict__ cvs, int n_full) {
  const size_t col = (size_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int chunk = 1 + blockIdx.y * 4 + (threadIdx.x >> 6);
  if (col >= n_cols || chunk > n_full) return;
  uint32_t cv[8], msg[16];
  iv(cv);
#pragma unroll
  for (int i = 0; i < 16; i++) msg[i] = (uint32_t)col * 0x9E3779B9u + i * 77 + chunk;
  for (int b = 0; b < 16; b++) {
    compress(cv, msg, (uint64_t)chunk, 64u, b == 0 ? CHUNK_START : b == 15 ? CHUNK_END : 0u);
    msg[b & 15] ^= cv[b & 7];
  }
  store8(cvs + ((size_t)chunk * n_cols + col) * 8, cv);
}

// two adjacent columns per lane: one 2N-word load per row, two compressions interleaved
template <class F>
__global__ __launch_bounds__(256) void v_two_cols(const uint32_t *__restrict__ m, size_t n_rows, size_t n_cols,
                                                  uint32_t *__restrict__ cvs, int n_full) {
  constexpr int N = F::N, EPB = 16 / N;
  const size_t col = 2 * ((size_t)blockIdx.x * 64 + (threadIdx.x & 63));
  const int chunk = 1 + blockIdx.y * 4 + (threadIdx.x >> 6);
  if (col >= n_cols || chunk > n_full) return;
  const size_t r_first = ((size_t)chunk * 256 - 8) / N;
  const uint32_t *colp = m + col * N;
  size_t e = r_first * n_cols * N;
  uint32_t cva[8], cvb[8];
  iv(cva);
  iv(cvb);
  for (int b = 0; b < 16; b++) {
    uint32_t ma[16], mb[16];
#pragma unroll
    for (int k = 0; k < EPB; k++) {
      if constexpr (N == 2) {
        const uint4 v = *reinterpret_cast<const uint4 *>(colp + e + (size_t)k * n_cols * N);
        ma[2 * k] = v.x; ma[2 * k + 1] = v.y; mb[2 * k] = v.z; mb[2 * k + 1] = v.w;
      } else {
        const uint4 v0 = *reinterpret_cast<const uint4 *>(colp + e + (size_t)k * n_cols * N);
        const uint4 v1 = *reinterpret_cast<const uint4 *>(colp + e + (size_t)k * n_cols * N + 4);
        ma[4 * k] = v0.x; ma[4 * k + 1] = v0.y; ma[4 * k + 2] = v0.z; ma[4 * k + 3] = v0.w;
        mb[4 * k] = v1.x; mb[4 * k + 1] = v1.y; mb[4 * k + 2] = v1.z; mb[4 * k + 3] = v1.w;
      }
    }
    e += (size_t)EPB * n_cols * N;
    const uint32_t fl = b == 0 ? CHUNK_START : b == 15 ? CHUNK_END : 0u;
    compress(cva, ma, (uint64_t)chunk, 64u, fl);
    compress(cvb, mb, (uint64_t)chunk, 64u, fl);
  }
  store8(cvs + ((size_t)chunk * n_cols + col) * 8, cva);
  store8(cvs + ((size_t)chunk * n_cols + col + 1) * 8, cvb);
}

}  // namespace
}  // namespace lcpc

struct Timer {
  hipEvent_t a, b;
  hipStream_t s;
  Timer(hipStream_t s_) : s(s_) {
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
  }
  float time(const std::function<void()> &fn, int reps) {
    fn();
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < reps; i++) fn();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
  }
};

template <class F>
void run(const char *name, size_t n_rows, size_t n_cols, hipStream_t s) {
  constexpr int N = F::N;
  const size_t words = n_rows * n_cols * N;
  uint32_t *cw, *cvs, *cvs2, *scratch;
  uint8_t *leaves;
  CK(hipMalloc(&cw, words * 4));
  std::vector<uint32_t> h(words);
  uint64_t x = 88172645463325252ull;
  for (size_t i = 0; i < words; i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    h[i] = (uint32_t)x;
  }
  // canonical values: clear the top bits of every element so each is < p
  for (size_t i = N - 1; i < words; i += N) h[i] &= 0x0fffffffu;
  CK(hipMemcpy(cw, h.data(), words * 4, hipMemcpyHostToDevice));
  const size_t total_words = 8 + n_rows * N;
  const int n_chunks = (int)((total_words + 255) / 256);
  const int n_full = (int)(total_words / 256) - 1;  // interior full chunks 1..n_full
  CK(hipMalloc(&cvs, (size_t)(n_chunks + 1) * n_cols * 32));
  CK(hipMalloc(&cvs2, (size_t)(n_chunks + 1) * n_cols * 32));
  CK(hipMalloc(&scratch, leaf_hash_scratch_bytes(F::ID, n_rows, n_cols) + 64));
  CK(hipMalloc(&leaves, n_cols * 32));
  Timer tm(s);
  const int reps = 10;
  const double bytes = (double)n_rows * n_cols * N * 4;
  dim3 grid((unsigned)((n_cols + 63) / 64), (unsigned)((n_chunks + 3) / 4));
  float ms = tm.time([&]() { CK(leaf_hashes(F::ID, cw, n_rows, n_cols, n_cols, leaves, scratch, s, true)); }, reps);
  printf("%s library leaves total        %.4f ms (%.2f TB/s)\n", name, ms, bytes / ms / 1e9);
  ms = tm.time([&]() {
    // (the library's grid: a block = 4 waves on 256 adjacent columns of one chunk)
    hipLaunchKernelGGL((k_leaf_chunks<F, true>), dim3((unsigned)((n_cols + 255) / 256), (unsigned)n_chunks),
                       dim3(256), 0, s, cw, n_rows, n_cols, n_cols, (size_t)1, cvs, leaves, n_chunks, (size_t)0, 0,
                       n_chunks, (size_t)0);
  }, reps);
  printf("%s library k_leaf_chunks       %.4f ms (%.2f TB/s)\n", name, ms, bytes / ms / 1e9);
  dim3 gi((unsigned)((n_cols + 63) / 64), (unsigned)((n_full + 3) / 4));
  const double ibytes = (double)n_full * 1024 * n_cols;
  ms = tm.time([&]() { hipLaunchKernelGGL((v_loads_only<F>), gi, dim3(256), 0, s, cw, n_rows, n_cols, cvs2, n_full); }, reps);
  printf("%s interior loads only         %.4f ms (%.2f TB/s)\n", name, ms, ibytes / ms / 1e9);
  ms = tm.time([&]() { hipLaunchKernelGGL((v_compute_only<F>), gi, dim3(256), 0, s, n_cols, cvs2, n_full); }, reps);
  printf("%s interior compress only      %.4f ms (%.1f G compress/s)\n", name, ms,
         (double)n_full * 16 * n_cols / ms / 1e6);
  dim3 g2((unsigned)((n_cols / 2 + 63) / 64), (unsigned)((n_full + 3) / 4));
  ms = tm.time([&]() { hipLaunchKernelGGL((v_two_cols<F>), g2, dim3(256), 0, s, cw, n_rows, n_cols, cvs2, n_full); }, reps);
  CK(hipStreamSynchronize(s));
  // compare interior chaining values with the library's
  std::vector<uint32_t> a((size_t)(n_chunks + 1) * n_cols * 8), b(a.size());
  CK(hipMemcpy(a.data(), cvs, a.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), cvs2, b.size() * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (int c = 1; c <= n_full; c++)
    for (size_t i = 0; i < n_cols * 8; i++) bad += a[(size_t)c * n_cols * 8 + i] != b[(size_t)c * n_cols * 8 + i];
  printf("%s interior two cols per lane  %.4f ms (%.2f TB/s)  %s\n", name, ms, ibytes / ms / 1e9,
         bad ? "MISMATCH" : "cvs match");
  CK(hipFree(cw));
  CK(hipFree(cvs));
  CK(hipFree(cvs2));
  CK(hipFree(scratch));
  CK(hipFree(leaves));
}

int main() {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  run<Ft63>("pos Ft63 9363x32768", 9363, 32768, s);
  run<Ft127>("cfg3 Ft127 512x65536", 512, 65536, s);
  return 0;
}
