// bench_native.cpp -- the bench.py step loop driven from C++ threads through the C ABI only
// (no Python): isolates host-side serialization from the Python layer.
// Usage: bench_native [pipeline] [steps] [log_len]
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/lcpc_mi.h"

#define CK(x)                                                                            \
  do {                                                                                   \
    int rc = (int)(x);                                                                   \
    if (rc) {                                                                            \
      printf("error %d at %s:%d: %s\n", rc, __FILE__, __LINE__, lcpc_last_error());      \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

int main(int argc, char **argv) {
  const int pipeline = argc > 1 ? atoi(argv[1]) : 4;
  const int steps = argc > 2 ? atoi(argv[2]) : 16;
  const int log_len = argc > 3 ? atoi(argv[3]) : 24;
  const size_t n = (size_t)1 << log_len;
  CK(lcpc_set_device(0));
  lcpc_encoding *enc = nullptr;
  CK(lcpc_ligero_new(LCPC_FT127, 1, 2, n, &enc));
  size_t nr, np, nc;
  lcpc_encoding_get_dims(enc, n, &nr, &np, &nc);
  std::vector<uint64_t> coeffs(2 * n), outer(2 * nr);
  CK(lcpc_field_random(LCPC_FT127, 0x1CDC2024, coeffs.data(), n));
  CK(lcpc_field_random(LCPC_FT127, 7, outer.data(), nr));
  void *d = nullptr;
  if (hipMalloc(&d, 16 * n) != hipSuccess) return 1;
  if (hipMemcpy(d, coeffs.data(), 16 * n, hipMemcpyHostToDevice) != hipSuccess) return 1;
  const size_t nco = lcpc_encoding_n_col_opens(enc);
  auto step = [&]() {
    lcpc_commit *c = nullptr;
    CK(lcpc_commit_new_device(enc, d, n, &c));
    uint8_t root[32];
    CK(lcpc_commit_get_root(c, root));
    const char *lab = "test transcript";
    lcpc_transcript *tr = lcpc_transcript_new((const uint8_t *)lab, strlen(lab));
    lcpc_transcript_append_message(tr, (const uint8_t *)"polycommit", 10, root, 32);
    uint8_t be[8];
    for (int i = 0; i < 8; i++) be[i] = (uint8_t)(nco >> (56 - 8 * i));
    lcpc_transcript_append_message(tr, (const uint8_t *)"ncols", 5, be, 8);
    lcpc_proof *p = nullptr;
    CK(lcpc_prove(c, outer.data(), nr, enc, tr, &p));
    lcpc_proof_free(p);
    lcpc_transcript_free(tr);
    lcpc_commit_free(c);
  };
  // persistent workers: each warms up (pinned staging, pool blocks) before the timed region
  std::atomic<int> ready(0), todo(steps);
  std::atomic<bool> go(false);
  std::chrono::steady_clock::time_point t0;
  std::vector<std::thread> th;
  for (int t = 0; t < pipeline; t++)
    th.emplace_back([&]() {
      step();
      ready.fetch_add(1);
      while (!go.load()) std::this_thread::yield();
      while (todo.fetch_sub(1) > 0) step();
    });
  while (ready.load() < pipeline) std::this_thread::yield();
  (void)hipDeviceSynchronize();
  t0 = std::chrono::steady_clock::now();
  go.store(true);
  for (auto &x : th) x.join();
  (void)hipDeviceSynchronize();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("pipeline %d: %d steps in %.3f s -> %.3f ms/step, %.3f G elem/s\n", pipeline, steps, s,
         1e3 * s / steps, steps * (double)n / s / 1e9);
  return 0;
}
