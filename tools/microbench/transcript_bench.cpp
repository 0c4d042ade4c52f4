// transcript_bench.cpp -- host throughput of the Merlin transcript (append_messages of 16-byte
// field reprs, as prove absorbs p_random / p_eval) and of bare Keccak-f[1600].
// Build: g++ -O3 -march=x86-64-v3 -I../../lcpc_proof_of_storage_amd/csrc transcript_bench.cpp \
//        ../../lcpc_proof_of_storage_amd/csrc/transcript.cpp -o transcript_bench
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "transcript.hpp"

using namespace lcpc;

int main() {
  const size_t n = 1 << 20;
  std::vector<uint8_t> msgs(n * 16);
  for (size_t i = 0; i < msgs.size(); i++) msgs[i] = (uint8_t)(i * 2654435761u >> 13);
  Transcript tr((const uint8_t *)"bench", 5);
  auto t0 = std::chrono::steady_clock::now();
  tr.append_messages((const uint8_t *)"$l//PR", 6, msgs.data(), 16, n);
  auto t1 = std::chrono::steady_clock::now();
  uint8_t out[32];
  tr.challenge_bytes((const uint8_t *)"x", 1, out, 32);
  const double ns = std::chrono::duration<double, std::nano>(t1 - t0).count() / n;
  uint64_t st[25] = {1};
  const int reps = 1 << 20;
  auto t2 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; i++) keccak_f1600(st);
  auto t3 = std::chrono::steady_clock::now();
  const double kns = std::chrono::duration<double, std::nano>(t3 - t2).count() / reps;
  printf("append_messages: %.2f ns per 16-byte element; keccak_f1600: %.1f ns; check %02x%02x %llx\n", ns, kns,
         out[0], out[1], (unsigned long long)st[0]);
  return 0;
}
