// keccak_variants.cpp -- Keccak-f[1600] schedules on the host CPU (A/B for transcript.cpp).
// Each variant is checked against the library's scalar permutation, then timed.
// Build: clang++ -O3 -std=c++20 -march=x86-64-v3 -I../../lcpc_proof_of_storage_amd/csrc \
//        keccak_variants.cpp ../../lcpc_proof_of_storage_amd/csrc/transcript.cpp -o keccak_variants
#include <immintrin.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "transcript.hpp"

namespace {
constexpr uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
    0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

// D form: theta's five D[x] are formed first (the column parities die there), so at most
// 25 lanes + 5 D values are live when b = rol(a ^ D) replaces each lane: no spills of the
// 32 vector registers.
__attribute__((target("avx512f,avx512vl"))) void keccak_avx512_d(uint64_t s[25]) {
  __m128i a00 = _mm_cvtsi64_si128((long long)s[0]);
  __m128i a01 = _mm_cvtsi64_si128((long long)s[1]);
  __m128i a02 = _mm_cvtsi64_si128((long long)s[2]);
  __m128i a03 = _mm_cvtsi64_si128((long long)s[3]);
  __m128i a04 = _mm_cvtsi64_si128((long long)s[4]);
  __m128i a05 = _mm_cvtsi64_si128((long long)s[5]);
  __m128i a06 = _mm_cvtsi64_si128((long long)s[6]);
  __m128i a07 = _mm_cvtsi64_si128((long long)s[7]);
  __m128i a08 = _mm_cvtsi64_si128((long long)s[8]);
  __m128i a09 = _mm_cvtsi64_si128((long long)s[9]);
  __m128i a10 = _mm_cvtsi64_si128((long long)s[10]);
  __m128i a11 = _mm_cvtsi64_si128((long long)s[11]);
  __m128i a12 = _mm_cvtsi64_si128((long long)s[12]);
  __m128i a13 = _mm_cvtsi64_si128((long long)s[13]);
  __m128i a14 = _mm_cvtsi64_si128((long long)s[14]);
  __m128i a15 = _mm_cvtsi64_si128((long long)s[15]);
  __m128i a16 = _mm_cvtsi64_si128((long long)s[16]);
  __m128i a17 = _mm_cvtsi64_si128((long long)s[17]);
  __m128i a18 = _mm_cvtsi64_si128((long long)s[18]);
  __m128i a19 = _mm_cvtsi64_si128((long long)s[19]);
  __m128i a20 = _mm_cvtsi64_si128((long long)s[20]);
  __m128i a21 = _mm_cvtsi64_si128((long long)s[21]);
  __m128i a22 = _mm_cvtsi64_si128((long long)s[22]);
  __m128i a23 = _mm_cvtsi64_si128((long long)s[23]);
  __m128i a24 = _mm_cvtsi64_si128((long long)s[24]);
  for (int r = 0; r < 24; r++) {
    const __m128i c0 = _mm_ternarylogic_epi64(_mm_ternarylogic_epi64(a00, a05, a10, 0x96), a15, a20, 0x96);
    const __m128i c1 = _mm_ternarylogic_epi64(_mm_ternarylogic_epi64(a01, a06, a11, 0x96), a16, a21, 0x96);
    const __m128i c2 = _mm_ternarylogic_epi64(_mm_ternarylogic_epi64(a02, a07, a12, 0x96), a17, a22, 0x96);
    const __m128i c3 = _mm_ternarylogic_epi64(_mm_ternarylogic_epi64(a03, a08, a13, 0x96), a18, a23, 0x96);
    const __m128i c4 = _mm_ternarylogic_epi64(_mm_ternarylogic_epi64(a04, a09, a14, 0x96), a19, a24, 0x96);
    const __m128i d0 = _mm_xor_si128(c4, _mm_rol_epi64(c1, 1));
    const __m128i d1 = _mm_xor_si128(c0, _mm_rol_epi64(c2, 1));
    const __m128i d2 = _mm_xor_si128(c1, _mm_rol_epi64(c3, 1));
    const __m128i d3 = _mm_xor_si128(c2, _mm_rol_epi64(c4, 1));
    const __m128i d4 = _mm_xor_si128(c3, _mm_rol_epi64(c0, 1));
    const __m128i b00 = _mm_xor_si128(a00, d0);
    const __m128i b10 = _mm_rol_epi64(_mm_xor_si128(a01, d1), 1);
    const __m128i b20 = _mm_rol_epi64(_mm_xor_si128(a02, d2), 62);
    const __m128i b05 = _mm_rol_epi64(_mm_xor_si128(a03, d3), 28);
    const __m128i b15 = _mm_rol_epi64(_mm_xor_si128(a04, d4), 27);
    const __m128i b16 = _mm_rol_epi64(_mm_xor_si128(a05, d0), 36);
    const __m128i b01 = _mm_rol_epi64(_mm_xor_si128(a06, d1), 44);
    const __m128i b11 = _mm_rol_epi64(_mm_xor_si128(a07, d2), 6);
    const __m128i b21 = _mm_rol_epi64(_mm_xor_si128(a08, d3), 55);
    const __m128i b06 = _mm_rol_epi64(_mm_xor_si128(a09, d4), 20);
    const __m128i b07 = _mm_rol_epi64(_mm_xor_si128(a10, d0), 3);
    const __m128i b17 = _mm_rol_epi64(_mm_xor_si128(a11, d1), 10);
    const __m128i b02 = _mm_rol_epi64(_mm_xor_si128(a12, d2), 43);
    const __m128i b12 = _mm_rol_epi64(_mm_xor_si128(a13, d3), 25);
    const __m128i b22 = _mm_rol_epi64(_mm_xor_si128(a14, d4), 39);
    const __m128i b23 = _mm_rol_epi64(_mm_xor_si128(a15, d0), 41);
    const __m128i b08 = _mm_rol_epi64(_mm_xor_si128(a16, d1), 45);
    const __m128i b18 = _mm_rol_epi64(_mm_xor_si128(a17, d2), 15);
    const __m128i b03 = _mm_rol_epi64(_mm_xor_si128(a18, d3), 21);
    const __m128i b13 = _mm_rol_epi64(_mm_xor_si128(a19, d4), 8);
    const __m128i b14 = _mm_rol_epi64(_mm_xor_si128(a20, d0), 18);
    const __m128i b24 = _mm_rol_epi64(_mm_xor_si128(a21, d1), 2);
    const __m128i b09 = _mm_rol_epi64(_mm_xor_si128(a22, d2), 61);
    const __m128i b19 = _mm_rol_epi64(_mm_xor_si128(a23, d3), 56);
    const __m128i b04 = _mm_rol_epi64(_mm_xor_si128(a24, d4), 14);
    a00 = _mm_ternarylogic_epi64(b00, b01, b02, 0xD2);
    a01 = _mm_ternarylogic_epi64(b01, b02, b03, 0xD2);
    a02 = _mm_ternarylogic_epi64(b02, b03, b04, 0xD2);
    a03 = _mm_ternarylogic_epi64(b03, b04, b00, 0xD2);
    a04 = _mm_ternarylogic_epi64(b04, b00, b01, 0xD2);
    a05 = _mm_ternarylogic_epi64(b05, b06, b07, 0xD2);
    a06 = _mm_ternarylogic_epi64(b06, b07, b08, 0xD2);
    a07 = _mm_ternarylogic_epi64(b07, b08, b09, 0xD2);
    a08 = _mm_ternarylogic_epi64(b08, b09, b05, 0xD2);
    a09 = _mm_ternarylogic_epi64(b09, b05, b06, 0xD2);
    a10 = _mm_ternarylogic_epi64(b10, b11, b12, 0xD2);
    a11 = _mm_ternarylogic_epi64(b11, b12, b13, 0xD2);
    a12 = _mm_ternarylogic_epi64(b12, b13, b14, 0xD2);
    a13 = _mm_ternarylogic_epi64(b13, b14, b10, 0xD2);
    a14 = _mm_ternarylogic_epi64(b14, b10, b11, 0xD2);
    a15 = _mm_ternarylogic_epi64(b15, b16, b17, 0xD2);
    a16 = _mm_ternarylogic_epi64(b16, b17, b18, 0xD2);
    a17 = _mm_ternarylogic_epi64(b17, b18, b19, 0xD2);
    a18 = _mm_ternarylogic_epi64(b18, b19, b15, 0xD2);
    a19 = _mm_ternarylogic_epi64(b19, b15, b16, 0xD2);
    a20 = _mm_ternarylogic_epi64(b20, b21, b22, 0xD2);
    a21 = _mm_ternarylogic_epi64(b21, b22, b23, 0xD2);
    a22 = _mm_ternarylogic_epi64(b22, b23, b24, 0xD2);
    a23 = _mm_ternarylogic_epi64(b23, b24, b20, 0xD2);
    a24 = _mm_ternarylogic_epi64(b24, b20, b21, 0xD2);
    a00 = _mm_xor_si128(a00, _mm_cvtsi64_si128((long long)RC[r]));
  }
  s[0] = (uint64_t)_mm_cvtsi128_si64(a00);
  s[1] = (uint64_t)_mm_cvtsi128_si64(a01);
  s[2] = (uint64_t)_mm_cvtsi128_si64(a02);
  s[3] = (uint64_t)_mm_cvtsi128_si64(a03);
  s[4] = (uint64_t)_mm_cvtsi128_si64(a04);
  s[5] = (uint64_t)_mm_cvtsi128_si64(a05);
  s[6] = (uint64_t)_mm_cvtsi128_si64(a06);
  s[7] = (uint64_t)_mm_cvtsi128_si64(a07);
  s[8] = (uint64_t)_mm_cvtsi128_si64(a08);
  s[9] = (uint64_t)_mm_cvtsi128_si64(a09);
  s[10] = (uint64_t)_mm_cvtsi128_si64(a10);
  s[11] = (uint64_t)_mm_cvtsi128_si64(a11);
  s[12] = (uint64_t)_mm_cvtsi128_si64(a12);
  s[13] = (uint64_t)_mm_cvtsi128_si64(a13);
  s[14] = (uint64_t)_mm_cvtsi128_si64(a14);
  s[15] = (uint64_t)_mm_cvtsi128_si64(a15);
  s[16] = (uint64_t)_mm_cvtsi128_si64(a16);
  s[17] = (uint64_t)_mm_cvtsi128_si64(a17);
  s[18] = (uint64_t)_mm_cvtsi128_si64(a18);
  s[19] = (uint64_t)_mm_cvtsi128_si64(a19);
  s[20] = (uint64_t)_mm_cvtsi128_si64(a20);
  s[21] = (uint64_t)_mm_cvtsi128_si64(a21);
  s[22] = (uint64_t)_mm_cvtsi128_si64(a22);
  s[23] = (uint64_t)_mm_cvtsi128_si64(a23);
  s[24] = (uint64_t)_mm_cvtsi128_si64(a24);
}

using Fn = void (*)(uint64_t *);
double time_ns(Fn f) {
  uint64_t st[25] = {1};
  double best = 1e30;
  for (int rep = 0; rep < 5; rep++) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < (1 << 18); i++) f(st);
    const auto t1 = std::chrono::steady_clock::now();
    const double ns = std::chrono::duration<double, std::nano>(t1 - t0).count() / (1 << 18);
    if (ns < best) best = ns;
  }
  return st[0] == 42 ? best + 1 : best;
}
}  // namespace

int main() {
  struct V { const char *name; Fn f; } vs[] = {{"scalar (library)", lcpc::keccak_f1600_scalar},
                                                {"avx512 (library)", lcpc::keccak_f1600_avx512},
                                                {"avx512 D form", keccak_avx512_d}};
  int bad = 0;
  for (auto &v : vs) {
    uint64_t a[25], b[25];
    for (int i = 0; i < 25; i++) a[i] = b[i] = 0x9e3779b97f4a7c15ULL * (i + 1);
    for (int k = 0; k < 3; k++) {
      lcpc::keccak_f1600_scalar(a);
      v.f(b);
    }
    const bool ok = std::memcmp(a, b, sizeof a) == 0;
    bad += !ok;
    printf("%-18s %7.1f ns per permutation %s\n", v.name, time_ns(v.f), ok ? "ok" : "MISMATCH");
  }
  return bad != 0;
}
