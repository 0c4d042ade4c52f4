// f127_host.hpp -- host-side Ft127 arithmetic for the matrix-core NTT microbenchmarks (exact,
// unsigned __int128; p = 0x6e754097ba20e0bf7f2bd90000000001, lcpc-test-fields/src/lib.rs:41-45).
// Canonical values (no Montgomery form) unless a name says otherwise.
#pragma once
#include <cstdint>
#include <cstring>

namespace f127h {
typedef unsigned __int128 u128;

constexpr u128 P = ((u128)0x6e754097ba20e0bfull << 64) | 0x7f2bd90000000001ull;

inline void mul_wide(u128 a, u128 b, u128 &hi, u128 &lo) {
  const uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64), b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64);
  const u128 p00 = (u128)a0 * b0, p01 = (u128)a0 * b1, p10 = (u128)a1 * b0, p11 = (u128)a1 * b1;
  const u128 mid = (p00 >> 64) + (uint64_t)p01 + (uint64_t)p10;
  lo = (mid << 64) | (uint64_t)p00;
  hi = p11 + (p01 >> 64) + (p10 >> 64) + (mid >> 64);
}

// (hi 2^128 + lo) mod p by shift-and-subtract over the 255-bit product (slow, exact)
inline u128 mod_wide(u128 hi, u128 lo) {
  u128 r = 0;
  for (int bit = 255; bit >= 0; bit--) {
    const int b = bit >= 128 ? (int)((hi >> (bit - 128)) & 1) : (int)((lo >> bit) & 1);
    // r = 2 r + b mod p  (r < p < 2^127: 2r + 1 < 2^128)
    r = (r << 1) | (u128)b;
    if (r >= P) r -= P;
  }
  return r;
}

inline u128 mul(u128 a, u128 b) {
  u128 hi, lo;
  mul_wide(a, b, hi, lo);
  return mod_wide(hi, lo);
}
inline u128 add(u128 a, u128 b) {
  u128 s = a + b;
  return s >= P ? s - P : s;
}
inline u128 sub(u128 a, u128 b) { return a >= b ? a - b : a + P - b; }
inline u128 pow(u128 a, u128 e) {
  u128 r = 1;
  while (e) {
    if (e & 1) r = mul(r, a);
    a = mul(a, a);
    e >>= 1;
  }
  return r;
}
// ROOT_OF_UNITY (canonical, order 2^40), SURVEY.md §8(a-1)
constexpr u128 ROOT = ((u128)0x3280b719bea9b43aull << 64) | 0xbb9ee4e683614688ull;
inline u128 root_of_order(int log) {  // w with w^(2^log) = 1
  u128 w = ROOT;
  for (int i = 0; i < 40 - log; i++) w = mul(w, w);
  return w;
}
inline u128 two_pow(int e) {
  u128 r = 1;
  for (int i = 0; i < e; i++) r = add(r, r);
  return r;
}
// 16 balanced base-256 digits (x < 2^127 - 2^120): byte a of (x + 0x80..80) XOR 0x80, as int8
inline void balanced(u128 x, int8_t d[16]) {
  u128 c = 0;
  for (int i = 0; i < 16; i++) c |= (u128)0x80 << (8 * i);
  const u128 v = x + c;
  for (int i = 0; i < 16; i++) d[i] = (int8_t)(uint8_t)(((v >> (8 * i)) & 0xff) ^ 0x80);
}
inline void to_words(u128 x, uint32_t w[4]) {
  for (int i = 0; i < 4; i++) w[i] = (uint32_t)(x >> (32 * i));
}
inline u128 from_words(const uint32_t w[4]) {
  u128 x = 0;
  for (int i = 3; i >= 0; i--) x = (x << 32) | w[i];
  return x;
}
}  // namespace f127h
