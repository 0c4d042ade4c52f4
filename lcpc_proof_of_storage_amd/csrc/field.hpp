// field.hpp -- prime-field arithmetic for gfx950 (CDNA4), 32-bit limbs, Montgomery form.
//
// Element layout = the reference's ff_derive internal representation (lcpc-test-fields
// src/lib.rs:13-70: `struct FtX([u64; N])`, value*R mod p with R = 2^(64N), limbs little
// endian), viewed as 2N little-endian u32 words.  Every result is fully reduced (< p), as
// ff_derive's, so the words written back are bit-identical to the reference's.
//
// Arithmetic: Montgomery multiplication on 32-bit words with v_mad_u64_u32 (32x32+64 -> 64 plus
// carry-out), add/sub with carry chains.  Every prime the reference declares has p = 1 mod 2^32,
// so -p^-1 mod 2^32 = 0xffffffff and p[0] = 1: the quotient word is m = -t0 and m*p[0] + t0
// contributes only a carry.  Those fields use product scanning (fe_mul_fips); CIOS
// (fe_mul_cios) is the generic path.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "field_params.hpp"

namespace lcpc {

template <class F>
struct Fe {
  uint32_t v[F::N];
};

template <class F>
__device__ __forceinline__ Fe<F> fe_zero() {
  Fe<F> r;
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = 0;
  return r;
}

template <class F>
__device__ __forceinline__ Fe<F> fe_one() {
  Fe<F> r;
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = F::ONE[i];
  return r;
}

template <class F>
__device__ __forceinline__ bool fe_is_zero(const Fe<F>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) o |= a.v[i];
  return o == 0;
}

template <class F>
__device__ __forceinline__ bool fe_eq(const Fe<F>& a, const Fe<F>& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) o |= a.v[i] ^ b.v[i];
  return o == 0;
}

// a < p (a canonical value: PrimeField::from_repr accepts it)
template <class F>
__device__ __forceinline__ bool fe_is_canonical(const Fe<F>& a) {
#pragma unroll
  for (int i = F::N - 1; i >= 0; i--) {
    if (a.v[i] != F::P[i]) return a.v[i] < F::P[i];
  }
  return false;
}

// r = a + b mod p  (a, b < p)
template <class F>
__device__ __forceinline__ Fe<F> fe_add(const Fe<F>& a, const Fe<F>& b) {
  Fe<F> t, u;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) t.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) u.v[i] = __builtin_subc(t.v[i], F::P[i], br, &br);
  // t >= p  <=>  carry out of the add, or no borrow out of t - p
  const bool take_u = c | (br ^ 1u);
  Fe<F> r;
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = take_u ? u.v[i] : t.v[i];
  return r;
}

// r = a - b mod p
template <class F>
__device__ __forceinline__ Fe<F> fe_sub(const Fe<F>& a, const Fe<F>& b) {
  Fe<F> t, u;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) t.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) u.v[i] = __builtin_addc(t.v[i], F::P[i], c, &c);
  Fe<F> r;
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = br ? u.v[i] : t.v[i];
  return r;
}

// a - b + p as an integer in [1, 2p) (no conditional correction): only as a MULTIPLICAND.
// With p < R/2 a Montgomery product of a value < 2p and one < p is < p (1 + 2p/R) < 2p before
// its final conditional subtraction, so fe_mul(fe_sub_lazy(a, b), w) == fe_mul(fe_sub(a, b), w)
// bit for bit; the DIF butterfly's twiddled output saves the select of fe_sub.
template <class F>
__device__ __forceinline__ Fe<F> fe_sub_lazy(const Fe<F>& a, const Fe<F>& b) {
  static_assert(F::P[F::N - 1] < 0x80000000u, "needs p < R / 2");
  Fe<F> t;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) t.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) t.v[i] = __builtin_addc(t.v[i], F::P[i], c, &c);
  return t;  // mod 2^(32N): a - b + p whether or not a - b borrowed
}

// ---- lazy residues in [0, 2p) (p < R/2, so 2p < R): the NTT passes keep every intermediate
// value in [0, 2p) and reduce once, at the final store (ntt_v2.hpp)
template <class F>
struct TwoP {
  static constexpr uint32_t limb(int i) {
    uint64_t c = 0, s = 0;
    for (int k = 0; k <= i; k++) {
      s = 2ull * F::P[k] + c;
      c = s >> 32;
    }
    return (uint32_t)s;
  }
};
// a + b for a, b < 2p: the sum (with its carry out) minus 2p when it is >= 2p, in [0, 2p)
template <class F>
__device__ __forceinline__ Fe<F> fe_add_2p(const Fe<F>& a, const Fe<F>& b) {
  static_assert(F::P[F::N - 1] < 0x80000000u, "needs p < R / 2");
  Fe<F> t, u, r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) t.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) u.v[i] = __builtin_subc(t.v[i], TwoP<F>::limb(i), br, &br);
  const bool take_u = c | (br ^ 1u);
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = take_u ? u.v[i] : t.v[i];
  return r;
}
// a - b for a, b < 2p, plus 2p when it borrowed: in [0, 2p)
template <class F>
__device__ __forceinline__ Fe<F> fe_sub_2p(const Fe<F>& a, const Fe<F>& b) {
  Fe<F> t, u, r;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) t.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) u.v[i] = __builtin_addc(t.v[i], TwoP<F>::limb(i), c, &c);
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = br ? u.v[i] : t.v[i];
  return r;
}
// x < 2p -> x mod p
template <class F>
__device__ __forceinline__ Fe<F> fe_reduce_2p(const Fe<F>& x) {
  Fe<F> u, r;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < F::N; i++) u.v[i] = __builtin_subc(x.v[i], F::P[i], br, &br);
#pragma unroll
  for (int i = 0; i < F::N; i++) r.v[i] = br ? x.v[i] : u.v[i];
  return r;
}

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * (uint64_t)b + c;
}

// Montgomery product a*b*R^-1 mod p, R = 2^(32N)  (CIOS, 32-bit words): any odd p
template <class F>
__device__ __forceinline__ Fe<F> fe_mul_cios(const Fe<F>& a, const Fe<F>& b) {
  constexpr int N = F::N;
  uint32_t t[N + 2];
#pragma unroll
  for (int i = 0; i < N + 2; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    // t += a * b[i]
    uint32_t carry = 0;
#pragma unroll
    for (int j = 0; j < N; j++) {
      uint64_t s = mad64(a.v[j], b.v[i], (uint64_t)t[j] + carry);
      t[j] = (uint32_t)s;
      carry = (uint32_t)(s >> 32);
    }
    {
      uint32_t c2 = 0;
      t[N] = __builtin_addc(t[N], carry, 0u, &c2);
      t[N + 1] = c2;
    }
    // t = (t + m p) / 2^32
    uint32_t c;
    if constexpr (F::NP == 0xffffffffu && F::P[0] == 1u) {
      // m = -t0; m*p0 + t0 = 2^32 * (t0 != 0)
      const uint32_t m = 0u - t[0];
      c = t[0] != 0u;
#pragma unroll
      for (int j = 1; j < N; j++) {
        uint64_t s = mad64(m, F::P[j], (uint64_t)t[j] + c);
        t[j - 1] = (uint32_t)s;
        c = (uint32_t)(s >> 32);
      }
    } else {
      const uint32_t m = t[0] * F::NP;
      uint64_t s0 = mad64(m, F::P[0], (uint64_t)t[0]);
      c = (uint32_t)(s0 >> 32);
#pragma unroll
      for (int j = 1; j < N; j++) {
        uint64_t s = mad64(m, F::P[j], (uint64_t)t[j] + c);
        t[j - 1] = (uint32_t)s;
        c = (uint32_t)(s >> 32);
      }
    }
    uint32_t c3 = 0;
    t[N - 1] = __builtin_addc(t[N], c, 0u, &c3);
    t[N] = t[N + 1] + c3;
  }
  // conditional final subtraction
  Fe<F> u, r;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; i++) u.v[i] = __builtin_subc(t[i], F::P[i], br, &br);
  const bool take_u = (t[N] != 0u) | (br ^ 1u);
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = take_u ? u.v[i] : t[i];
  return r;
}

// v_mad_u64_u32 with its carry-out (the compiler's own selection for a 64-bit multiply-add
// discards the carry, so every accumulation step would cost extra adds and moves)
__device__ __forceinline__ uint64_t mad_co_vv(uint32_t a, uint32_t b, uint64_t c, uint64_t &cm) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(cm) : "v"(a), "v"(b), "v"(c));
  return d;
}
__device__ __forceinline__ uint64_t mad_co_vs(uint32_t a, uint32_t b, uint64_t c, uint64_t &cm) {
  uint64_t d;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(cm) : "v"(a), "s"(b), "v"(c));
  return d;
}
// x + carry (the SGPR lane mask written by mad_co_*)
__device__ __forceinline__ uint32_t add_carry(uint32_t x, uint64_t cm) {
  uint32_t d;
  uint64_t co;
  asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(d), "=s"(co) : "v"(x), "s"(cm));
  return d;
}

// Column transition of the product scanning below for k < N: m = 0 - lo (its borrow is lo != 0),
// then the next column's 64-bit addend is (hi + borrow, r2 + carry), two add-with-carry written
// straight into the addend's halves (no select, no 64-bit add, fewer moves;
// tools/microbench/femul2.hip: Ft127 486 -> 503 G mul/s, Ft63 1638 -> 1701, bit-identical).
__device__ __forceinline__ void fips_col_step(uint32_t lo, uint32_t hi, uint32_t r2, uint32_t &m, uint32_t &nlo,
                                              uint32_t &nhi) {
  uint64_t c0, c1, c2;
  asm("v_sub_co_u32_e64 %0, %3, 0, %6\n\t"
      "v_addc_co_u32_e64 %1, %4, %7, 0, %3\n\t"
      "v_addc_co_u32_e64 %2, %5, %8, 0, %4"
      : "=&v"(m), "=&v"(nlo), "=&v"(nhi), "=&s"(c0), "=&s"(c1), "=&s"(c2)
      : "v"(lo), "v"(hi), "v"(r2));
}

// Carry-free mads of column k of fe_mul_fips (bit s: product a_s b_(k-s) for s < N, reduction
// m_(s-N) p_(k-s+N) for s >= N).  A column starts from an addend below 2^37 (the previous
// column's high word and at most 2N + 1 carries).  A mad whose worst-case product keeps the
// running sum below 2^64 cannot carry out, so its carry fold is dropped.  Such mads are taken
// smallest bound first.  Every p has p_(N-1) < 2^31 (p < R / 2), so m p_(N-1) < 2^63; in the lazy
// product b < p, so b_(N-1) <= p_(N-1) as well.  Ft127: the mads with p_1 (0.50 of 2^64),
// p_3 (0.43) and, lazy, b_3 (0.43) -- 10 of the 28 mads need no fold (8 without b < p).
template <class F, bool LAZY>
__host__ __device__ constexpr uint32_t fips_free_mask(int k) {
  constexpr int N = F::N;
  using u128 = unsigned __int128;
  const u128 lim = ((u128)1 << 64) - 1;
  const u128 w = 0xffffffffu;
  u128 bound[2 * N] = {};
  bool cand[2 * N] = {};
  for (int i = 0; i < N; i++) {
    const int j = k - i;
    if (j >= 0 && j < N) {
      cand[i] = true;
      bound[i] = w * ((LAZY && j == N - 1) ? (u128)F::P[N - 1] : w);
    }
    if (i < k && j >= 1 && j < N) {
      cand[N + i] = true;
      bound[N + i] = w * (u128)F::P[j];
    }
  }
  u128 sum = (u128)1 << 37;
  uint32_t mask = 0;
  for (;;) {
    int best = -1;
    for (int s = 0; s < 2 * N; s++)
      if (cand[s] && !((mask >> s) & 1u) && (best < 0 || bound[s] < bound[best])) best = s;
    if (best < 0 || sum + bound[best] > lim) break;
    sum += bound[best];
    mask |= 1u << best;
  }
  return mask;
}

// Montgomery product for p = 1 mod 2^32 (every field the reference declares): finely integrated
// product scanning.  Column k accumulates a_i b_(k-i) and m_i p_(k-i) into a 96-bit (acc, r2)
// with one carry-out mad + one add-with-carry per product; for k < N the quotient word is
// m_k = -acc mod 2^32 (-p^-1 = -1 mod 2^32) and m_k p_0 = m_k only clears the low word, leaving
// a carry iff it was nonzero.  Each carry is folded into r2 one product later, so the SGPR a
// mad writes is not read by the very next instruction.  tools/microbench/femul_variants.hip:
// Ft127 366 -> 465 G mul/s on MI355X, bit-identical to the CIOS form.  Round 6: the mads
// fips_free_mask proves cannot carry go first in their column, without a fold.
template <class F, bool LAZY = false>
__device__ __forceinline__ Fe<F> fe_mul_fips(const Fe<F>& a, const Fe<F>& b) {
  constexpr int N = F::N;
  static_assert(F::P[N - 1] < 0x7fffff00u, "fips_free_mask's addend bound needs p < R / 2");
  uint32_t m[N], out[N];
  uint64_t acc = 0;
  uint32_t r2 = 0;
  // column 0 alone: a0 b0 <= (2^32 - 1)^2 cannot carry out of 64 bits, and its high word is at
  // most 2^32 - 2, so hi + (lo != 0) cannot carry either: m0 = -lo, next addend (hi + borrow, 0)
  // -- two instructions after the product instead of a carry fold and a three-instruction step
  {
    const uint64_t p0 = (uint64_t)a.v[0] * b.v[0];
    uint32_t nlo;
    uint64_t c0, c1;
    asm("v_sub_co_u32_e64 %0, %2, 0, %4\n\t"
        "v_addc_co_u32_e64 %1, %3, %5, 0, %2"
        : "=&v"(m[0]), "=&v"(nlo), "=&s"(c0), "=&s"(c1)
        : "v"((uint32_t)p0), "v"((uint32_t)(p0 >> 32)));
    acc = nlo;
  }
  auto column = [&]<int k>() {
    constexpr uint32_t fm = fips_free_mask<F, LAZY>(k);
    // the carry-free mads first: the same v_mad_u64_u32 with its carry-out mask left unread (the
    // compiler's own 64-bit multiply-add selection adds a separate 64-bit add)
    uint64_t unused;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j >= 0 && j < N && ((fm >> i) & 1u)) acc = mad_co_vv(a.v[i], b.v[j], acc, unused);
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < N && ((fm >> (N + i)) & 1u)) acc = mad_co_vs(m[i], F::P[j], acc, unused);
    }
    uint64_t cprev = 0, ccur;
    bool have = false;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (j < 0 || j >= N || ((fm >> i) & 1u)) continue;
      acc = mad_co_vv(a.v[i], b.v[j], acc, ccur);
      if (have) r2 = add_carry(r2, cprev);
      cprev = ccur;
      have = true;
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i >= k || j < 1 || j >= N || ((fm >> (N + i)) & 1u)) continue;
      acc = mad_co_vs(m[i], F::P[j], acc, ccur);
      if (have) r2 = add_carry(r2, cprev);
      cprev = ccur;
      have = true;
    }
    if (have) r2 = add_carry(r2, cprev);
    if constexpr (k < N) {
      uint32_t nlo, nhi;
      fips_col_step((uint32_t)acc, (uint32_t)(acc >> 32), r2, m[k], nlo, nhi);
      acc = ((uint64_t)nhi << 32) | nlo;
    } else {
      out[k - N] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)r2 << 32);
    }
    r2 = 0;
  };
  [&]<int... Ks>(std::integer_sequence<int, Ks...>) {
    (column.template operator()<Ks + 1>(), ...);
  }(std::make_integer_sequence<int, 2 * N - 1>{});
  // out + acc * 2^(32N) < 2p: one conditional subtraction
  Fe<F> u, r;
  if constexpr (LAZY) {  // a < 2p, b < p: the value is < p (1 + 2p/R) < 2p < R, so acc == 0
#pragma unroll
    for (int i = 0; i < N; i++) r.v[i] = out[i];
    return r;
  }
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; i++) u.v[i] = __builtin_subc(out[i], F::P[i], br, &br);
  const bool take_u = ((uint32_t)acc != 0u) | (br ^ 1u);
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = take_u ? u.v[i] : out[i];
  return r;
}

// a * b R^-1 in [0, 2p) for a < 2p, b < p (no final subtraction)
template <class F>
__device__ __forceinline__ Fe<F> fe_mul_lazy(const Fe<F>& a, const Fe<F>& b) {
  static_assert(F::NP == 0xffffffffu && F::P[0] == 1u, "p = 1 mod 2^32");
  static_assert(F::P[F::N - 1] < 0x80000000u, "needs p < R / 2");
  return fe_mul_fips<F, true>(a, b);
}

// Largest K with K * p < R = 2^(32N) (a safe bound from the top word): a sum of K products,
// each < p^2, stays below p R, so one Montgomery reduction of the sum lands in [0, 2p).
template <class F>
constexpr int fe_dot_kmax() {
  return (int)((1ull << 32) / ((uint64_t)F::P[F::N - 1] + 1));
}

// sum_k a[k] b[k] R^-1 mod p with ONE reduction (lazy: the K double-width products are added
// before reducing): K N^2 + N (N - 1) carry-out mads and one final subtraction, instead of K
// full Montgomery products and K - 1 modular additions.  Requires p = 1 mod 2^32 and
// K <= fe_dot_kmax<F>() (Ft127: 2, Ft63: 3, Ft255: 2, Ft253_192: 7).
template <class F, int K>
__device__ __forceinline__ Fe<F> fe_dot(const Fe<F>* a, const Fe<F>* b) {
  constexpr int N = F::N;
  static_assert(F::NP == 0xffffffffu && F::P[0] == 1u, "p = 1 mod 2^32");
  static_assert(K >= 1 && K <= fe_dot_kmax<F>(), "K products would exceed p R");
  uint32_t m[N], out[N];
  uint64_t acc = 0;
  uint32_t r2 = 0;
#pragma unroll
  for (int k = 0; k < 2 * N; k++) {
    uint64_t cprev = 0, ccur;
    bool have = false;
#pragma unroll
    for (int q = 0; q < K; q++) {
#pragma unroll
      for (int i = 0; i < N; i++) {
        const int j = k - i;
        if (j < 0 || j >= N) continue;
        acc = mad_co_vv(a[q].v[i], b[q].v[j], acc, ccur);
        if (have) r2 = add_carry(r2, cprev);
        cprev = ccur;
        have = true;
      }
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i >= k || j < 1 || j >= N) continue;
      acc = mad_co_vs(m[i], F::P[j], acc, ccur);
      if (have) r2 = add_carry(r2, cprev);
      cprev = ccur;
      have = true;
    }
    if (have) r2 = add_carry(r2, cprev);
    if (k < N) {
      uint32_t nlo, nhi;
      fips_col_step((uint32_t)acc, (uint32_t)(acc >> 32), r2, m[k], nlo, nhi);
      acc = ((uint64_t)nhi << 32) | nlo;
    } else {
      out[k - N] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)r2 << 32);
    }
    r2 = 0;
  }
  Fe<F> u, r;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; i++) u.v[i] = __builtin_subc(out[i], F::P[i], br, &br);
  const bool take_u = ((uint32_t)acc != 0u) | (br ^ 1u);
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = take_u ? u.v[i] : out[i];
  return r;
}

template <class F>
__device__ __forceinline__ Fe<F> fe_mul(const Fe<F>& a, const Fe<F>& b) {
  if constexpr (F::NP == 0xffffffffu && F::P[0] == 1u)
    return fe_mul_fips<F>(a, b);
  else
    return fe_mul_cios<F>(a, b);
}

template <class F>
__device__ __forceinline__ Fe<F> fe_sqr(const Fe<F>& a) {
  return fe_mul<F>(a, a);
}

// a^e for a small exponent (square-and-multiply, MSB first)
template <class F>
__device__ __forceinline__ Fe<F> fe_pow(Fe<F> a, uint64_t e) {
  Fe<F> acc = fe_one<F>();
  while (e) {
    if (e & 1) acc = fe_mul<F>(acc, a);
    a = fe_sqr<F>(a);
    e >>= 1;
  }
  return acc;
}

// canonical (non-Montgomery) value of a: a * R^-1 mod p (Montgomery reduction of a
// single-width value; a < p so the result is < p without a final subtraction)
template <class F>
__device__ __forceinline__ Fe<F> fe_from_mont_generic(const Fe<F>& a) {
  constexpr int N = F::N;
  uint32_t t[N + 1];
#pragma unroll
  for (int i = 0; i < N; i++) t[i] = a.v[i];
  t[N] = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint32_t m = t[0] * F::NP;
    uint64_t s0 = mad64(m, F::P[0], (uint64_t)t[0]);
    uint32_t c = (uint32_t)(s0 >> 32);
#pragma unroll
    for (int j = 1; j < N; j++) {
      uint64_t s = mad64(m, F::P[j], (uint64_t)t[j] + c);
      t[j - 1] = (uint32_t)s;
      c = (uint32_t)(s >> 32);
    }
    t[N - 1] = t[N] + c;
    t[N] = 0;
  }
  Fe<F> r;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = t[i];
  return r;
}

// the same reduction in product-scanning form for p = 1 mod 2^32 (b = 1 in fe_mul_fips: only
// the N (N - 1) quotient products m_i p_j remain, each one carry-out mad)
template <class F>
__device__ __forceinline__ Fe<F> fe_from_mont_fips(const Fe<F>& a) {
  constexpr int N = F::N;
  uint32_t m[N], out[N];
  uint64_t acc = 0;
  uint32_t r2 = 0;
#pragma unroll
  for (int k = 0; k < 2 * N; k++) {
    if (k < N) acc += a.v[k];  // acc < 2^40 here: no carry out
    uint64_t cprev = 0, ccur;
    bool have = false;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int j = k - i;
      if (i >= k || j < 1 || j >= N) continue;
      acc = mad_co_vs(m[i], F::P[j], acc, ccur);
      if (have) r2 = add_carry(r2, cprev);
      cprev = ccur;
      have = true;
    }
    if (have) r2 = add_carry(r2, cprev);
    if (k < N) {
      uint32_t nlo, nhi;
      fips_col_step((uint32_t)acc, (uint32_t)(acc >> 32), r2, m[k], nlo, nhi);
      acc = ((uint64_t)nhi << 32) | nlo;
    } else {
      out[k - N] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)r2 << 32);
    }
    r2 = 0;
  }
  Fe<F> r;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = out[i];
  return r;
}

template <class F>
__device__ __forceinline__ Fe<F> fe_from_mont(const Fe<F>& a) {
  if constexpr (F::NP == 0xffffffffu && F::P[0] == 1u)
    return fe_from_mont_fips<F>(a);
  else
    return fe_from_mont_generic<F>(a);
}

// Montgomery form of a canonical value a < p: a * R^2 * R^-1
template <class F>
__device__ __forceinline__ Fe<F> fe_to_mont(const Fe<F>& a) {
  Fe<F> r2;
#pragma unroll
  for (int i = 0; i < F::N; i++) r2.v[i] = F::R2[i];
  return fe_mul<F>(a, r2);
}

// 32-bit words of to_repr(a) as they appear in a byte stream read as little-endian u32:
// ff_derive's to_repr is the canonical value little endian (big endian for Ft253_192).
template <class F>
__device__ __forceinline__ void fe_repr_words(const Fe<F>& a, uint32_t* w) {
  const Fe<F> c = fe_from_mont<F>(a);
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    if constexpr (F::BE_REPR)
      w[i] = __builtin_bswap32(c.v[F::N - 1 - i]);
    else
      w[i] = c.v[i];
  }
}

// repr words of a value already in canonical form (no Montgomery conversion)
template <class F>
__device__ __forceinline__ void fe_canon_repr_words(const Fe<F>& c, uint32_t* w) {
#pragma unroll
  for (int i = 0; i < F::N; i++) {
    if constexpr (F::BE_REPR)
      w[i] = __builtin_bswap32(c.v[F::N - 1 - i]);
    else
      w[i] = c.v[i];
  }
}

// ---------------------------------------------------------------- memory
// Elements are 8/16/24/32 bytes; move them with the widest aligned vector loads.
template <class F>
__device__ __forceinline__ Fe<F> fe_load(const uint32_t* __restrict__ base, size_t idx) {
  Fe<F> r;
  const uint32_t* p = base + idx * F::N;
  if constexpr (F::N % 4 == 0) {
#pragma unroll
    for (int k = 0; k < F::N / 4; k++) {
      uint4 q = reinterpret_cast<const uint4*>(p)[k];
      r.v[4 * k] = q.x;
      r.v[4 * k + 1] = q.y;
      r.v[4 * k + 2] = q.z;
      r.v[4 * k + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < F::N / 2; k++) {
      uint2 q = reinterpret_cast<const uint2*>(p)[k];
      r.v[2 * k] = q.x;
      r.v[2 * k + 1] = q.y;
    }
  }
  return r;
}

template <class F>
__device__ __forceinline__ void fe_store(uint32_t* __restrict__ base, size_t idx, const Fe<F>& x) {
  uint32_t* p = base + idx * F::N;
  if constexpr (F::N % 4 == 0) {
#pragma unroll
    for (int k = 0; k < F::N / 4; k++)
      reinterpret_cast<uint4*>(p)[k] =
          make_uint4(x.v[4 * k], x.v[4 * k + 1], x.v[4 * k + 2], x.v[4 * k + 3]);
  } else {
#pragma unroll
    for (int k = 0; k < F::N / 2; k++)
      reinterpret_cast<uint2*>(p)[k] = make_uint2(x.v[2 * k], x.v[2 * k + 1]);
  }
}

// field dispatch helper: calls fn.template operator()<F>()
template <class Fn>
inline auto dispatch_field(int fid, Fn&& fn) {
  switch (fid) {
    case 0: return fn.template operator()<Ft63>();
    case 1: return fn.template operator()<Ft127>();
    case 2: return fn.template operator()<Ft191>();
    case 3: return fn.template operator()<Ft255>();
    default: return fn.template operator()<Ft253_192>();
  }
}

}  // namespace lcpc
