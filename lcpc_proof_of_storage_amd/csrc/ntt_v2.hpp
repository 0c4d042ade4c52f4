// ntt_v2.hpp -- register-round NTT passes with one LDS exchange (gfx950).
//
// Same contract and four-step decomposition as ntt_impl.hpp (fffft::fft_io, out[bitrev(j)] =
// sum_i in[i] w^(ij)).  What changes is the data movement per workgroup:
//   pass A: round 0 of the column DIF loads its 2^R elements straight from HBM (lanes = adjacent
//           columns: coalesced row segments), rounds exchange through one padded LDS tile, and
//           the last round applies the inter-pass twiddle and stores straight to HBM (again
//           lanes = adjacent columns).  With HALFZ (n_valid <= n/2, rate-1/2 Ligero rows) the
//           upper half of every column is known zero: it is never loaded and the first stage
//           degenerates to (a, a*w) -- no add/sub.
//   pass B: round 0 loads contiguous block positions (lanes = adjacent positions), the last
//           round goes through LDS once more so the final stores are contiguous rows.
// Block size T threads, tile S x CW elements, 2^R = S*CW/T elements per thread per round.
#pragma once
#include "field.hpp"
#include "kernels.hpp"
#include "prof.hpp"

// LCPC_NTT_LAZY (default 1): butterflies keep residues in [0, 2p) (no final subtraction in the
// twiddle products), and pass B's final store reduces to [0, p).
#ifndef LCPC_NTT_LAZY
#define LCPC_NTT_LAZY 1
#endif

namespace lcpc {
namespace ntt_v2 {

#if LCPC_NTT_LAZY
template <class F>
__device__ __forceinline__ Fe<F> NTT_MUL(const Fe<F> &a, const Fe<F> &b) { return fe_mul_lazy<F>(a, b); }
#else
template <class F>
__device__ __forceinline__ Fe<F> NTT_MUL(const Fe<F> &a, const Fe<F> &b) { return fe_mul<F>(a, b); }
#endif

__device__ __forceinline__ int brev(int x, int bits) {
  return bits ? (int)(__builtin_bitreverse32((uint32_t)x) >> (32 - bits)) : 0;
}

// Stages S0 .. S0+RR-1 of the 2^LOG_S-point DIF on the K = 2^RR register elements
// x[j] = v[b + j*GL] (GL = 2^(LOG_S-S0-RR), b = b_lo + multiple of GL*K, b_lo < GL).
// HALFZ: x[j] == 0 for j >= K/2 on entry (only meaningful for S0 == 0).
template <class F, int LOG_S, int S0, int RR, bool HALFZ>
__device__ __forceinline__ void dif_regs(Fe<F> *x, int b_lo, const Fe<F> *tw) {
  constexpr int LOG_GL = LOG_S - S0 - RR;
  constexpr int GL = 1 << LOG_GL;
  constexpr int K = 1 << RR;
#pragma unroll
  for (int qq = 0; qq < RR; qq++) {
    const int s = S0 + qq;
    const int h = 1 << (RR - 1 - qq);
#pragma unroll
    for (int j = 0; j < K; j++) {
      if (j & h) continue;
      const int jm = j & (h - 1);
      const bool triv = (LOG_GL == 0 && jm == 0);
      if (HALFZ && qq == 0) {
        const Fe<F> a = x[j];
#if LCPC_NTT_LAZY
        x[j + h] = triv ? a : fe_mul_lazy<F>(a, tw[(b_lo + jm * GL) << s]);
#else
        x[j + h] = triv ? a : fe_mul<F>(a, tw[(b_lo + jm * GL) << s]);
#endif
      } else {
        const Fe<F> a = x[j], c = x[j + h];
#if LCPC_NTT_LAZY
        // residues in [0, 2p) throughout; the final store reduces (k_pass_b)
        x[j] = fe_add_2p<F>(a, c);
        const Fe<F> d = fe_sub_2p<F>(a, c);
        x[j + h] = triv ? d : fe_mul_lazy<F>(d, tw[(b_lo + jm * GL) << s]);
#else
        x[j] = fe_add<F>(a, c);
        x[j + h] = triv ? fe_sub<F>(a, c) : fe_mul<F>(fe_sub_lazy<F>(a, c), tw[(b_lo + jm * GL) << s]);
#endif
      }
    }
  }
}

// round size for round starting at stage S0
template <int LOG_S, int R, int S0>
constexpr int rr_of() {
  return (LOG_S - S0) < R ? (LOG_S - S0) : R;
}

// middle rounds: LDS -> registers -> LDS, lanes = adjacent vectors (v fastest)
template <class F, int LOG_S, int LOG_CW, int LOG_T, int R, int S0, int LAST_S0>
__device__ __forceinline__ void mid_rounds(Fe<F> *tile, const Fe<F> *tw, int tid) {
  if constexpr (S0 < LAST_S0) {
    constexpr int RR = rr_of<LOG_S, R, S0>();
    constexpr int CW = 1 << LOG_CW, LD = CW > 1 ? CW + 1 : 1;
    constexpr int LOG_GL = LOG_S - S0 - RR;
    constexpr int GL = 1 << LOG_GL, K = 1 << RR;
    constexpr int ITEMS = (1 << (LOG_S - RR)) * CW;
    for (int item = tid; item < ITEMS; item += (1 << LOG_T)) {
      const int v = item & (CW - 1), q = item >> LOG_CW;
      const int b_lo = q & (GL - 1);
      const int b = b_lo + ((q >> LOG_GL) << (LOG_GL + RR));
      Fe<F> x[K];
#pragma unroll
      for (int j = 0; j < K; j++) x[j] = tile[(b + j * GL) * LD + v];
      dif_regs<F, LOG_S, S0, RR, false>(x, b_lo, tw);
#pragma unroll
      for (int j = 0; j < K; j++) tile[(b + j * GL) * LD + v] = x[j];
    }
    __syncthreads();
    mid_rounds<F, LOG_S, LOG_CW, LOG_T, R, S0 + RR, LAST_S0>(tile, tw, tid);
  }
}

template <int LOG_S, int R>
constexpr int last_s0() {  // first stage of the last round
  int s0 = 0;
  while (LOG_S - s0 > R) s0 += R;
  return s0;
}

// CANON: the inter-pass multiplier is w^e R^-1 (the canonical words of w^e), applied to every
// element including e = 0, so the whole transform comes out scaled by R^-1 -- i.e. in canonical
// form (see ntt_rows' canon_out).  tw2: the inter-pass twiddles w^(c bitrev(t)) laid out [t][c]
// (NttPlan::d_tw2 / d_tw2_canon), so the lanes of a store (adjacent columns c) load adjacent
// twiddles.
template <class F, int LOG_S, int LOG_CW, int LOG_T, bool HALFZ, bool CANON>
__global__ __launch_bounds__(1 << LOG_T) void k_pass_a(const uint32_t *__restrict__ src,
                                                       size_t src_stride, size_t n_valid,
                                                       uint32_t *__restrict__ dst,
                                                       size_t dst_stride,
                                                       const uint32_t *__restrict__ twn,
                                                       const uint32_t *__restrict__ tw2,
                                                       int log_n, uint32_t *__restrict__ copy,
                                                       size_t copy_stride) {
  constexpr int S = 1 << LOG_S, CW = 1 << LOG_CW, LD = CW > 1 ? CW + 1 : 1, T = 1 << LOG_T;
  constexpr int R = LOG_S + LOG_CW - LOG_T;
  static_assert(R >= 1 && R <= LOG_S, "tile / thread shape");
  constexpr int LS0 = last_s0<LOG_S, R>();
  constexpr bool ONE_ROUND = LS0 == 0;
  __shared__ __align__(16) uint32_t smem[((ONE_ROUND ? 0 : S * LD) + S / 2) * F::N];
  Fe<F> *tw = reinterpret_cast<Fe<F> *>(smem);
  Fe<F> *tile = tw + S / 2;
  const int tid = threadIdx.x;
  const int log_m = log_n - LOG_S;
  const int groups = 1 << (log_m - LOG_CW);
  const size_t row = blockIdx.x / groups;
  const size_t c0 = (size_t)(blockIdx.x % groups) << LOG_CW;
  for (int e = tid; e < S / 2; e += T) tw[e] = fe_load<F>(twn, (size_t)e << log_m);

  const uint32_t *in = src + row * src_stride * F::N;
  uint32_t *out = dst + row * dst_stride * F::N;
  uint32_t *cp = copy ? copy + row * copy_stride * F::N : nullptr;
  // ---- round 0 straight from HBM (exactly one item per thread: ITEMS = CW * S / 2^R = T)
  {
    constexpr int RR = rr_of<LOG_S, R, 0>();
    constexpr int K = 1 << RR, LOG_GL = LOG_S - RR, GL = 1 << LOG_GL;
    const int v = tid & (CW - 1), q = tid >> LOG_CW;  // q < GL
    const size_t c = c0 + v;
    Fe<F> x[K];
#pragma unroll
    for (int j = 0; j < K; j++) {
      if (HALFZ && j >= K / 2) {
        x[j] = fe_zero<F>();
      } else {
        const size_t pos = c + ((size_t)(q + j * GL) << log_m);
        if (pos < n_valid) {
          x[j] = fe_load<F>(in, pos);
          if (cp) fe_store<F>(cp, pos, x[j]);  // coalesced: lanes = adjacent columns
        } else {
          x[j] = fe_zero<F>();
        }
      }
    }
    __syncthreads();  // twiddle table
    dif_regs<F, LOG_S, 0, RR, HALFZ>(x, q, tw);
    if constexpr (ONE_ROUND) {
#pragma unroll
      for (int j = 0; j < K; j++) {
        const int t = q + j * GL;  // GL == 1 here
        const size_t at = c + ((size_t)t << log_m);  // (also the [t][c] twiddle's index)
        Fe<F> y = x[j];
        if (CANON || (c && t)) y = NTT_MUL<F>(y, fe_load<F>(tw2, at));  // (w^0 = 1 otherwise)
        fe_store<F>(out, at, y);
      }
      return;
    } else {
#pragma unroll
      for (int j = 0; j < K; j++) tile[(q + j * GL) * LD + v] = x[j];
    }
  }
  if constexpr (!ONE_ROUND) {
    __syncthreads();
    mid_rounds<F, LOG_S, LOG_CW, LOG_T, R, rr_of<LOG_S, R, 0>(), LS0>(tile, tw, tid);
    // ---- last round: LDS -> registers -> twiddle -> HBM
    constexpr int RR = LOG_S - LS0;
    constexpr int K = 1 << RR;
    constexpr int ITEMS = (1 << (LOG_S - RR)) * CW;
    for (int item = tid; item < ITEMS; item += T) {
      const int v = item & (CW - 1), q = item >> LOG_CW;
      const int b = q << RR;  // GL == 1
      Fe<F> x[K];
#pragma unroll
      for (int j = 0; j < K; j++) x[j] = tile[(b + j) * LD + v];
      dif_regs<F, LOG_S, LS0, RR, false>(x, 0, tw);
      const size_t c = c0 + v;
#pragma unroll
      for (int j = 0; j < K; j++) {
        const int t = b + j;
        const size_t at = c + ((size_t)t << log_m);  // (also the [t][c] twiddle's index)
        Fe<F> y = x[j];
        if (CANON || (c && t)) y = NTT_MUL<F>(y, fe_load<F>(tw2, at));  // (w^0 = 1 otherwise)
        fe_store<F>(out, at, y);
      }
    }
  }
}

template <class F, int LOG_S, int LOG_CW, int LOG_T>
__global__ __launch_bounds__(1 << LOG_T) void k_pass_b(uint32_t *__restrict__ data, size_t stride,
                                                       const uint32_t *__restrict__ twn,
                                                       int log_n) {
  constexpr int S = 1 << LOG_S, CW = 1 << LOG_CW, LD = CW > 1 ? CW + 1 : 1, T = 1 << LOG_T;
  constexpr int R = LOG_S + LOG_CW - LOG_T;
  static_assert(R >= 1 && R <= LOG_S, "tile / thread shape");
  __shared__ __align__(16) uint32_t smem[(S * LD + S / 2) * F::N];
  Fe<F> *tw = reinterpret_cast<Fe<F> *>(smem);
  Fe<F> *tile = tw + S / 2;
  const int tid = threadIdx.x;
  const int log_blocks = log_n - LOG_S;
  const int groups = 1 << (log_blocks - LOG_CW);
  const size_t row = blockIdx.x / groups;
  const size_t b0 = (size_t)(blockIdx.x % groups) << LOG_CW;
  for (int e = tid; e < S / 2; e += T) tw[e] = fe_load<F>(twn, (size_t)e << log_blocks);
  uint32_t *io = data + (row * stride + b0 * S) * F::N;
  // ---- round 0 from HBM: lanes = adjacent positions of one block
  {
    constexpr int RR = rr_of<LOG_S, R, 0>();
    constexpr int K = 1 << RR, LOG_GL = LOG_S - RR, GL = 1 << LOG_GL;
    const int q = tid & (GL - 1), v = tid >> LOG_GL;
    Fe<F> x[K];
#pragma unroll
    for (int j = 0; j < K; j++) x[j] = fe_load<F>(io, (size_t)v * S + q + j * GL);
    __syncthreads();
    dif_regs<F, LOG_S, 0, RR, false>(x, q, tw);
#pragma unroll
    for (int j = 0; j < K; j++) tile[(q + j * GL) * LD + v] = x[j];
  }
  __syncthreads();
  mid_rounds<F, LOG_S, LOG_CW, LOG_T, R, rr_of<LOG_S, R, 0>(), LOG_S>(tile, tw, tid);
  for (int idx = tid; idx < S * CW; idx += T) {
    const int v = idx >> LOG_S, t = idx & (S - 1);
#if LCPC_NTT_LAZY
    fe_store<F>(io, idx, fe_reduce_2p<F>(tile[t * LD + v]));
#else
    fe_store<F>(io, idx, tile[t * LD + v]);
#endif
  }
}

template <class F, int LOG_S, int LOG_CW, int LOG_T, bool HALFZ, bool CANON = false>
hipError_t launch_a(const uint32_t *src, size_t ss, size_t nv, uint32_t *dst, size_t ds,
                    const uint32_t *tw, int log_n, size_t n_rows, hipStream_t s, uint32_t *cp,
                    size_t cs, const uint32_t *tw2) {
  const size_t groups = (size_t)1 << (log_n - LOG_S - LOG_CW);
  prof::Scope ps("ntt_pass_a", s);
  hipLaunchKernelGGL((k_pass_a<F, LOG_S, LOG_CW, LOG_T, HALFZ, CANON>), dim3((unsigned)(n_rows * groups)),
                     dim3(1 << LOG_T), 0, s, src, ss, nv, dst, ds, tw, tw2, log_n, cp, cs);
  return hipGetLastError();
}

template <class F, int LOG_S, int LOG_CW, int LOG_T>
hipError_t launch_b(uint32_t *dst, size_t ds, const uint32_t *tw, int log_n, size_t n_rows,
                    hipStream_t s) {
  const size_t groups = (size_t)1 << (log_n - LOG_S - LOG_CW);
  prof::Scope ps("ntt_pass_b", s);
  hipLaunchKernelGGL((k_pass_b<F, LOG_S, LOG_CW, LOG_T>), dim3((unsigned)(n_rows * groups)),
                     dim3(1 << LOG_T), 0, s, dst, ds, tw, log_n);
  return hipGetLastError();
}

}  // namespace ntt_v2
}  // namespace lcpc
