// ntt_v1.hpp -- the first (v1) NTT pass kernels: 256 threads, whole tile staged in LDS,
// radix-2^R rounds with three LDS round trips.  Kept only as the A/B baseline of
// tools/microbench/nttbench.hip (the product uses csrc/ntt_v2.hpp).
#pragma once
#include "../../lcpc_proof_of_storage_amd/csrc/ntt_impl.hpp"

namespace lcpc {
namespace ntt_v1 {
using ntt_detail::NTHREADS;
using ntt_detail::bitrev;
using ntt_detail::k_ntt_small;

// One radix-2^RR round of the S-point DIF (stages S0 .. S0+RR-1) on CW vectors in LDS.
template <class F, int LOG_S, int LOG_CW, int S0, int RR>
__device__ __forceinline__ void dif_round(Fe<F> *tile, const Fe<F> *tw, int tid) {
  constexpr int CW = 1 << LOG_CW, LD = CW + 1;
  constexpr int LOG_GL = LOG_S - S0 - RR;  // log2 of the smallest gap in this round
  constexpr int GL = 1 << LOG_GL;
  constexpr int K = 1 << RR;
  constexpr int ITEMS = (1 << (LOG_S - RR)) * CW;
  for (int item = tid; item < ITEMS; item += NTHREADS) {
    const int v = item & (CW - 1);
    const int q = item >> LOG_CW;
    const int b_lo = q & (GL - 1);
    const int b = b_lo + ((q >> LOG_GL) << (LOG_GL + RR));
    Fe<F> x[K];
#pragma unroll
    for (int j = 0; j < K; j++) x[j] = tile[(b + j * GL) * LD + v];
#pragma unroll
    for (int qq = 0; qq < RR; qq++) {
      const int s = S0 + qq;
      const int h = 1 << (RR - 1 - qq);
#pragma unroll
      for (int j = 0; j < K; j++) {
        if (j & h) continue;
        const Fe<F> a = x[j], c = x[j + h];
        x[j] = fe_add<F>(a, c);
        const Fe<F> d = fe_sub<F>(a, c);
        const int jm = j & (h - 1);
        if (LOG_GL == 0 && jm == 0) {
          x[j + h] = d;  // twiddle w^0
        } else {
          const int e = (b_lo + jm * GL) << s;
          x[j + h] = fe_mul<F>(d, tw[e]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < K; j++) tile[(b + j * GL) * LD + v] = x[j];
  }
}

template <class F, int LOG_S, int LOG_CW, int R, int S0>
__device__ __forceinline__ void dif_all(Fe<F> *tile, const Fe<F> *tw, int tid) {
  if constexpr (S0 < LOG_S) {
    constexpr int RR = (LOG_S - S0) < R ? (LOG_S - S0) : R;
    dif_round<F, LOG_S, LOG_CW, S0, RR>(tile, tw, tid);
    __syncthreads();
    dif_all<F, LOG_S, LOG_CW, R, S0 + RR>(tile, tw, tid);
  }
}

template <class F, int LOG_S, int LOG_E>
__global__ __launch_bounds__(NTHREADS) void k_ntt_pass_a(const uint32_t *__restrict__ src,
                                                         size_t src_stride, size_t n_valid,
                                                         uint32_t *__restrict__ dst,
                                                         size_t dst_stride,
                                                         const uint32_t *__restrict__ twn,
                                                         int log_n) {
  constexpr int LOG_CW = LOG_E - LOG_S;
  constexpr int S = 1 << LOG_S, CW = 1 << LOG_CW, LD = CW + 1;
  constexpr int R = LOG_E - 8;
  __shared__ __align__(16) uint32_t smem[(S * LD + S / 2) * F::N];
  Fe<F> *tile = reinterpret_cast<Fe<F> *>(smem);
  Fe<F> *tw = tile + S * LD;
  const int tid = threadIdx.x;
  const int log_m = log_n - LOG_S;
  const int groups = 1 << (log_m - LOG_CW);
  const size_t row = blockIdx.x / groups;
  const size_t c0 = (size_t)(blockIdx.x % groups) << LOG_CW;

  for (int e = tid; e < S / 2; e += NTHREADS) tw[e] = fe_load<F>(twn, (size_t)e << log_m);
  const uint32_t *in = src + row * src_stride * F::N;
  for (int idx = tid; idx < S * CW; idx += NTHREADS) {
    const int t = idx >> LOG_CW, v = idx & (CW - 1);
    const size_t pos = c0 + v + ((size_t)t << log_m);
    tile[t * LD + v] = pos < n_valid ? fe_load<F>(in, pos) : fe_zero<F>();
  }
  __syncthreads();
  dif_all<F, LOG_S, LOG_CW, R, 0>(tile, tw, tid);

  uint32_t *out = dst + row * dst_stride * F::N;
  for (int idx = tid; idx < S * CW; idx += NTHREADS) {
    const int t = idx >> LOG_CW, v = idx & (CW - 1);
    const size_t c = c0 + v;
    const size_t e = c * (size_t)bitrev(t, LOG_S);
    Fe<F> x = tile[t * LD + v];
    if (e) x = fe_mul<F>(x, fe_load<F>(twn, e));
    fe_store<F>(out, c + ((size_t)t << log_m), x);
  }
}

template <class F, int LOG_S, int LOG_E>
__global__ __launch_bounds__(NTHREADS) void k_ntt_pass_b(uint32_t *__restrict__ data,
                                                         size_t stride,
                                                         const uint32_t *__restrict__ twn,
                                                         int log_n) {
  constexpr int LOG_CW = LOG_E - LOG_S;
  constexpr int S = 1 << LOG_S, CW = 1 << LOG_CW, LD = CW + 1;
  constexpr int R = LOG_E - 8;
  __shared__ __align__(16) uint32_t smem[(S * LD + S / 2) * F::N];
  Fe<F> *tile = reinterpret_cast<Fe<F> *>(smem);
  Fe<F> *tw = tile + S * LD;
  const int tid = threadIdx.x;
  const int log_blocks = log_n - LOG_S;  // contiguous S-blocks per row
  const int groups = 1 << (log_blocks - LOG_CW);
  const size_t row = blockIdx.x / groups;
  const size_t b0 = (size_t)(blockIdx.x % groups) << LOG_CW;

  for (int e = tid; e < S / 2; e += NTHREADS) tw[e] = fe_load<F>(twn, (size_t)e << log_blocks);
  uint32_t *io = data + (row * stride + b0 * S) * F::N;
  for (int idx = tid; idx < S * CW; idx += NTHREADS) {
    const int v = idx >> LOG_S, t = idx & (S - 1);
    tile[t * LD + v] = fe_load<F>(io, idx);
  }
  __syncthreads();
  dif_all<F, LOG_S, LOG_CW, R, 0>(tile, tw, tid);
  for (int idx = tid; idx < S * CW; idx += NTHREADS) {
    const int v = idx >> LOG_S, t = idx & (S - 1);
    fe_store<F>(io, idx, tile[t * LD + v]);
  }
}

template <class F>
constexpr int log_elems() {
  return F::N >= 8 ? 11 : 12;  // 64 KiB-class tiles; 32-byte fields use 2^11
}

template <class F, int LOG_S>
hipError_t launch_a(const uint32_t *src, size_t ss, size_t nv, uint32_t *dst, size_t ds,
                    const uint32_t *tw, int log_n, size_t n_rows, hipStream_t s) {
  constexpr int LE = log_elems<F>();
  const size_t groups = (size_t)1 << (log_n - LOG_S - (LE - LOG_S));
  prof::Scope ps("ntt_pass_a", s);
  hipLaunchKernelGGL((k_ntt_pass_a<F, LOG_S, LE>), dim3(n_rows * groups), dim3(NTHREADS), 0, s,
                     src, ss, nv, dst, ds, tw, log_n);
  return hipGetLastError();
}

template <class F, int LOG_S>
hipError_t launch_b(uint32_t *dst, size_t ds, const uint32_t *tw, int log_n, size_t n_rows,
                    hipStream_t s) {
  constexpr int LE = log_elems<F>();
  const size_t groups = (size_t)1 << (log_n - LOG_S - (LE - LOG_S));
  prof::Scope ps("ntt_pass_b", s);
  hipLaunchKernelGGL((k_ntt_pass_b<F, LOG_S, LE>), dim3(n_rows * groups), dim3(NTHREADS), 0, s,
                     dst, ds, tw, log_n);
  return hipGetLastError();
}

template <class F, int LO, int HI, class Fn>
hipError_t dispatch_logs(int l, Fn &&fn) {
  if constexpr (LO > HI) {
    return hipErrorInvalidValue;
  } else {
    if (l == LO) return fn.template operator()<LO>();
    return dispatch_logs<F, LO + 1, HI>(l, fn);
  }
}

template <class F>
hipError_t ntt_rows_v1(const NttPlan &p, const uint32_t *src, size_t ss, size_t nv, uint32_t *dst,
                      size_t ds, size_t n_rows, hipStream_t s) {
  if (n_rows == 0) return hipSuccess;
  if (p.log_n == 0) {  // length-1 transform is the identity (fffft returns early)
    return hipMemcpy2DAsync(dst, ds * F::N * 4, src, ss * F::N * 4, nv ? F::N * 4 : 0, n_rows,
                            hipMemcpyDeviceToDevice, s);
  }
  if (p.log_n <= 12) {
    prof::Scope ps("ntt_small", s);
    hipLaunchKernelGGL((k_ntt_small<F>), dim3(n_rows), dim3(NTHREADS), 0, s, src, ss, nv, dst, ds,
                       p.d_tw, p.log_n, (uint32_t *)nullptr, (size_t)0, 0);
    return hipGetLastError();
  }
  constexpr int LE = log_elems<F>();
  hipError_t e = dispatch_logs<F, 6, LE>(p.l1, [&]<int L>() {
    return launch_a<F, L>(src, ss, nv, dst, ds, p.d_tw, p.log_n, n_rows, s);
  });
  if (e != hipSuccess) return e;
  return dispatch_logs<F, 6, LE>(p.l2, [&]<int L>() {
    return launch_b<F, L>(dst, ds, p.d_tw, p.log_n, n_rows, s);
  });
}

}  // namespace ntt_v1
}  // namespace lcpc
