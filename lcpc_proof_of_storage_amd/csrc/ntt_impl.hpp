// ntt_impl.hpp -- Ligero Reed-Solomon encode (fffft::fft_io semantics) on gfx950.
//
// Replaces LigeroEncodingRho::encode -> FieldFFT::fft_io_pc (lcpc-ligero-pc/src/lib.rs:162-164)
// as called row-parallel by commit (lcpc-2d/src/lib.rs:677-682) and by verify on single rows
// (lcpc-2d/src/lib.rs:913-918, 944-950).  Output contract (bit-exact): for a length-n row
// whose first n_valid entries are the coefficients and the rest zero,
//     out[bitrev_log_n(j)] = sum_i in[i] * w^(i*j),   w = ROOT_OF_UNITY^(2^(S - log_n)).
//
// Four-step decomposition, n = 2^l1 * 2^l2, i = c + M t (M = 2^l2, t < 2^l1), j = j1 + 2^l1 j2:
//   pass A (per column c): Y_c[j1] = sum_t x[c + M t] w_{2^l1}^(t j1), stored DIF-style at
//           t' = bitrev_l1(j1), times w^(c j1); zero padding is applied while loading, so the
//           coefficient matrix is read directly (no padded copy);
//   pass B (per contiguous block t'): the 2^l2-point DIF over c, in place.
// Position t' M + c' then holds X_{j1 + 2^l1 j2} with j1 = bitrev(t'), j2 = bitrev(c'), which
// is exactly out[bitrev_log_n(j)].
//
// Passes (ntt_v2.hpp): each workgroup owns a tile of CW sub-FFT vectors; the first radix-2^R
// round reads HBM directly, rounds exchange through one padded LDS tile, and pass A's last round
// applies the inter-pass twiddle and writes HBM directly.  Rows of length <= 2^12 use a single
// whole-row-in-LDS kernel (k_ntt_small).  The last DIF stage of every sub-FFT has twiddle 1 and
// is multiplication-free at compile time.
#pragma once
#include "field.hpp"
#include "kernels.hpp"
#include "ntt_row1.hpp"
#include "ntt_v2.hpp"
#include "prof.hpp"

#include <cstdlib>

namespace lcpc {
namespace ntt_detail {

constexpr int NTHREADS = 256;

template <class F>
__global__ void k_tw_table(uint32_t *__restrict__ tw, int log_n, int inverse) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)1 << log_n;
  if (e >= n) return;
  Fe<F> w;
#pragma unroll
  for (int i = 0; i < F::N; i++) w.v[i] = inverse ? F::ROOT_INV[i] : F::ROOT[i];
  for (int i = 0; i < F::S - log_n; i++) w = fe_sqr<F>(w);
  fe_store<F>(tw, e, fe_pow<F>(w, e));
}

__device__ __forceinline__ int bitrev(int x, int bits) {
  return bits ? (int)(__builtin_bitreverse32((uint32_t)x) >> (32 - bits)) : 0;
}

// Whole row in LDS (log_n <= 12): plain radix-2 DIF stages.
template <class F>
__global__ __launch_bounds__(NTHREADS) void k_ntt_small(const uint32_t *__restrict__ src,
                                                        size_t src_stride, size_t n_valid,
                                                        uint32_t *__restrict__ dst,
                                                        size_t dst_stride,
                                                        const uint32_t *__restrict__ twn,
                                                        int log_n, uint32_t *__restrict__ copy,
                                                        size_t copy_stride, int canon) {
  __shared__ __align__(16) uint32_t smem[4096 * F::N];
  Fe<F> *buf = reinterpret_cast<Fe<F> *>(smem);
  const size_t row = blockIdx.x;
  const int n = 1 << log_n;
  const uint32_t *in = src + row * src_stride * F::N;
  uint32_t *cp = copy ? copy + row * copy_stride * F::N : nullptr;
  for (int i = threadIdx.x; i < n; i += NTHREADS) {
    if ((size_t)i < n_valid) {
      buf[i] = fe_load<F>(in, i);
      if (cp) fe_store<F>(cp, i, buf[i]);
    } else {
      buf[i] = fe_zero<F>();
    }
  }
  for (int gap = n / 2; gap > 0; gap /= 2) {
    __syncthreads();
    const int nchunks = n / (2 * gap);
    for (int i = threadIdx.x; i < n / 2; i += NTHREADS) {
      const int chunk = i / gap, j = i % gap;
      const int base = chunk * 2 * gap;
      const Fe<F> a = buf[base + j], b = buf[base + j + gap];
      buf[base + j] = fe_add<F>(a, b);
      buf[base + j + gap] = j ? fe_mul<F>(fe_sub_lazy<F>(a, b), fe_load<F>(twn, (size_t)nchunks * j))
                              : fe_sub<F>(a, b);
    }
  }
  __syncthreads();
  uint32_t *out = dst + row * dst_stride * F::N;
  for (int i = threadIdx.x; i < n; i += NTHREADS) fe_store<F>(out, i, canon ? fe_from_mont<F>(buf[i]) : buf[i]);
}

// Per-field tile shapes for the v2 passes (tools/microbench/nttbench.hip sweep on MI355X):
// R = log2(elements per thread per round), E = log2(tile elements per workgroup).
template <class F>
struct Shape;
template <>
struct Shape<Ft63> {
  static constexpr int R = 3, E = 12;
};
template <>
struct Shape<Ft127> {
  static constexpr int R = 3, E = 11;
};
template <>
struct Shape<Ft255> {
  static constexpr int R = 2, E = 10;
};
template <>
struct Shape<Ft253_192> {
  static constexpr int R = 2, E = 10;
};
template <>
struct Shape<Ft191> {
  static constexpr int R = 2, E = 10;
};

template <int LOG_S, int E>
constexpr int log_cw() {
  return E > LOG_S ? E - LOG_S : 0;
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
__global__ void k_from_mont_rows(uint32_t *__restrict__ m, size_t stride, size_t n_rows) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < n_rows) fe_store<F>(m, r * stride, fe_from_mont<F>(fe_load<F>(m, r * stride)));
}

template <class F>
hipError_t ntt_rows_t(const NttPlan &p, const uint32_t *src, size_t ss, size_t nv, uint32_t *dst,
                      size_t ds, size_t n_rows, hipStream_t s, uint32_t *cp, size_t cs, bool canon) {
  if (n_rows == 0) return hipSuccess;
  if (canon && !p.d_tw_canon) return hipErrorInvalidValue;
  if (p.log_n > 12 && !(canon ? p.d_tw2_canon : p.d_tw2)) return hipErrorInvalidValue;
  if (p.log_n == 0) {  // length-1 transform is the identity (fffft returns early)
    if (cp && nv) {
      hipError_t e = hipMemcpy2DAsync(cp, cs * F::N * 4, src, ss * F::N * 4, F::N * 4, n_rows,
                                      hipMemcpyDeviceToDevice, s);
      if (e != hipSuccess) return e;
    }
    if (!nv) return hipMemset2DAsync(dst, ds * F::N * 4, 0, F::N * 4, n_rows, s);
    hipError_t e = hipMemcpy2DAsync(dst, ds * F::N * 4, src, ss * F::N * 4, F::N * 4, n_rows,
                                    hipMemcpyDeviceToDevice, s);
    if (e != hipSuccess || !canon) return e;
    hipLaunchKernelGGL((k_from_mont_rows<F>), dim3((unsigned)((n_rows + 255) / 256)), dim3(256), 0, s, dst, ds,
                       n_rows);
    return hipGetLastError();
  }
  if (p.log_n <= 12) {
    prof::Scope ps("ntt_small", s);
    hipLaunchKernelGGL((k_ntt_small<F>), dim3(n_rows), dim3(NTHREADS), 0, s, src, ss, nv, dst, ds,
                       p.d_tw, p.log_n, cp, cs, canon ? 1 : 0);
    return hipGetLastError();
  }
  constexpr int R = Shape<F>::R, E = Shape<F>::E;
  const bool halfz = 2 * nv <= ((size_t)1 << p.log_n);
  if constexpr (F::ID == 0) {
    // PoS default dims: element rows take the four-step pair (2.57 ms per 1 GiB request against
    // 2.97 for the one-pass kernel on elements) unless the encoding asks for the
    // one-pass row kernel (ntt_row1.hpp; LCPC_ROW_KERNEL_ONEPASS)
    if (p.log_n == ntt_row1::LOG_N && halfz && p.row_kernel == 2)
      return ntt_row1::launch<F>(p, src, ss, nv, dst, ds, n_rows, s, cp, cs, canon);
  }
  constexpr int HI = F::N >= 8 ? 11 : 12;  // LDS budget of 32-byte fields
  auto pass_a = [&]<int L, int CW, int T = L + CW - R>() {
    // the inter-pass twiddles in [t][c] layout (canonical words for canon_out)
    const uint32_t *t2 = canon ? p.d_tw2_canon : p.d_tw2;
    if (halfz && canon)
      return ntt_v2::launch_a<F, L, CW, T, true, true>(src, ss, nv, dst, ds, p.d_tw, p.log_n, n_rows, s, cp, cs, t2);
    if (halfz)
      return ntt_v2::launch_a<F, L, CW, T, true>(src, ss, nv, dst, ds, p.d_tw, p.log_n, n_rows, s, cp, cs, t2);
    if (canon)
      return ntt_v2::launch_a<F, L, CW, T, false, true>(src, ss, nv, dst, ds, p.d_tw, p.log_n, n_rows, s, cp, cs, t2);
    return ntt_v2::launch_a<F, L, CW, T, false>(src, ss, nv, dst, ds, p.d_tw, p.log_n, n_rows, s, cp, cs, t2);
  };
  hipError_t e;
  if constexpr (F::ID == 1) {
    // cfg2 (2^14-point rows, 128 rows per 2^20-coefficient commitment): both passes over 32
    // vectors of 128 points in 1024 threads, radix-2^2 register rounds -- one launch holds only
    // 1024 tiles of the default shape (one partial wave of blocks), and twice the waves per CU
    // hide its load and store phases: 0.059 against 0.066 ms for the pair
    // (tools/microbench/nttbench.hip mode 2, profiles/r05_nttbench_cfg2.txt)
    if (p.log_n == 14 && p.l1 == 7) {
      if ((e = pass_a.template operator()<7, 5, 10>()) != hipSuccess) return e;
      return ntt_v2::launch_b<F, 7, 5, 10>(dst, ds, p.d_tw, p.log_n, n_rows, s);
    }
  }
  if constexpr (F::ID == 0) {
    // PoS default dims (n_cols = 2^15, ntt_plan_init's l1 = 8): pass A over 32 columns of
    // 256-point DIFs in 1024 threads (tools/microbench/nttbench.hip mode 5, fastest split).
    if (p.log_n == 15 && p.l1 == 8)
      e = pass_a.template operator()<8, 5>();
    else
      e = dispatch_logs<F, 6, HI>(p.l1, [&]<int L>() { return pass_a.template operator()<L, log_cw<L, E>()>(); });
  } else {
    e = dispatch_logs<F, 6, HI>(p.l1, [&]<int L>() { return pass_a.template operator()<L, log_cw<L, E>()>(); });
  }
  if (e != hipSuccess) return e;
  return dispatch_logs<F, 7, HI>(p.l2, [&]<int L>() {
    constexpr int CW = log_cw<L, E>();
    constexpr int T = L + CW - R;
    return ntt_v2::launch_b<F, L, CW, T>(dst, ds, p.d_tw, p.log_n, n_rows, s);
  });
}

}  // namespace ntt_detail
}  // namespace lcpc
