// sdig.hip -- Brakedown / SDIG encode on gfx950 (see sdig.hpp).
//
// Layout: the codeword of R rows is element-major, cw[j][b] = element j of row b.  A sparse
// level y = M x becomes, for every output j and row b, y[j][b] = sum_k val[k] * x[idx[k]][b]
// over the nonzeros k of output row j (CSR).  Threads are (j, b) pairs with b fastest: the R
// threads of one output read the same nonzero (one broadcast load) and R adjacent elements of
// one input (a coalesced R * B-byte run), so no gather is scattered even though the matrix is.
// Field sums are exact, so the CSR order (vs sprs' CSC dot) cannot change a bit.
//
// Ft127 runs the levels on the int8 matrix cores instead (k_spmm_mfma), with the digit
// decomposition of collapse_mfma.hpp: the matrix values are the small, reused operand (each one
// multiplies R codeword elements), so every nonzero val_k is expanded into the balanced digits
// h[k][a][u] of H_ka = val_k 2^(8a) mod p, and an output is
//     Y[u][b] = sum_(k, a) h[k][a][u] d_a(x[idx_k][b])          (one exact int32 GEMM per output)
//     y[b]   = REDC(sum_u Y[u][b] 2^(8u)) = sum_k val_k x[idx_k][b]  (Montgomery, bit-identical)
// A wave owns one output and TILES x 16 rows; each v_mfma_i32_16x16x64_i8 takes 4 nonzeros
// (K = 4 x 16 digits) x 16 rows (N) x the 16 digit positions (M).  A 16-byte codeword element
// is one lane's B fragment straight from the element-major layout, so the VALU work per
// (nonzero, row) is the 8-op balanced-digit conversion, against ~22 v_mad_u64_u32 + carries of
// the VALU product.  The h digits are derived in the kernel, once per (nonzero, wave): the 64
// lanes of a 4-nonzero group are its 64 (k, a) pairs, each computes H_ka with one Montgomery
// product, and a 16 x 16 byte transpose through LDS gives every lane its A fragment.  Reading a
// 16-B value per nonzero instead of a 256-B digit table cuts ~18 % of a level's gather traffic.
#include <cstdlib>

#include "collapse_mfma.hpp"
#include "field.hpp"
#include "kernels.hpp"
#include "prof.hpp"
#include "sdig.hpp"

namespace lcpc {

namespace {

template <class F>
__global__ __launch_bounds__(256) void k_spmm(const uint32_t *__restrict__ ptr,
                                              const uint32_t *__restrict__ idx,
                                              const uint32_t *__restrict__ val,
                                              const uint32_t *__restrict__ x,
                                              uint32_t *__restrict__ y, size_t m, uint32_t R,
                                              uint32_t b0, uint32_t nb) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= m * nb) return;
  const size_t j = t / nb;
  const uint32_t b = b0 + (uint32_t)(t - j * nb);
  Fe<F> acc = fe_zero<F>();
  const uint32_t k1 = ptr[j + 1];
  uint32_t k = ptr[j];
  // K nonzeros per step, one Montgomery reduction per K products (fe_dot, lazy reduction)
  constexpr int K = fe_dot_kmax<F>() < 4 ? fe_dot_kmax<F>() : 4;
  for (; k + K <= k1; k += K) {
    Fe<F> v[K], xs[K];
#pragma unroll
    for (int q = 0; q < K; q++) {
      v[q] = fe_load<F>(val, k + q);
      xs[q] = fe_load<F>(x, (size_t)idx[k + q] * R + b);
    }
    acc = fe_add<F>(acc, fe_dot<F, K>(v, xs));
  }
  for (; k < k1; k++)
    acc = fe_add<F>(acc, fe_mul<F>(fe_load<F>(val, k), fe_load<F>(x, (size_t)idx[k] * R + b)));
  fe_store<F>(y, j * R + b, acc);
}

// One wave per output j (4 per block), rows [b0, b0 + 16 TILES) with b0 = 16 TILES blockIdx.y.
// Lane (n = lane & 15, g = lane >> 4): A fragment = h of padded nonzero 4q + g at digit
// position n; B fragment of tile t = the digits of x[idx][b0 + 16 t + n].  The output's
// neighbour list (pidx) is staged in LDS first.  |Y| < 2^27 needs at most 512 nonzeros per
// output (checked when the plan is built).
//
// The A fragment: lane (n, g) computes H = gval[4q + g] 2^(8n) mod p (a = n; the Montgomery
// product with the constant 2^(8n) R mod p) and its balanced digits, i.e. bytes u = 0..15 of
// h[k][a = n][.]; the fragment wants bytes a = 0..15 of h[k][.][u = n].  The 16 lanes of a group
// exchange them through LDS as dwords (T[g][u / 4][a]), and each lane picks byte n % 4 of the 16
// dwords it reads with three v_perm_b32 per output dword.
constexpr int SPMM_MAX_GROUPS = 128;  // 512 nonzeros
__device__ __forceinline__ uint32_t pick4(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t sel_lo,
                                          uint32_t sel_hi) {
  // bytes (beta of d0, beta of d1, beta of d2, beta of d3); sel_lo = {beta, 4 + beta, 0x0c, 0x0c}
  const uint32_t t = __builtin_amdgcn_perm(d1, d0, sel_lo);
  const uint32_t s = __builtin_amdgcn_perm(d3, d2, sel_lo);
  return __builtin_amdgcn_perm(s, t, sel_hi);
}
// SPLIT = 4 (the small levels): the four waves of a block share ONE output and take its
// 4-nonzero groups in turn (wave w: groups w, w + 4, ...); their int32 digit sums are added
// through LDS before the one reduction.  A level with few outputs is latency-bound -- each wave's
// groups are a dependent gather -> MFMA chain -- and this cuts that chain by four.
template <class F, int TILES, int SPLIT = 1>
__global__ __launch_bounds__(256) void k_spmm_mfma(const uint32_t *__restrict__ gptr,
                                                   const uint32_t *__restrict__ pidx,
                                                   const uint32_t *__restrict__ gval,
                                                   const uint32_t *__restrict__ x,
                                                   uint32_t *__restrict__ y, size_t m, uint32_t R,
                                                   uint32_t row0, uint32_t row_end) {
  static_assert(F::N == 4, "Ft127 layout");
  __shared__ int red[4][TILES][16][17];
  __shared__ uint32_t nbr[4][4 * SPMM_MAX_GROUPS];
  __shared__ uint32_t tr[4][2][4][4][16];  // [wave][buffer][g][u / 4][a]
  static_assert(SPLIT == 1 || SPLIT == 4, "one output per wave, or per block of four waves");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t j = SPLIT == 1 ? (size_t)blockIdx.x * 4 + wave : (size_t)blockIdx.x;
  if (j >= m) return;  // whole waves (SPLIT: the whole block) only: they synchronise below
  const int n = lane & 15, g = lane >> 4;
  const size_t b0 = row0 + (size_t)blockIdx.y * TILES * 16;
  const uint32_t q0 = gptr[j], nq = gptr[j + 1] - q0;
  uint32_t *nb = nbr[wave];
  for (uint32_t i = lane; i < 4 * nq; i += 64) nb[i] = pidx[4 * (size_t)q0 + i];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // this lane's multiplier 2^(8n) R mod p and byte selectors
  Fe<F> pw = fe_zero<F>();
  pw.v[n >> 2] = 1u << (8 * (n & 3));
  const Fe<F> pn = fe_to_mont<F>(pw);
  const uint32_t beta = (uint32_t)(n & 3);
  const uint32_t sel_lo = beta | ((4u + beta) << 8) | 0x0c0c0000u, sel_hi = 0x05040100u;
  const uint4 *x4 = reinterpret_cast<const uint4 *>(x);
  const uint4 *v4 = reinterpret_cast<const uint4 *>(gval);
  bool rowok[TILES];
#pragma unroll
  for (int t = 0; t < TILES; t++) rowok[t] = b0 + 16 * t + n < row_end;
  cmfma::v4i acc[TILES];
#pragma unroll
  for (int t = 0; t < TILES; t++) acc[t] = cmfma::v4i{0, 0, 0, 0};
  auto load = [&](uint32_t q, uint4 *xv, uint4 &vv) {
    const size_t kk = 4 * ((size_t)q0 + q) + g;
    const size_t id = nb[4 * q + g];
    vv = v4[kk];
#pragma unroll
    for (int t = 0; t < TILES; t++)
      xv[t] = rowok[t] ? x4[id * R + b0 + 16 * t + n] : make_uint4(0, 0, 0, 0);
  };
  uint4 xc[TILES], xn[TILES], vc, vn;
  const uint32_t q_first = SPLIT == 1 ? 0u : (uint32_t)wave;
  if (q_first < nq) load(q_first, xc, vc);
  for (uint32_t q = q_first; q < nq; q += SPLIT) {
    const bool more = q + SPLIT < nq;
    if (more) load(q + SPLIT, xn, vn);
    // A fragment of group q
    Fe<F> v;
    v.v[0] = vc.x; v.v[1] = vc.y; v.v[2] = vc.z; v.v[3] = vc.w;
    const Fe<F> h = fe_mul<F>(v, pn);
    const cmfma::v4i hd = cmfma::balanced_digits(h.v[0], h.v[1], h.v[2], h.v[3]);
    uint32_t(*T)[4][16] = tr[wave][(q / SPLIT) & 1];
    T[g][0][n] = (uint32_t)hd.x;
    T[g][1][n] = (uint32_t)hd.y;
    T[g][2][n] = (uint32_t)hd.z;
    T[g][3][n] = (uint32_t)hd.w;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint4 *row = reinterpret_cast<const uint4 *>(T[g][n >> 2]);
    const uint4 r0 = row[0], r1 = row[1], r2 = row[2], r3 = row[3];
    const cmfma::v4i av = cmfma::v4i{(int)pick4(r0.x, r0.y, r0.z, r0.w, sel_lo, sel_hi),
                                     (int)pick4(r1.x, r1.y, r1.z, r1.w, sel_lo, sel_hi),
                                     (int)pick4(r2.x, r2.y, r2.z, r2.w, sel_lo, sel_hi),
                                     (int)pick4(r3.x, r3.y, r3.z, r3.w, sel_lo, sel_hi)};
#pragma unroll
    for (int t = 0; t < TILES; t++) {
      const cmfma::v4i d = cmfma::balanced_digits(xc[t].x, xc[t].y, xc[t].z, xc[t].w);
      acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, d, acc[t], 0, 0, 0);
    }
    if (more) {
#pragma unroll
      for (int t = 0; t < TILES; t++) xc[t] = xn[t];
      vc = vn;
    }
  }
  // C/D layout: lane holds digit positions u = 4 g + i of row n of each tile; through this
  // wave's LDS slice, then one output row per lane (tiles 4 at a time)
  int(*rw)[16][17] = red[wave];
#pragma unroll
  for (int t = 0; t < TILES; t++) {
    rw[t][4 * g + 0][n] = acc[t].x;
    rw[t][4 * g + 1][n] = acc[t].y;
    rw[t][4 * g + 2][n] = acc[t].z;
    rw[t][4 * g + 3][n] = acc[t].w;
  }
  if constexpr (SPLIT == 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int p = 0; p < TILES; p += 4) {
      const int t = p + g;
      const size_t b = b0 + 16 * (size_t)t + n;
      if (t < TILES && b < row_end) {
        int Y[16];
#pragma unroll
        for (int u = 0; u < 16; u++) Y[u] = rw[t][u][n];
        fe_store<F>(y, j * R + b, cmfma::recombine_redc<F>(Y));
      }
    }
  } else {
    __syncthreads();  // every wave's partial digit sums are in red[]
    // thread (t, n): the four waves' sums for row n of tile t, then the one reduction
    for (int i = threadIdx.x; i < TILES * 16; i += 256) {
      const int t = i >> 4, r = i & 15;
      const size_t b = b0 + 16 * (size_t)t + r;
      if (b < row_end) {
        int Y[16];
#pragma unroll
        for (int u = 0; u < 16; u++) Y[u] = red[0][t][u][r] + red[1][t][u][r] + red[2][t][u][r] + red[3][t][u][r];
        fe_store<F>(y, j * R + b, cmfma::recombine_redc<F>(Y));
      }
    }
  }
}

// encode::reed_solomon (encode.rs:97-110): out[k] = sum_j in[j] (k+1)^j by Horner, per row b
template <class F>
__global__ __launch_bounds__(256) void k_reed_solomon(const uint32_t *__restrict__ in, size_t m,
                                                      uint32_t *__restrict__ out, size_t n_out,
                                                      uint32_t R, uint32_t b0, uint32_t nb) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_out * nb) return;
  const size_t k = t / nb;
  const uint32_t b = b0 + (uint32_t)(t - k * nb);
  Fe<F> x = fe_zero<F>();  // the point k + 1 (k < 2^32), into Montgomery form by one multiply
  x.v[0] = (uint32_t)(k + 1);
  x = fe_to_mont<F>(x);
  Fe<F> r = fe_zero<F>();
  for (size_t jj = m; jj-- > 0;) r = fe_add<F>(fe_mul<F>(r, x), fe_load<F>(in, jj * R + b));
  fe_store<F>(out, k * R + b, r);
}

// 32 x 32 element tiles through LDS (padded row: no repeated bank pattern down a column).
// MODE: TR_PLAIN copies elements; TR_FROM_MONT writes canonical values (the PoS on-disk repr);
// TR_TO_MONT reads canonical values, flags any that is not < p in *bad (from_repr's check).
// Source elements at flat offset r * ss + c >= n_flat also read as zero.  With `copy`, the
// (zero-padded) source is also written row-major to copy[r * cs + c] as it is read.
template <class F, int MODE>
__global__ __launch_bounds__(256) void k_transpose(const uint32_t *__restrict__ src, size_t rows,
                                                   size_t cols, size_t ss, size_t nv,
                                                   uint32_t *__restrict__ dst, size_t ds,
                                                   uint32_t *__restrict__ bad, size_t n_flat,
                                                   uint32_t *__restrict__ copy, size_t cs) {
  __shared__ Fe<F> tile[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const size_t c0 = (size_t)blockIdx.x * 32, r0 = (size_t)blockIdx.y * 32;
  bool ok = true;
  for (int i = ty; i < 32; i += 8) {
    const size_t r = r0 + i, c = c0 + tx;
    Fe<F> x = (r < rows && c < cols && c < nv && r * ss + c < n_flat) ? fe_load<F>(src, r * ss + c)
                                                                      : fe_zero<F>();
    if (copy && r < rows && c < cols) fe_store<F>(copy, r * cs + c, x);  // lanes = adjacent columns
    if constexpr (MODE == TR_TO_MONT) {
      ok &= fe_is_canonical<F>(x);
      x = fe_to_mont<F>(x);
    }
    tile[i][tx] = x;
  }
  if constexpr (MODE == TR_TO_MONT) {
    if (!ok) atomicOr(bad, 1u);
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const size_t c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) {
      if constexpr (MODE == TR_FROM_MONT)
        fe_store<F>(dst, c * ds + r, fe_from_mont<F>(tile[tx][i]));
      else
        fe_store<F>(dst, c * ds + r, tile[tx][i]);
    }
  }
}

// rows per wave of k_spmm_mfma: chunks of at most 8 tiles of 16 rows, as few tiles as cover R
// (9 or 10 tiles per wave -- two commitments' 144 rows in one wave -- measured slower in round 4:
// 13.9-14.1 against 16.1 G/s; no longer built)
constexpr int MFMA_MAX_TILES = 8;
inline void mfma_tiling(size_t R, int &tiles, unsigned &chunks) {
  const size_t per = 16 * (size_t)MFMA_MAX_TILES;
  chunks = (unsigned)((R + per - 1) / per);
  tiles = (int)((R + 16 * chunks - 1) / (16 * chunks));
}

// levels with fewer outputs than this take the split kernel (four waves per output): the
// expander's small levels (SdigCode3 at cfg4: pre2-pre5 and post2-post5, 8-1864 outputs) are
// latency chains of 8-19 groups per wave, 15-26 us each with one wave per output
constexpr size_t SPMM_SPLIT_BELOW = 2048;

template <class F, int TILES>
void launch_spmm_mfma(const CsrDev &M, const uint32_t *x, uint32_t *y, size_t R, size_t b0, size_t nb,
                      unsigned chunks, hipStream_t s) {
  if (M.rows < SPMM_SPLIT_BELOW)
    hipLaunchKernelGGL((k_spmm_mfma<F, TILES, 4>), dim3((unsigned)M.rows, chunks), dim3(256), 0, s, M.gptr, M.pidx,
                       M.gval, x, y, M.rows, (uint32_t)R, (uint32_t)b0, (uint32_t)(b0 + nb));
  else
    hipLaunchKernelGGL((k_spmm_mfma<F, TILES>), dim3((unsigned)((M.rows + 3) / 4), chunks), dim3(256), 0, s,
                       M.gptr, M.pidx, M.gval, x, y, M.rows, (uint32_t)R, (uint32_t)b0, (uint32_t)(b0 + nb));
}

// y = M x on rows [b0, b0 + nb) of the element-major vectors (R rows)
template <class F>
hipError_t spmm(const SdigPlan &p, const CsrDev &M, const uint32_t *x, uint32_t *y, size_t R, size_t b0,
                size_t nb, hipStream_t s) {
  const size_t n = M.rows * nb;
  if (!n) return hipSuccess;
  if constexpr (F::N == 4 && F::ID == 1) {
    if (p.mfma) {
      int tiles;
      unsigned chunks;
      mfma_tiling(nb, tiles, chunks);
      switch (tiles) {
        case 1: launch_spmm_mfma<F, 1>(M, x, y, R, b0, nb, chunks, s); break;
        case 2: launch_spmm_mfma<F, 2>(M, x, y, R, b0, nb, chunks, s); break;
        case 3: launch_spmm_mfma<F, 3>(M, x, y, R, b0, nb, chunks, s); break;
        case 4: launch_spmm_mfma<F, 4>(M, x, y, R, b0, nb, chunks, s); break;
        case 5: launch_spmm_mfma<F, 5>(M, x, y, R, b0, nb, chunks, s); break;
        case 6: launch_spmm_mfma<F, 6>(M, x, y, R, b0, nb, chunks, s); break;
        case 7: launch_spmm_mfma<F, 7>(M, x, y, R, b0, nb, chunks, s); break;
        default: launch_spmm_mfma<F, 8>(M, x, y, R, b0, nb, chunks, s); break;
      }
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((k_spmm<F>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, M.ptr, M.idx,
                     M.val, x, y, M.rows, (uint32_t)R, (uint32_t)b0, (uint32_t)nb);
  return hipGetLastError();
}

template <class F>
hipError_t encode_rows_slice(const SdigPlan &p, uint32_t *cw, size_t R, size_t b0, size_t nb, uint32_t *tmp,
                             hipStream_t s) {
  constexpr int N = F::N;
  const int L = (int)p.pre.size();
  hipError_t e;
  // precodes all the way down (encode.rs:46-59): input [in_start, in_end), output right after
  size_t in_start = 0;
  for (int i = 0; i + 1 < L; i++) {
    const CsrDev &M = p.pre[i];
    const size_t in_end = in_start + M.cols;
    if ((e = spmm<F>(p, M, cw + in_start * R * N, cw + in_end * R * N, R, b0, nb, s)) != hipSuccess) return e;
    in_start = in_end;
  }
  // last precode into scratch, then Reed-Solomon into the codeword (:61-74)
  const CsrDev &ML = p.pre[L - 1];
  const size_t in_end = in_start + ML.cols;
  if ((e = spmm<F>(p, ML, cw + in_start * R * N, tmp, R, b0, nb, s)) != hipSuccess) return e;
  const size_t n_rs = p.post[L - 1].cols;
  if (n_rs * nb) {
    hipLaunchKernelGGL((k_reed_solomon<F>), dim3((unsigned)((n_rs * nb + 255) / 256)), dim3(256), 0,
                       s, tmp, ML.rows, cw + in_end * R * N, n_rs, (uint32_t)R, (uint32_t)b0, (uint32_t)nb);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  // postcodes in reverse (:76-90): input [in_start, out_start), output at out_start
  size_t in_pos = in_end + ML.rows, out_pos = in_end + n_rs;
  for (int i = L - 1; i >= 0; i--) {
    in_pos -= p.pre[i].rows;
    const CsrDev &Q = p.post[i];
    if (out_pos - in_pos != Q.cols) return hipErrorInvalidValue;
    if ((e = spmm<F>(p, Q, cw + in_pos * R * N, cw + out_pos * R * N, R, b0, nb, s)) != hipSuccess) return e;
    out_pos += Q.rows;
  }
  if (in_pos != p.pre[0].cols || out_pos != p.n_cols) return hipErrorInvalidValue;
  return hipSuccess;
}

template <class F>
hipError_t encode_cm(const SdigPlan &p, uint32_t *cw, size_t R, uint32_t *tmp, hipStream_t s) {
  // (the whole chain over all R rows: running it on row slices so that a level's input stays in
  // the infinity cache measured slower, 1.14-2.0 against 0.85 ms)
  prof::Scope ps("sdig_encode", s);
  return encode_rows_slice<F>(p, cw, R, 0, R, tmp, s);
}

}  // namespace

hipError_t sdig_plan_mfma(SdigPlan &plan, const std::vector<CsrHost> &pre, const std::vector<CsrHost> &post,
                          hipStream_t s);

hipError_t sdig_plan_upload(SdigPlan &plan, int fid, const std::vector<CsrHost> &pre,
                            const std::vector<CsrHost> &post, hipStream_t s) {
  const int N = field_words(fid);
  auto bytes_of = [&](const CsrHost &h) {
    const size_t a = ((h.rows + 1) * 4 + 255) & ~(size_t)255;
    const size_t b = (h.idx.size() * 4 + 255) & ~(size_t)255;
    const size_t c = (h.idx.size() * N * 4 + 255) & ~(size_t)255;
    return a + b + c;
  };
  size_t total = 0;
  for (const auto &h : pre) total += bytes_of(h);
  for (const auto &h : post) total += bytes_of(h);
  hipError_t e = hipMalloc(&plan.d_buf, total ? total : 256);
  if (e != hipSuccess) return e;
  plan.fid = fid;
  plan.n_per_row = pre[0].cols;
  plan.n_cols = sdig_codeword_length(pre, post);
  plan.tmp_elems = pre.back().rows;
  uint8_t *cur = (uint8_t *)plan.d_buf;
  auto put = [&](const CsrHost &h, CsrDev &d) -> hipError_t {
    d.rows = h.rows;
    d.cols = h.cols;
    d.nnz = h.idx.size();
    const size_t a = ((h.rows + 1) * 4 + 255) & ~(size_t)255;
    const size_t b = (h.idx.size() * 4 + 255) & ~(size_t)255;
    const size_t c = (h.idx.size() * N * 4 + 255) & ~(size_t)255;
    d.ptr = (const uint32_t *)cur;
    d.idx = (const uint32_t *)(cur + a);
    d.val = (const uint32_t *)(cur + a + b);
    hipError_t r = hipMemcpyAsync(cur, h.ptr.data(), (h.rows + 1) * 4, hipMemcpyHostToDevice, s);
    if (r == hipSuccess && d.nnz)
      r = hipMemcpyAsync(cur + a, h.idx.data(), d.nnz * 4, hipMemcpyHostToDevice, s);
    if (r == hipSuccess && d.nnz)  // u64 limbs == little-endian u32 words
      r = hipMemcpyAsync(cur + a + b, h.val.data(), d.nnz * N * 4, hipMemcpyHostToDevice, s);
    cur += a + b + c;
    return r;
  };
  plan.pre.assign(pre.size(), CsrDev{});
  plan.post.assign(post.size(), CsrDev{});
  for (size_t i = 0; i < pre.size(); i++)
    if ((e = put(pre[i], plan.pre[i])) != hipSuccess) return e;
  for (size_t i = 0; i < post.size(); i++)
    if ((e = put(post[i], plan.post[i])) != hipSuccess) return e;
  if ((e = sdig_plan_mfma(plan, pre, post, s)) != hipSuccess) return e;
  return hipStreamSynchronize(s);  // host vectors may be freed after return
}

// The matrix-core forms of every level (Ft127; LCPC_NO_MFMA=1 keeps the VALU kernel for A/B
// runs).  Every output needs at most 4 SPMM_MAX_GROUPS nonzeros (the int32 accumulator bound).
hipError_t sdig_plan_mfma(SdigPlan &plan, const std::vector<CsrHost> &pre, const std::vector<CsrHost> &post,
                          hipStream_t s) {
  plan.mfma = false;
  if (plan.fid != Ft127::ID || no_mfma()) return hipSuccess;
  std::vector<const CsrHost *> hs;
  std::vector<CsrDev *> ds;
  for (size_t i = 0; i < pre.size(); i++) hs.push_back(&pre[i]), ds.push_back(&plan.pre[i]);
  for (size_t i = 0; i < post.size(); i++) hs.push_back(&post[i]), ds.push_back(&plan.post[i]);
  struct Form {
    std::vector<uint32_t> gptr, pidx;
    std::vector<uint64_t> gval;  // 2 u64 limbs per padded nonzero
  };
  std::vector<Form> f(hs.size());
  size_t total = 0;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  for (size_t m = 0; m < hs.size(); m++) {
    const CsrHost &h = *hs[m];
    Form &F = f[m];
    F.gptr.assign(h.rows + 1, 0);
    for (size_t j = 0; j < h.rows; j++) {
      const size_t nz = h.ptr[j + 1] - h.ptr[j];
      if (nz > 4 * (size_t)SPMM_MAX_GROUPS) return hipSuccess;  // VALU kernel for this plan
      F.gptr[j + 1] = F.gptr[j] + (uint32_t)((nz + 3) / 4);
    }
    const size_t groups = F.gptr[h.rows];
    F.pidx.assign(4 * groups, 0);
    F.gval.assign(8 * groups, 0);
    for (size_t j = 0; j < h.rows; j++)
      for (uint32_t k = h.ptr[j], q = 4 * F.gptr[j]; k < h.ptr[j + 1]; k++, q++) {
        F.pidx[q] = h.idx[k];
        F.gval[2 * q] = h.val[2 * (size_t)k];
        F.gval[2 * q + 1] = h.val[2 * (size_t)k + 1];
      }
    total += al((h.rows + 1) * 4) + al(4 * groups * 4) + al(4 * groups * 16);
  }
  hipError_t e = hipMalloc(&plan.d_mfma, total ? total : 256);
  if (e != hipSuccess) return e;
  uint8_t *cur = (uint8_t *)plan.d_mfma;
  for (size_t m = 0; m < hs.size() && e == hipSuccess; m++) {
    const CsrHost &h = *hs[m];
    CsrDev &d = *ds[m];
    const Form &F = f[m];
    d.groups = F.gptr[h.rows];
    d.gptr = (const uint32_t *)cur;
    d.pidx = (const uint32_t *)(cur + al((h.rows + 1) * 4));
    d.gval = (const uint32_t *)(cur + al((h.rows + 1) * 4) + al(4 * d.groups * 4));
    e = hipMemcpyAsync((void *)d.gptr, F.gptr.data(), F.gptr.size() * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && d.groups)
      e = hipMemcpyAsync((void *)d.pidx, F.pidx.data(), F.pidx.size() * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess && d.groups)
      e = hipMemcpyAsync((void *)d.gval, F.gval.data(), F.gval.size() * 8, hipMemcpyHostToDevice, s);
    cur += al((h.rows + 1) * 4) + al(4 * d.groups * 4) + al(4 * d.groups * 16);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);  // the host forms are freed on return
  if (e == hipSuccess) plan.mfma = true;
  return e;
}

void sdig_plan_free(SdigPlan &plan) {
  if (plan.d_buf) (void)hipFree(plan.d_buf);
  if (plan.d_mfma) (void)hipFree(plan.d_mfma);
  plan.d_buf = nullptr;
  plan.d_mfma = nullptr;
  plan.mfma = false;
  plan.pre.clear();
  plan.post.clear();
}

hipError_t sdig_encode_cm(const SdigPlan &plan, uint32_t *cw, size_t R, uint32_t *tmp,
                          hipStream_t s) {
  if (R == 0) return hipSuccess;
  return dispatch_field(plan.fid, [&]<class F>() { return encode_cm<F>(plan, cw, R, tmp, s); });
}

hipError_t transpose_elems(int fid, const uint32_t *src, size_t rows, size_t cols,
                           size_t src_stride, size_t n_valid, uint32_t *dst, size_t dst_stride,
                           hipStream_t s, int mode, uint32_t *bad, size_t n_flat, uint32_t *copy,
                           size_t copy_stride) {
  if (!rows || !cols) return hipSuccess;
  if (mode == TR_TO_MONT && !bad) return hipErrorInvalidValue;
  if (copy && mode == TR_TO_MONT) return hipErrorInvalidValue;  // (the copy holds the source words)
  return dispatch_field(fid, [&]<class F>() {
    prof::Scope ps("transpose", s);
    dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32));
    if (mode == TR_FROM_MONT)
      hipLaunchKernelGGL((k_transpose<F, TR_FROM_MONT>), grid, dim3(256), 0, s, src, rows, cols,
                         src_stride, n_valid, dst, dst_stride, bad, n_flat, copy, copy_stride);
    else if (mode == TR_TO_MONT)
      hipLaunchKernelGGL((k_transpose<F, TR_TO_MONT>), grid, dim3(256), 0, s, src, rows, cols,
                         src_stride, n_valid, dst, dst_stride, bad, n_flat, copy, copy_stride);
    else
      hipLaunchKernelGGL((k_transpose<F, TR_PLAIN>), grid, dim3(256), 0, s, src, rows, cols,
                         src_stride, n_valid, dst, dst_stride, bad, n_flat, copy, copy_stride);
    return hipGetLastError();
  });
}

}  // namespace lcpc
