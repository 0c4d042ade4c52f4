// pos.hip -- proof-of-storage producers around the commitment (proof-of-storage/src).
//
//   k_pack7      DataField::from_byte_vec for WriteableFt63 (fields/data_field.rs:38-46,
//                fields/writable_ft63.rs:35-40): 7 little-endian data bytes per element, zero
//                padded, stored as the element's RAW u64 limb (no Montgomery conversion).
//   k_unpack7    field_vec_to_byte_vec (data_field.rs:57-62): the low 7 bytes of every limb.
//   k_bitrev_scale / inverse plan
//                decode_row = fffft ifft_oi (lcpc_online.rs:568-574): with P the bit reversal
//                and fwd_w = P F_w (the encode kernels), ifft_oi(y) = n^-1 P fwd_{w^-1}(P y).
//   k_powers     form_side_vectors_for_polynomial_evaluation_from_point (lcpc_online.rs:603-627)
// verifiable_polynomial_evaluation (lcpc_online.rs:454-484) is collapse_rows over the encoded
// matrix (collapse.hip).
//
// Byte kernels move 8 elements (56 bytes = 7 aligned u64) per thread; k_pack7 stages a block's
// bytes and elements through LDS so its global loads and stores are coalesced 16-byte vectors.
#include "field.hpp"
#include "kernels.hpp"
#include "pos.hpp"
#include "prof.hpp"

namespace lcpc {

namespace {

// element k = bits [56k, 56k + 56) of the 448-bit little-endian run q
__device__ __forceinline__ uint64_t pack7_elem(const uint64_t q[7], int k) {
  const int bit = 56 * k, wi = bit >> 6, sh = bit & 63;
  uint64_t v = q[wi] >> sh;
  if (sh > 8 && wi + 1 < 7) v |= q[wi + 1] << (64 - sh);
  return v & 0x00ffffffffffffffull;
}

// A block packs 2048 elements (14336 bytes): the bytes come in as coalesced 16-byte loads into
// LDS, each thread unpacks its 56-byte run from there, and the 16 KiB of elements go out through
// LDS again as coalesced 16-byte stores (a lane's 7 and 8 u64 accesses straight to memory are
// 56 and 64 bytes apart across the wave).  A partial last block takes the per-thread path.
constexpr int PACK_EL = 2048, PACK_BYTES = 7 * PACK_EL;
__global__ __launch_bounds__(256) void k_pack7(const uint8_t *__restrict__ bytes, size_t n_bytes,
                                               uint64_t *__restrict__ out, size_t n_elems) {
  __shared__ __align__(16) uint64_t s_in[PACK_BYTES / 8];
  __shared__ __align__(16) uint64_t s_out[PACK_EL];
  const int tid = threadIdx.x;
  const size_t eb = (size_t)blockIdx.x * PACK_EL, bb = (size_t)blockIdx.x * PACK_BYTES;
  // (the API guarantees 8-byte buffers; the 16-byte path needs both 16-byte aligned)
  const bool a16 = (((uintptr_t)bytes | (uintptr_t)out) & 15) == 0;
  if (a16 && eb + PACK_EL <= n_elems && bb + PACK_BYTES <= n_bytes) {
    const uint4 *src = reinterpret_cast<const uint4 *>(bytes + bb);  // 16-byte aligned
    uint4 *si = reinterpret_cast<uint4 *>(s_in);
#pragma unroll
    for (int i = tid; i < PACK_BYTES / 16; i += 256) si[i] = src[i];
    __syncthreads();
    uint64_t q[7];
#pragma unroll
    for (int i = 0; i < 7; i++) q[i] = s_in[7 * tid + i];
#pragma unroll
    for (int k = 0; k < 8; k++) s_out[8 * tid + k] = pack7_elem(q, k);
    __syncthreads();
    uint4 *dst = reinterpret_cast<uint4 *>(out + eb);
    const uint4 *so = reinterpret_cast<const uint4 *>(s_out);
#pragma unroll
    for (int i = tid; i < PACK_EL / 2; i += 256) dst[i] = so[i];
    return;
  }
  const size_t t = (size_t)blockIdx.x * PACK_EL / 8 + tid;
  const size_t e0 = 8 * t;
  if (e0 >= n_elems) return;
  const size_t b0 = 56 * t;
  if (b0 + 56 <= n_bytes && e0 + 8 <= n_elems) {
    const uint64_t *w = reinterpret_cast<const uint64_t *>(bytes + b0);  // 8-byte aligned
    uint64_t q[7];
#pragma unroll
    for (int i = 0; i < 7; i++) q[i] = w[i];
#pragma unroll
    for (int k = 0; k < 8; k++) out[e0 + k] = pack7_elem(q, k);
  } else {
    for (size_t e = e0; e < e0 + 8 && e < n_elems; e++) {
      uint64_t v = 0;
      for (int k = 0; k < 7; k++) {
        const size_t b = 7 * e + k;
        if (b < n_bytes) v |= (uint64_t)bytes[b] << (8 * k);
      }
      out[e] = v;
    }
  }
}

__global__ __launch_bounds__(256) void k_unpack7(const uint64_t *__restrict__ elems, size_t n_elems,
                                                 uint8_t *__restrict__ out, size_t n_bytes) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t e0 = 8 * t, b0 = 56 * t;
  if (b0 >= n_bytes) return;
  if (b0 + 56 <= n_bytes && e0 + 8 <= n_elems) {
    uint64_t q[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint64_t v = elems[e0 + k] & 0x00ffffffffffffffull;
      const int bit = 56 * k, wi = bit >> 6, sh = bit & 63;
      q[wi] |= v << sh;
      if (sh > 8 && wi + 1 < 7) q[wi + 1] |= v >> (64 - sh);
    }
    uint64_t *w = reinterpret_cast<uint64_t *>(out + b0);
#pragma unroll
    for (int i = 0; i < 7; i++) w[i] = q[i];
  } else {
    for (size_t b = b0; b < b0 + 56 && b < n_bytes; b++) {
      const size_t e = b / 7;
      out[b] = e < n_elems ? (uint8_t)(elems[e] >> (8 * (b % 7))) : 0;
    }
  }
}

// out[r][bitrev(i)] = in[r][i] * scale   (scale given canonical, converted here)
template <class F>
__global__ __launch_bounds__(256) void k_bitrev_scale(const uint32_t *__restrict__ in,
                                                      uint32_t *__restrict__ out, int log_n,
                                                      size_t n_rows, Fe<F> scale_canon,
                                                      int do_scale) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)1 << log_n;
  if (t >= n * n_rows) return;
  const size_t r = t >> log_n, i = t & (n - 1);
  const size_t j = log_n ? (size_t)(__builtin_bitreverse64((uint64_t)i) >> (64 - log_n)) : 0;
  Fe<F> v = fe_load<F>(in, t);
  if (do_scale) v = fe_mul<F>(v, fe_to_mont<F>(scale_canon));
  fe_store<F>(out, r * n + j, v);
}

// m[r][j] <-> m[r][bitrev(j)], one thread per pair end j (the one with j < bitrev(j) swaps)
template <class F>
__global__ __launch_bounds__(256) void k_bitrev_inplace(uint32_t *__restrict__ m, size_t stride, int log_n,
                                                        size_t n_rows) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)1 << log_n;
  if (t >= n * n_rows) return;
  const size_t r = t >> log_n, i = t & (n - 1);
  const size_t j = log_n ? (size_t)(__builtin_bitreverse64((uint64_t)i) >> (64 - log_n)) : 0;
  if (i >= j) return;
  const Fe<F> a = fe_load<F>(m, r * stride + i), b = fe_load<F>(m, r * stride + j);
  fe_store<F>(m, r * stride + i, b);
  fe_store<F>(m, r * stride + j, a);
}

// dst[i] = base^(i * step_exp)  for i < n  (Montgomery)
template <class F>
__global__ __launch_bounds__(256) void k_powers(const uint32_t *__restrict__ base, uint64_t step_exp,
                                                size_t n, uint32_t *__restrict__ dst) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fe<F> b = fe_load<F>(base, 0);
  Fe<F> s = fe_pow<F>(b, step_exp);     // base^step
  fe_store<F>(dst, i, fe_pow<F>(s, (uint64_t)i));
}

}  // namespace

hipError_t pos_pack7(const uint8_t *bytes, size_t n_bytes, uint64_t *out, hipStream_t s) {
  const size_t n = (n_bytes + 6) / 7;
  if (!n) return hipSuccess;
  prof::Scope ps("pos_pack7", s);
  hipLaunchKernelGGL(k_pack7, dim3((unsigned)((n + PACK_EL - 1) / PACK_EL)), dim3(256), 0, s, bytes, n_bytes,
                     out, n);
  return hipGetLastError();
}

hipError_t pos_unpack7(const uint64_t *elems, size_t n_elems, uint8_t *out, size_t n_bytes,
                       hipStream_t s) {
  if (!n_bytes) return hipSuccess;
  const size_t threads = (n_bytes + 55) / 56;
  hipLaunchKernelGGL(k_unpack7, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, elems, n_elems,
                     out, n_bytes);
  return hipGetLastError();
}

hipError_t bitrev_scale(int fid, const uint32_t *in, uint32_t *out, int log_n, size_t n_rows,
                        const uint32_t *scale_canon_words, hipStream_t s) {
  const size_t total = ((size_t)1 << log_n) * n_rows;
  if (!total) return hipSuccess;
  return dispatch_field(fid, [&]<class F>() {
    Fe<F> sc{};
    if (scale_canon_words)
      for (int i = 0; i < F::N; i++) sc.v[i] = scale_canon_words[i];
    hipLaunchKernelGGL((k_bitrev_scale<F>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, in,
                       out, log_n, n_rows, sc, scale_canon_words ? 1 : 0);
    return hipGetLastError();
  });
}

hipError_t bitrev_rows_inplace(int fid, uint32_t *m, size_t stride, int log_n, size_t n_rows, hipStream_t s) {
  const size_t total = ((size_t)1 << log_n) * n_rows;
  if (!total || log_n == 0) return hipSuccess;
  return dispatch_field(fid, [&]<class F>() {
    hipLaunchKernelGGL((k_bitrev_inplace<F>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, m, stride,
                       log_n, n_rows);
    return hipGetLastError();
  });
}

hipError_t powers(int fid, const uint32_t *base, uint64_t step_exp, size_t n, uint32_t *dst,
                  hipStream_t s) {
  if (!n) return hipSuccess;
  return dispatch_field(fid, [&]<class F>() {
    hipLaunchKernelGGL((k_powers<F>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, base, step_exp,
                       n, dst);
    return hipGetLastError();
  });
}

}  // namespace lcpc
