// ntt_row1.hpp -- the 2^15-point Ft63 row encode in ONE pass (the proof-of-storage default
// dims: 16384 coefficients -> 32768 per row, 9363 rows per 1 GiB file; lcpc_online.rs:80-239
// commits them through LigeroEncodingRho::encode, lcpc-ligero-pc/src/lib.rs:162-164).
// Same contract as ntt_impl.hpp (fffft::fft_io, out[bitrev(j)] = sum_i in[i] w^(ij)), rate-1/2
// rows only (n_valid <= n / 2).
//
// One 1024-thread workgroup per row. The row (256 KiB) stays in registers, 32 elements per
// thread, and the 15 radix-2 DIF stages run as three radix-32 rounds over the index bits
// i = (hi << 10) | (mid << 5) | lo:
//   round 1: stages 0-4   (bits 14-10)  thread (mid, lo) holds hi  = 0..31
//   round 2: stages 5-9   (bits 9-5)    thread (hi, lo)  holds mid = 0..31
//   round 3: stages 10-14 (bits 4-0)    thread (hi, mid) holds lo  = 0..31
// Rounds exchange through one 128 KiB LDS buffer in two halves. The half is a bit that the
// writer's and the reader's thread numbering put at the SAME thread-id bit >= 6 (lo's top bit at
// bit 9 for exchange 1, hi's top bit at bit 8 for exchange 2), so each half is written and read
// back by the same 8 waves and no thread ever holds more than its own 32 elements. The output
// goes through LDS once more so the stores are contiguous 16-byte vectors.
//
// Against the four-step pair (k_pass_a + k_pass_b) at the PoS dims: no intermediate round trip
// (2 x 2.45 GB of HBM per 1 GiB request) and no inter-pass twiddle products; round 3's twiddles
// are w^(1024 k) with k known at compile time, so its trivial products drop out.
// CANON: the row is scaled by R^-1 on the way in -- the sum branch of the (HALFZ) first stage by
// a Montgomery reduction, the product branch through the canonical-word twiddle table -- so the
// Montgomery words written out are the canonical values (the ntt_rows canon_out contract).
#pragma once
#include "field.hpp"
#include "kernels.hpp"
#include "prof.hpp"

#include <cstdlib>

namespace lcpc {
namespace ntt_row1 {

constexpr int LOG_N = 15;
// Which rows take this kernel (NttPlan::row_kernel, LCPC_ROW_KERNEL_AUTO): the file-image commit
// (2.75 ms per 1 GiB request against 2.93 for k_pack7 + the four-step pair); element rows keep the
// four-step pair (2.57 against 2.97 ms) unless the encoding asks for this one.  The
// round-4 variants that measured slower -- persistent workgroups with an LDS-DMA prefetch, outputs
// stored from registers, the four-step pair unpacking in pass A -- are no longer built.

// element (hi, mid, lo & 15) of the half lo >> 4 (exchange 1); the XOR spreads a ds_read's lanes
// (16 values of hi) over 16 bank pairs
__device__ __forceinline__ int x1_at(int hi, int mid, int l4) { return (((hi << 5) | mid) << 4) | (l4 ^ (hi & 15)); }
// element (hi & 15, mid, lo) of the half hi >> 4 (exchange 2)
__device__ __forceinline__ int x2_at(int hi, int mid, int lo) {
  return ((hi & 15) << 10) | (mid << 5) | (lo ^ (hi & 15));
}

template <class F>
__device__ __forceinline__ void bfly(Fe<F> &a, Fe<F> &b, const Fe<F> &w) {
  const Fe<F> s = fe_add_2p<F>(a, b);
  b = fe_mul_lazy<F>(fe_sub_2p<F>(a, b), w);
  a = s;
}
template <class F>
__device__ __forceinline__ void bfly1(Fe<F> &a, Fe<F> &b) {  // twiddle 1
  const Fe<F> s = fe_add_2p<F>(a, b);
  b = fe_sub_2p<F>(a, b);
  a = s;
}
template <class F>
__device__ __forceinline__ Fe<F> lds_ld(const uint2 *t, int i) {
  const uint2 q = t[i];
  Fe<F> r;
  r.v[0] = q.x;
  r.v[1] = q.y;
  return r;
}
template <class F>
__device__ __forceinline__ void lds_st(uint2 *t, int i, const Fe<F> &x) {
  t[i] = make_uint2(x.v[0], x.v[1]);
}

// one DIF stage over the 32 register elements: pairs (j, j + HS), twiddle index tw_at(jm)
template <class F, int HS, class TwAt>
__device__ __forceinline__ void reg_stage(Fe<F> *x, TwAt &&tw_at) {
#pragma unroll
  for (int j = 0; j < 32; j++) {
    if (j & HS) continue;
    bfly<F>(x[j], x[j + HS], tw_at(j & (HS - 1)));
  }
}
// round 3's stage S (10..14): twiddle w^(jm << S) = wtab[jm << (S - 5)], 1 for jm = 0
template <class F, int S>
__device__ __forceinline__ void lo_stage(Fe<F> *x, const uint2 *wtab) {
  constexpr int HS = 16 >> (S - 10);
#pragma unroll
  for (int j = 0; j < 32; j++) {
    if (j & HS) continue;
    const int jm = j & (HS - 1);
    if (jm == 0)
      bfly1<F>(x[j], x[j + HS]);
    else
      bfly<F>(x[j], x[j + HS], lds_ld<F>(wtab, jm << (S - 5)));
  }
}

// tw: w^e (Montgomery, e < n); tw0: the first stage's table (canonical words when CANON).
// BYTES: src is a proof-of-storage file image of n_valid bytes, 7 little-endian bytes per element
// (DataField::from_byte_vec for WriteableFt63, fields/data_field.rs:38-46: the element's raw u64
// limb, zero-padded), row r = elements [16384 r, 16384 (r + 1)); the row's 112 KiB are staged in
// the exchange buffer with coalesced 16-byte loads and each thread unpacks its 16 elements from
// there -- k_pack7 fused into the encode (no element image written and read back).
constexpr int ROW_BYTES = 7 << 14;  // one row of the file image

// PF (file images): at the start of round 3 each thread touches one 128-byte line of
// the image row PF_DIST rows ahead (LDS-DMA into a 4 KiB scratch block: 139 KiB of LDS, still one
// workgroup per CU) -- the row the XCD's next free CU most likely takes next
// (workgroups go round-robin over the 8 XCDs, 32 CUs each) -- so that its byte load hits L2
constexpr int PF_DIST = 256;

// one dword of each 128-byte line of image row `ahead` by LDS-DMA (no VGPR destination; nothing
// waits on it before the next barrier), into a scratch block no one reads
__device__ __forceinline__ void pf_row(const uint32_t *src, size_t n_valid, size_t ahead, int tid, uint32_t *scratch) {
  const size_t b = ahead * (size_t)ROW_BYTES + 128 * (size_t)tid;
  if (ahead < gridDim.x && tid < ROW_BYTES / 128 && b + 4 <= n_valid)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void *)(reinterpret_cast<const uint8_t *>(src) + b),
        (__attribute__((address_space(3))) void *)(scratch + (tid & ~63)), 4, 0, 0);
}

// PF: where the prefetch is issued -- 0 none, 1 round 3's start (the default), 2 round 2's start,
// 3 the output phase's start (A/B: LCPC_ROW1_PREFETCH).  GLDS: a whole row's bytes are staged by
// LDS-DMA (global_load_lds_dwordx4: no VGPR round trip, no ds_write) instead of loads + ds_write
// (A/B: LCPC_ROW1_GLDS)
template <class F, bool CANON, bool COPY, bool BYTES, int PF = 0, bool GLDS = false>
__global__ __launch_bounds__(1024) void k_row_ntt15(const uint32_t *__restrict__ src, size_t src_stride,
                                                    size_t n_valid, uint32_t *__restrict__ dst, size_t dst_stride,
                                                    const uint32_t *__restrict__ tw,
                                                    const uint32_t *__restrict__ tw0,
                                                    uint32_t *__restrict__ copy, size_t copy_stride) {
  static_assert(F::N == 2, "8-byte fields");
  __shared__ __align__(16) uint2 xbuf[16384];  // half a row
  __shared__ uint2 wtab[512];                   // w^(32 k)
  __shared__ uint32_t pf_scratch[BYTES && PF ? 1024 : 1];
  const int tid = threadIdx.x;
  const size_t row = blockIdx.x;
  if (tid < 512) wtab[tid] = reinterpret_cast<const uint2 *>(tw)[32 * tid];
  Fe<F> x[32];
  {
    // ---- round 1: thread (mid, lo), lo's top bit at thread-id bit 9
    {
      const int lo = ((tid >> 9) << 4) | (tid & 15), mid = (tid >> 4) & 31;
      const int tl = (mid << 5) | lo;
      if constexpr (BYTES) {
        const size_t row0 = row * (size_t)ROW_BYTES;
        const uint8_t *rb = reinterpret_cast<const uint8_t *>(src) + row0;
        uint4 *sb = reinterpret_cast<uint4 *>(xbuf);
        if (GLDS && row0 + ROW_BYTES <= n_valid) {
          // a wave's 64 lanes take 64 consecutive 16-byte units: LDS base + lane x 16 is sb[i]
#pragma unroll
          for (int k = 0; k < ROW_BYTES / 16 / 1024; k++) {
            const int i = tid + 1024 * k;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(rb + 16 * (size_t)i),
                (__attribute__((address_space(3))) void *)(sb + (i & ~63)), 16, 0, 0);
          }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else
        for (int i = tid; i < ROW_BYTES / 16; i += 1024) {
          const size_t b = row0 + 16 * (size_t)i;
          if (b + 16 <= n_valid) {
            sb[i] = reinterpret_cast<const uint4 *>(rb)[i];
          } else {  // the file's last bytes: zero padded
            uint32_t w[4] = {0, 0, 0, 0};
            for (int k = 0; k < 16; k++)
              if (b + k < n_valid) w[k >> 2] |= (uint32_t)rb[16 * i + k] << (8 * (k & 3));
            sb[i] = make_uint4(w[0], w[1], w[2], w[3]);
          }
        }
      }
      if constexpr (BYTES) __syncthreads();  // the staged row (every wave's part) is in
      const uint32_t *in = src + row * src_stride * 2;
#pragma unroll
      for (int h = 0; h < 16; h++) {
        const int pos = (h << 10) | tl;
        Fe<F> a = fe_zero<F>();
        if constexpr (BYTES) {
          const uint32_t *sw = reinterpret_cast<const uint32_t *>(xbuf);
          const int b = 7 * pos, d = b >> 2, sh = b & 3;
          const uint32_t d0 = sw[d], d1 = sw[d + 1], d2 = sw[d + 2];  // (d + 2 < 32768: inside xbuf)
          a.v[0] = __builtin_amdgcn_alignbyte(d1, d0, sh);
          a.v[1] = __builtin_amdgcn_alignbyte(d2, d1, sh) & 0xffffffu;
          if constexpr (COPY) fe_store<F>(copy + row * copy_stride * 2, pos, a);
        } else if ((size_t)pos < n_valid) {
          a = fe_load<F>(in, pos);
          if constexpr (COPY) fe_store<F>(copy + row * copy_stride * 2, pos, a);
        }
        // stage 0 with x[h + 16] = 0: (a, a w^e)
        x[h + 16] = fe_mul_lazy<F>(a, fe_load<F>(tw0, pos));
        if constexpr (CANON)
          x[h] = fe_from_mont<F>(a);
        else
          x[h] = a;
      }
      if constexpr (BYTES) __syncthreads();  // every input read before exchange 1 reuses xbuf
      reg_stage<F, 8>(x, [&](int jm) { return fe_load<F>(tw, ((jm << 10) | tl) << 1); });
      reg_stage<F, 4>(x, [&](int jm) { return fe_load<F>(tw, ((jm << 10) | tl) << 2); });
      reg_stage<F, 2>(x, [&](int jm) { return fe_load<F>(tw, ((jm << 10) | tl) << 3); });
      reg_stage<F, 1>(x, [&](int jm) { return fe_load<F>(tw, ((jm << 10) | tl) << 4); });
      // ---- exchange 1: (mid, lo) -> (hi, lo), halves by lo >> 4
      const int lo2 = ((tid >> 9) << 4) | ((tid >> 4) & 15), hi2 = (((tid >> 8) & 1) << 4) | (tid & 15);
      auto xchg = [&](int ph) {
        if ((tid >> 9) == ph) {
#pragma unroll
          for (int h = 0; h < 32; h++) lds_st<F>(xbuf, x1_at(h, mid, lo & 15), x[h]);
        }
        __syncthreads();
        if ((tid >> 9) == ph) {
#pragma unroll
          for (int m = 0; m < 32; m++) x[m] = lds_ld<F>(xbuf, x1_at(hi2, m, lo2 & 15));
        }
        __syncthreads();
      };
      xchg(0);
      xchg(1);
    }
    // ---- round 2: thread (hi, lo) holds mid = 0..31; twiddles w^(((jm << 5) | lo) << s)
    if constexpr (BYTES && PF == 2) pf_row(src, n_valid, row + PF_DIST, tid, pf_scratch);
    {
      const int lo = ((tid >> 9) << 4) | ((tid >> 4) & 15), hi = (((tid >> 8) & 1) << 4) | (tid & 15);
      reg_stage<F, 16>(x, [&](int jm) { return lds_ld<F>(wtab, (jm << 5) | lo); });
      reg_stage<F, 8>(x, [&](int jm) { return lds_ld<F>(wtab, ((jm << 5) | lo) << 1); });
      reg_stage<F, 4>(x, [&](int jm) { return lds_ld<F>(wtab, ((jm << 5) | lo) << 2); });
      reg_stage<F, 2>(x, [&](int jm) { return lds_ld<F>(wtab, ((jm << 5) | lo) << 3); });
      reg_stage<F, 1>(x, [&](int jm) { return lds_ld<F>(wtab, ((jm << 5) | lo) << 4); });
      // ---- exchange 2: (hi, lo) -> (hi, mid), halves by hi >> 4 (thread-id bit 8 in both)
      const int mid3 = ((tid >> 9) << 4) | ((tid >> 4) & 15);
      auto xchg = [&](int ph) {
        if (((tid >> 8) & 1) == ph) {
#pragma unroll
          for (int m = 0; m < 32; m++) lds_st<F>(xbuf, x2_at(hi, m, lo), x[m]);
        }
        __syncthreads();
        if (((tid >> 8) & 1) == ph) {
#pragma unroll
          for (int l = 0; l < 32; l++) x[l] = lds_ld<F>(xbuf, x2_at(hi, mid3, l));
        }
        __syncthreads();
      };
      xchg(0);
      xchg(1);
    }
    // ---- round 3: thread (hi, mid) holds lo = 0..31; twiddles w^(jm << s) = wtab[jm << (s - 5)]
    if constexpr (BYTES && PF == 1) pf_row(src, n_valid, row + PF_DIST, tid, pf_scratch);
    const int mid = ((tid >> 9) << 4) | ((tid >> 4) & 15), hi = (((tid >> 8) & 1) << 4) | (tid & 15);
    lo_stage<F, 10>(x, wtab);
    lo_stage<F, 11>(x, wtab);
    lo_stage<F, 12>(x, wtab);
    lo_stage<F, 13>(x, wtab);
    lo_stage<F, 14>(x, wtab);
    {
      // ---- out: through LDS in halves (hi >> 4), 16-byte units u = ((hi & 15) << 9) | (mid << 4) | (lo >> 1)
      //      stored at u ^ (hi & 7): a ds_write's 64 lanes land on 8 distinct 16-byte bank slots
      if constexpr (BYTES && PF == 3) pf_row(src, n_valid, row + PF_DIST, tid, pf_scratch);
      uint4 *ubuf = reinterpret_cast<uint4 *>(xbuf);
      uint4 *out = reinterpret_cast<uint4 *>(dst + row * dst_stride * 2);
      auto store_half = [&](int ph) {
        if (((tid >> 8) & 1) == ph) {
#pragma unroll
          for (int lp = 0; lp < 16; lp++) {
            const Fe<F> a = fe_reduce_2p<F>(x[2 * lp]), b = fe_reduce_2p<F>(x[2 * lp + 1]);
            const int u = ((hi & 15) << 9) | (mid << 4) | lp;
            ubuf[u ^ (hi & 7)] = make_uint4(a.v[0], a.v[1], b.v[0], b.v[1]);
          }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const int u = (k << 10) | tid;
          out[(ph << 13) | u] = ubuf[u ^ ((u >> 9) & 7)];
        }
      };
      store_half(0);
      __syncthreads();
      store_half(1);
    }
  }
}

template <class F, bool CANON, bool COPY, bool BYTES, int PF = 0, bool GLDS = false>
hipError_t launch_t(const NttPlan &p, const uint32_t *src, size_t ss, size_t nv, uint32_t *dst, size_t ds,
                    size_t n_rows, hipStream_t s, uint32_t *cp, size_t cs) {
  const uint32_t *tw0 = CANON ? p.d_tw_canon : p.d_tw;
  prof::Scope ps("ntt_row1", s);
  hipLaunchKernelGGL((k_row_ntt15<F, CANON, COPY, BYTES, PF, GLDS>), dim3((unsigned)n_rows), dim3(1024), 0, s, src, ss, nv,
                     dst, ds, p.d_tw, tw0, cp, cs);
  return hipGetLastError();
}

template <class F>
hipError_t launch(const NttPlan &p, const uint32_t *src, size_t ss, size_t nv, uint32_t *dst, size_t ds,
                  size_t n_rows, hipStream_t s, uint32_t *cp, size_t cs, bool canon) {
  if (canon && cp) return launch_t<F, true, true, false>(p, src, ss, nv, dst, ds, n_rows, s, cp, cs);
  if (canon) return launch_t<F, true, false, false>(p, src, ss, nv, dst, ds, n_rows, s, cp, cs);
  if (cp) return launch_t<F, false, true, false>(p, src, ss, nv, dst, ds, n_rows, s, cp, cs);
  return launch_t<F, false, false, false>(p, src, ss, nv, dst, ds, n_rows, s, cp, cs);
}

// the proof-of-storage commit from the file image (BYTES above): canonical output, coefficient copy;
// the file's ragged last row (if any) is zero padded as it is staged
// the L2 prefetch above is the default: the kernel 2.51 -> 2.34 ms per 1 GiB request serially,
// the cfg5 line's median 36.1 -> 37.6 G el/s over eight interleaved pairs
// (profiles/r06_row1_prefetch_ab.json); LCPC_ROW1_PREFETCH=0 turns it off for A/B runs (read once)
inline int row1_prefetch() {
  static const int mode = [] {
    const char *e = std::getenv("LCPC_ROW1_PREFETCH");
    return (e && e[0] >= '0' && e[0] <= '3' && !e[1]) ? e[0] - '0' : 1;
  }();
  return mode;
}

// the LDS-DMA staging is the default with the round-3 prefetch: the kernel 2.36 -> 2.29 ms per
// 1 GiB request serially, the cfg5 line's median 35.1 -> 36.3 G el/s over four interleaved pairs
// (profiles/r06_row1_glds_ab.json); LCPC_ROW1_GLDS=0 stages through VGPRs + ds_write (read once)
inline bool row1_glds() {
  static const bool on = [] {
    const char *e = std::getenv("LCPC_ROW1_GLDS");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <class F>
hipError_t launch_bytes(const NttPlan &p, const uint8_t *bytes, size_t n_bytes, uint32_t *dst, size_t ds,
                        size_t n_rows, hipStream_t s, uint32_t *cp, size_t cs) {
  const uint32_t *b = reinterpret_cast<const uint32_t *>(bytes);
  if (row1_glds() && row1_prefetch() == 1)
    return launch_t<F, true, true, true, 1, true>(p, b, 0, n_bytes, dst, ds, n_rows, s, cp, cs);
  switch (row1_prefetch()) {
    case 0: return launch_t<F, true, true, true, 0>(p, b, 0, n_bytes, dst, ds, n_rows, s, cp, cs);
    case 2: return launch_t<F, true, true, true, 2>(p, b, 0, n_bytes, dst, ds, n_rows, s, cp, cs);
    case 3: return launch_t<F, true, true, true, 3>(p, b, 0, n_bytes, dst, ds, n_rows, s, cp, cs);
    default: return launch_t<F, true, true, true, 1>(p, b, 0, n_bytes, dst, ds, n_rows, s, cp, cs);
  }
}

}  // namespace ntt_row1
}  // namespace lcpc
