// blake3.hip -- column leaves and Merkle tree of an lcpc-2d commitment on gfx950.
//
// Replaces merkleize -> hash_columns / merkle_tree / merkle_layer (lcpc-2d/src/lib.rs:720-815)
// with D = blake3::Hasher (blake3 1.5):
//   leaf[j]  = BLAKE3(32 zero bytes || to_repr(comm[0][j]) || ... || to_repr(comm[n_rows-1][j]))
//   node     = BLAKE3(left || right)            (a 64-byte message, not a BLAKE3 parent node)
//   hashes   = [leaves (next_pow2(n_cols), zero-padded) | level 1 | ... | root]
// plus the opening-side gathers (open_column, :818-855) and the verifier's path check
// (verify_column_path, :985-1012).
//
// Leaves: the leaf message of a column is 32 + n_rows * B bytes (8224 B at 512 x Ft127), i.e.
// several 1-KiB BLAKE3 chunks.  One thread owns one (column, chunk): a wave is 64 adjacent
// columns of the same chunk, so every element load is a fully coalesced 1-KiB row segment of
// the row-major codeword (no transpose).  Chunk chaining values of multi-chunk leaves go to a
// [chunk][column] scratch (coalesced both ways) and a second kernel folds them with BLAKE3's
// left-balanced tree (pairwise per level, odd node carried up, ROOT on the last parent).
#include <cstdlib>

#include "field.hpp"
#include "kernels.hpp"
#include "prof.hpp"

namespace lcpc {

namespace {

constexpr uint32_t IV0 = 0x6A09E667u, IV1 = 0xBB67AE85u, IV2 = 0x3C6EF372u, IV3 = 0xA54FF53Au,
                   IV4 = 0x510E527Fu, IV5 = 0x9B05688Cu, IV6 = 0x1F83D9ABu, IV7 = 0x5BE0CD19u;
enum : uint32_t { CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8 };

// message schedule: round r uses m[SCHED[r][i]]  (permutation 2,6,3,10,7,0,4,13,1,11,12,5,9,14,15,8)
__host__ __device__ constexpr int sched(int r, int i) {
  constexpr int P[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
  int x = i;
  for (int k = 0; k < r; k++) x = P[x];
  return x;
}

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_rotateright32(x, n); }

#define B3G(a, b, c, d, mx, my)          \
  a = a + b + (mx);                      \
  d = rotr(d ^ a, 16);                   \
  c = c + d;                             \
  b = rotr(b ^ c, 12);                   \
  a = a + b + (my);                      \
  d = rotr(d ^ a, 8);                    \
  c = c + d;                             \
  b = rotr(b ^ c, 7);

// cv = first half of compress(cv, m, counter, len, flags)
__device__ __forceinline__ void compress(uint32_t cv[8], const uint32_t m[16], uint64_t counter,
                                         uint32_t block_len, uint32_t flags) {
  uint32_t s0 = cv[0], s1 = cv[1], s2 = cv[2], s3 = cv[3], s4 = cv[4], s5 = cv[5], s6 = cv[6],
           s7 = cv[7];
  uint32_t s8 = IV0, s9 = IV1, s10 = IV2, s11 = IV3;
  uint32_t s12 = (uint32_t)counter, s13 = (uint32_t)(counter >> 32), s14 = block_len, s15 = flags;
#pragma unroll
  for (int r = 0; r < 7; r++) {
    B3G(s0, s4, s8, s12, m[sched(r, 0)], m[sched(r, 1)]);
    B3G(s1, s5, s9, s13, m[sched(r, 2)], m[sched(r, 3)]);
    B3G(s2, s6, s10, s14, m[sched(r, 4)], m[sched(r, 5)]);
    B3G(s3, s7, s11, s15, m[sched(r, 6)], m[sched(r, 7)]);
    B3G(s0, s5, s10, s15, m[sched(r, 8)], m[sched(r, 9)]);
    B3G(s1, s6, s11, s12, m[sched(r, 10)], m[sched(r, 11)]);
    B3G(s2, s7, s8, s13, m[sched(r, 12)], m[sched(r, 13)]);
    B3G(s3, s4, s9, s14, m[sched(r, 14)], m[sched(r, 15)]);
  }
  cv[0] = s0 ^ s8;
  cv[1] = s1 ^ s9;
  cv[2] = s2 ^ s10;
  cv[3] = s3 ^ s11;
  cv[4] = s4 ^ s12;
  cv[5] = s5 ^ s13;
  cv[6] = s6 ^ s14;
  cv[7] = s7 ^ s15;
}

__device__ __forceinline__ void iv(uint32_t cv[8]) {
  cv[0] = IV0; cv[1] = IV1; cv[2] = IV2; cv[3] = IV3;
  cv[4] = IV4; cv[5] = IV5; cv[6] = IV6; cv[7] = IV7;
}

// BLAKE3 of a 64-byte message (one chunk, one block) = lcpc-2d Merkle node.
__device__ __forceinline__ void hash64(const uint32_t m[16], uint32_t out[8]) {
  iv(out);
  compress(out, m, 0, 64, CHUNK_START | CHUNK_END | ROOT);
}

__device__ __forceinline__ void parent_cv(const uint32_t l[8], const uint32_t r[8], bool root,
                                          uint32_t out[8]) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    m[i] = l[i];
    m[8 + i] = r[i];
  }
  iv(out);
  compress(out, m, 0, 64, PARENT | (root ? ROOT : 0u));
}

__device__ __forceinline__ void load8(const uint32_t *p, uint32_t v[8]) {
  const uint4 a = reinterpret_cast<const uint4 *>(p)[0], b = reinterpret_cast<const uint4 *>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void store8(uint32_t *p, const uint32_t v[8]) {
  reinterpret_cast<uint4 *>(p)[0] = make_uint4(v[0], v[1], v[2], v[3]);
  reinterpret_cast<uint4 *>(p)[1] = make_uint4(v[4], v[5], v[6], v[7]);
}

// Slot of the chaining value of (col, chunk) in a chunk range [chunk0, chunk_end): [chunk][col],
// or with blk > 0 the row-shard exchange's layout [col / blk][chunk][col % blk] (each destination
// rank's column block contiguous, ready to send).
__device__ __forceinline__ size_t cv_slot(size_t col, int chunk, int chunk0, int chunk_end, size_t n_cols,
                                          size_t blk) {
  const size_t c = (size_t)(chunk - chunk0);
  return blk ? ((col / blk) * (size_t)(chunk_end - chunk0) + c) * blk + col % blk : c * n_cols + col;
}

// acc += sum_k u[k] el[k] R^-1 over k in [K0, EPB), in fe_dot groups of at most fe_dot_kmax
// products per reduction (bit-identical to summing fe_mul products: the same values mod p)
template <class F, int K0, int EPB>
__device__ __forceinline__ void dot_groups(Fe<F> &acc, const Fe<F> *u, const Fe<F> *el) {
  if constexpr (K0 < EPB) {
    constexpr int KM = fe_dot_kmax<F>() < 1 ? 1 : fe_dot_kmax<F>();
    constexpr int G = (EPB - K0) < KM ? (EPB - K0) : KM;
    acc = fe_add<F>(acc, fe_dot<F, G>(u + K0, el + K0));
    dot_groups<F, K0 + G, EPB>(acc, u, el);
  }
}

// The chaining value of chunk `chunk` of one column's leaf message (column pointer colp, element
// row r at colp + (r - row0) row_stride).  Message word w of a column: w < 8 is the zero prefix,
// else word (w-8) % N of element row (w-8) / N.  N in {2, 4, 8} divides both 8 and 16, so every
// 16-word block holds whole elements.  A one-chunk message gets ROOT (it is the leaf).
// EVAL: also *acc = sum over the chunk's rows r of left[r] * element (Montgomery products of the
// Montgomery left[r] and the canonical codeword: canonical results, as collapse_rows gives them).
template <class F, bool CANON, bool EVAL = false>
__device__ __forceinline__ void chunk_cv_rm(const uint32_t *__restrict__ colp, size_t n_rows, size_t row_stride,
                                            size_t row0, int chunk, int n_chunks, uint32_t cv[8],
                                            const uint32_t *__restrict__ left = nullptr, Fe<F> *acc = nullptr) {
  constexpr int N = F::N;
  static_assert(16 % N == 0 && 8 % N == 0, "element must tile a BLAKE3 block");
  const size_t total_words = 8 + n_rows * N;
  const size_t w0 = (size_t)chunk * 256;
  const size_t cw = total_words - w0 < 256 ? total_words - w0 : 256;
  const int nb = (int)((cw + 15) / 16);
  iv(cv);
  constexpr int EPB = 16 / N;  // elements per 64-byte block
  // element e of the block starting at word gw: stream word gw + e N - 8 (negative: prefix)
  auto fetch = [&](size_t gw, Fe<F> *raw) {
#pragma unroll
    for (int k = 0; k < EPB; k++) {
      const long long ew = (long long)gw + k * N - 8;
      const size_t row = ew < 0 ? n_rows : (size_t)ew / N;
      raw[k] = row < n_rows ? fe_load<F>(colp, (row - row0) * row_stride) : fe_zero<F>();
    }
  };
  auto to_msg = [&](const Fe<F> *el, uint32_t *msg) {
#pragma unroll
    for (int k = 0; k < EPB; k++) {
      uint32_t w[N];
      if constexpr (CANON)
        fe_canon_repr_words<F>(el[k], w);
      else
        fe_repr_words<F>(el[k], w);
#pragma unroll
      for (int i = 0; i < N; i++) msg[k * N + i] = w[i];
    }
  };
  // left[r] * element summed into *acc for the elements of rows r0, r0 + 1, ... (n of them)
  auto eval_acc = [&](const Fe<F> *el, size_t r0) {  // a whole block of EPB rows
    if constexpr (EVAL) {
      Fe<F> u[EPB];
#pragma unroll
      for (int k = 0; k < EPB; k++) u[k] = fe_load<F>(left, r0 + k);
      dot_groups<F, 0, EPB>(*acc, u, el);
    }
  };
  // Interior chunks (a wave-uniform case: 16 full blocks, every row present, no zero prefix):
  // one strided pointer walk without per-element bounds checks, blocks in ping-pong pairs so
  // the next block's loads overlap this block's 7 rounds without register copies.
  {
    const size_t r_first = w0 >= 8 ? (w0 - 8) / N : 0;
    if (chunk > 0 && cw == 256 && r_first >= row0 && r_first + 16 * EPB <= n_rows) {
      size_t e = (r_first - row0) * row_stride;
      Fe<F> ea[EPB], eb[EPB];
      uint32_t msg[16];
#pragma unroll
      for (int k = 0; k < EPB; k++) ea[k] = fe_load<F>(colp, e + k * row_stride);
      e += EPB * row_stride;
      for (int b = 0; b < 16; b += 2) {
#pragma unroll
        for (int k = 0; k < EPB; k++) eb[k] = fe_load<F>(colp, e + k * row_stride);
        e += EPB * row_stride;
        to_msg(ea, msg);
        eval_acc(ea, r_first + (size_t)b * EPB);
        compress(cv, msg, (uint64_t)chunk, 64u, b == 0 ? CHUNK_START : 0u);
        if (b + 2 < 16) {
#pragma unroll
          for (int k = 0; k < EPB; k++) ea[k] = fe_load<F>(colp, e + k * row_stride);
          e += EPB * row_stride;
        }
        to_msg(eb, msg);
        eval_acc(eb, r_first + (size_t)(b + 1) * EPB);
        compress(cv, msg, (uint64_t)chunk, 64u, b + 1 == 15 ? CHUNK_END : 0u);
      }
      return;
    }
  }
  // general case (the zero prefix, the ragged last chunk): the next block's elements are
  // loaded before the current block is compressed, so HBM latency overlaps the 7 rounds
  Fe<F> cur[EPB], nxt[EPB];
  fetch(w0, cur);
  for (int b = 0; b < nb; b++) {
    const size_t gw = w0 + 16 * (size_t)b;
    if (b + 1 < nb) fetch(gw + 16, nxt);
    uint32_t msg[16];
#pragma unroll
    for (int k = 0; k < EPB; k++) {
      const long long ew = (long long)gw + k * N - 8;
      uint32_t w[N];
      if (ew < 0 || (size_t)ew / N >= n_rows) {
#pragma unroll
        for (int i = 0; i < N; i++) w[i] = 0;
      } else {
        if constexpr (CANON) {
          fe_canon_repr_words<F>(cur[k], w);
        } else {
          fe_repr_words<F>(cur[k], w);
        }
        if constexpr (EVAL) *acc = fe_add<F>(*acc, fe_mul<F>(fe_load<F>(left, (size_t)ew / N), cur[k]));
      }
#pragma unroll
      for (int i = 0; i < N; i++) msg[k * N + i] = w[i];
    }
    const size_t left = cw - 16 * (size_t)b;
    const uint32_t blen = left >= 16 ? 64u : (uint32_t)(4 * left);
    uint32_t flags = b == 0 ? CHUNK_START : 0u;
    if (b == nb - 1) flags |= CHUNK_END | (n_chunks == 1 ? ROOT : 0u);
    compress(cv, msg, (uint64_t)chunk, blen, flags);
#pragma unroll
    for (int k = 0; k < EPB; k++) cur[k] = nxt[k];
  }
}

// One thread per (column, chunk) of a row-major matrix.  The launch covers chunks [chunk0,
// chunk_end) of messages of n_rows rows; m holds rows [row0, ...) (a row shard: every row those
// chunks read is present), and chaining values go to cvs[chunk - chunk0][col] (cv_slot).
template <class F, bool CANON>
__global__ __launch_bounds__(256) void k_leaf_chunks(const uint32_t *__restrict__ m,
                                                     size_t n_rows, size_t n_cols,
                                                     size_t row_stride, size_t col_stride,
                                                     uint32_t *__restrict__ cvs,
                                                     uint8_t *__restrict__ leaves, int n_chunks,
                                                     size_t row0, int chunk0, int chunk_end, size_t blk) {
  // a block = 4 waves on 256 adjacent columns of one chunk (every wave of a block does the same
  // amount of work; a chunk per wave left the waves of chunks >= n_chunks idle)
  const size_t col = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int chunk = chunk0 + blockIdx.y;
  if (col >= n_cols || chunk >= chunk_end) return;
  uint32_t cv[8];
  chunk_cv_rm<F, CANON>(m + col * col_stride * F::N, n_rows, row_stride, row0, chunk, n_chunks, cv);
  if (n_chunks == 1 && leaves) {
    store8(reinterpret_cast<uint32_t *>(leaves + 32 * col), cv);
  } else {
    store8(cvs + cv_slot(col, chunk, chunk0, chunk_end, n_cols, blk) * 8, cv);
  }
}

// k_leaf_chunks over a whole canonical row-major codeword (one rank, every row present) that also
// leaves each (chunk, column)'s share of u^T Enc(M) in partials[chunk][col]: the proof-of-storage
// request's evaluation (lcpc_online.rs:454-484) without a second pass over the codeword
template <class F>
__global__ __launch_bounds__(256) void k_leaf_chunks_eval(const uint32_t *__restrict__ m, size_t n_rows,
                                                          size_t n_cols, size_t row_stride,
                                                          uint32_t *__restrict__ cvs, uint8_t *__restrict__ leaves,
                                                          int n_chunks, const uint32_t *__restrict__ left,
                                                          uint32_t *__restrict__ partials) {
  const size_t col = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int chunk = blockIdx.y;
  if (col >= n_cols || chunk >= n_chunks) return;
  uint32_t cv[8];
  Fe<F> acc = fe_zero<F>();
  chunk_cv_rm<F, true, true>(m + col * F::N, n_rows, row_stride, 0, chunk, n_chunks, cv, left, &acc);
  if (n_chunks == 1 && leaves)
    store8(reinterpret_cast<uint32_t *>(leaves + 32 * col), cv);
  else
    store8(cvs + ((size_t)chunk * n_cols + col) * 8, cv);
  fe_store<F>(partials, (size_t)chunk * n_cols + col, acc);
}

// The same chunks for a column-major matrix ([column][row], a column's message words contiguous
// in memory: the SDIG commitments and the PoS column files).  Read lane-per-column, every load of
// a wave touches 64 columns n_rows * B bytes apart; here the wave loads each 64-byte block of its
// 64 columns cooperatively instead -- 4 adjacent lanes read one column's block, so a load
// instruction covers 16 columns x 64 contiguous bytes -- and hands the blocks over through LDS
// (rows padded to 80 B so the per-column reads are bank-conflict free).  Needs
// n_rows * N % 4 == 0 (16-B aligned columns); the message word w of a column is memory word w - 8
// of the column (w >= 8), and a 4-word unit lies wholly inside or outside the message.
// fuse2: a two-chunk message hashed whole by one wave (grid.y = 1, leaves written directly).
template <class F, bool CANON>
__global__ __launch_bounds__(256) void k_leaf_chunks_cm(const uint32_t *__restrict__ m, size_t n_rows,
                                                        size_t n_cols, uint32_t *__restrict__ cvs,
                                                        uint8_t *__restrict__ leaves, int n_chunks, int fuse2) {
  constexpr int N = F::N;
  static_assert(16 % N == 0 && 8 % N == 0, "element must tile a BLAKE3 block");
  constexpr int EPB = 16 / N;
  __shared__ uint4 stage[4][64][5];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t col0 = ((size_t)blockIdx.x * 4 + wave) * 64, col = col0 + lane;
  if (col0 >= n_cols) return;  // whole waves
  const size_t msg_words = 8 + n_rows * N;  // the column's message, in words
  const int unit = lane & 3, csub = lane >> 2;
  // block b (of the chunk starting at message word w0): this lane's 4 loads, unit `unit` (words
  // 4 unit .. +3) of column col0 + csub + 16 i
  auto gload = [&](size_t w0, int b, uint4 r[4]) {
    const size_t w = w0 + 16 * (size_t)b + 4 * unit;  // message word
    const bool in = w >= 8 && w < msg_words;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const size_t c = col0 + csub + 16 * i;
      r[i] = in && c < n_cols ? reinterpret_cast<const uint4 *>(m + c * n_rows * N + (w - 8))[0]
                              : make_uint4(0, 0, 0, 0);
    }
  };
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto lput = [&](const uint4 r[4]) {
#pragma unroll
    for (int i = 0; i < 4; i++) stage[wave][csub + 16 * i][unit] = r[i];
    wave_sync();
  };
  // one chunk's chaining value (its blocks staged through LDS, the next block's loads in flight
  // while this one compresses)
  auto chunk_cv = [&](int chunk, uint32_t cv[8]) {
    const size_t w0 = (size_t)chunk * 256;
    const size_t cw = msg_words - w0 < 256 ? msg_words - w0 : 256;
    const int nb = (int)((cw + 15) / 16);
    iv(cv);
    uint4 r[4];
    gload(w0, 0, r);
    lput(r);
    for (int b = 0; b < nb; b++) {
      const bool more = b + 1 < nb;
      if (more) gload(w0, b + 1, r);
      uint32_t msg[16];
      {
        const uint4 *row = stage[wave][lane];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint4 q = row[k];
          msg[4 * k] = q.x; msg[4 * k + 1] = q.y; msg[4 * k + 2] = q.z; msg[4 * k + 3] = q.w;
        }
      }
      wave_sync();  // every lane has read block b before block b + 1 overwrites the stage
      // element words -> repr words (Montgomery -> canonical unless CANON); the zero prefix and
      // words past the message stay zero either way (from_mont(0) = 0, and they load as zero)
#pragma unroll
      for (int k = 0; k < EPB; k++) {
        Fe<F> e;
#pragma unroll
        for (int i = 0; i < N; i++) e.v[i] = msg[k * N + i];
        uint32_t w[N];
        if constexpr (CANON)
          fe_canon_repr_words<F>(e, w);
        else
          fe_repr_words<F>(e, w);
#pragma unroll
        for (int i = 0; i < N; i++) msg[k * N + i] = w[i];
      }
      const size_t left = cw - 16 * (size_t)b;
      const uint32_t blen = left >= 16 ? 64u : (uint32_t)(4 * left);
      uint32_t flags = b == 0 ? CHUNK_START : 0u;
      if (b == nb - 1) flags |= CHUNK_END | (n_chunks == 1 ? ROOT : 0u);
      compress(cv, msg, (uint64_t)chunk, blen, flags);
      if (more) lput(r);
    }
  };
  uint32_t cv[8];
  if (fuse2) {
    // a two-chunk message (cfg4's 1184-byte leaves) whole in one wave: both chaining values in
    // registers and their ROOT parent, no scratch round trip and no merge launch
    uint32_t cv1[8], leaf[8];
    chunk_cv(0, cv);
    chunk_cv(1, cv1);
    parent_cv(cv, cv1, true, leaf);
    if (col < n_cols) store8(reinterpret_cast<uint32_t *>(leaves + 32 * col), leaf);
    return;
  }
  const int chunk = blockIdx.y;
  chunk_cv(chunk, cv);
  if (col >= n_cols) return;
  if (n_chunks == 1 && leaves) {
    store8(reinterpret_cast<uint32_t *>(leaves + 32 * col), cv);
  } else {
    store8(cvs + ((size_t)chunk * n_cols + col) * 8, cv);
  }
}

// The same chunks for an element that does not tile a 64-byte block (Ft191: 24 bytes, so
// elements straddle blocks and chunks).  A block of stream words [gw, gw + 16) starts at word
// `off` of element e0 = floor((gw - 8) / N); the 4 elements e0 .. e0 + 3 cover it (off + 16 <=
// N - 1 + 16 <= 4N), elements outside [0, n_rows) -- the 32-byte zero prefix, the tail -- read
// as zero words.  `off` is the same for every lane of a wave (lanes = columns of one chunk), so
// the word selection is a uniform switch, not a dynamic register index.
template <class F, bool CANON>
__global__ __launch_bounds__(256) void k_leaf_chunks_words(const uint32_t *__restrict__ m, size_t n_rows,
                                                           size_t n_cols, size_t row_stride, size_t col_stride,
                                                           uint32_t *__restrict__ cvs, uint8_t *__restrict__ leaves,
                                                           int n_chunks, size_t row0, int chunk0, int chunk_end,
                                                           size_t blk) {
  constexpr int N = F::N;
  static_assert(4 * N >= N - 1 + 16, "four elements cover a block");
  const size_t col = (size_t)blockIdx.x * 256 + threadIdx.x;  // 4 waves, 256 columns, one chunk
  const int chunk = chunk0 + blockIdx.y;
  if (col >= n_cols || chunk >= chunk_end) return;
  const size_t total_words = 8 + n_rows * N;
  const size_t w0 = (size_t)chunk * 256;
  const size_t cw = total_words - w0 < 256 ? total_words - w0 : 256;
  const int nb = (int)((cw + 15) / 16);
  uint32_t cv[8];
  iv(cv);
  const uint32_t *colp = m + col * col_stride * N;
  // elements that start before the end of the launch's chunk range: a row shard holds exactly
  // those (its range ends on an element boundary), so nothing past it is ever loaded
  const size_t w_end = (size_t)chunk_end * 256;
  for (int b = 0; b < nb; b++) {
    const long long sw0 = (long long)(w0 + 16 * (size_t)b) - 8;  // stream word of the block's word 0
    const long long e0 = sw0 >= 0 ? sw0 / N : -((-sw0 + N - 1) / N);
    const int off = (int)(sw0 - e0 * N);
    uint32_t w[4 * N];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const long long e = e0 + k;
      uint32_t r[N];
      if (e < 0 || (size_t)e >= n_rows || 8 + (size_t)e * N >= w_end) {
#pragma unroll
        for (int i = 0; i < N; i++) r[i] = 0;
      } else {
        const Fe<F> x = fe_load<F>(colp, ((size_t)e - row0) * row_stride);
        if constexpr (CANON)
          fe_canon_repr_words<F>(x, r);
        else
          fe_repr_words<F>(x, r);
      }
#pragma unroll
      for (int i = 0; i < N; i++) w[k * N + i] = r[i];
    }
    uint32_t msg[16];
    switch (off) {
#define LCPC_SEL(o)                                        \
  case o:                                                  \
    if constexpr (o + 16 <= 4 * N) {                       \
      _Pragma("unroll") for (int i = 0; i < 16; i++) msg[i] = w[o + i]; \
    }                                                      \
    break;
      LCPC_SEL(0) LCPC_SEL(1) LCPC_SEL(2) LCPC_SEL(3) LCPC_SEL(4) LCPC_SEL(5) LCPC_SEL(6) LCPC_SEL(7)
#undef LCPC_SEL
      default: break;
    }
    const size_t left = cw - 16 * (size_t)b;
    const uint32_t blen = left >= 16 ? 64u : (uint32_t)(4 * left);
    uint32_t flags = b == 0 ? CHUNK_START : 0u;
    if (b == nb - 1) flags |= CHUNK_END | (n_chunks == 1 ? ROOT : 0u);
    compress(cv, msg, (uint64_t)chunk, blen, flags);
  }
  if (n_chunks == 1 && leaves) {
    store8(reinterpret_cast<uint32_t *>(leaves + 32 * col), cv);
  } else {
    store8(cvs + cv_slot(col, chunk, chunk0, chunk_end, n_cols, blk) * 8, cv);
  }
}

// Fold `count` chaining values of column col -- chunk slots first, first + stride, ... of the
// [chunk][col] scratch -- pairwise per level, an odd node carried up (BLAKE3's left-balanced tree
// over those chunks), in place; the result lands in slot `first`.  ROOT marks the last parent when
// this fold is the whole tree.
__device__ __forceinline__ void fold_cvs(uint32_t *__restrict__ cvs, size_t n_cols, size_t col, int first,
                                         int count, int stride, bool root, uint32_t o[8]) {
  int nodes = count;
  uint32_t l[8], r[8];
  auto slot = [&](int i) { return cvs + ((size_t)(first + i * stride) * n_cols + col) * 8; };
  while (nodes > 1) {
    const int pairs = nodes / 2;
    for (int i = 0; i < pairs; i++) {
      load8(slot(2 * i), l);
      load8(slot(2 * i + 1), r);
      parent_cv(l, r, root && nodes == 2, o);
      store8(slot(i), o);
    }
    if (nodes & 1) {
      load8(slot(nodes - 1), l);
      store8(slot(pairs), l);
    }
    nodes = pairs + (nodes & 1);
  }
  load8(slot(0), o);
}

// Chunk groups of the leaf merge: groups of MERGE_GROUP consecutive chunks, aligned, are whole
// subtrees of the pairwise fold (an aligned block of 2^k nodes pairs only within itself for k
// levels, and a ragged last group's own pairwise fold is the node the whole-tree fold carries up),
// so the fold runs in two passes: every group in parallel, then each column's group nodes.
constexpr int MERGE_GROUP = 8;

// pass 1 (more than one group): one thread per (column, group); the group's node goes to its
// first chunk slot
__global__ __launch_bounds__(256) void k_leaf_merge_groups(uint32_t *__restrict__ cvs, size_t n_cols,
                                                           int n_chunks) {
  const size_t col = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  if (col >= n_cols) return;
  const int first = g * MERGE_GROUP;
  const int count = n_chunks - first < MERGE_GROUP ? n_chunks - first : MERGE_GROUP;
  uint32_t o[8];
  fold_cvs(cvs, n_cols, col, first, count, 1, false, o);
}

// one thread per column folds its `count` nodes (slots 0, stride, 2 stride, ...) into the leaf:
// the group nodes after pass 1 (stride MERGE_GROUP), or every chunk (stride 1)
__global__ __launch_bounds__(256) void k_leaf_merge(uint32_t *__restrict__ cvs, size_t n_cols, int count,
                                                    int stride, uint8_t *__restrict__ leaves) {
  const size_t col = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= n_cols) return;
  uint32_t o[8];
  fold_cvs(cvs, n_cols, col, 0, count, stride, true, o);
  store8(reinterpret_cast<uint32_t *>(leaves + 32 * col), o);
}

// Up to 2 groups (16 chunks, e.g. cfg3's 9) one serial fold per column is as short as the two
// passes and saves a launch (measured: 256-thread blocks 21.5 us at cfg3, 64-thread 29 us); longer
// leaves (PoS: 74 chunks, 0.16 -> 0.09 ms) fold in two passes of 64-thread blocks, so pass 2's
// one thread per column still spreads over every SIMD.
hipError_t launch_leaf_merge(uint32_t *cvs, size_t n_cols, int n_chunks, uint8_t *leaves, hipStream_t s) {
  prof::Scope ps("leaf_merge", s);
  const unsigned bx = (unsigned)((n_cols + 63) / 64);
  const int n_groups = (n_chunks + MERGE_GROUP - 1) / MERGE_GROUP;
  if (n_groups <= 2) {
    hipLaunchKernelGGL(k_leaf_merge, dim3((unsigned)((n_cols + 255) / 256)), dim3(256), 0, s, cvs, n_cols, n_chunks,
                       1, leaves);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_leaf_merge_groups, dim3(bx, (unsigned)n_groups), dim3(64), 0, s, cvs, n_cols, n_chunks);
  hipLaunchKernelGGL(k_leaf_merge, dim3(bx), dim3(64), 0, s, cvs, n_cols, (n_chunks + MERGE_GROUP - 1) / MERGE_GROUP,
                     MERGE_GROUP, leaves);
  return hipGetLastError();
}

// Merkle levels: each workgroup folds 2^levels consecutive nodes of level `lvl` (starting at
// element offset in_off of `hashes`) into one node, writing every intermediate level.
// node(level l+1, i) = BLAKE3(node(l, 2i) || node(l, 2i+1)).
__global__ __launch_bounds__(256) void k_merkle(uint8_t *__restrict__ hashes, size_t np2,
                                                int lvl, int levels) {
  __shared__ __align__(16) uint32_t buf[2][256 * 8];
  const int tid = threadIdx.x;
  size_t n_in = np2 >> lvl;
  size_t base_in = 2 * np2 - 2 * n_in;  // offset of level lvl
  const int width = 1 << levels;         // input nodes per workgroup (<= 512)
  const size_t first = (size_t)blockIdx.x * width;
  // level lvl -> lvl+1 straight from global
  int cur = 0;
  for (int i = tid; i < width / 2; i += 256) {
    uint32_t msg[16], o[8];
    load8(reinterpret_cast<const uint32_t *>(hashes + 32 * (base_in + first + 2 * i)), msg);
    load8(reinterpret_cast<const uint32_t *>(hashes + 32 * (base_in + first + 2 * i + 1)), msg + 8);
    hash64(msg, o);
#pragma unroll
    for (int k = 0; k < 8; k++) buf[cur][i * 8 + k] = o[k];
    store8(reinterpret_cast<uint32_t *>(hashes + 32 * (base_in + n_in + first / 2 + i)), o);
  }
  base_in += n_in;
  n_in /= 2;
  size_t f = first / 2;
  for (int l = 1; l < levels; l++) {
    __syncthreads();
    const int cnt = width >> (l + 1);
    for (int i = tid; i < cnt; i += 256) {
      uint32_t msg[16], o[8];
#pragma unroll
      for (int k = 0; k < 16; k++) msg[k] = buf[cur][2 * i * 8 + k];
      hash64(msg, o);
#pragma unroll
      for (int k = 0; k < 8; k++) buf[cur ^ 1][i * 8 + k] = o[k];
      store8(reinterpret_cast<uint32_t *>(hashes + 32 * (base_in + n_in + f / 2 + i)), o);
    }
    cur ^= 1;
    base_in += n_in;
    n_in /= 2;
    f /= 2;
  }
}

template <class F>
__global__ void k_gather_cols(const uint32_t *__restrict__ m, size_t n_rows, size_t n_cols,
                              const uint64_t *__restrict__ idx, size_t n_idx,
                              uint32_t *__restrict__ cols, int col_major, int canon) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_idx * n_rows) return;
  const size_t k = t / n_rows, r = t % n_rows;
  const size_t at = col_major ? idx[k] * n_rows + r : r * n_cols + idx[k];
  const Fe<F> x = fe_load<F>(m, at);
  fe_store<F>(cols, t, canon ? fe_to_mont<F>(x) : x);
}

__global__ void k_gather_paths(const uint8_t *__restrict__ hashes, size_t np2,
                               const uint64_t *__restrict__ idx, size_t n_idx, size_t path_len,
                               uint8_t *__restrict__ paths) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_idx * path_len) return;
  const size_t k = t / path_len, i = t % path_len;
  const size_t base = 2 * np2 - 2 * (np2 >> i);
  const size_t other = (idx[k] >> i) ^ 1;
  uint32_t v[8];
  load8(reinterpret_cast<const uint32_t *>(hashes + 32 * (base + other)), v);
  store8(reinterpret_cast<uint32_t *>(paths + 32 * t), v);
}

__global__ void k_path_checks(const uint8_t *__restrict__ leaves, const uint8_t *__restrict__ paths,
                              size_t n, size_t path_len, const uint64_t *__restrict__ idx,
                              const uint8_t *__restrict__ root, uint32_t *__restrict__ flags) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  uint32_t h[8], msg[16];
  load8(reinterpret_cast<const uint32_t *>(leaves + 32 * k), h);
  size_t col = idx[k];
  for (size_t i = 0; i < path_len; i++) {
    uint32_t p[8];
    load8(reinterpret_cast<const uint32_t *>(paths + 32 * (k * path_len + i)), p);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      msg[q] = (col & 1) ? p[q] : h[q];
      msg[8 + q] = (col & 1) ? h[q] : p[q];
    }
    hash64(msg, h);
    col >>= 1;
  }
  uint32_t rt[8];
  load8(reinterpret_cast<const uint32_t *>(root), rt);
  uint32_t diff = 0;
#pragma unroll
  for (int q = 0; q < 8; q++) diff |= h[q] ^ rt[q];
  flags[k] = diff == 0;
}

}  // namespace

size_t leaf_hash_scratch_bytes(int fid, size_t n_rows, size_t n_cols) {
  const size_t words = 8 + n_rows * (size_t)field_words(fid);
  const size_t n_chunks = (words + 255) / 256;
  return n_chunks > 1 ? n_chunks * n_cols * 32 : 0;
}

static hipError_t leaf_hashes_strided(int fid, const uint32_t *m, size_t n_rows, size_t n_cols,
                                      size_t row_stride, size_t col_stride, uint8_t *leaves,
                                      void *scratch, hipStream_t s, bool canon) {
  if (n_cols == 0) return hipSuccess;
  const size_t words = 8 + n_rows * (size_t)field_words(fid);
  const int n_chunks = (int)((words + 255) / 256);
  dim3 grid((unsigned)((n_cols + 255) / 256), (unsigned)n_chunks);
  bool leaves_done = false;
  hipError_t e = dispatch_field(fid, [&]<class F>() {
    if constexpr (16 % F::N == 0 && 8 % F::N == 0) {
      prof::Scope ps("leaf_chunks", s);
      if (row_stride == 1 && col_stride == n_rows && (n_rows * F::N) % 4 == 0) {  // column-major, 16-B aligned
        const int fuse2 = n_chunks == 2 && leaves;
        const dim3 g2(grid.x, fuse2 ? 1 : grid.y);
        if (canon)
          hipLaunchKernelGGL((k_leaf_chunks_cm<F, true>), g2, dim3(256), 0, s, m, n_rows, n_cols,
                             (uint32_t *)scratch, leaves, n_chunks, fuse2);
        else
          hipLaunchKernelGGL((k_leaf_chunks_cm<F, false>), g2, dim3(256), 0, s, m, n_rows, n_cols,
                             (uint32_t *)scratch, leaves, n_chunks, fuse2);
        leaves_done = fuse2;  // (the leaves are written: no merge)
        return hipGetLastError();
      }
      if (canon)
        hipLaunchKernelGGL((k_leaf_chunks<F, true>), grid, dim3(256), 0, s, m, n_rows, n_cols, row_stride,
                           col_stride, (uint32_t *)scratch, leaves, n_chunks, (size_t)0, 0, n_chunks, (size_t)0);
      else
        hipLaunchKernelGGL((k_leaf_chunks<F, false>), grid, dim3(256), 0, s, m, n_rows, n_cols, row_stride,
                           col_stride, (uint32_t *)scratch, leaves, n_chunks, (size_t)0, 0, n_chunks, (size_t)0);
      return hipGetLastError();
    } else {
      prof::Scope ps("leaf_chunks", s);
      if (canon)
        hipLaunchKernelGGL((k_leaf_chunks_words<F, true>), grid, dim3(256), 0, s, m, n_rows, n_cols, row_stride,
                           col_stride, (uint32_t *)scratch, leaves, n_chunks, (size_t)0, 0, n_chunks, (size_t)0);
      else
        hipLaunchKernelGGL((k_leaf_chunks_words<F, false>), grid, dim3(256), 0, s, m, n_rows, n_cols, row_stride,
                           col_stride, (uint32_t *)scratch, leaves, n_chunks, (size_t)0, 0, n_chunks, (size_t)0);
      return hipGetLastError();
    }
  });
  if (e != hipSuccess || n_chunks == 1 || leaves_done) return e;
  return launch_leaf_merge((uint32_t *)scratch, n_cols, n_chunks, leaves, s);
}

size_t leaf_n_chunks(int fid, size_t n_rows) {
  return (8 + n_rows * (size_t)field_words(fid) + 255) / 256;
}

hipError_t leaf_chunk_cvs(int fid, const uint32_t *m, size_t row0, size_t n_rows, size_t n_cols,
                          size_t stride, size_t chunk_lo, size_t chunk_hi, uint32_t *cvs,
                          hipStream_t s, bool canon, size_t blk, size_t col_stride) {
  if (n_cols == 0 || chunk_hi <= chunk_lo) return hipSuccess;
  const int n_chunks = (int)leaf_n_chunks(fid, n_rows);
  dim3 grid((unsigned)((n_cols + 255) / 256), (unsigned)(chunk_hi - chunk_lo));
  return dispatch_field(fid, [&]<class F>() {
    if constexpr (16 % F::N == 0 && 8 % F::N == 0) {
      prof::Scope ps("leaf_chunks", s);
      if (canon)
        hipLaunchKernelGGL((k_leaf_chunks<F, true>), grid, dim3(256), 0, s, m, n_rows, n_cols, stride,
                           col_stride, cvs, (uint8_t *)nullptr, n_chunks, row0, (int)chunk_lo,
                           (int)chunk_hi, blk);
      else
        hipLaunchKernelGGL((k_leaf_chunks<F, false>), grid, dim3(256), 0, s, m, n_rows, n_cols, stride,
                           col_stride, cvs, (uint8_t *)nullptr, n_chunks, row0, (int)chunk_lo,
                           (int)chunk_hi, blk);
      return hipGetLastError();
    } else {
      prof::Scope ps("leaf_chunks", s);
      if (canon)
        hipLaunchKernelGGL((k_leaf_chunks_words<F, true>), grid, dim3(256), 0, s, m, n_rows, n_cols, stride,
                           col_stride, cvs, (uint8_t *)nullptr, n_chunks, row0, (int)chunk_lo, (int)chunk_hi,
                           blk);
      else
        hipLaunchKernelGGL((k_leaf_chunks_words<F, false>), grid, dim3(256), 0, s, m, n_rows, n_cols, stride,
                           col_stride, cvs, (uint8_t *)nullptr, n_chunks, row0, (int)chunk_lo, (int)chunk_hi,
                           blk);
      return hipGetLastError();
    }
  });
}

hipError_t leaves_from_cvs(uint32_t *cvs, size_t n_cols, int n_chunks, uint8_t *leaves,
                           hipStream_t s) {
  if (!n_cols) return hipSuccess;
  if (n_chunks == 1) return hipMemcpyAsync(leaves, cvs, n_cols * 32, hipMemcpyDeviceToDevice, s);
  return launch_leaf_merge(cvs, n_cols, n_chunks, leaves, s);
}

hipError_t leaf_hashes(int fid, const uint32_t *m, size_t n_rows, size_t n_cols, size_t stride,
                       uint8_t *leaves, void *scratch, hipStream_t s, bool canon) {
  return leaf_hashes_strided(fid, m, n_rows, n_cols, stride, 1, leaves, scratch, s, canon);
}

hipError_t leaf_hashes_eval(int fid, const uint32_t *m, size_t n_rows, size_t n_cols, size_t stride,
                            uint8_t *leaves, void *scratch, const uint32_t *left, uint32_t *partials,
                            hipStream_t s) {
  if (n_cols == 0) return hipSuccess;
  const int n_chunks = (int)leaf_n_chunks(fid, n_rows);
  const dim3 grid((unsigned)((n_cols + 255) / 256), (unsigned)n_chunks);
  hipError_t e = dispatch_field(fid, [&]<class F>() -> hipError_t {
    if constexpr (16 % F::N == 0 && 8 % F::N == 0) {
      prof::Scope ps("leaf_chunks", s);
      hipLaunchKernelGGL((k_leaf_chunks_eval<F>), grid, dim3(256), 0, s, m, n_rows, n_cols, stride,
                         (uint32_t *)scratch, leaves, n_chunks, left, partials);
      return hipGetLastError();
    } else {
      return hipErrorInvalidValue;  // (callers check leaf_eval_fusable first)
    }
  });
  if (e != hipSuccess || n_chunks == 1) return e;
  return launch_leaf_merge((uint32_t *)scratch, n_cols, n_chunks, leaves, s);
}

bool leaf_eval_fusable(int fid) { return field_words(fid) == 2 || field_words(fid) == 4 || field_words(fid) == 8; }

hipError_t leaf_hashes_cols(int fid, const uint32_t *cols, size_t n_rows, size_t n_cols,
                            uint8_t *leaves, void *scratch, hipStream_t s, bool canon) {
  // cols laid out [column][row]
  return leaf_hashes_strided(fid, cols, n_rows, n_cols, 1, n_rows, leaves, scratch, s, canon);
}

hipError_t merkle_tree(uint8_t *hashes, size_t np2, hipStream_t s) {
  int lvl = 0;
  size_t n = np2;
  while (n > 1) {
    int levels = 0;
    while (levels < 9 && ((size_t)1 << (levels + 1)) <= n) levels++;
    const size_t blocks = n >> levels;
    prof::Scope ps("merkle", s);
    hipLaunchKernelGGL(k_merkle, dim3((unsigned)blocks), dim3(256), 0, s, hashes, np2, lvl, levels);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    lvl += levels;
    n >>= levels;
  }
  return hipSuccess;
}

namespace {
// Row shards: rank g's subtree over column block g ([B leaves | B/2 | ... | 1], B a power of
// two) is level l, positions [g B/2^l, (g + 1) B/2^l) of the whole tree.  One thread per
// 16 bytes of digest.
__global__ __launch_bounds__(256) void k_assemble_subtrees(const uint4 *__restrict__ subs, size_t B, size_t G,
                                                           uint4 *__restrict__ tree) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t per = 2 * B - 1;
  if (t >= 2 * G * per) return;
  const size_t dig = t >> 1, g = dig / per, sidx = dig - g * per;
  size_t off = 0, w = B, l = 0;
  while (sidx >= off + w) {
    off += w;
    w >>= 1;
    l++;
  }
  const size_t nc = G * B, lvl_off = 2 * nc - 2 * (nc >> l);
  tree[2 * (lvl_off + g * w + (sidx - off)) + (t & 1)] = subs[t];
}
}  // namespace

hipError_t assemble_subtrees(const uint8_t *subs, size_t B, size_t G, uint8_t *tree, hipStream_t s) {
  const size_t n = 2 * G * (2 * B - 1);
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_assemble_subtrees, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const uint4 *)subs, B,
                     G, (uint4 *)tree);
  return hipGetLastError();
}

hipError_t merkle_tree_io(const uint8_t *ins, size_t n_ins, uint8_t *outs, hipStream_t s) {
  // requires outs to directly follow ins in one buffer (as lcpc-2d's `hashes` split)
  if (outs != ins + 32 * n_ins) return hipErrorInvalidValue;
  return merkle_tree(const_cast<uint8_t *>(ins), n_ins, s);
}

hipError_t gather_columns(int fid, const uint32_t *m, size_t n_rows, size_t n_cols,
                          const uint64_t *idx, size_t n_idx, uint32_t *cols, hipStream_t s,
                          bool col_major, bool canon) {
  const size_t n = n_idx * n_rows;
  if (!n) return hipSuccess;
  return dispatch_field(fid, [&]<class F>() {
    prof::Scope ps("gather_cols", s);
    hipLaunchKernelGGL((k_gather_cols<F>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, m,
                       n_rows, n_cols, idx, n_idx, cols, col_major ? 1 : 0, canon ? 1 : 0);
    return hipGetLastError();
  });
}

hipError_t gather_paths(const uint8_t *hashes, size_t n_hashes, const uint64_t *idx, size_t n_idx,
                        size_t path_len, uint8_t *paths, hipStream_t s) {
  const size_t n = n_idx * path_len;
  if (!n) return hipSuccess;
  const size_t np2 = (n_hashes + 1) / 2;
  hipLaunchKernelGGL(k_gather_paths, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, hashes,
                     np2, idx, n_idx, path_len, paths);
  return hipGetLastError();
}

hipError_t path_checks(const uint8_t *leaves, const uint8_t *paths, size_t n, size_t path_len,
                       const uint64_t *idx, const uint8_t *root, uint32_t *flags, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_path_checks, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, s, leaves, paths,
                     n, path_len, idx, root, flags);
  return hipGetLastError();
}

}  // namespace lcpc
