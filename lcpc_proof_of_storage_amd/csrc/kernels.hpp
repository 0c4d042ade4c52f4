// kernels.hpp -- host-side launchers of the gfx950 kernels (internal to liblcpc_mi.so).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/lcpc_fft_convention.h"

namespace lcpc {

// Bytes per element of field `fid` (8, 16, 24, 32) and 32-bit words per element.
int field_words(int fid);
inline int field_bytes(int fid) { return 4 * field_words(fid); }
bool field_gpu_supported(int fid);

// ------------------------------------------------------------------ NTT (Ligero encode)
// fffft::fft_io semantics on rows of length n = 2^log_n: out[bitrev(j)] = sum_i in[i] w^(ij),
// w = ROOT_OF_UNITY^(2^(S - log_n)).  Two passes (four-step):
//   pass A: 2^l1-point DIF down each of the 2^l2 columns of the row viewed as [2^l1][2^l2],
//           input zero-padded past n_valid, then the inter-pass twiddle w^(c * bitrev(t'));
//   pass B: 2^l2-point DIF along each contiguous block.
// LCPC_NO_MFMA=1: VALU kernels instead of the int8 matrix-core ones (A/B runs; identical results)
bool no_mfma();

struct NttPlan {
  int fid = -1;
  int log_n = 0, l1 = 0, l2 = 0;
  // an ifft_oi plan (its rows are the inner DIF of the inverse: never reordered by ntt_rows)
  bool inverse = false;
  uint32_t *d_tw = nullptr;        // w^e, e in [0, n): n elements (Montgomery)
  uint32_t *d_tw_canon = nullptr;  // forward plans: the same values' canonical words (below)
  // pass A's inter-pass twiddles w^(c * bitrev_l1(t)) laid out [t][c] (t < 2^l1, c < 2^l2): the
  // lanes of a pass-A store are adjacent columns c, so their twiddle loads are contiguous (from
  // the flat table they were c * bitrev(t) apart, one cache line per lane); log_n > 12 only
  uint32_t *d_tw2 = nullptr;
  uint32_t *d_tw2_canon = nullptr;  // forward plans: canonical words
  // which kernel encodes the PoS-dims rows (2^15-point Ft63, rate 1/2): LCPC_ROW_KERNEL_AUTO (the
  // measured choice: the one-pass kernel for file images, the four-step pair for element rows),
  // _FOURSTEP or _ONEPASS (lcpc_encoding_set_row_kernel)
  int row_kernel = 0;
};
// the [t][c] table above for a pass-A split l1 from a flat table tw (n = 2^log_n elements)
hipError_t ntt_tw2_table(int fid, const uint32_t *tw, int log_n, int l1, uint32_t *out, hipStream_t s);
hipError_t ntt_plan_init(NttPlan &p, int fid, int log_n, bool inverse, hipStream_t s);
void ntt_plan_free(NttPlan &p);
// rows r in [0, n_rows): in = src + r * src_stride (elements), n_valid leading elements
// (rest zero); out = dst + r * dst_stride (n elements).  src may alias dst only if
// src_stride == dst_stride and n_valid == n (in-place full-length transform).
// copy (optional): the n_valid input coefficients of row r are also written to
// copy + r * copy_stride by the first pass, which reads them anyway (commit keeps its own
// coefficient matrix without a separate device-to-device copy).
// canon_out: the outputs are written in canonical form instead of Montgomery form.  The
// transform is linear, so pass A multiplies by w^e R^-1 -- whose Montgomery words are the
// canonical words of w^e (d_tw_canon) -- at no extra cost, and every output's Montgomery words
// become its canonical value: commitments hash their codeword without a per-element
// conversion (the Merkle leaves are over canonical bytes).
// Forward plans follow include/lcpc_fft_convention.h: with LCPC_FFT_OUTPUT_BITREV = 0 the rows are
// reordered to natural order after the transform (bitrev_rows_inplace).
hipError_t ntt_rows(const NttPlan &p, const uint32_t *src, size_t src_stride, size_t n_valid,
                    uint32_t *dst, size_t dst_stride, size_t n_rows, hipStream_t s,
                    uint32_t *copy = nullptr, size_t copy_stride = 0, bool canon_out = false);
// m[r][j] <-> m[r][bitrev_log_n(j)] in place, rows r < n_rows of stride `stride` elements
hipError_t bitrev_rows_inplace(int fid, uint32_t *m, size_t stride, int log_n, size_t n_rows, hipStream_t s);
// The proof-of-storage file image encoded straight into a commitment (ntt_row1.hpp BYTES): row r
// = WriteableFt63 elements [n_per_row r, n_per_row (r + 1)) of the n_bytes-byte image, 7 bytes per
// element (zero padded); canonical output, the coefficient matrix written to copy.  Only at the
// one-pass kernel's shape (ntt_rows_pos_bytes_ok), 16-byte-aligned bytes.
bool ntt_rows_pos_bytes_ok(const NttPlan &p, size_t n_per_row);
bool ntt_row1_bytes(const NttPlan &p);  // whether the file-image commit takes the one-pass kernel (p.row_kernel)
hipError_t ntt_rows_pos_bytes(const NttPlan &p, const uint8_t *bytes, size_t n_bytes, uint32_t *dst,
                              size_t dst_stride, size_t n_rows, hipStream_t s, uint32_t *copy, size_t copy_stride);

// ------------------------------------------------------------------ BLAKE3 / Merkle
// leaf[j] = BLAKE3(32 zero bytes || repr(m[0][j]) || ... || repr(m[n_rows-1][j]))
// for j in [0, n_cols); m is row-major with row stride `stride` elements.
// canon: the matrix holds canonical values (ntt_rows canon_out) instead of Montgomery form.
size_t leaf_hash_scratch_bytes(int fid, size_t n_rows, size_t n_cols);
hipError_t leaf_hashes(int fid, const uint32_t *m, size_t n_rows, size_t n_cols, size_t stride,
                       uint8_t *leaves, void *scratch, hipStream_t s, bool canon = false);
// Row shards: chaining values of chunks [chunk_lo, chunk_hi) of every column's leaf message
// (messages of n_rows rows in total) from a row-major shard m holding rows [row0, ...);
// cvs[(chunk - chunk_lo) * n_cols + col] (8 words), or with blk > 0 the exchange layout
// cvs[((col / blk) * (chunk_hi - chunk_lo) + chunk - chunk_lo) * blk + col % blk].  Chunk c starts
// at message byte 1024 c.  col_stride: elements between columns (1: row-major m; the shard's row
// count with stride 1: an element-major [n_cols][rows] shard).
size_t leaf_n_chunks(int fid, size_t n_rows);
hipError_t leaf_chunk_cvs(int fid, const uint32_t *m, size_t row0, size_t n_rows, size_t n_cols,
                          size_t stride, size_t chunk_lo, size_t chunk_hi, uint32_t *cvs,
                          hipStream_t s, bool canon = false, size_t blk = 0, size_t col_stride = 1);
// leaf digests from all n_chunks chaining values ([chunk][col] layout; cvs is clobbered)
hipError_t leaves_from_cvs(uint32_t *cvs, size_t n_cols, int n_chunks, uint8_t *leaves,
                           hipStream_t s);
// leaf_hashes of a canonical row-major codeword that also writes each (chunk, column)'s share of
// u^T Enc(M): partials[chunk][col] = sum over the chunk's rows r of left[r] * m[r][col]
// (Montgomery left, canonical results; leaf_n_chunks(fid, n_rows) x n_cols elements).  Fields
// whose element tiles a BLAKE3 block only (leaf_eval_fusable).
bool leaf_eval_fusable(int fid);
hipError_t leaf_hashes_eval(int fid, const uint32_t *m, size_t n_rows, size_t n_cols, size_t stride,
                            uint8_t *leaves, void *scratch, const uint32_t *left, uint32_t *partials,
                            hipStream_t s);
// same, for a [column][row] matrix (opened columns of a proof)
hipError_t leaf_hashes_cols(int fid, const uint32_t *cols, size_t n_rows, size_t n_cols,
                            uint8_t *leaves, void *scratch, hipStream_t s, bool canon = false);
// hashes = [leaves (np2) | level 1 (np2/2) | ... | root]; fills every level above the leaves
hipError_t merkle_tree(uint8_t *hashes, size_t np2, hipStream_t s);
// generic Merkle over ins (n_ins = outs + 1 nodes, power of two) -> outs
hipError_t merkle_tree_io(const uint8_t *ins, size_t n_ins, uint8_t *outs, hipStream_t s);
// row shards: G subtrees of 2B - 1 digests (column block g, levels leaves..root, B a power of
// two) into levels 0..log2(B) of the whole tree of G B leaves ([leaves | level 1 | ...] layout)
hipError_t assemble_subtrees(const uint8_t *subs, size_t B, size_t G, uint8_t *tree, hipStream_t s);

// ------------------------------------------------------------------ prover helpers
// out[t][c] = sum_r tensors[t][r] * coeffs[r][c]   (t < n_tensors, c < n_per_row)
size_t collapse_scratch_bytes(int fid, size_t n_rows, size_t n_per_row, int n_tensors);
hipError_t collapse_rows(int fid, const uint32_t *coeffs, size_t n_rows, size_t n_per_row,
                         const uint32_t *tensors, int n_tensors, uint32_t *out, void *scratch,
                         hipStream_t s);
// out[c] = sum_k vecs[k][c] (n_vecs vectors of len elements)
hipError_t collapse_fold_rows(int fid, const uint32_t *vecs, size_t n_vecs, size_t len, uint32_t *out,
                              hipStream_t s);
// cols[k][r] = m[r][idx[k]] (m row-major) or m[idx[k]][r] (col_major); canon: m holds
// canonical values and the gathered columns are converted to Montgomery form;
// paths[k][i] = sibling digests of leaf idx[k]
hipError_t gather_columns(int fid, const uint32_t *m, size_t n_rows, size_t n_cols,
                          const uint64_t *idx, size_t n_idx, uint32_t *cols, hipStream_t s,
                          bool col_major = false, bool canon = false);
hipError_t gather_paths(const uint8_t *hashes, size_t n_hashes, const uint64_t *idx,
                        size_t n_idx, size_t path_len, uint8_t *paths, hipStream_t s);

// ------------------------------------------------------------------ verifier helpers
// dots[k][t] = sum_r tensors[t][r] * cols[k][r]; ok[k] bit t set iff dots == enc[t][idx[k]]
hipError_t column_checks(int fid, const uint32_t *cols, size_t n_cols_open, size_t n_rows,
                         const uint32_t *tensors, int n_tensors, const uint32_t *encs,
                         size_t enc_len, const uint64_t *idx, uint32_t *flags, hipStream_t s);
// path[k] check against root: flags[k] = 1 iff the Merkle path of leaf k verifies
hipError_t path_checks(const uint8_t *leaves, const uint8_t *paths, size_t n, size_t path_len,
                       const uint64_t *idx, const uint8_t *root, uint32_t *flags,
                       hipStream_t s);
// out = sum_i a[i] * b[i]
hipError_t dot(int fid, const uint32_t *a, const uint32_t *b, size_t n, uint32_t *out,
               void *scratch, hipStream_t s);
// elementwise Montgomery <-> canonical conversion (device); with bad non-null, canonical
// inputs that are not < p set *bad = 1
hipError_t convert(int fid, const uint32_t *in, uint32_t *out, size_t n, bool to_mont,
                   hipStream_t s, uint32_t *bad = nullptr);
// bytes (a multiple of 8, 8-byte aligned pointers) copied by a kernel on stream s; either side
// may be device-mapped page-locked host memory (over_link: then a capped grid)
hipError_t copy_words(void *dst, const void *src, size_t bytes, hipStream_t s, bool over_link = true);
// chunk-local self-test entry: out = a * b elementwise (Montgomery)
hipError_t mul_elementwise(int fid, const uint32_t *a, const uint32_t *b, uint32_t *out,
                           size_t n, hipStream_t s);

}  // namespace lcpc
