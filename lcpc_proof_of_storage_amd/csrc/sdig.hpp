// sdig.hpp -- Brakedown / SDIG expander-code encoding (lcpc-brakedown-pc) for gfx950.
//
// Host side (sdig_host.cpp): the code parameters of SdigSpecification (codespec.rs:17-232), the
// encoding dimensions of SdigEncodingS (lib.rs:54-137), and matgen::generate (matgen.rs:28-188)
// -- the random sparse precode / postcode matrices, drawn from ChaCha20Rng::seed_from_u64(seed)
// with set_stream(level) exactly as the reference draws them, then stored output-major (CSR) so
// that every output element is a gather over its nonzeros.
//
// Device side (sdig.hip): encode::encode (encode.rs:36-94) on an ELEMENT-MAJOR codeword
// [n_cols][R] for R rows at once: every nonzero multiplies a contiguous run of R elements (one
// per row), so the gathers of a wave are coalesced; the reference's segment arithmetic (inputs
// [in_start, in_end), outputs after them, R-S on the last precode output, postcodes in reverse
// over [precode_i output || everything after]) is unchanged.
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace lcpc {

struct SdigSpec {
  size_t an, ad, bn, bd, rn, rd, blen;  // alpha, beta, r as fractions; base-case length
};
// SdigCode1..6 (codespec.rs:169-232); nullptr for another id
const SdigSpec *sdig_spec(int code);
// SdigEncodingS::_n_col_opens (lib.rs:57-61)
size_t sdig_n_col_opens(int code);
// SdigEncodingS::new (lib.rs:103-110) / new_ml (:114-123) -> n_per_row (0 if invalid)
size_t sdig_new_np(int code, int num_bits, size_t len);
size_t sdig_new_ml_np(int code, int num_bits, size_t n_vars);

// matgen::get_dims (matgen.rs:56-111): per level (n_i, m_i, d_i) of the precode and postcode
int sdig_level_dims(int code, size_t n, double log2p, std::vector<std::array<size_t, 3>> &pre,
                    std::vector<std::array<size_t, 3>> &post);

// A code matrix of shape rows x cols (CsMat::new_csc((m, n), ...)), stored by output row.
struct CsrHost {
  size_t rows = 0, cols = 0;
  std::vector<uint32_t> ptr;  // rows + 1
  std::vector<uint32_t> idx;  // input index of each nonzero
  std::vector<uint64_t> val;  // nonzero values, `limbs` u64 Montgomery words each
};

// matgen::generate for field (limbs, num_bits, p): false if n <= baselen
bool sdig_generate(int limbs, int num_bits, const uint64_t *p, int code, size_t n, uint64_t seed,
                   std::vector<CsrHost> &pre, std::vector<CsrHost> &post);
// encode::codeword_length (encode.rs:18-33)
size_t sdig_codeword_length(const std::vector<CsrHost> &pre, const std::vector<CsrHost> &post);

// ------------------------------------------------------------------ device plan
struct CsrDev {
  size_t rows = 0, cols = 0, nnz = 0;
  const uint32_t *ptr = nullptr, *idx = nullptr, *val = nullptr;
  // Ft127 matrix-core form (sdig.hip, k_spmm_mfma): every output's nonzeros padded to groups of
  // 4; gptr[j] = first group of output j, pidx = input index per padded nonzero, gval = its
  // value (16 B, zero for pads; the kernel derives the digits of val 2^(8a) mod p itself)
  const uint32_t *gptr = nullptr, *pidx = nullptr, *gval = nullptr;
  size_t groups = 0;
};
struct SdigPlan {
  int fid = -1;
  size_t n_per_row = 0, n_cols = 0;
  std::vector<CsrDev> pre, post;
  size_t tmp_elems = 0;      // scratch elements per row (last precode output)
  void *d_buf = nullptr;     // one allocation holding every matrix
  void *d_mfma = nullptr;    // the matrix-core forms (Ft127), when every level has one
  bool mfma = false;
};
hipError_t sdig_plan_upload(SdigPlan &plan, int fid, const std::vector<CsrHost> &pre,
                            const std::vector<CsrHost> &post, hipStream_t s);
void sdig_plan_free(SdigPlan &plan);
// In place on cw = [n_cols][R] (element-major; elements [0, n_per_row) hold the message of every
// row): writes the rest of every codeword.  tmp holds tmp_elems * R elements.
hipError_t sdig_encode_cm(const SdigPlan &plan, uint32_t *cw, size_t R, uint32_t *tmp,
                          hipStream_t s);

// dst[c][r] = src[r][c] (element units, row strides src_stride / dst_stride) for r < rows,
// c < cols; source columns c >= n_valid, and flat source offsets r * src_stride + c >= n_flat,
// read as zero.  mode TR_FROM_MONT stores canonical values; TR_TO_MONT reads canonical values
// into Montgomery form and sets *bad = 1 if any is not < p.  `copy` (TR_PLAIN only) also
// receives the zero-padded source row-major: copy[r * copy_stride + c], r < rows, c < cols.
enum { TR_PLAIN = 0, TR_FROM_MONT = 1, TR_TO_MONT = 2 };
hipError_t transpose_elems(int fid, const uint32_t *src, size_t rows, size_t cols,
                           size_t src_stride, size_t n_valid, uint32_t *dst, size_t dst_stride,
                           hipStream_t s, int mode = TR_PLAIN, uint32_t *bad = nullptr,
                           size_t n_flat = SIZE_MAX, uint32_t *copy = nullptr, size_t copy_stride = 0);

}  // namespace lcpc
