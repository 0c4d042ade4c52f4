// pos.hpp -- launchers of the proof-of-storage producer kernels (pos.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace lcpc {

// DataField::from_byte_vec (WriteableFt63): ceil(n_bytes / 7) raw u64 limbs
hipError_t pos_pack7(const uint8_t *bytes, size_t n_bytes, uint64_t *out, hipStream_t s);
// field_vec_to_byte_vec truncated to n_bytes
hipError_t pos_unpack7(const uint64_t *elems, size_t n_elems, uint8_t *out, size_t n_bytes,
                       hipStream_t s);
// out[r][bitrev(i)] = in[r][i] (* scale, given as canonical words, if non-null); rows of 2^log_n
hipError_t bitrev_scale(int fid, const uint32_t *in, uint32_t *out, int log_n, size_t n_rows,
                        const uint32_t *scale_canon_words, hipStream_t s);
// dst[i] = base^(i * step_exp)
hipError_t powers(int fid, const uint32_t *base, uint64_t step_exp, size_t n, uint32_t *dst,
                  hipStream_t s);

}  // namespace lcpc
