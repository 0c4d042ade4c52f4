// transcript.hpp -- host-side Fiat-Shamir plumbing of lcpc-2d prove/verify.
//
// merlin 2.0 Transcript (STROBE-128 over Keccak-f[1600]), rand_chacha 0.3 ChaCha20Rng,
// rand 0.8 Uniform<usize>, and ff_derive's Field::random -- the serial host steps the
// reference runs between its parallel loops (lcpc-2d/src/lib.rs:899-941, 1055-1110).  They
// are inherently sequential (a sponge), cost O(kB) per challenge, and feed the GPU kernels
// their tensors and column indices.  No field arithmetic happens here: Field::random only
// draws limbs and compares them with p (rejection sampling on the Montgomery limbs).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

namespace lcpc {

void keccak_f1600(uint64_t st[25]);         // the fastest the host CPU runs (AVX-512F if present)
void keccak_f1600_scalar(uint64_t st[25]);  // any x86-64
void keccak_f1600_avx512(uint64_t st[25]);  // needs AVX-512F
const char *keccak_impl();                  // "avx512" or "scalar"


class Strobe128 {
 public:
  explicit Strobe128(const uint8_t *proto, size_t n);
  void meta_ad(const uint8_t *d, size_t n, bool more);
  void ad(const uint8_t *d, size_t n, bool more);
  void prf(uint8_t *d, size_t n, bool more);
  // n merlin append_message(label, msg_i) records (ln, ml <= 64), absorbed block by block
  void append_records(const uint8_t *label, size_t ln, const uint8_t *msgs, size_t ml, size_t n);
  template <size_t LN, size_t ML>
  void append_records_t(const uint8_t *label, size_t ln, const uint8_t *msgs, size_t ml, size_t n);

 private:
  void run_f();
  void absorb(const uint8_t *d, size_t n);
  void squeeze(uint8_t *d, size_t n);
  void begin_op(uint8_t flags, bool more);
  uint8_t *bytes() { return reinterpret_cast<uint8_t *>(st_); }
  alignas(8) uint64_t st_[25];
  uint8_t pos_ = 0, pos_begin_ = 0, cur_flags_ = 0;
};

class Transcript {
 public:
  explicit Transcript(const uint8_t *label, size_t n);
  void append_message(const uint8_t *label, size_t ln, const uint8_t *msg, size_t mn);
  // append_message(label, m) for every m in msgs (n_msgs messages of msg_len bytes each)
  void append_messages(const uint8_t *label, size_t ln, const uint8_t *msgs, size_t msg_len,
                       size_t n_msgs);
  void challenge_bytes(const uint8_t *label, size_t ln, uint8_t *dst, size_t n);

 private:
  Strobe128 s_;
};

class ChaCha20Rng {
 public:
  explicit ChaCha20Rng(const uint8_t seed[32], int rounds = 20);
  static ChaCha20Rng seed_from_u64(uint64_t state, int rounds = 20);
  uint32_t next_u32();
  uint64_t next_u64();
  void set_stream(uint64_t stream);

 private:
  void refill();
  uint32_t key_[8];
  uint64_t counter_ = 0, stream_ = 0;
  int rounds_;
  uint32_t buf_[64];
  int index_ = 64;
};

// rand 0.8 Uniform::new(low, high).sample(rng) for usize (64-bit)
uint64_t uniform_usize(ChaCha20Rng &rng, uint64_t low, uint64_t high);

// ff_derive Field::random: `limbs` u64 words, top masked to num_bits, accept iff < p (p as u64 limbs)
void field_random(ChaCha20Rng &rng, int limbs, int num_bits, const uint64_t *p, uint64_t *out,
                  size_t n);

}  // namespace lcpc
