// issue_cost.hip -- per-class VALU issue cost on gfx950, for the Ligero encode's cycle model
// (the instruction counts are profiles/r05_encode_isa_attribution.txt).
//
// Each kernel runs ITERS iterations of a fixed block of one instruction class on 8 independent
// register streams (so it measures issue throughput, not a dependency chain), in waves of 64,
// at k = 1, 2, 4 (and 8) waves per SIMD: 1024 * k waves in blocks of 256 threads, one wave per
// SIMD per block.  Every wave reads the shader clock (clock64 = s_memtime) around its loop, so
//   cost = (its elapsed shader cycles) / (instructions it issued) / k
// is the SIMD issue cycles one wave-instruction of the class costs when k waves share the SIMD
// (the waves run concurrently: a throughput-bound SIMD interleaves them).  The kernel's HIP-event
// time gives the same figure through the measured shader clock (clock64 against wall_clock64).
// Each wave also records its hardware slot (HW_ID: SIMD, CU, SE; XCC_ID) so the report shows the
// waves-per-SIMD the dispatcher actually produced.
//
// Classes: the ones pass A / pass B issue (k_pass_a<Ft127, 8, 3, 8>: 812 v_mad_u64_u32, 1216
// v_addc/v_subb with SGPR carries, 213 v_add_co, 193 v_cndmask, 98 v_mov, 1038 s_nop 0 per
// thread), plus the pattern the compiler emits for the multi-limb carry chains: each link reads
// the SGPR carry the previous link wrote, a one-wait-state hazard on gfx950 (s_nop 0 between).
//
//   hipcc -O3 --offload-arch=gfx950 -o issue_cost issue_cost.hip && ./issue_cost
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <map>
#include <set>
#include <vector>

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                            \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

constexpr int ITERS = 16384;

enum Mode { MAD = 0, ADDC, ADDCO, CND, MOV, ADD32, NOP_PAIR, HAZARD, NOP_ONLY, CND_SGPR, CND_CMP, BFI, SUBB_MASK,
            ADD32_E64, ADD32_LIT, CHAIN_VCC, MAD_VCC_CHAIN, XOR32, ALIGNBIT, ADD3, PERM, BITOP3, N_MODES };
static const char *NAMES[N_MODES] = {
    "v_mad_u64_u32",
    "v_addc_co_u32 (independent SGPR carries)",
    "v_add_co_u32 (SGPR carry out)",
    "v_cndmask_b32",
    "v_mov_b32",
    "v_add_u32 (reference: full-rate)",
    "v_add_u32 + s_nop 0 (pair)",
    "carry chain: add(c)_co + s_nop 0 per link",
    "s_nop 0 alone",
    "v_cndmask_b32_e64 (SGPR-pair mask)",
    "v_cmp_gt_u32 + v_cndmask_b32 (vcc just written)",
    "v_bfi_b32 (VGPR mask select)",
    "v_subb_co_u32 (0 - borrow: a VGPR mask)",
    "v_add_u32_e64 (the same add, 8-byte encoding)",
    "v_add_u32_e32 + 32-bit literal (8 bytes)",
    "carry chain through VCC, e32 forms (4 bytes)",
    "mad_u64 (carry to VCC) + v_addc_co_u32_e32 fold",
    "v_xor_b32",
    "v_alignbit_b32 (rotate)",
    "v_add3_u32",
    "v_perm_b32",
    "v_bitop3_b32 (3-input xor)",
};
// instructions (VALU + s_nop) per stream per iteration, and VALU ones among them
static const int INSTR[N_MODES] = {1, 1, 1, 1, 1, 1, 2, 2, 1, 1, 2, 1, 1, 1, 1, 1, 2, 1, 1, 1, 1, 1};
static const int VALU[N_MODES] = {1, 1, 1, 1, 1, 1, 1, 1, 0, 1, 2, 1, 1, 1, 1, 1, 2, 1, 1, 1, 1, 1};

struct WaveRec {
  uint64_t cycles;
  uint32_t hw_id, xcc_id;
};

template <int MODE>
__global__ __launch_bounds__(256) void k_issue(WaveRec *rec, uint32_t seed) {
  uint32_t a[8], b[8];
  uint64_t c[8];
  for (int i = 0; i < 8; i++) {
    a[i] = threadIdx.x * 7 + seed + i;
    b[i] = blockIdx.x * 13 + seed * 3 + i;
    c[i] = (uint64_t)a[i] << 7;
  }
  asm volatile("s_mov_b64 vcc, -1" ::: "vcc");
  __syncthreads();
  const uint64_t t0 = clock64();
  // one asm statement per iteration holding all 8 streams' instructions: the compiler's hazard
  // recognizer treats an inline-asm block as opaque and pads its boundary with s_nop, so the
  // block must be long for that padding to vanish in the count (it is reported: see main);
  // within a block the instructions are exactly the ones named
#define V8(I) "+v"(a[I])
  for (int it = 0; it < ITERS; it++) {
    if constexpr (MODE == MAD) {
      asm volatile(
          "v_mad_u64_u32 %0, vcc, %8, %16, %0\n\tv_mad_u64_u32 %1, vcc, %9, %17, %1\n\t"
          "v_mad_u64_u32 %2, vcc, %10, %18, %2\n\tv_mad_u64_u32 %3, vcc, %11, %19, %3\n\t"
          "v_mad_u64_u32 %4, vcc, %12, %20, %4\n\tv_mad_u64_u32 %5, vcc, %13, %21, %5\n\t"
          "v_mad_u64_u32 %6, vcc, %14, %22, %6\n\tv_mad_u64_u32 %7, vcc, %15, %23, %7"
          : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7])
          : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]),
            "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
          : "vcc");
    } else if constexpr (MODE == ADDC) {  // 8 independent carry chains, one SGPR pair each
      asm volatile(
          "v_addc_co_u32 %0, s[40:41], %0, %8, s[40:41]\n\tv_addc_co_u32 %1, s[42:43], %1, %9, s[42:43]\n\t"
          "v_addc_co_u32 %2, s[44:45], %2, %10, s[44:45]\n\tv_addc_co_u32 %3, s[46:47], %3, %11, s[46:47]\n\t"
          "v_addc_co_u32 %4, s[48:49], %4, %12, s[48:49]\n\tv_addc_co_u32 %5, s[50:51], %5, %13, s[50:51]\n\t"
          "v_addc_co_u32 %6, s[52:53], %6, %14, s[52:53]\n\tv_addc_co_u32 %7, s[54:55], %7, %15, s[54:55]"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
          : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53",
            "s54", "s55");
    } else if constexpr (MODE == ADDCO) {
      asm volatile(
          "v_add_co_u32 %0, s[40:41], %0, %8\n\tv_add_co_u32 %1, s[42:43], %1, %9\n\t"
          "v_add_co_u32 %2, s[44:45], %2, %10\n\tv_add_co_u32 %3, s[46:47], %3, %11\n\t"
          "v_add_co_u32 %4, s[48:49], %4, %12\n\tv_add_co_u32 %5, s[50:51], %5, %13\n\t"
          "v_add_co_u32 %6, s[52:53], %6, %14\n\tv_add_co_u32 %7, s[54:55], %7, %15"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
          : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53",
            "s54", "s55");
    } else if constexpr (MODE == CND) {
      asm volatile(
          "v_cndmask_b32 %0, %0, %8, vcc\n\tv_cndmask_b32 %1, %1, %9, vcc\n\t"
          "v_cndmask_b32 %2, %2, %10, vcc\n\tv_cndmask_b32 %3, %3, %11, vcc\n\t"
          "v_cndmask_b32 %4, %4, %12, vcc\n\tv_cndmask_b32 %5, %5, %13, vcc\n\t"
          "v_cndmask_b32 %6, %6, %14, vcc\n\tv_cndmask_b32 %7, %7, %15, vcc"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
          : "vcc");
    } else if constexpr (MODE == MOV) {
      asm volatile(
          "v_mov_b32 %0, %9\n\tv_mov_b32 %1, %10\n\tv_mov_b32 %2, %11\n\tv_mov_b32 %3, %12\n\t"
          "v_mov_b32 %4, %13\n\tv_mov_b32 %5, %14\n\tv_mov_b32 %6, %15\n\tv_mov_b32 %7, %8"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]));
    } else if constexpr (MODE == ADD32) {
      asm volatile(
          "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %9\n\tv_add_u32 %2, %2, %10\n\tv_add_u32 %3, %3, %11\n\t"
          "v_add_u32 %4, %4, %12\n\tv_add_u32 %5, %5, %13\n\tv_add_u32 %6, %6, %14\n\tv_add_u32 %7, %7, %15"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]));
    } else if constexpr (MODE == NOP_PAIR) {
      asm volatile(
          "v_add_u32 %0, %0, %8\n\ts_nop 0\n\tv_add_u32 %1, %1, %9\n\ts_nop 0\n\t"
          "v_add_u32 %2, %2, %10\n\ts_nop 0\n\tv_add_u32 %3, %3, %11\n\ts_nop 0\n\t"
          "v_add_u32 %4, %4, %12\n\ts_nop 0\n\tv_add_u32 %5, %5, %13\n\ts_nop 0\n\t"
          "v_add_u32 %6, %6, %14\n\ts_nop 0\n\tv_add_u32 %7, %7, %15\n\ts_nop 0"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]));
    } else if constexpr (MODE == HAZARD) {
      // the encode's carry chain: each add-with-carry reads the SGPR carry the previous one
      // wrote (a gfx950 hazard: one wait state, the compiler's s_nop 0) -- 8 chain links
      asm volatile(
          "v_add_co_u32 %0, s[40:41], %0, %8\n\ts_nop 0\n\tv_addc_co_u32 %1, s[40:41], %1, %9, s[40:41]\n\ts_nop 0\n\t"
          "v_addc_co_u32 %2, s[40:41], %2, %10, s[40:41]\n\ts_nop 0\n\tv_addc_co_u32 %3, s[40:41], %3, %11, s[40:41]\n\ts_nop 0\n\t"
          "v_add_co_u32 %4, s[40:41], %4, %12\n\ts_nop 0\n\tv_addc_co_u32 %5, s[40:41], %5, %13, s[40:41]\n\ts_nop 0\n\t"
          "v_addc_co_u32 %6, s[40:41], %6, %14, s[40:41]\n\ts_nop 0\n\tv_addc_co_u32 %7, s[40:41], %7, %15, s[40:41]\n\ts_nop 0"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
          : "s40", "s41");
    } else if constexpr (MODE == NOP_ONLY) {
      asm volatile("s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0");
    } else if constexpr (MODE == CND_SGPR) {
      asm volatile(
          "v_cndmask_b32_e64 %0, %0, %8, s[40:41]\n\tv_cndmask_b32_e64 %1, %1, %9, s[40:41]\n\t"
          "v_cndmask_b32_e64 %2, %2, %10, s[40:41]\n\tv_cndmask_b32_e64 %3, %3, %11, s[40:41]\n\t"
          "v_cndmask_b32_e64 %4, %4, %12, s[40:41]\n\tv_cndmask_b32_e64 %5, %5, %13, s[40:41]\n\t"
          "v_cndmask_b32_e64 %6, %6, %14, s[40:41]\n\tv_cndmask_b32_e64 %7, %7, %15, s[40:41]"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
          : "s40", "s41");
    } else if constexpr (MODE == CND_CMP) {  // the field add's pattern: a compare, then its select
      asm volatile(
          "v_cmp_gt_u32 vcc, %0, %8\n\tv_cndmask_b32 %0, %0, %8, vcc\n\t"
          "v_cmp_gt_u32 vcc, %1, %9\n\tv_cndmask_b32 %1, %1, %9, vcc\n\t"
          "v_cmp_gt_u32 vcc, %2, %10\n\tv_cndmask_b32 %2, %2, %10, vcc\n\t"
          "v_cmp_gt_u32 vcc, %3, %11\n\tv_cndmask_b32 %3, %3, %11, vcc\n\t"
          "v_cmp_gt_u32 vcc, %4, %12\n\tv_cndmask_b32 %4, %4, %12, vcc\n\t"
          "v_cmp_gt_u32 vcc, %5, %13\n\tv_cndmask_b32 %5, %5, %13, vcc\n\t"
          "v_cmp_gt_u32 vcc, %6, %14\n\tv_cndmask_b32 %6, %6, %14, vcc\n\t"
          "v_cmp_gt_u32 vcc, %7, %15\n\tv_cndmask_b32 %7, %7, %15, vcc"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
          : "vcc");
    } else if constexpr (MODE == BFI) {
      asm volatile(
          "v_bfi_b32 %0, %8, %0, %9\n\tv_bfi_b32 %1, %9, %1, %10\n\tv_bfi_b32 %2, %10, %2, %11\n\t"
          "v_bfi_b32 %3, %11, %3, %12\n\tv_bfi_b32 %4, %12, %4, %13\n\tv_bfi_b32 %5, %13, %5, %14\n\t"
          "v_bfi_b32 %6, %14, %6, %15\n\tv_bfi_b32 %7, %15, %7, %8"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]));
    } else if constexpr (MODE == ADD32_E64) {
      asm volatile(
          "v_add_u32_e64 %0, %0, %8\n\tv_add_u32_e64 %1, %1, %9\n\tv_add_u32_e64 %2, %2, %10\n\tv_add_u32_e64 %3, %3, %11\n\t"
          "v_add_u32_e64 %4, %4, %12\n\tv_add_u32_e64 %5, %5, %13\n\tv_add_u32_e64 %6, %6, %14\n\tv_add_u32_e64 %7, %7, %15"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]));
    } else if constexpr (MODE == ADD32_LIT) {
      asm volatile(
          "v_add_u32 %0, 0x12345, %0\n\tv_add_u32 %1, 0x12346, %1\n\tv_add_u32 %2, 0x12347, %2\n\tv_add_u32 %3, 0x12348, %3\n\t"
          "v_add_u32 %4, 0x12349, %4\n\tv_add_u32 %5, 0x1234a, %5\n\tv_add_u32 %6, 0x1234b, %6\n\tv_add_u32 %7, 0x1234c, %7"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7));
    } else if constexpr (MODE == CHAIN_VCC) {  // two 4-limb additions, carries in VCC (e32)
      asm volatile(
          "v_add_co_u32_e32 %0, vcc, %0, %8\n\tv_addc_co_u32_e32 %1, vcc, %1, %9, vcc\n\t"
          "v_addc_co_u32_e32 %2, vcc, %2, %10, vcc\n\tv_addc_co_u32_e32 %3, vcc, %3, %11, vcc\n\t"
          "v_add_co_u32_e32 %4, vcc, %4, %12\n\tv_addc_co_u32_e32 %5, vcc, %5, %13, vcc\n\t"
          "v_addc_co_u32_e32 %6, vcc, %6, %14, vcc\n\tv_addc_co_u32_e32 %7, vcc, %7, %15, vcc"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
          : "vcc");
    } else if constexpr (MODE == MAD_VCC_CHAIN) {  // product scanning with the carry folded via VCC
      asm volatile(
          "v_mad_u64_u32 %0, vcc, %8, %16, %0\n\tv_addc_co_u32_e32 %9, vcc, 0, %9, vcc\n\t"
          "v_mad_u64_u32 %1, vcc, %10, %17, %1\n\tv_addc_co_u32_e32 %11, vcc, 0, %11, vcc\n\t"
          "v_mad_u64_u32 %2, vcc, %12, %18, %2\n\tv_addc_co_u32_e32 %13, vcc, 0, %13, vcc\n\t"
          "v_mad_u64_u32 %3, vcc, %14, %19, %3\n\tv_addc_co_u32_e32 %15, vcc, 0, %15, vcc\n\t"
          "v_mad_u64_u32 %4, vcc, %8, %20, %4\n\tv_addc_co_u32_e32 %9, vcc, 0, %9, vcc\n\t"
          "v_mad_u64_u32 %5, vcc, %10, %21, %5\n\tv_addc_co_u32_e32 %11, vcc, 0, %11, vcc\n\t"
          "v_mad_u64_u32 %6, vcc, %12, %22, %6\n\tv_addc_co_u32_e32 %13, vcc, 0, %13, vcc\n\t"
          "v_mad_u64_u32 %7, vcc, %14, %23, %7\n\tv_addc_co_u32_e32 %15, vcc, 0, %15, vcc"
          : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]), "+v"(c[5]), "+v"(c[6]), "+v"(c[7]),
            "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
          : "vcc");
    } else if constexpr (MODE == XOR32 || MODE == ALIGNBIT || MODE == ADD3 || MODE == PERM || MODE == BITOP3) {
#define OP3(OPS)                                                                                              \
  asm volatile(OPS : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)                                  \
               : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]))
      if constexpr (MODE == XOR32)
        OP3("v_xor_b32 %0, %0, %8\n\tv_xor_b32 %1, %1, %9\n\tv_xor_b32 %2, %2, %10\n\tv_xor_b32 %3, %3, %11\n\t"
            "v_xor_b32 %4, %4, %12\n\tv_xor_b32 %5, %5, %13\n\tv_xor_b32 %6, %6, %14\n\tv_xor_b32 %7, %7, %15");
      else if constexpr (MODE == ALIGNBIT)
        OP3("v_alignbit_b32 %0, %0, %0, 12\n\tv_alignbit_b32 %1, %1, %1, 12\n\tv_alignbit_b32 %2, %2, %2, 12\n\t"
            "v_alignbit_b32 %3, %3, %3, 12\n\tv_alignbit_b32 %4, %4, %4, 12\n\tv_alignbit_b32 %5, %5, %5, 12\n\t"
            "v_alignbit_b32 %6, %6, %6, 12\n\tv_alignbit_b32 %7, %7, %7, 12");
      else if constexpr (MODE == ADD3)
        OP3("v_add3_u32 %0, %0, %8, %9\n\tv_add3_u32 %1, %1, %9, %10\n\tv_add3_u32 %2, %2, %10, %11\n\t"
            "v_add3_u32 %3, %3, %11, %12\n\tv_add3_u32 %4, %4, %12, %13\n\tv_add3_u32 %5, %5, %13, %14\n\t"
            "v_add3_u32 %6, %6, %14, %15\n\tv_add3_u32 %7, %7, %15, %8");
      else if constexpr (MODE == PERM)
        OP3("v_perm_b32 %0, %0, %0, %8\n\tv_perm_b32 %1, %1, %1, %8\n\tv_perm_b32 %2, %2, %2, %8\n\t"
            "v_perm_b32 %3, %3, %3, %8\n\tv_perm_b32 %4, %4, %4, %8\n\tv_perm_b32 %5, %5, %5, %8\n\t"
            "v_perm_b32 %6, %6, %6, %8\n\tv_perm_b32 %7, %7, %7, %8");
      else
        OP3("v_bitop3_b32 %0, %0, %8, %9 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %9, %10 bitop3:0x96\n\tv_bitop3_b32 %2, %2, %10, %11 bitop3:0x96\n\t"
            "v_bitop3_b32 %3, %3, %11, %12 bitop3:0x96\n\tv_bitop3_b32 %4, %4, %12, %13 bitop3:0x96\n\tv_bitop3_b32 %5, %5, %13, %14 bitop3:0x96\n\t"
            "v_bitop3_b32 %6, %6, %14, %15 bitop3:0x96\n\tv_bitop3_b32 %7, %7, %15, %8 bitop3:0x96");
#undef OP3
    } else {
      asm volatile(
          "v_subb_co_u32 %0, s[40:41], 0, %8, s[40:41]\n\tv_subb_co_u32 %1, s[42:43], 0, %9, s[42:43]\n\t"
          "v_subb_co_u32 %2, s[44:45], 0, %10, s[44:45]\n\tv_subb_co_u32 %3, s[46:47], 0, %11, s[46:47]\n\t"
          "v_subb_co_u32 %4, s[48:49], 0, %12, s[48:49]\n\tv_subb_co_u32 %5, s[50:51], 0, %13, s[50:51]\n\t"
          "v_subb_co_u32 %6, s[52:53], 0, %14, s[52:53]\n\tv_subb_co_u32 %7, s[54:55], 0, %15, s[54:55]"
          : V8(0), V8(1), V8(2), V8(3), V8(4), V8(5), V8(6), V8(7)
          : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7])
          : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53",
            "s54", "s55");
    }
  }
#undef V8
  const uint64_t t1 = clock64();
  uint32_t acc = 0;
  for (int i = 0; i < 8; i++) acc ^= a[i] ^ b[i] ^ (uint32_t)c[i] ^ (uint32_t)(c[i] >> 32);
  if ((threadIdx.x & 63) == 0) {
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    WaveRec r;
    r.cycles = t1 - t0 + (acc == 0x9e3779b9u ? 1 : 0);  // (keeps the streams live)
    r.hw_id = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
    r.xcc_id = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    rec[wave] = r;
  }
}

__global__ void k_clock(uint64_t *out) {
  const uint64_t c0 = clock64(), w0 = wall_clock64();
  uint64_t c1 = c0, w1 = w0;
  while (w1 - w0 < 2000000) {  // 20 ms of the 100 MHz constant clock
    c1 = clock64();
    w1 = wall_clock64();
  }
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = w1 - w0;
  }
}

template <int MODE>
int run(int k, int n_cu, double clock_mhz, FILE *js, bool first) {
  const int waves = n_cu * 4 * k, blocks = waves / 4;
  WaveRec *d;
  CHECK(hipMalloc(&d, waves * sizeof(WaveRec)));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_issue<MODE>, dim3(blocks), dim3(256), 0, 0, d, 1u);  // warm-up
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_issue<MODE>, dim3(blocks), dim3(256), 0, 0, d, 2u);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<WaveRec> h(waves);
  CHECK(hipMemcpy(h.data(), d, waves * sizeof(WaveRec), hipMemcpyDeviceToHost));
  std::map<uint64_t, int> per_simd;
  std::vector<double> cyc;
  for (auto &r : h) {
    // (XCC, SE, SH, CU, SIMD) -- HW_ID: simd [5:4], cu [11:8], sh [12], se [15:13]
    const uint64_t key = ((uint64_t)r.xcc_id << 32) | (r.hw_id & 0xFF30u);
    per_simd[key]++;
    cyc.push_back((double)r.cycles);
  }
  int max_w = 0;
  for (auto &kv : per_simd) max_w = std::max(max_w, kv.second);
  std::sort(cyc.begin(), cyc.end());
  const double med = cyc[cyc.size() / 2];
  const double instr = (double)ITERS * 8 * INSTR[MODE], valu = (double)ITERS * 8 * VALU[MODE];
  // SIMD cycles per wave-instruction: a wave's cycles / its instructions / the waves sharing its SIMD
  const double c_instr = med / instr / k;
  const double c_valu = valu ? med / valu / k : 0;
  // the same from the kernel time: SIMD-cycles available / wave-instructions issued
  const double sim_cycles = ms * 1e-3 * clock_mhz * 1e6 * n_cu * 4;
  const double c_event = sim_cycles / (instr * waves);
  printf("%-44s k=%d  simds=%zu max_waves/simd=%d  median wave %.0f cyc  %.2f cyc/instr  %.2f cyc/VALU  "
         "(kernel %.3f ms -> %.2f cyc/instr)\n",
         NAMES[MODE], k, per_simd.size(), max_w, med, c_instr, c_valu, ms, c_event);
  fprintf(js, "%s{\"class\": \"%s\", \"waves_per_simd\": %d, \"simds_used\": %zu, \"max_waves_per_simd\": %d, "
              "\"median_wave_cycles\": %.0f, \"cycles_per_instr\": %.4f, \"cycles_per_valu\": %.4f, "
              "\"kernel_ms\": %.4f, \"cycles_per_instr_from_event\": %.4f}",
          first ? "" : ",\n", NAMES[MODE], k, per_simd.size(), max_w, med, c_instr, c_valu, ms, c_event);
  CHECK(hipFree(d));
  return 0;
}

int main(int argc, char **argv) {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int n_cu = prop.multiProcessorCount;
  uint64_t *dc, hc[2];
  CHECK(hipMalloc(&dc, 16));
  hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, 0, dc);
  CHECK(hipMemcpy(hc, dc, 16, hipMemcpyDeviceToHost));
  int wall_khz = 0;
  CHECK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0));
  const double clock_mhz = (double)hc[0] / ((double)hc[1] / (wall_khz * 1e3)) / 1e6;
  printf("%s: %d CUs, shader clock %.0f MHz (clock64 over wall_clock64 at %d kHz, idle-ish GPU)\n", prop.name,
         n_cu, clock_mhz, wall_khz);
  FILE *js = fopen(argc > 1 ? argv[1] : "issue_cost.json", "w");
  fprintf(js, "{\"device\": \"%s\", \"cus\": %d, \"shader_clock_mhz\": %.1f, \"iters\": %d, \"rows\": [\n",
          prop.name, n_cu, clock_mhz, ITERS);
  bool first = true;
  for (int k : {1, 2, 4, 8}) {
    int rc = 0;
    rc |= run<MAD>(k, n_cu, clock_mhz, js, first);
    first = false;
    rc |= run<ADDC>(k, n_cu, clock_mhz, js, false);
    rc |= run<ADDCO>(k, n_cu, clock_mhz, js, false);
    rc |= run<CND>(k, n_cu, clock_mhz, js, false);
    rc |= run<MOV>(k, n_cu, clock_mhz, js, false);
    rc |= run<ADD32>(k, n_cu, clock_mhz, js, false);
    rc |= run<NOP_PAIR>(k, n_cu, clock_mhz, js, false);
    rc |= run<HAZARD>(k, n_cu, clock_mhz, js, false);
    rc |= run<NOP_ONLY>(k, n_cu, clock_mhz, js, false);
    rc |= run<CND_SGPR>(k, n_cu, clock_mhz, js, false);
    rc |= run<CND_CMP>(k, n_cu, clock_mhz, js, false);
    rc |= run<BFI>(k, n_cu, clock_mhz, js, false);
    rc |= run<SUBB_MASK>(k, n_cu, clock_mhz, js, false);
    rc |= run<ADD32_E64>(k, n_cu, clock_mhz, js, false);
    rc |= run<ADD32_LIT>(k, n_cu, clock_mhz, js, false);
    rc |= run<CHAIN_VCC>(k, n_cu, clock_mhz, js, false);
    rc |= run<MAD_VCC_CHAIN>(k, n_cu, clock_mhz, js, false);
    rc |= run<XOR32>(k, n_cu, clock_mhz, js, false);
    rc |= run<ALIGNBIT>(k, n_cu, clock_mhz, js, false);
    rc |= run<ADD3>(k, n_cu, clock_mhz, js, false);
    rc |= run<PERM>(k, n_cu, clock_mhz, js, false);
    rc |= run<BITOP3>(k, n_cu, clock_mhz, js, false);
    if (rc) return rc;
  }
  fprintf(js, "\n]}\n");
  fclose(js);
  return 0;
}
