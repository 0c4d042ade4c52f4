// lcpc_host.cpp -- host orchestration and C ABI of liblcpc_mi.so (see include/lcpc_mi.h).
//
// The reference's lcpc-2d commit / prove / verify (lcpc-2d/src/lib.rs:651-1123) restated for
// one MI355X: every field operation and every hash runs in the gfx950 kernels (ntt*.hip,
// blake3.hip, collapse.hip); this file only sequences them, moves the proof-sized vectors
// across PCIe, and runs the inherently serial Fiat-Shamir steps (transcript.cpp).
// There is no CPU fallback: with no usable HIP device every compute entry point fails with
// LCPC_ERR_NO_DEVICE.
#include "host_internal.hpp"

using namespace lcpc;
using namespace lcpc_host;

// ---------------------------------------------------------------- internal helpers
namespace {
lcpc_status make_rs_encoding(int fid, size_t n_per_row, size_t n_cols, size_t nco, size_t ndt,
                             lcpc_encoding **out) {
  if (!out) return fail(LCPC_ERR_INVALID_ARG, "null out");
  if (!valid_field(fid)) return fail(LCPC_ERR_INVALID_ARG, "unknown field");
  if (!field_gpu_supported(fid)) return fail(LCPC_ERR_UNSUPPORTED, "field has no gfx950 kernels");
  // LigeroEncodingRho::_dims_ok (lib.rs:114-118) is asserted by new_from_dims
  if (!(n_per_row < n_cols) || !n_cols || (n_cols & (n_cols - 1)))
    return fail(LCPC_ERR_INVALID_ARG, "dims_ok failed: need n_per_row < n_cols, n_cols = 2^k");
  const int log_n = (int)log2_np2(n_cols);
  const FieldInfo fi = field_info(fid);
  if (log_n > fi.s) return fail(LCPC_FFT_TOO_BIG, "FFTError::TooBig: log2(n_cols) > S");
  lcpc_status st;
  Device *dev = get_device(g_device, &st);
  if (!dev) return st;
  auto e = std::make_unique<lcpc_encoding>();
  e->fid = fid;
  e->n_per_row = n_per_row;
  e->n_cols = n_cols;
  e->n_col_opens = nco;
  e->n_degree_tests = ndt;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  hipError_t he = ntt_plan_init(e->plan, fid, log_n, false, lease.s);
  if (he == hipErrorInvalidValue) return fail(LCPC_ERR_UNSUPPORTED, "n_cols beyond the supported NTT range");
  HIP_TRY(he);
  HIP_TRY(hipStreamSynchronize(lease.s));
  e->dev = dev;
  *out = e.release();
  return LCPC_OK;
}

// SdigEncodingS::_new_from_np1 / new_from_dims (lcpc-brakedown-pc/src/lib.rs:69-137) with the
// n_per_row already chosen; want_cols = 0 accepts the generated codeword length.
lcpc_status make_sdig_encoding(int fid, int code, size_t n_per_row, size_t want_cols, uint64_t seed,
                               lcpc_encoding **out) {
  if (!out) return fail(LCPC_ERR_INVALID_ARG, "null out");
  if (!valid_field(fid)) return fail(LCPC_ERR_INVALID_ARG, "unknown field");
  if (!field_gpu_supported(fid)) return fail(LCPC_ERR_UNSUPPORTED, "field has no gfx950 kernels");
  const SdigSpec *sp = sdig_spec(code);
  if (!sp) return fail(LCPC_ERR_INVALID_ARG, "SDIG code id must be 1..6");
  if (!(n_per_row > sp->blen))  // matgen::get_dims asserts n > baselen
    return fail(LCPC_ERR_INVALID_ARG, "SDIG: n_per_row must exceed the code's base length");
  if (n_per_row > 0xffffffffu) return fail(LCPC_ERR_INVALID_ARG, "SDIG: n_per_row too large");
  lcpc_status st;
  Device *dev = get_device(g_device, &st);
  if (!dev) return st;
  const FieldInfo fi = field_info(fid);
  std::vector<CsrHost> pre, post;
  if (!sdig_generate(fi.limbs, fi.num_bits, fi.p, code, n_per_row, seed, pre, post))
    return fail(LCPC_ERR_INVALID_ARG, "SDIG: matrix generation failed");
  const size_t nc = sdig_codeword_length(pre, post);
  if (want_cols && want_cols != nc)  // new_from_dims asserts n_cols == codeword_length
    return fail(LCPC_ERR_INVALID_ARG, "SDIG: n_cols does not match the code's codeword length");
  auto e = std::make_unique<lcpc_encoding>();
  e->fid = fid;
  e->kind = KIND_SDIG;
  e->code = code;
  e->seed = seed;
  e->n_per_row = n_per_row;
  e->n_cols = nc;
  e->n_col_opens = sdig_n_col_opens(code);
  e->n_degree_tests = lcpc_n_degree_tests(128, nc, fi.num_bits - 1);
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  HIP_TRY(sdig_plan_upload(e->sdig, fid, pre, post, lease.s));
  e->dev = dev;
  *out = e.release();
  return LCPC_OK;
}

// Host -> device upload of `bytes` bytes in blocks of `block` bytes on a copy stream of its own,
// each block handed to on_block(off, n) -- which queues the block's compute on `s` -- as soon as s
// has been ordered after the block's copy: the DMA of block k + 1 overlaps the kernels of block k.
// A page-locked source (hipHostMalloc / registered) is read by the DMA engine directly; a pageable
// one (lcpc_commit_new's source is the caller's &[F], lcpc-2d/src/lib.rs:651: normally pageable)
// goes through the runtime's own pageable path, block by block (measured against staging it
// through two page-locked slots of this thread: 40.5 / 40.8 against 38.9 / 40.2 GB/s at cfg3,
// profiles/r06_h2d_pageable_ab.json).  Returns with the copies queued; s is ordered after all of
// them.
struct UploadStats {
  bool pinned = false;
  size_t blocks = 0;
};
inline thread_local UploadStats t_last_upload;
// this thread's upload events (one "block landed" event per block in flight, and the
// destination's "taken" record on the consuming stream), per current device
struct UploadEvents {
  hipEvent_t e[3] = {};
  int dev = -1;
  ~UploadEvents() { reset(); }
  void reset() {
    for (hipEvent_t &x : e) {
      if (x) (void)hipEventDestroy(x);
      x = nullptr;
    }
  }
  bool ready() {
    int cur = -1;
    if (hipGetDevice(&cur) != hipSuccess) return false;
    if (cur != dev) {
      reset();
      dev = cur;
    }
    for (hipEvent_t &x : e)
      if (!x && hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) {
        x = nullptr;
        return false;
      }
    return true;
  }
};
inline thread_local UploadEvents t_upload_ev;

template <class OnBlock>
lcpc_status h2d_blocks(Device *dev, uint8_t *d_dst, const uint8_t *h_src, size_t bytes, size_t block,
                       hipStream_t s, OnBlock &&on_block) {
  t_last_upload = {};
  if (!bytes) return LCPC_OK;
  block = std::max<size_t>(block, 4096);
  t_last_upload.pinned = host_dev_ptr(h_src) != nullptr;
  if (!t_upload_ev.ready()) return fail(LCPC_ERR_DEVICE, "hipEventCreate");
  hipStream_t cs = dev->acquire_stream(POOL_BULK);
  if (!cs) return fail(LCPC_ERR_DEVICE, "no HIP stream");
  // (the copies stay queued on cs, and s waits on them: the stream goes back to the pool at once,
  // work still queued on it ordered like any pooled stream's; the events are this thread's,
  // reused only after its caller drains s)
  struct Release {
    Device *dev;
    hipStream_t cs;
    bool ordered = false;  // s waits on every copy queued so far
    ~Release() {
      // an early return may leave a copy that s never waited on: it writes a buffer the caller
      // releases with a fence on s alone, so drain it here
      if (!ordered) (void)hipStreamSynchronize(cs);
      dev->release_stream(cs, POOL_BULK);
    }
  } rel{dev, cs};
  // d_dst was taken from the pool on s (a reused block's fence wait is queued there): the copy
  // stream writes it only after s has passed that point
  HIP_TRY(hipEventRecord(t_upload_ev.e[2], s));
  HIP_TRY(hipStreamWaitEvent(cs, t_upload_ev.e[2], 0));
  size_t k = 0;
  for (size_t off = 0; off < bytes; off += block, k++) {
    const size_t n = std::min(block, bytes - off);
    hipEvent_t landed = t_upload_ev.e[k & 1];
    rel.ordered = false;
    HIP_TRY(hipMemcpyAsync(d_dst + off, h_src + off, n, hipMemcpyHostToDevice, cs));
    HIP_TRY(hipEventRecord(landed, cs));
    HIP_TRY(hipStreamWaitEvent(s, landed, 0));
    rel.ordered = true;
    lcpc_status st = on_block(off, n);
    if (st) return st;
  }
  t_last_upload.blocks = k;
  return LCPC_OK;
}

// upload block: about 8 MiB, whole rows of `row_bytes` (at least one)
inline size_t upload_block(size_t row_bytes) {
  const size_t target = (size_t)8 << 20;
  return std::max<size_t>(1, target / std::max<size_t>(row_bytes, 1)) * row_bytes;
}

// src_bytes != 0: d_src is a device proof-of-storage file image of src_bytes bytes, 7 per
// WriteableFt63 element (len = ceil(src_bytes / 7)), packed as DataField::from_byte_vec does
// (fields/data_field.rs:38-46) -- at the PoS default dims straight into the one-pass encode
// eval_left / eval_out (n_rows / n_cols elements, host): also u^T Enc(M) over the new codeword
// (lcpc_online.rs:454-484, as lcpc_pos_eval_encoded), fused into the leaf hashing's pass over
// the codeword where the leaf kernel can carry it (leaf_eval_fusable), else one more pass after it
lcpc_status commit_device(const lcpc_encoding *e, const void *d_src, bool src_is_host, size_t len,
                          lcpc_commit **out, size_t src_bytes = 0, const uint64_t *eval_left = nullptr,
                          uint64_t *eval_out = nullptr) {
  prof::HostScope hs_total("host_commit_total");
  if (!e || !out) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  const size_t np = e->n_per_row, nc = e->n_cols;
  const size_t n_rows = (len + np - 1) / np;  // LcEncoding::get_dims
  // commit's assertions (lcpc-2d/src/lib.rs:659-661) -> invalid argument
  if (len == 0 || n_rows * np < len || (n_rows - 1) * np >= len)
    return fail(LCPC_ERR_INVALID_ARG, "commit: coefficient count incompatible with dims");
  if (encoding_dims_ok(e, np, nc) != LCPC_OK) return fail(LCPC_ERR_INVALID_ARG, "commit: dims_ok");
  const size_t np2 = next_pow2(nc);
  if (np2 == 0) return fail(LCPC_PROVER_TOO_BIG, "n_cols too large");
  Device *dev = e->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  hipStream_t s = lease.s;
  const int fid = e->fid, wb = field_bytes(fid);
  DBuf packed;  // bytes off the fused path: the element image (at function scope: no block-exit drain)
  DBuf image;   // a host file image's device copy
  const uint8_t *src_b = nullptr;
  bool host_image = false;  // src_b fills block by block from the host (encoded as blocks land)
  if (src_bytes) {
    if (fid != LCPC_FT63) return fail(LCPC_ERR_INVALID_ARG, "file image: WriteableFt63 only");
    const bool fuse = e->kind != KIND_SDIG && ntt_row1_bytes(e->plan) && ntt_rows_pos_bytes_ok(e->plan, np);
    if (src_is_host) {
      const size_t padded = (src_bytes + 15) / 16 * 16 + 16;
      HIP_TRY(image.alloc(dev, padded));
      // (only the padding past the file: the upload writes the rest on its own stream)
      HIP_TRY(hipMemsetAsync(image.as<uint8_t>() + src_bytes, 0, padded - src_bytes, s));
      if (fuse) {
        src_b = image.as<uint8_t>();
        host_image = true;
      } else {
        lcpc_status st = h2d_blocks(dev, image.as<uint8_t>(), (const uint8_t *)d_src, src_bytes, (size_t)8 << 20, s,
                                    [](size_t, size_t) { return LCPC_OK; });
        if (st) return st;
        d_src = image.p;
      }
      src_is_host = false;
    } else if (fuse && !((uintptr_t)d_src & 15)) {
      src_b = (const uint8_t *)d_src;
    }
    if (!src_b) {
      HIP_TRY(packed.alloc(dev, len * 8));
      HIP_TRY(pos_pack7((const uint8_t *)d_src, src_bytes, packed.as<uint64_t>(), s));
      d_src = packed.p;
    }
  }
  auto c = std::make_unique<lcpc_commit>();
  c->fid = fid;
  c->dev = dev;
  c->n_rows = n_rows;
  c->n_cols = nc;
  c->n_per_row = np;
  c->n_hashes = 2 * np2 - 1;
  // coeffs, zero padded to n_rows * n_per_row (:665, :669-674); comm row r = encode(coeffs
  // row r || zeros) (:677-682)
  HIP_TRY(c->coeffs.alloc(dev, n_rows * np * wb));
  HIP_TRY(c->comm.alloc(dev, n_rows * nc * wb));
  uint8_t *cf = c->coeffs.as<uint8_t>();
  uint8_t *cm = c->comm.as<uint8_t>();
  DBuf tmp;  // (SDIG scratch; at function scope, so that no block exit drains the stream)
  if (e->kind == KIND_SDIG) {
    // element-major codeword [n_cols][n_rows]: the message part is the coefficient matrix
    // transposed, the SDIG levels fill the rest, and each leaf is a contiguous column.  The
    // codeword is held canonical: the transpose writes canonical values, and every level is a
    // sum of Montgomery products by Montgomery constants (SpMM values, Reed-Solomon points), so
    // canonical inputs give canonical outputs -- the leaves then hash it without a per-element
    // conversion, as the Ligero codeword (opened columns convert back, as there)
    c->col_major = true;
    c->canon = true;
    if (src_is_host) {
      lcpc_status st = h2d_blocks(dev, cf, (const uint8_t *)d_src, len * wb, (size_t)8 << 20, s,
                                  [](size_t, size_t) { return LCPC_OK; });
      if (st) return st;
      if (n_rows * np > len) HIP_TRY(hipMemsetAsync(cf + len * wb, 0, (n_rows * np - len) * wb, s));
      HIP_TRY(transpose_elems(fid, (const uint32_t *)cf, n_rows, np, np, np, (uint32_t *)cm, n_rows, s,
                              TR_FROM_MONT));
    } else {
      // one pass over the caller's coefficients writes both the transposed message part and
      // the commitment's zero-padded row-major copy (no separate device-to-device copy)
      HIP_TRY(transpose_elems(fid, (const uint32_t *)d_src, n_rows, np, np, np, (uint32_t *)cm, n_rows, s,
                              TR_FROM_MONT, nullptr, len, (uint32_t *)cf, np));
    }
    HIP_TRY(tmp.alloc(dev, e->sdig.tmp_elems * n_rows * wb));
    HIP_TRY(sdig_encode_cm(e->sdig, (uint32_t *)cm, n_rows, tmp.as<uint32_t>(), s));
  } else if (src_is_host) {
    // the caller's rows land in the commitment's coefficient matrix block by block, each block's
    // rows encoded as soon as they are there (the copy of the next block overlaps)
    c->canon = true;
    const size_t row_b = np * wb, total = len * wb;
    lcpc_status st = h2d_blocks(dev, cf, (const uint8_t *)d_src, total, upload_block(row_b), s,
                                [&](size_t off, size_t n) -> lcpc_status {
      const bool last = off + n == total;
      const size_t r0 = off / row_b, r1 = last ? n_rows : (off + n) / row_b;
      if (last && n_rows * np > len) HIP_TRY(hipMemsetAsync(cf + total, 0, (n_rows * np - len) * wb, s));
      if (r1 > r0)
        HIP_TRY(ntt_rows(e->plan, (const uint32_t *)(cf + r0 * row_b), np, np, (uint32_t *)(cm + r0 * nc * wb), nc,
                         r1 - r0, s, nullptr, 0, true));
      return LCPC_OK;
    });
    if (st) return st;
  } else if (host_image) {
    // a host file image: uploaded block by block (whole rows of 7 n_per_row bytes), each block's
    // rows unpacked and encoded by the one-pass kernel as soon as they are there
    c->canon = true;
    const size_t row_b = 7 * np;
    lcpc_status st = h2d_blocks(dev, image.as<uint8_t>(), (const uint8_t *)d_src, src_bytes, upload_block(row_b), s,
                                [&](size_t off, size_t n) -> lcpc_status {
      const bool last = off + n == src_bytes;
      const size_t r0 = off / row_b, r1 = last ? n_rows : (off + n) / row_b;
      if (r1 > r0)
        HIP_TRY(ntt_rows_pos_bytes(e->plan, src_b + r0 * row_b, src_bytes - r0 * row_b,
                                   (uint32_t *)(cm + r0 * nc * wb), nc, r1 - r0, s, (uint32_t *)(cf + r0 * np * wb), np));
      return LCPC_OK;
    });
    if (st) return st;
  } else if (src_b) {
    // the file image, unpacked inside the encode, which also writes the coefficient matrix
    c->canon = true;
    HIP_TRY(ntt_rows_pos_bytes(e->plan, src_b, src_bytes, (uint32_t *)cm, nc, n_rows, s, (uint32_t *)cf, np));
  } else {
    // full rows are encoded straight from the caller's buffer; the first NTT pass writes the
    // commitment's own coefficient copy as it reads them (no separate D2D copy)
    c->canon = true;
    const size_t full = len / np, tail = len - full * np;
    HIP_TRY(ntt_rows(e->plan, (const uint32_t *)d_src, np, np, (uint32_t *)cm, nc, full, s,
                     (uint32_t *)cf, np, true));
    if (tail) {
      uint8_t *last = cf + full * np * wb;
      HIP_TRY(hipMemcpyAsync(last, (const uint8_t *)d_src + full * np * wb, tail * wb,
                             hipMemcpyDeviceToDevice, s));
      HIP_TRY(hipMemsetAsync(last + tail * wb, 0, (np - tail) * wb, s));
      HIP_TRY(ntt_rows(e->plan, (const uint32_t *)last, np, np, (uint32_t *)(cm + full * nc * wb),
                       nc, 1, s, nullptr, 0, true));
    }
  }
  // Merkle tree (:685-697, merkleize :720-734); leaves past n_cols stay zero digests
  HIP_TRY(c->hashes.alloc(dev, c->n_hashes * 32));
  if (np2 > nc) HIP_TRY(hipMemsetAsync(c->hashes.as<uint8_t>() + nc * 32, 0, (np2 - nc) * 32, s));
  DBuf scratch, dleft, partials, dsum;
  HIP_TRY(scratch.alloc(dev, leaf_hash_scratch_bytes(fid, n_rows, nc)));
  const bool eval = eval_left && eval_out;
  const bool fused = eval && !c->col_major && c->canon && leaf_eval_fusable(fid);
  if (eval) {
    if (c->col_major) return fail(LCPC_ERR_UNSUPPORTED, "u^T Enc(M): row-major (Ligero) commitments only");
    lcpc_status st = upload(dev, dleft, eval_left, n_rows * wb);
    if (st) return st;
    HIP_TRY(dsum.alloc(dev, nc * wb));
  }
  if (c->col_major) {
    HIP_TRY(leaf_hashes_cols(fid, c->comm.as<uint32_t>(), n_rows, nc, c->hashes.as<uint8_t>(), scratch.p, s,
                             c->canon));
  } else if (fused) {
    // the leaf pass also sums each (chunk, column)'s share of u^T Enc(M); the shares fold below
    const size_t n_chunks = leaf_n_chunks(fid, n_rows);
    HIP_TRY(partials.alloc(dev, n_chunks * nc * wb));
    HIP_TRY(leaf_hashes_eval(fid, c->comm.as<uint32_t>(), n_rows, nc, nc, c->hashes.as<uint8_t>(), scratch.p,
                             dleft.as<uint32_t>(), partials.as<uint32_t>(), s));
    HIP_TRY(collapse_fold_rows(fid, partials.as<uint32_t>(), n_chunks, nc, dsum.as<uint32_t>(), s));
  } else {
    HIP_TRY(leaf_hashes(fid, c->comm.as<uint32_t>(), n_rows, nc, nc, c->hashes.as<uint8_t>(), scratch.p, s,
                        c->canon));
    if (eval) {
      DBuf cs;
      HIP_TRY(cs.alloc(dev, collapse_scratch_bytes(fid, n_rows, nc, 1)));
      HIP_TRY(collapse_rows(fid, c->comm.as<uint32_t>(), n_rows, nc, dleft.as<uint32_t>(), 1, dsum.as<uint32_t>(),
                            cs.p, s));
    }
  }
  HIP_TRY(merkle_tree(c->hashes.as<uint8_t>(), np2, s));
  if (eval) {
    // over a canonical matrix the Montgomery products come out as canonical values
    if (c->canon) HIP_TRY(convert(fid, dsum.as<uint32_t>(), dsum.as<uint32_t>(), nc, true, s));
    HIP_TRY(d2h_staged(eval_out, dsum.p, nc * wb, s));
  }
  uint8_t *h_root = (uint8_t *)t_pin[PIN_OUTER].get(32);
  if (!h_root) return fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
  HIP_TRY(d2h(h_root, c->hashes.as<uint8_t>() + (c->n_hashes - 1) * 32, 32, s));
  HIP_TRY(hipStreamSynchronize(s));
  // this commit's work is complete: its scratch needs no fence
  tmp.settle();
  scratch.settle();
  packed.settle();
  image.settle();
  std::memcpy(c->root, h_root, 32);
  c->coeffs.settle();
  c->comm.settle();
  c->hashes.settle();
  *out = c.release();
  return LCPC_OK;
}
}  // namespace

// ================================================================= C ABI
extern "C" {

int lcpc_abi_version(void) { return LCPC_ABI_VERSION; }
const char *lcpc_last_error(void) { return g_err.c_str(); }

lcpc_status lcpc_set_device(int device) {
  if (device < 0) return fail(LCPC_ERR_INVALID_ARG, "negative device");
  g_device = device;
  lcpc_status st;
  return get_device(device, &st) ? LCPC_OK : st;
}

int lcpc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

lcpc_status lcpc_field_random(lcpc_field f, uint64_t seed, uint64_t *out, size_t n) {
  // F::random(&mut ChaCha20Rng::seed_from_u64(seed)) x n (ff_derive; rand_core 0.6)
  if (!valid_field(f) || (!out && n)) return fail(LCPC_ERR_INVALID_ARG, "field / out");
  ChaCha20Rng rng = ChaCha20Rng::seed_from_u64(seed);
  const FieldInfo fi = field_info(f);
  field_random(rng, fi.limbs, fi.num_bits, fi.p, out, n);
  return LCPC_OK;
}

int lcpc_field_limbs(lcpc_field f) { return valid_field(f) ? field_info(f).limbs : 0; }
int lcpc_field_num_bits(lcpc_field f) { return valid_field(f) ? field_info(f).num_bits : 0; }

size_t lcpc_log2(size_t v) { return log2_np2(v); }

size_t lcpc_n_degree_tests(size_t lambda, size_t len, size_t flog2) {
  const size_t den = flog2 - log2_np2(len);
  return (lambda + den - 1) / den;
}

size_t lcpc_ligero_n_col_opens(size_t rho_num, size_t rho_den) {
  const double rho = (double)rho_num / (double)rho_den;
  const double den = std::log2((1.0 + rho) / 2.0);
  return (size_t)std::ceil(-128.0 / den);
}

lcpc_status lcpc_ligero_get_dims(lcpc_field f, size_t rn, size_t rd, size_t len, size_t *nr,
                                 size_t *npr, size_t *nc) {
  // LigeroEncodingRho::_get_dims (lcpc-ligero-pc/src/lib.rs:70-112)
  if (!valid_field(f) || !(rn < rd) || len == 0 || !nr || !npr || !nc)
    return fail(LCPC_ERR_INVALID_ARG, "get_dims arguments");
  const FieldInfo fi = field_info(f);
  const size_t flog2 = fi.num_bits - 1;
  const double rho = (double)rn / (double)rd;
  const size_t nco = lcpc_ligero_n_col_opens(rn, rd);
  const double lncf = (double)(nco * len);
  const double ndt = (double)lcpc_n_degree_tests(128, (size_t)std::ceil(std::sqrt(lncf) / rho), flog2);
  const size_t nc1 = next_pow2((size_t)std::ceil(std::sqrt(lncf / ndt) / rho));
  if (fi.s < 63 && nc1 > ((size_t)1 << fi.s)) return fail(LCPC_PROVER_TOO_BIG, "n_cols > 2^S");
  const size_t np1 = nc1 * rn / rd;
  if (np1 == 0) return fail(LCPC_ERR_INVALID_ARG, "degenerate dims");
  const size_t nr1 = (len + np1 - 1) / np1;
  const size_t nd1 = lcpc_n_degree_tests(128, nc1, flog2);
  const size_t nc2 = nc1 / 2, np2 = np1 / 2;
  if (np2 == 0)  // the reference divides by np2 = 0 here and panics
    return fail(LCPC_ERR_INVALID_ARG, "get_dims: len too small (n_per_row / 2 == 0)");
  const size_t nr2 = (len + np2 - 1) / np2;
  const size_t nd2 = lcpc_n_degree_tests(128, nc2, flog2);
  const size_t sz1 = nco * nr1 + (1 + nd1) * np1;
  const size_t sz2 = nco * nr2 + (1 + nd2) * np2;
  if (sz1 < sz2) {
    *nr = nr1; *npr = np1; *nc = nc1;
  } else {
    *nr = nr2; *npr = np2; *nc = nc2;
  }
  return LCPC_OK;
}

lcpc_status lcpc_ligero_new_from_dims(lcpc_field f, size_t rn, size_t rd, size_t n_per_row,
                                      size_t n_cols, lcpc_encoding **out) {
  if (!valid_field(f) || !(rn < rd)) return fail(LCPC_ERR_INVALID_ARG, "rate");
  const size_t nco = lcpc_ligero_n_col_opens(rn, rd);
  const size_t ndt = lcpc_n_degree_tests(128, n_cols, field_info(f).num_bits - 1);
  return make_rs_encoding(f, n_per_row, n_cols, nco, ndt, out);
}

lcpc_status lcpc_ligero_new(lcpc_field f, size_t rn, size_t rd, size_t len, lcpc_encoding **out) {
  size_t nr, np, nc;
  lcpc_status st = lcpc_ligero_get_dims(f, rn, rd, len, &nr, &np, &nc);
  if (st != LCPC_OK) return st;
  return lcpc_ligero_new_from_dims(f, rn, rd, np, nc, out);
}

lcpc_status lcpc_ligero_new_ml(lcpc_field f, size_t rn, size_t rd, size_t n_vars,
                               lcpc_encoding **out) {
  // LigeroEncodingRho::new_ml (lib.rs:130-136)
  if (n_vars >= 63) return fail(LCPC_ERR_INVALID_ARG, "n_vars");
  const size_t n_mon = (size_t)1 << n_vars;
  size_t nr, np, nc;
  lcpc_status st = lcpc_ligero_get_dims(f, rn, rd, n_mon, &nr, &np, &nc);
  if (st != LCPC_OK) return st;
  if ((nr & (nr - 1)) || (np & (np - 1)) || nr * np != n_mon)
    return fail(LCPC_ERR_INVALID_ARG, "new_ml: dims are not powers of two");
  return lcpc_ligero_new_from_dims(f, rn, rd, np, nc, out);
}

lcpc_status lcpc_rs_encoding_new(lcpc_field f, size_t n_per_row, size_t n_cols, size_t nco,
                                 size_t ndt, lcpc_encoding **out) {
  return make_rs_encoding(f, n_per_row, n_cols, nco, ndt, out);
}

size_t lcpc_sdig_n_col_opens(int code) { return sdig_n_col_opens(code); }

lcpc_status lcpc_sdig_get_n_per_row(lcpc_field f, int code, size_t len, size_t *n_per_row) {
  if (!valid_field(f) || !sdig_spec(code) || !n_per_row || len == 0)
    return fail(LCPC_ERR_INVALID_ARG, "sdig_get_n_per_row arguments");
  *n_per_row = sdig_new_np(code, field_info(f).num_bits, len);
  return LCPC_OK;
}

lcpc_status lcpc_sdig_new(lcpc_field f, int code, size_t len, uint64_t seed, lcpc_encoding **out) {
  // SdigEncodingS::new (lcpc-brakedown-pc/src/lib.rs:103-110)
  if (!valid_field(f) || !sdig_spec(code) || len == 0)
    return fail(LCPC_ERR_INVALID_ARG, "sdig_new arguments");
  return make_sdig_encoding(f, code, sdig_new_np(code, field_info(f).num_bits, len), 0, seed, out);
}

lcpc_status lcpc_sdig_new_ml(lcpc_field f, int code, size_t n_vars, uint64_t seed,
                             lcpc_encoding **out) {
  // SdigEncodingS::new_ml (lib.rs:114-123)
  if (!valid_field(f) || !sdig_spec(code) || n_vars >= 63)
    return fail(LCPC_ERR_INVALID_ARG, "sdig_new_ml arguments");
  return make_sdig_encoding(f, code, sdig_new_ml_np(code, field_info(f).num_bits, n_vars), 0, seed, out);
}

lcpc_status lcpc_sdig_new_from_dims(lcpc_field f, int code, size_t n_per_row, size_t n_cols,
                                    uint64_t seed, lcpc_encoding **out) {
  // SdigEncodingS::new_from_dims (lib.rs:126-137)
  if (n_cols == 0) return fail(LCPC_ERR_INVALID_ARG, "n_cols");
  return make_sdig_encoding(f, code, n_per_row, n_cols, seed, out);
}

int lcpc_encoding_kind(const lcpc_encoding *e) { return e->kind; }

size_t lcpc_encoding_matrix_nnz(const lcpc_encoding *e) {
  size_t nnz = 0;
  for (const auto &m : e->sdig.pre) nnz += m.nnz;
  for (const auto &m : e->sdig.post) nnz += m.nnz;
  return nnz;
}

void lcpc_encoding_free(lcpc_encoding *e) { delete e; }
lcpc_field lcpc_encoding_field(const lcpc_encoding *e) { return (lcpc_field)e->fid; }

void lcpc_encoding_get_dims(const lcpc_encoding *e, size_t len, size_t *nr, size_t *np, size_t *nc) {
  *nr = (len + e->n_per_row - 1) / e->n_per_row;
  *np = e->n_per_row;
  *nc = e->n_cols;
}
int lcpc_encoding_dims_ok(const lcpc_encoding *e, size_t np, size_t nc) {
  return encoding_dims_ok(e, np, nc) == LCPC_OK;
}
size_t lcpc_encoding_n_col_opens(const lcpc_encoding *e) { return e->n_col_opens; }
size_t lcpc_encoding_n_degree_tests(const lcpc_encoding *e) { return e->n_degree_tests; }
size_t lcpc_encoding_n_per_row(const lcpc_encoding *e) { return e->n_per_row; }
size_t lcpc_encoding_n_cols(const lcpc_encoding *e) { return e->n_cols; }
lcpc_status lcpc_encoding_set_row_kernel(lcpc_encoding *e, int kernel) {
  if (!e || kernel < LCPC_ROW_KERNEL_AUTO || kernel > LCPC_ROW_KERNEL_ONEPASS)
    return fail(LCPC_ERR_INVALID_ARG, "row kernel");
  e->plan.row_kernel = kernel;
  return LCPC_OK;
}

lcpc_status lcpc_reserve(const lcpc_encoding *e, size_t len, size_t count) {
  if (!e || !len) return fail(LCPC_ERR_INVALID_ARG, "reserve arguments");
  Device *dev = e->dev;
  HIP_TRY(hipSetDevice(dev->id));
  const size_t wb = (size_t)field_bytes(e->fid), np = e->n_per_row, nc = e->n_cols, nco = e->n_col_opens;
  const size_t nr = (len + np - 1) / np, np2 = next_pow2(nc), pl = log2_np2(nc);
  // the blocks commit_device and lcpc_prove ask of the pool, by size
  std::vector<size_t> sizes = {nr * np * wb, nr * nc * wb, (2 * np2 - 1) * 32,
                               leaf_hash_scratch_bytes(e->fid, nr, nc), 2 * nr * wb, 2 * np * wb,
                               collapse_scratch_bytes(e->fid, nr, np, 2), np * wb, nco * 8, nco * nr * wb,
                               nco * pl * 32};
  if (e->kind == KIND_SDIG) sizes.push_back(e->sdig.tmp_elems * nr * wb);
  std::vector<void *> blocks;
  lcpc_status st = LCPC_OK;
  for (size_t k = 0; k < count && !st; k++)
    for (size_t b : sizes) {
      void *p = nullptr;
      if (dev->alloc(&p, b) != hipSuccess) {
        st = fail(LCPC_ERR_OUT_OF_MEMORY, "reserve: device pool");
        break;
      }
      blocks.push_back(p);
    }
  for (void *p : blocks) dev->release(p);
  std::vector<hipStream_t> lo, hi;
  for (size_t k = 0; k < count; k++) {
    lo.push_back(dev->acquire_stream(POOL_BULK));
    hi.push_back(dev->acquire_stream(POOL_PROVER));
  }
  for (hipStream_t s : lo)
    if (s) dev->release_stream(s, POOL_BULK);
  for (hipStream_t s : hi)
    if (s) dev->release_stream(s, POOL_PROVER);
  // the page-locked blocks of `count` proofs (p_random, p_eval, columns, paths)
  const size_t ndt = e->n_degree_tests;
  std::vector<void *> pins;
  for (size_t k = 0; k < count; k++)
    for (size_t b : {ndt * np * wb, np * wb, nco * nr * wb, nco * pl * 32})
      if (b >= PinnedHeap::MIN)
        if (void *p = g_pinned_heap.get(b)) pins.push_back(p);
  for (void *p : pins) g_pinned_heap.put(p);
  return st;
}

lcpc_status lcpc_prepare_thread(const lcpc_encoding *e, size_t n_rows) {
  if (!e) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  // the sizes lcpc_prove asks of each thread-local slot
  const size_t wb = (size_t)field_bytes(e->fid), np = e->n_per_row, nco = e->n_col_opens;
  const size_t ndt = e->n_degree_tests, pl = log2_np2(e->n_cols);
  (void)ndt;
  (void)pl;
  // (p_random, p_eval and the columns land in the proof's own page-locked vectors)
  const size_t want[PIN_N] = {2 * np * wb, 1, 1, 1, nco * 8, n_rows * wb, n_rows * wb, 1, 1};
  for (int i = 0; i < PIN_N; i++)
    if (!t_pin[i].get(std::max<size_t>(1, want[i]))) return fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
  t_eval_repr.reserve(np * wb);
  return LCPC_OK;
}

static lcpc_status encode_rows_chunk(const lcpc_encoding *e, uint64_t *rows, size_t n_rows, size_t stride) {
  Device *dev = e->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  const int wb = field_bytes(e->fid);
  DBuf d;
  HIP_TRY(d.alloc(dev, n_rows * e->n_cols * wb));
  HIP_TRY(hipMemcpy2DAsync(d.p, e->n_cols * wb, rows, stride * wb, e->n_cols * wb, n_rows,
                           hipMemcpyHostToDevice, lease.s));
  lcpc_status st = encode_rows_any(e, d.as<uint32_t>(), e->n_cols, e->n_cols, d.as<uint32_t>(),
                                   e->n_cols, n_rows, lease.s);
  if (st) return st;
  HIP_TRY(hipMemcpy2DAsync(rows, stride * wb, d.p, e->n_cols * wb, e->n_cols * wb, n_rows,
                           hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_encode_rows(const lcpc_encoding *e, uint64_t *rows, size_t n_rows, size_t stride) {
  if (!e || (!rows && n_rows)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (stride < e->n_cols) return fail(LCPC_ERR_INVALID_ARG, "row stride < n_cols");
  if (n_rows == 0) return LCPC_OK;
  // The rows are the caller's pageable memory, so one stream's H2D -> encode -> D2H runs
  // serially.  Chunks of ~16 MiB on up to 8 host threads (each with its own leased stream)
  // overlap one chunk's copies with another's kernels, as concurrent per-row callers do
  // (tools/encode_rows_bench.py at the cfg3 row size: 62 GB/s of H2D + D2H for 16 callers
  // against 52 GB/s for the whole batch on one stream).
  const size_t row_bytes = e->n_cols * (size_t)field_bytes(e->fid);
  const size_t chunk = std::max<size_t>(1, ((size_t)16 << 20) / row_bytes);
  const size_t n_chunks = (n_rows + chunk - 1) / chunk;
  if (n_chunks < 2) return encode_rows_chunk(e, rows, n_rows, stride);
  const size_t T = std::min<size_t>(8, n_chunks);
  std::atomic<size_t> next{0};
  std::mutex mu;
  lcpc_status first = LCPC_OK;
  std::string msg;
  auto work = [&] {
    for (size_t k; (k = next.fetch_add(1)) < n_chunks;) {
      const size_t r0 = k * chunk, nr = std::min(chunk, n_rows - r0);
      const lcpc_status st = encode_rows_chunk(e, rows + r0 * stride * (size_t)field_info(e->fid).limbs, nr, stride);
      if (st) {
        std::lock_guard<std::mutex> lk(mu);
        if (!first) first = st, msg = g_err;
        next.store(n_chunks);
      }
    }
  };
  std::vector<std::thread> th;
  for (size_t i = 1; i < T; i++) th.emplace_back(work);
  work();
  for (auto &t : th) t.join();
  return first ? fail(first, msg) : LCPC_OK;
}

lcpc_status lcpc_encode(const lcpc_encoding *e, uint64_t *inp, size_t len) {
  // fffft::fft_io_pc: the slice length must equal the precomputation length
  if (!e || !inp) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (e->kind == KIND_SDIG && len != e->n_cols)  // encode.rs:42 asserts the codeword length
    return fail(LCPC_ERR_INVALID_ARG, "SDIG encode: slice length != codeword length");
  if (len != e->n_cols) {
    if (len == 0 || (len & (len - 1))) return fail(LCPC_FFT_NOT_POWER_OF_TWO, "FFTError::NotPowerOfTwo");
    if ((int)log2_np2(len) > field_info(e->fid).s) return fail(LCPC_FFT_TOO_BIG, "FFTError::TooBig");
    return fail(LCPC_FFT_WRONG_SIZE_PRECOMP, "FFTError::WrongSizePrecomp");
  }
  return lcpc_encode_rows(e, inp, 1, len);
}

lcpc_status lcpc_encode_rows_device(const lcpc_encoding *e, const void *d_src, size_t src_stride,
                                    size_t n_valid, void *d_dst, size_t dst_stride, size_t n_rows,
                                    void *stream) {
  if (!e || !d_dst || (!d_src && n_valid)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (n_valid > e->n_cols || dst_stride < e->n_cols)
    return fail(LCPC_ERR_INVALID_ARG, "encode_rows_device: bad lengths");
  Device *dev = e->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  hipStream_t s = stream ? (hipStream_t)stream : lease.s;
  StreamAs on_s(s);  // (SDIG's scratch codeword: taken and fenced on the stream that uses it)
  lcpc_status st = encode_rows_any(e, (const uint32_t *)d_src, src_stride, n_valid,
                                   (uint32_t *)d_dst, dst_stride, n_rows, s);
  if (st) return st;
  if (!stream) HIP_TRY(hipStreamSynchronize(s));
  return LCPC_OK;
}

// ---------------------------------------------------------------- commit
lcpc_status lcpc_commit_new(const lcpc_encoding *e, const uint64_t *coeffs, size_t len,
                            lcpc_commit **out) {
  if (!coeffs) return fail(LCPC_ERR_INVALID_ARG, "null coeffs");
  return commit_device(e, coeffs, true, len, out);
}

lcpc_status lcpc_commit_new_device(const lcpc_encoding *e, const void *d_coeffs, size_t len,
                                   lcpc_commit **out) {
  if (!d_coeffs) return fail(LCPC_ERR_INVALID_ARG, "null coeffs");
  return commit_device(e, d_coeffs, false, len, out);
}

lcpc_status lcpc_pos_commit_bytes_device(const lcpc_encoding *e, const void *d_bytes, size_t n_bytes,
                                         lcpc_commit **out) {
  if (!d_bytes || !n_bytes) return fail(LCPC_ERR_INVALID_ARG, "null or empty file image");
  if ((uintptr_t)d_bytes & 7) return fail(LCPC_ERR_INVALID_ARG, "device file image must be 8-byte aligned");
  return commit_device(e, d_bytes, false, (n_bytes + 6) / 7, out, n_bytes);  // 7 data bytes per element
}

lcpc_status lcpc_pos_commit_eval_bytes_device(const lcpc_encoding *e, const void *d_bytes, size_t n_bytes,
                                              const uint64_t *left, size_t n_rows, uint64_t *eval_out,
                                              lcpc_commit **out) {
  if (!e || !d_bytes || !n_bytes || !left || !eval_out) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if ((uintptr_t)d_bytes & 7) return fail(LCPC_ERR_INVALID_ARG, "device file image must be 8-byte aligned");
  const size_t len = (n_bytes + 6) / 7;
  if (!e->n_per_row || n_rows != (len + e->n_per_row - 1) / e->n_per_row)
    return fail(LCPC_ERR_INVALID_ARG, "left vector length != the commitment's n_rows");
  return commit_device(e, d_bytes, false, len, out, n_bytes, left, eval_out);
}

lcpc_status lcpc_pos_commit_bytes(const lcpc_encoding *e, const uint8_t *bytes, size_t n_bytes, lcpc_commit **out) {
  if (!bytes || !n_bytes) return fail(LCPC_ERR_INVALID_ARG, "null or empty file image");
  return commit_device(e, bytes, true, (n_bytes + 6) / 7, out, n_bytes);
}

int lcpc_last_upload_pinned(void) { return t_last_upload.pinned ? 1 : 0; }

void lcpc_commit_free(lcpc_commit *c) {
  if (!c) return;
  Device *dev = c->dev;
  Lease lease(dev);
  (void)hipSetDevice(dev->id);
  (void)hipStreamSynchronize(lease.s);
  delete c;
}

lcpc_status lcpc_commit_get_root(const lcpc_commit *c, uint8_t root[32]) {
  std::memcpy(root, c->root, 32);
  return LCPC_OK;
}
size_t lcpc_commit_n_rows(const lcpc_commit *c) { return c->n_rows; }
size_t lcpc_commit_n_cols(const lcpc_commit *c) { return c->n_cols; }
size_t lcpc_commit_n_per_row(const lcpc_commit *c) { return c->n_per_row; }
size_t lcpc_commit_n_hashes(const lcpc_commit *c) { return c->n_hashes; }
const void *lcpc_commit_device_comm(const lcpc_commit *c) { return c->comm.p; }
const void *lcpc_commit_device_coeffs(const lcpc_commit *c) { return c->coeffs.p; }

static lcpc_status copy_out(const lcpc_commit *c, void *dst, const void *src, size_t bytes) {
  Lease lease(c->dev);
  HIP_TRY(hipSetDevice(c->dev->id));
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}
lcpc_status lcpc_commit_copy_comm(const lcpc_commit *c, uint64_t *out) {
  const size_t bytes = c->n_rows * c->n_cols * field_bytes(c->fid);
  if (c->canon && !c->col_major) {  // canonical on the device -> the reference's Montgomery words
    Lease lease(c->dev);
    HIP_TRY(hipSetDevice(c->dev->id));
    DBuf mm;
    HIP_TRY(mm.alloc(c->dev, bytes));
    HIP_TRY(convert(c->fid, c->comm.as<uint32_t>(), mm.as<uint32_t>(), c->n_rows * c->n_cols, true, lease.s));
    HIP_TRY(hipMemcpyAsync(out, mm.p, bytes, hipMemcpyDeviceToHost, lease.s));
    HIP_TRY(hipStreamSynchronize(lease.s));
    return LCPC_OK;
  }
  if (!c->col_major) return copy_out(c, out, c->comm.p, bytes);
  // element-major on the device -> the reference's row-major Vec<F>
  Lease lease(c->dev);
  HIP_TRY(hipSetDevice(c->dev->id));
  DBuf rm;
  HIP_TRY(rm.alloc(c->dev, bytes));
  HIP_TRY(transpose_elems(c->fid, c->comm.as<uint32_t>(), c->n_cols, c->n_rows, c->n_rows, c->n_rows,
                          rm.as<uint32_t>(), c->n_cols, lease.s));
  if (c->canon) HIP_TRY(convert(c->fid, rm.as<uint32_t>(), rm.as<uint32_t>(), c->n_rows * c->n_cols, true, lease.s));
  HIP_TRY(hipMemcpyAsync(out, rm.p, bytes, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}
int lcpc_commit_col_major(const lcpc_commit *c) { return c->col_major ? 1 : 0; }
int lcpc_commit_comm_canonical(const lcpc_commit *c) { return c->canon ? 1 : 0; }
lcpc_status lcpc_commit_copy_coeffs(const lcpc_commit *c, uint64_t *out) {
  return copy_out(c, out, c->coeffs.p, c->n_rows * c->n_per_row * field_bytes(c->fid));
}
lcpc_status lcpc_commit_copy_hashes(const lcpc_commit *c, uint8_t *out) {
  return copy_out(c, out, c->hashes.p, c->n_hashes * 32);
}

lcpc_status lcpc_commit_from_parts(lcpc_field f, size_t n_rows, size_t n_cols, size_t n_per_row,
                                   const uint64_t *comm, const uint64_t *coeffs, const uint8_t *hashes,
                                   size_t n_hashes, lcpc_commit **out) {
  // LcCommit's Deserialize (WrappedLcCommit::unwrap, lcpc-2d/src/lib.rs:193-229): the fields as
  // given (row-major Montgomery comm and coeffs, the hashes in commit order, root last), loaded
  // into HBM so that prove / open_column run on them.  The reference takes any lengths and fails
  // later (check_comm, or a panic in open_column); here the lengths must be the ones commit
  // produces, else LCPC_ERR_INVALID_ARG.
  if (!out || (!comm && n_rows * n_cols) || (!coeffs && n_rows * n_per_row) || !hashes)
    return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (!valid_field(f) || !field_gpu_supported(f)) return fail(LCPC_ERR_UNSUPPORTED, "field");
  if (!n_rows || !n_cols || n_per_row > n_cols || n_hashes != 2 * next_pow2(n_cols) - 1)
    return fail(LCPC_ERR_INVALID_ARG, "commitment parts of inconsistent sizes");
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  auto c = std::make_unique<lcpc_commit>();
  c->fid = f;
  c->dev = dev;
  c->n_rows = n_rows;
  c->n_cols = n_cols;
  c->n_per_row = n_per_row;
  c->n_hashes = n_hashes;
  const size_t wb = field_bytes(f);
  if ((st = upload(dev, c->comm, comm, n_rows * n_cols * wb))) return st;
  if ((st = upload(dev, c->coeffs, coeffs, n_rows * n_per_row * wb))) return st;
  if ((st = upload(dev, c->hashes, hashes, n_hashes * 32))) return st;
  std::memcpy(c->root, hashes + (n_hashes - 1) * 32, 32);
  HIP_TRY(hipStreamSynchronize(lease.s));
  for (auto *b : {&c->comm, &c->coeffs, &c->hashes}) b->settle();
  *out = c.release();
  return LCPC_OK;
}

lcpc_status lcpc_check_comm(const lcpc_commit *c, const lcpc_encoding *e) {
  // check_comm (lcpc-2d/src/lib.rs:703-718); buffer sizes hold by construction
  if (!c || !e) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  const bool hashlen = c->n_hashes != 2 * next_pow2(c->n_cols) - 1;
  if (hashlen || encoding_dims_ok(e, c->n_per_row, c->n_cols) != LCPC_OK || c->fid != e->fid)
    return fail(LCPC_PROVER_COMMIT, "ProverError::Commit");
  return LCPC_OK;
}

lcpc_status lcpc_open_column(const lcpc_commit *c, size_t column, uint64_t *col_out,
                             uint8_t *path_out) {
  // open_column (lcpc-2d/src/lib.rs:818-855)
  if (!c) return fail(LCPC_ERR_INVALID_ARG, "null commit");
  if (column >= c->n_cols) return fail(LCPC_PROVER_COLUMN_NUMBER, "ProverError::ColumnNumber");
  Device *dev = c->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  const uint64_t idx = column;
  const size_t path_len = log2_np2(c->n_cols);
  DBuf didx, dcol, dpath;
  lcpc_status st = upload(dev, didx, &idx, 8);
  if (st) return st;
  const int wb = field_bytes(c->fid);
  HIP_TRY(dcol.alloc(dev, c->n_rows * wb));
  HIP_TRY(dpath.alloc(dev, path_len * 32));
  HIP_TRY(gather_columns(c->fid, c->comm.as<uint32_t>(), c->n_rows, c->n_cols, didx.as<uint64_t>(), 1,
                         dcol.as<uint32_t>(), lease.s, c->col_major, c->canon));
  HIP_TRY(gather_paths(c->hashes.as<uint8_t>(), c->n_hashes, didx.as<uint64_t>(), 1, path_len,
                       dpath.as<uint8_t>(), lease.s));
  if (col_out) HIP_TRY(hipMemcpyAsync(col_out, dcol.p, c->n_rows * wb, hipMemcpyDeviceToHost, lease.s));
  if (path_out && path_len)
    HIP_TRY(hipMemcpyAsync(path_out, dpath.p, path_len * 32, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

// ---------------------------------------------------------------- transcript
lcpc_transcript *lcpc_transcript_new(const uint8_t *label, size_t n) {
  return new lcpc_transcript(label, n);
}
lcpc_transcript *lcpc_transcript_from_ops(const lcpc_transcript_ops *ops) {
  if (!ops || !ops->append_message || !ops->challenge_bytes) {
    fail(LCPC_ERR_INVALID_ARG, "transcript ops need append_message and challenge_bytes");
    return nullptr;
  }
  return new lcpc_transcript(*ops);
}
int lcpc_transcript_status(const lcpc_transcript *t) { return t ? t->cb_status : 0; }
lcpc_transcript *lcpc_transcript_clone(const lcpc_transcript *t) {
  if (!t) return nullptr;
  if (t->external) {  // the caller's state lives on its side of the boundary
    fail(LCPC_ERR_UNSUPPORTED, "a caller-owned (ops) transcript cannot be cloned here; clone it on the caller's side");
    return nullptr;
  }
  return new lcpc_transcript(*t);
}
void lcpc_transcript_free(lcpc_transcript *t) { delete t; }
void lcpc_transcript_append_message(lcpc_transcript *t, const uint8_t *l, size_t ln,
                                    const uint8_t *m, size_t mn) {
  t->append_message(l, ln, m, mn);
}
void lcpc_transcript_append_messages(lcpc_transcript *t, const uint8_t *l, size_t ln, const uint8_t *msgs,
                                     size_t msg_len, size_t n_msgs) {
  t->append_messages(l, ln, msgs, msg_len, n_msgs);
}
void lcpc_transcript_challenge_bytes(lcpc_transcript *t, const uint8_t *l, size_t ln, uint8_t *d,
                                     size_t n) {
  t->challenge_bytes(l, ln, d, n);
}

// ---------------------------------------------------------------- prove
lcpc_status lcpc_prove(const lcpc_commit *c, const uint64_t *outer, size_t outer_len,
                       const lcpc_encoding *e, lcpc_transcript *tr, lcpc_proof **out) {
  // prove (lcpc-2d/src/lib.rs:1034-1123)
  prof::HostScope hs_total("host_prove_total");
  if (!c || !e || !tr || !out) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  lcpc_status st = lcpc_check_comm(c, e);
  if (st) return st;
  if (outer_len != c->n_rows || (!outer && outer_len))
    return fail(LCPC_PROVER_OUTER_TENSOR, "ProverError::OuterTensor");
  Device *dev = c->dev;
  Lease lease(dev, POOL_PROVER);
  HIP_TRY(hipSetDevice(dev->id));
  hipStream_t s = lease.s;
  const int fid = c->fid, wb = field_bytes(fid), limbs = wb / 8;
  const size_t nr = c->n_rows, np = c->n_per_row, ndt = e->n_degree_tests, nco = e->n_col_opens;
  auto p = std::make_unique<lcpc_proof>();
  p->fid = fid;
  p->n_cols = c->n_cols;
  p->n_per_row = np;
  p->n_rows = nr;
  p->ndt = ndt;
  p->nco = nco;
  p->path_len = log2_np2(c->n_cols);

  // the proof's own vectors are page-locked (pinned_vector): results land there by DMA
  p->p_random.resize(ndt * np * limbs);
  p->p_eval.resize(np * limbs);
  uint8_t *h_prand = (uint8_t *)p->p_random.data();
  uint8_t *h_peval = (uint8_t *)p->p_eval.data();
  uint8_t *h_tens = (uint8_t *)t_pin[PIN_TENSOR].get(nr * wb);
  uint8_t *h_outer = (uint8_t *)t_pin[PIN_OUTER].get(nr * wb);
  if (!h_tens || !h_outer) return fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
  std::memcpy(h_outer, outer, nr * wb);

  // tensors on device: [t_i | outer] -- the evaluation tensor rides along with the first
  // degree test so the coefficient matrix is read once for both (results are independent).
  DBuf dtens, dres, scratch;
  HIP_TRY(dtens.alloc(dev, 2 * nr * wb));
  HIP_TRY(dres.alloc(dev, 2 * np * wb));
  HIP_TRY(scratch.alloc(dev, collapse_scratch_bytes(fid, nr, np, 2)));
  HIP_TRY(h2d(dtens.as<uint8_t>() + nr * wb, h_outer, nr * wb, s));
  std::vector<uint64_t> tensor;
  const uint8_t *repr = nullptr;
  bool eval_done = false;
  // the evaluation's repr bytes, converted in the first round's GPU round trip (its absorb comes
  // after the last degree test's): one round trip fewer on the proof's serial path
  std::vector<uint8_t> &eval_repr = t_eval_repr;
  bool eval_repr_ready = false;
  for (size_t i = 0; i < ndt; i++) {
    {
      prof::HostScope hs("host_prove_round_issue");
      challenge_tensor(*tr, fid, nr, tensor);
      if ((st = transcript_status(tr))) return st;
      std::memcpy(h_tens, tensor.data(), nr * wb);
      HIP_TRY(h2d(dtens.p, h_tens, nr * wb, s));
      const int nt = eval_done ? 1 : 2;
      HIP_TRY(collapse_rows(fid, c->coeffs.as<uint32_t>(), nr, np, dtens.as<uint32_t>(), nt,
                            dres.as<uint32_t>(), scratch.p, s));
      HIP_TRY(d2h(h_prand + i * np * wb, dres.p, np * wb, s));
      if (!eval_done) {
        HIP_TRY(d2h(h_peval, dres.as<uint8_t>() + np * wb, np * wb, s));
        eval_done = true;
      }
    }
    const bool with_eval = i == 0;  // round 0 also holds the evaluation (dres[np, 2 np))
    {
      prof::HostScope hs("host_prove_gpu_wait");
      st = to_repr_host(dev, fid, dres.as<uint32_t>(), with_eval ? 2 * np : np, &repr);  // syncs the stream
    }
    if (st) return st;
    if (with_eval) {
      eval_repr.assign(repr + np * wb, repr + 2 * np * wb);
      eval_repr_ready = true;
    }
    {
      prof::HostScope hs("host_prove_transcript");
      tr->append_messages(LABEL_PR, 6, repr, wb, np);
    }
    if ((st = transcript_status(tr))) return st;
  }
  const uint32_t *d_eval = dres.as<uint32_t>() + np * limbs * 2;  // second collapse output
  if (!eval_done) {
    HIP_TRY(collapse_rows(fid, c->coeffs.as<uint32_t>(), nr, np, dtens.as<uint32_t>() + nr * limbs * 2, 1,
                          dres.as<uint32_t>(), scratch.p, s));
    HIP_TRY(d2h(h_peval, dres.p, np * wb, s));
    d_eval = dres.as<uint32_t>();
  }
  if (eval_repr_ready) {
    repr = eval_repr.data();
  } else {
    prof::HostScope hs("host_prove_gpu_wait");
    st = to_repr_host(dev, fid, d_eval, np, &repr);
  }
  if (st) return st;
  {
    prof::HostScope hs("host_prove_transcript");
    tr->append_messages(LABEL_PE, 6, repr, wb, np);
  }

  // columns (:1101-1115)
  challenge_columns(*tr, c->n_cols, nco, p->col_idx);
  if ((st = transcript_status(tr))) return st;
  p->cols.resize(nco * nr * limbs);
  p->paths.resize(nco * p->path_len * 32);
  uint8_t *h_cols = (uint8_t *)p->cols.data();
  uint8_t *h_paths = p->paths.data();
  uint8_t *h_idx = (uint8_t *)t_pin[PIN_PATHS].get(std::max<size_t>(1, nco * 8));
  if (!h_idx) return fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
  std::memcpy(h_idx, p->col_idx.data(), nco * 8);
  DBuf didx, dcols, dpaths;
  HIP_TRY(didx.alloc(dev, nco * 8));
  if (nco) HIP_TRY(h2d(didx.p, h_idx, nco * 8, s));
  HIP_TRY(dcols.alloc(dev, nco * nr * wb));
  HIP_TRY(dpaths.alloc(dev, nco * p->path_len * 32));
  HIP_TRY(gather_columns(fid, c->comm.as<uint32_t>(), nr, c->n_cols, didx.as<uint64_t>(), nco,
                         dcols.as<uint32_t>(), s, c->col_major, c->canon));
  HIP_TRY(gather_paths(c->hashes.as<uint8_t>(), c->n_hashes, didx.as<uint64_t>(), nco, p->path_len,
                       dpaths.as<uint8_t>(), s));
  if (nco) {
    HIP_TRY(d2h(h_cols, dcols.p, nco * nr * wb, s));
    if (p->path_len)
      HIP_TRY(d2h(h_paths, dpaths.p, nco * p->path_len * 32, s));
  }
  {
    prof::HostScope hs("host_prove_cols_wait");
    HIP_TRY(hipStreamSynchronize(s));
  }
  *out = p.release();
  return LCPC_OK;
}

void lcpc_proof_free(lcpc_proof *p) { delete p; }
size_t lcpc_proof_n_cols(const lcpc_proof *p) { return p->n_cols; }
size_t lcpc_proof_n_per_row(const lcpc_proof *p) { return p->n_per_row; }
size_t lcpc_proof_n_rows(const lcpc_proof *p) { return p->n_rows; }
size_t lcpc_proof_n_degree_tests(const lcpc_proof *p) { return p->ndt; }
size_t lcpc_proof_n_col_opens(const lcpc_proof *p) { return p->nco; }
size_t lcpc_proof_path_len(const lcpc_proof *p) { return p->path_len; }
lcpc_field lcpc_proof_field(const lcpc_proof *p) { return (lcpc_field)p->fid; }

lcpc_status lcpc_proof_copy_p_eval(const lcpc_proof *p, uint64_t *out) {
  std::memcpy(out, p->p_eval.data(), p->p_eval.size() * 8);
  return LCPC_OK;
}
lcpc_status lcpc_proof_copy_p_random(const lcpc_proof *p, size_t i, uint64_t *out) {
  if (i >= p->ndt) return fail(LCPC_ERR_INVALID_ARG, "degree test index");
  const size_t n = p->n_per_row * (field_bytes(p->fid) / 8);
  std::memcpy(out, p->p_random.data() + i * n, n * 8);
  return LCPC_OK;
}
lcpc_status lcpc_proof_copy_column(const lcpc_proof *p, size_t k, uint64_t *col, uint8_t *path) {
  if (k >= p->nco) return fail(LCPC_ERR_INVALID_ARG, "column index");
  const size_t n = p->n_rows * (field_bytes(p->fid) / 8);
  if (col) std::memcpy(col, p->cols.data() + k * n, n * 8);
  if (path && p->path_len) std::memcpy(path, p->paths.data() + k * p->path_len * 32, p->path_len * 32);
  return LCPC_OK;
}

lcpc_status lcpc_proof_from_parts(lcpc_field f, size_t n_cols, size_t n_per_row, size_t n_rows,
                                  size_t ndt, size_t nco, size_t path_len, const uint64_t *p_eval,
                                  const uint64_t *p_random, const uint64_t *cols,
                                  const uint8_t *paths, lcpc_proof **out) {
  if (!valid_field(f) || !out) return fail(LCPC_ERR_INVALID_ARG, "field / out");
  auto p = std::make_unique<lcpc_proof>();
  const size_t limbs = field_info(f).limbs;
  p->fid = f;
  p->n_cols = n_cols;
  p->n_per_row = n_per_row;
  p->n_rows = n_rows;
  p->ndt = ndt;
  p->nco = nco;
  p->path_len = path_len;
  p->p_eval.assign(p_eval, p_eval + n_per_row * limbs);
  if (ndt) p->p_random.assign(p_random, p_random + ndt * n_per_row * limbs);
  if (nco) p->cols.assign(cols, cols + nco * n_rows * limbs);
  if (nco && path_len) p->paths.assign(paths, paths + nco * path_len * 32);
  *out = p.release();
  return LCPC_OK;
}

// ---------------------------------------------------------------- verify
lcpc_status lcpc_verify(const uint8_t root[32], const uint64_t *outer, size_t outer_len,
                        const uint64_t *inner, size_t inner_len, const lcpc_proof *p,
                        const lcpc_encoding *e, lcpc_transcript *tr, uint64_t *eval_out) {
  // verify (lcpc-2d/src/lib.rs:862-982)
  if (!root || !p || !e || !tr) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  const size_t nco = e->n_col_opens;
  if (nco != p->nco || nco == 0) return fail(LCPC_VERIFIER_NUM_COL_OPENS, "VerifierError::NumColOpens");
  const size_t nr = p->n_rows, nc = p->n_cols, np = p->n_per_row;
  if (inner_len != np) return fail(LCPC_VERIFIER_INNER_TENSOR, "VerifierError::InnerTensor");
  if (outer_len != nr) return fail(LCPC_VERIFIER_OUTER_TENSOR, "VerifierError::OuterTensor");
  if (encoding_dims_ok(e, np, nc) != LCPC_OK || p->fid != e->fid)
    return fail(LCPC_VERIFIER_ENCODING_DIMS, "VerifierError::EncodingDims");
  const size_t ndt = e->n_degree_tests;
  if (p->ndt != ndt) return fail(LCPC_VERIFIER_ENCODING_DIMS, "proof has a different number of degree tests");
  const int fid = e->fid, wb = field_bytes(fid), limbs = wb / 8;
  Device *dev = e->dev;
  Lease lease(dev, POOL_HIGH);
  HIP_TRY(hipSetDevice(dev->id));
  hipStream_t s = lease.s;

  // device copies: tensors [ndt | outer] (n_rows each), encodings [ndt + 1][n_cols]
  DBuf dtens, denc, dvec, didx, dcols, dpaths, dleaves, dflags, dpflags, scratch, dinner, dout, droot;
  HIP_TRY(dtens.alloc(dev, (ndt + 1) * nr * wb));
  HIP_TRY(denc.alloc(dev, (ndt + 1) * nc * wb));
  HIP_TRY(hipMemcpyAsync(dtens.as<uint8_t>() + ndt * nr * wb, outer, nr * wb, hipMemcpyHostToDevice, s));
  std::vector<uint64_t> tensor;
  const uint8_t *repr = nullptr;
  lcpc_status st;
  for (size_t i = 0; i < ndt; i++) {
    challenge_tensor(*tr, fid, nr, tensor);
    HIP_TRY(hipMemcpyAsync(dtens.as<uint8_t>() + i * nr * wb, tensor.data(), nr * wb,
                           hipMemcpyHostToDevice, s));
    st = upload(dev, dvec, p->p_random.data() + i * np * limbs, np * wb);
    if (st) return st;
    st = encode_rows_any(e, dvec.as<uint32_t>(), np, np, denc.as<uint32_t>() + i * nc * limbs * 2, nc, 1, s);
    if (st) return st;
    st = to_repr_host(dev, fid, dvec.as<uint32_t>(), np, &repr);
    if (st) return st;
    tr->append_messages(LABEL_PR, 6, repr, wb, np);
    if ((st = transcript_status(tr))) return st;
  }
  st = upload(dev, dvec, p->p_eval.data(), np * wb);
  if (st) return st;
  st = to_repr_host(dev, fid, dvec.as<uint32_t>(), np, &repr);
  if (st) return st;
  tr->append_messages(LABEL_PE, 6, repr, wb, np);
  std::vector<uint64_t> idx;
  challenge_columns(*tr, nc, nco, idx);
  if ((st = transcript_status(tr))) return st;
  st = encode_rows_any(e, dvec.as<uint32_t>(), np, np, denc.as<uint32_t>() + ndt * nc * limbs * 2, nc, 1, s);
  if (st) return st;

  // per-column checks (:953-974)
  st = upload(dev, didx, idx.data(), nco * 8);
  if (st) return st;
  st = upload(dev, dcols, p->cols.data(), nco * nr * wb);
  if (st) return st;
  st = upload(dev, dpaths, p->paths.data(), nco * p->path_len * 32);
  if (st) return st;
  st = upload(dev, droot, root, 32);
  if (st) return st;
  HIP_TRY(dflags.alloc(dev, nco * (ndt + 1) * 4));
  HIP_TRY(dpflags.alloc(dev, nco * 4));
  HIP_TRY(dleaves.alloc(dev, nco * 32));
  HIP_TRY(scratch.alloc(dev, leaf_hash_scratch_bytes(fid, nr, nco)));
  HIP_TRY(column_checks(fid, dcols.as<uint32_t>(), nco, nr, dtens.as<uint32_t>(), (int)(ndt + 1),
                        denc.as<uint32_t>(), nc, didx.as<uint64_t>(), dflags.as<uint32_t>(), s));
  HIP_TRY(leaf_hashes_cols(fid, dcols.as<uint32_t>(), nr, nco, dleaves.as<uint8_t>(), scratch.p, s));
  HIP_TRY(path_checks(dleaves.as<uint8_t>(), dpaths.as<uint8_t>(), nco, p->path_len,
                      didx.as<uint64_t>(), droot.as<uint8_t>(), dpflags.as<uint32_t>(), s));
  std::vector<uint32_t> flags(nco * (ndt + 1)), pflags(nco);
  HIP_TRY(hipMemcpyAsync(flags.data(), dflags.p, flags.size() * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(pflags.data(), dpflags.p, pflags.size() * 4, hipMemcpyDeviceToHost, s));
  // final inner product (:977-981)
  st = upload(dev, dinner, inner, np * wb);
  if (st) return st;
  HIP_TRY(dout.alloc(dev, wb));
  HIP_TRY(dot(fid, dinner.as<uint32_t>(), dvec.as<uint32_t>(), np, dout.as<uint32_t>(), nullptr, s));
  std::vector<uint64_t> ev(limbs);
  HIP_TRY(hipMemcpyAsync(ev.data(), dout.p, wb, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (size_t k = 0; k < nco; k++) {
    bool rnd = true;
    for (size_t i = 0; i < ndt; i++) rnd &= flags[k * (ndt + 1) + i] != 0;
    const bool ev_ok = flags[k * (ndt + 1) + ndt] != 0;
    if (!rnd) return fail(LCPC_VERIFIER_COLUMN_DEGREE, "VerifierError::ColumnDegree");
    if (!ev_ok) return fail(LCPC_VERIFIER_COLUMN_EVAL, "VerifierError::ColumnEval");
    if (!pflags[k]) return fail(LCPC_VERIFIER_COLUMN_PATH, "VerifierError::ColumnPath");
  }
  if (eval_out) std::memcpy(eval_out, ev.data(), wb);
  return LCPC_OK;
}

// prove / verify over a caller-owned transcript for the length of one call (the reference's
// `&mut Transcript` argument, lcpc-2d/src/lib.rs:319-326, 547-556)
lcpc_status lcpc_prove_ops(const lcpc_commit *c, const uint64_t *outer, size_t outer_len, const lcpc_encoding *e,
                           const lcpc_transcript_ops *ops, lcpc_proof **out) {
  if (!ops || !ops->append_message || !ops->challenge_bytes)
    return fail(LCPC_ERR_INVALID_ARG, "transcript ops need append_message and challenge_bytes");
  lcpc_transcript tr(*ops);
  return lcpc_prove(c, outer, outer_len, e, &tr, out);
}
lcpc_status lcpc_verify_ops(const uint8_t root[32], const uint64_t *outer, size_t outer_len, const uint64_t *inner,
                            size_t inner_len, const lcpc_proof *p, const lcpc_encoding *e,
                            const lcpc_transcript_ops *ops, uint64_t *eval_out) {
  if (!ops || !ops->append_message || !ops->challenge_bytes)
    return fail(LCPC_ERR_INVALID_ARG, "transcript ops need append_message and challenge_bytes");
  lcpc_transcript tr(*ops);
  return lcpc_verify(root, outer, outer_len, inner, inner_len, p, e, &tr, eval_out);
}

// ---------------------------------------------------------------- free functions

lcpc_status lcpc_collapse_columns(lcpc_field f, const uint64_t *coeffs, const uint64_t *tensor,
                                  uint64_t *poly, size_t n_rows, size_t n_per_row) {
  if (!valid_field(f)) return fail(LCPC_ERR_INVALID_ARG, "field");
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  const int wb = field_bytes(f);
  DBuf dc, dt, dp, scratch;
  if ((st = upload(dev, dc, coeffs, n_rows * n_per_row * wb))) return st;
  if ((st = upload(dev, dt, tensor, n_rows * wb))) return st;
  HIP_TRY(dp.alloc(dev, n_per_row * wb));
  HIP_TRY(scratch.alloc(dev, collapse_scratch_bytes(f, n_rows, n_per_row, 1)));
  HIP_TRY(collapse_rows(f, dc.as<uint32_t>(), n_rows, n_per_row, dt.as<uint32_t>(), 1, dp.as<uint32_t>(),
                        scratch.p, lease.s));
  HIP_TRY(hipMemcpyAsync(poly, dp.p, n_per_row * wb, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_merkle_tree(const uint8_t *ins, size_t n_ins, uint8_t *outs) {
  if (!n_ins || (n_ins & (n_ins - 1))) return fail(LCPC_ERR_INVALID_ARG, "ins.len() must be 2^k");
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf d;
  HIP_TRY(d.alloc(dev, (2 * n_ins - 1) * 32));
  HIP_TRY(hipMemcpyAsync(d.p, ins, n_ins * 32, hipMemcpyHostToDevice, lease.s));
  HIP_TRY(merkle_tree(d.as<uint8_t>(), n_ins, lease.s));
  if (n_ins > 1)
    HIP_TRY(hipMemcpyAsync(outs, d.as<uint8_t>() + n_ins * 32, (n_ins - 1) * 32, hipMemcpyDeviceToHost,
                           lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_hash_columns(lcpc_field f, const uint64_t *comm, size_t n_rows, size_t n_cols,
                              uint8_t *out) {
  if (!valid_field(f) || !field_gpu_supported(f)) return fail(LCPC_ERR_UNSUPPORTED, "field");
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  const int wb = field_bytes(f);
  DBuf dm, dl, scratch;
  if ((st = upload(dev, dm, comm, n_rows * n_cols * wb))) return st;
  HIP_TRY(dl.alloc(dev, n_cols * 32));
  HIP_TRY(scratch.alloc(dev, leaf_hash_scratch_bytes(f, n_rows, n_cols)));
  HIP_TRY(leaf_hashes(f, dm.as<uint32_t>(), n_rows, n_cols, n_cols, dl.as<uint8_t>(), scratch.p, lease.s));
  HIP_TRY(hipMemcpyAsync(out, dl.p, n_cols * 32, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

int lcpc_verify_column_path(lcpc_field f, const uint64_t *col, size_t n_rows, const uint8_t *path,
                            size_t path_len, size_t col_num, const uint8_t root[32]) {
  if (!valid_field(f) || !field_gpu_supported(f)) return 0;
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return 0;
  Lease lease(dev);
  if (hipSetDevice(dev->id) != hipSuccess) return 0;
  const int wb = field_bytes(f);
  DBuf dc, dp, di, dr, dl, dfl, scratch;
  const uint64_t idx = col_num;
  if (upload(dev, dc, col, n_rows * wb) || upload(dev, dp, path, path_len * 32) ||
      upload(dev, di, &idx, 8) || upload(dev, dr, root, 32))
    return 0;
  if (dl.alloc(dev, 32) || dfl.alloc(dev, 4) || scratch.alloc(dev, leaf_hash_scratch_bytes(f, n_rows, 1)))
    return 0;
  if (leaf_hashes_cols(f, dc.as<uint32_t>(), n_rows, 1, dl.as<uint8_t>(), scratch.p, lease.s) ||
      path_checks(dl.as<uint8_t>(), dp.as<uint8_t>(), 1, path_len, di.as<uint64_t>(), dr.as<uint8_t>(),
                  dfl.as<uint32_t>(), lease.s))
    return 0;
  uint32_t flag = 0;
  if (hipMemcpyAsync(&flag, dfl.p, 4, hipMemcpyDeviceToHost, lease.s) ||
      hipStreamSynchronize(lease.s))
    return 0;
  return flag != 0;
}

lcpc_status lcpc_hash_field_columns(lcpc_field f, const uint64_t *cols, size_t n_rows, size_t n_cols,
                                    uint8_t *out) {
  // hash_field_vec_to_digest / hash_column_to_digest (lcpc_online.rs:431-452) for n_cols
  // columns given one after another ([n_cols][n_rows])
  if (!valid_field(f) || !field_gpu_supported(f)) return fail(LCPC_ERR_UNSUPPORTED, "field");
  if ((!cols && n_rows * n_cols) || (!out && n_cols)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (!n_cols) return LCPC_OK;
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  const int wb = field_bytes(f);
  DBuf dm, dl, scratch;
  if ((st = upload(dev, dm, cols, n_rows * n_cols * wb))) return st;
  HIP_TRY(dl.alloc(dev, n_cols * 32));
  HIP_TRY(scratch.alloc(dev, leaf_hash_scratch_bytes(f, n_rows, n_cols)));
  HIP_TRY(leaf_hashes_cols(f, dm.as<uint32_t>(), n_rows, n_cols, dl.as<uint8_t>(), scratch.p, lease.s));
  HIP_TRY(hipMemcpyAsync(out, dl.p, n_cols * 32, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_verify_leaf_paths(const uint8_t *leaves, const uint8_t *paths, size_t n,
                                   size_t path_len, const uint64_t *idx, const uint8_t root[32],
                                   uint8_t *ok) {
  // client_online_verify_column_paths_without_full_columns (lcpc_online.rs:280-318): ok[k] = 1
  // iff the path of leaf digest k at column idx[k] hashes up to root
  if ((!leaves || !paths || !idx || !ok) && n) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (!root) return fail(LCPC_ERR_INVALID_ARG, "null root");
  if (!n) return LCPC_OK;
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf dl, dp, di, dr, dfl;
  if ((st = upload(dev, dl, leaves, n * 32)) || (st = upload(dev, dp, paths, n * path_len * 32 + 32)) ||
      (st = upload(dev, di, idx, n * 8)) || (st = upload(dev, dr, root, 32)))
    return st;
  HIP_TRY(dfl.alloc(dev, n * 4));
  HIP_TRY(path_checks(dl.as<uint8_t>(), dp.as<uint8_t>(), n, path_len, di.as<uint64_t>(), dr.as<uint8_t>(),
                      dfl.as<uint32_t>(), lease.s));
  std::vector<uint32_t> fl(n);
  HIP_TRY(hipMemcpyAsync(fl.data(), dfl.p, n * 4, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  for (size_t k = 0; k < n; k++) ok[k] = fl[k] ? 1 : 0;
  return LCPC_OK;
}

lcpc_status lcpc_verify_column_values(lcpc_field f, const uint64_t *cols, size_t n, size_t n_rows,
                                      const uint64_t *tensor, const uint64_t *values, size_t n_values,
                                      const uint64_t *idx, uint8_t *ok) {
  // verify_column_value (lcpc-2d/src/lib.rs:1014-1030) for n columns at once, also
  // verify_proper_partial_polynomial_evaluation's check (lcpc_online.rs:487-516): ok[k] = 1 iff
  // sum_r tensor[r] cols[k][r] == values[idx[k]]
  if (!valid_field(f) || !field_gpu_supported(f)) return fail(LCPC_ERR_UNSUPPORTED, "field");
  if ((!cols || !idx || !ok) && n) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if ((!tensor && n_rows) || (!values && n_values)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  for (size_t k = 0; k < n; k++)
    if (idx[k] >= n_values) return fail(LCPC_ERR_INVALID_ARG, "value index out of range");
  if (!n) return LCPC_OK;
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  const int wb = field_bytes(f);
  DBuf dc, dt, dv, di, dfl;
  if ((st = upload(dev, dc, cols, n * n_rows * wb)) || (st = upload(dev, dt, tensor, n_rows * wb)) ||
      (st = upload(dev, dv, values, n_values * wb)) || (st = upload(dev, di, idx, n * 8)))
    return st;
  HIP_TRY(dfl.alloc(dev, n * 4));
  HIP_TRY(column_checks(f, dc.as<uint32_t>(), n, n_rows, dt.as<uint32_t>(), 1, dv.as<uint32_t>(), n_values,
                        di.as<uint64_t>(), dfl.as<uint32_t>(), lease.s));
  std::vector<uint32_t> fl(n);
  HIP_TRY(hipMemcpyAsync(fl.data(), dfl.p, n * 4, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  for (size_t k = 0; k < n; k++) ok[k] = fl[k] ? 1 : 0;
  return LCPC_OK;
}

int lcpc_verify_column_value(lcpc_field f, const uint64_t *col, const uint64_t *tensor,
                             size_t n_rows, const uint64_t *poly_eval) {
  if (!valid_field(f)) return 0;
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return 0;
  Lease lease(dev);
  if (hipSetDevice(dev->id) != hipSuccess) return 0;
  const int wb = field_bytes(f);
  DBuf dc, dt, de, di, dfl;
  const uint64_t zero = 0;
  if (upload(dev, dc, col, n_rows * wb) || upload(dev, dt, tensor, n_rows * wb) ||
      upload(dev, de, poly_eval, wb) || upload(dev, di, &zero, 8) || dfl.alloc(dev, 4))
    return 0;
  if (column_checks(f, dc.as<uint32_t>(), 1, n_rows, dt.as<uint32_t>(), 1, de.as<uint32_t>(), 1,
                    di.as<uint64_t>(), dfl.as<uint32_t>(), lease.s))
    return 0;
  uint32_t flag = 0;
  if (hipMemcpyAsync(&flag, dfl.p, 4, hipMemcpyDeviceToHost, lease.s) ||
      hipStreamSynchronize(lease.s))
    return 0;
  return flag != 0;
}

}  // extern "C"

// ================================================================= proof-of-storage producers
namespace {

// n^-1 mod p for n = 2^log_n | p - 1, canonical: p - (p - 1) / n
void inv_pow2_canon(int fid, int log_n, uint32_t *words) {
  const FieldInfo fi = field_info(fid);
  uint64_t q[4] = {0, 0, 0, 0}, r[4] = {0, 0, 0, 0};
  for (int i = 0; i < fi.limbs; i++) q[i] = fi.p[i];
  q[0] -= 1;  // p odd: no borrow
  for (int k = 0; k < log_n; k++) {  // q >>= 1 (multi-limb)
    for (int i = 0; i < fi.limbs; i++) {
      q[i] >>= 1;
      if (i + 1 < fi.limbs) q[i] |= q[i + 1] << 63;
    }
  }
  uint64_t br = 0;
  for (int i = 0; i < fi.limbs; i++) {
    const uint64_t a = fi.p[i], b = q[i];
    const uint64_t d = a - b - br;
    br = (a < b) || (a - b < br);
    r[i] = d;
  }
  for (int i = 0; i < fi.limbs; i++) {
    words[2 * i] = (uint32_t)r[i];
    words[2 * i + 1] = (uint32_t)(r[i] >> 32);
  }
}

lcpc_status check_fft_len(int fid, size_t len) {
  if (len == 0 || (len & (len - 1))) return fail(LCPC_FFT_NOT_POWER_OF_TWO, "FFTError::NotPowerOfTwo");
  if ((int)log2_np2(len) > field_info(fid).s) return fail(LCPC_FFT_TOO_BIG, "FFTError::TooBig");
  return LCPC_OK;
}

// Encode `len` host elements with e into a temporary row-major codeword (Leaves /
// ColumnsWithoutPath requests, lcpc_online.rs:144-224): no commitment, no Merkle tree.
lcpc_status encode_matrix(const lcpc_encoding *e, const uint64_t *elems, size_t len, DBuf &comm,
                          size_t *n_rows_out, hipStream_t s) {
  const size_t np = e->n_per_row, nc = e->n_cols;
  const size_t n_rows = (len + np - 1) / np;
  const int wb = field_bytes(e->fid);
  DBuf coeffs;
  HIP_TRY(coeffs.alloc(e->dev, n_rows * np * wb));
  HIP_TRY(hipMemcpyAsync(coeffs.p, elems, len * wb, hipMemcpyHostToDevice, s));
  if (n_rows * np > len)
    HIP_TRY(hipMemsetAsync(coeffs.as<uint8_t>() + len * wb, 0, (n_rows * np - len) * wb, s));
  HIP_TRY(comm.alloc(e->dev, n_rows * nc * wb));
  lcpc_status st = encode_rows_any(e, coeffs.as<uint32_t>(), np, np, comm.as<uint32_t>(), nc, n_rows, s);
  if (st) return st;
  *n_rows_out = n_rows;
  return LCPC_OK;
}

}  // namespace

extern "C" {

lcpc_status lcpc_pos_bytes_to_field_device(const void *d_bytes, size_t n_bytes, void *d_out,
                                           void *stream) {
  if ((!d_bytes || !d_out) && n_bytes) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (((uintptr_t)d_bytes & 7) || ((uintptr_t)d_out & 7))
    return fail(LCPC_ERR_INVALID_ARG, "device buffers must be 8-byte aligned");
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  hipStream_t s = stream ? (hipStream_t)stream : lease.s;
  HIP_TRY(pos_pack7((const uint8_t *)d_bytes, n_bytes, (uint64_t *)d_out, s));
  if (!stream) HIP_TRY(hipStreamSynchronize(s));
  return LCPC_OK;
}

lcpc_status lcpc_pos_bytes_to_field(const uint8_t *bytes, size_t n_bytes, uint64_t *out,
                                    size_t *n_out) {
  if ((!bytes || !out) && n_bytes) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  const size_t n = (n_bytes + 6) / 7;
  if (n_out) *n_out = n;
  if (!n) return LCPC_OK;
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf db, de;
  if ((st = upload(dev, db, bytes, n_bytes))) return st;
  HIP_TRY(de.alloc(dev, n * 8));
  HIP_TRY(pos_pack7(db.as<uint8_t>(), n_bytes, de.as<uint64_t>(), lease.s));
  HIP_TRY(hipMemcpyAsync(out, de.p, n * 8, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_pos_field_to_bytes(const uint64_t *elems, size_t n, uint8_t *out,
                                    size_t expected_len) {
  if ((!elems && n) || (!out && expected_len)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (expected_len > 7 * n) return fail(LCPC_ERR_INVALID_ARG, "expected_len > 7 * n");
  if (!expected_len) return LCPC_OK;
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf de, db;
  if ((st = upload(dev, de, elems, n * 8))) return st;
  HIP_TRY(db.alloc(dev, expected_len));
  HIP_TRY(pos_unpack7(de.as<uint64_t>(), n, db.as<uint8_t>(), expected_len, lease.s));
  HIP_TRY(hipMemcpyAsync(out, db.p, expected_len, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

void lcpc_pos_default_dims(size_t field_len, size_t *n_per_row, size_t *n_cols, size_t *soundness) {
  // get_aspect_ratio_default_from_field_len (networking/server.rs:1139-1158): f32 sqrt
  const size_t w = (size_t)std::ceil(std::sqrt((float)field_len));
  const size_t np = (w & (w - 1)) == 0 ? w : next_pow2(w);  // fields::is_power_of_two
  const size_t nc = next_pow2(np + 1);
  // get_soundness_from_matrix_dims (:1160-1170)
  const double den = std::log2((1.0 + (double)np / (double)nc) / 2.0);
  const size_t th = (size_t)std::ceil(-128.0 / den);
  if (n_per_row) *n_per_row = np;
  if (n_cols) *n_cols = nc;
  if (soundness) *soundness = th < nc ? th : nc;
}

lcpc_status lcpc_pos_column_indices(uint64_t seed, size_t amount, size_t max_index, uint64_t *out,
                                    size_t *n_out) {
  // get_column_indicies_from_random_seed (networking/client.rs:443-456): ChaCha8Rng +
  // IteratorRandom::choose_multiple (rand 0.8 reservoir; gen_index = gen_range(0..ub as u32))
  if (!out && amount) return fail(LCPC_ERR_INVALID_ARG, "null out");
  ChaCha20Rng rng = ChaCha20Rng::seed_from_u64(seed, 8);
  size_t filled = 0;
  for (size_t i = 0; i < max_index && filled < amount; i++) out[filled++] = i;
  if (filled == amount) {
    for (size_t i = 0; amount + i < max_index; i++) {
      const size_t ub = i + 1 + amount;
      size_t k;
      if (ub <= 0xffffffffu) {
        const uint32_t range = (uint32_t)ub;
        const uint32_t zone = (range << __builtin_clz(range)) - 1;
        for (;;) {
          const uint64_t m = (uint64_t)rng.next_u32() * range;
          if ((uint32_t)m <= zone) {
            k = (size_t)(m >> 32);
            break;
          }
        }
      } else {
        const uint64_t zone = ((uint64_t)ub << __builtin_clzll((uint64_t)ub)) - 1;
        for (;;) {
          const unsigned __int128 m = (unsigned __int128)rng.next_u64() * ub;
          if ((uint64_t)m <= zone) {
            k = (size_t)(m >> 64);
            break;
          }
        }
      }
      if (k < amount) out[k] = amount + i;
    }
  }
  if (n_out) *n_out = filled;
  return LCPC_OK;
}

lcpc_status lcpc_pos_side_vectors(lcpc_field f, const uint64_t *x, size_t n_rows, size_t n_cols,
                                  uint64_t *left, uint64_t *right) {
  // form_side_vectors_for_polynomial_evaluation_from_point (lcpc_online.rs:603-627):
  // right = [1, x, ..., x^(n_cols-1)], left = [1, x^n_cols, x^(2 n_cols), ...]
  if (!valid_field(f) || !x || (!left && n_rows) || (!right && n_cols))
    return fail(LCPC_ERR_INVALID_ARG, "side vector arguments");
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  const int wb = field_bytes(f);
  DBuf dx, dl, dr;
  if ((st = upload(dev, dx, x, wb))) return st;
  HIP_TRY(dl.alloc(dev, n_rows * wb));
  HIP_TRY(dr.alloc(dev, n_cols * wb));
  HIP_TRY(powers(f, dx.as<uint32_t>(), 1, n_cols, dr.as<uint32_t>(), lease.s));
  HIP_TRY(powers(f, dx.as<uint32_t>(), (uint64_t)n_cols, n_rows, dl.as<uint32_t>(), lease.s));
  if (n_cols) HIP_TRY(hipMemcpyAsync(right, dr.p, n_cols * wb, hipMemcpyDeviceToHost, lease.s));
  if (n_rows) HIP_TRY(hipMemcpyAsync(left, dl.p, n_rows * wb, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_pos_eval_encoded(const lcpc_commit *c, const uint64_t *left, size_t n_rows,
                                  uint64_t *out) {
  // verifiable_polynomial_evaluation (lcpc_online.rs:454-484): out[j] = sum_r left[r] comm[r][j]
  if (!c || !left || !out) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (n_rows != c->n_rows) return fail(LCPC_ERR_INVALID_ARG, "left vector length != n_rows");
  if (c->col_major) return fail(LCPC_ERR_UNSUPPORTED, "row-major (Ligero) commitments only");
  Device *dev = c->dev;
  Lease lease(dev, POOL_HIGH);
  HIP_TRY(hipSetDevice(dev->id));
  const int wb = field_bytes(c->fid);
  DBuf dt, dout, scratch;
  lcpc_status st;
  if ((st = upload(dev, dt, left, n_rows * wb))) return st;
  HIP_TRY(dout.alloc(dev, c->n_cols * wb));
  HIP_TRY(scratch.alloc(dev, collapse_scratch_bytes(c->fid, n_rows, c->n_cols, 1)));
  HIP_TRY(collapse_rows(c->fid, c->comm.as<uint32_t>(), n_rows, c->n_cols, dt.as<uint32_t>(), 1,
                        dout.as<uint32_t>(), scratch.p, lease.s));
  // over a canonical matrix the Montgomery products come out as canonical values
  if (c->canon) HIP_TRY(convert(c->fid, dout.as<uint32_t>(), dout.as<uint32_t>(), c->n_cols, true, lease.s));
  HIP_TRY(d2h_staged(out, dout.p, c->n_cols * wb, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_ifft_oi_rows(lcpc_field f, uint64_t *rows, size_t n_rows, size_t len) {
  // fffft::ifft_oi on each row (decode_row, lcpc_online.rs:568-574): bit-reversed evaluations
  // in, natural-order coefficients out
  if (!valid_field(f) || (!rows && n_rows)) return fail(LCPC_ERR_INVALID_ARG, "arguments");
  if (!field_gpu_supported(f)) return fail(LCPC_ERR_UNSUPPORTED, "field has no gfx950 kernels");
  lcpc_status st = check_fft_len(f, len);
  if (st) return st;
  if (n_rows == 0) return LCPC_OK;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  const int log_n = (int)log2_np2(len);
  const int wb = field_bytes(f);
  NttPlan plan;
  hipError_t he = ntt_plan_init(plan, f, log_n, true, lease.s);
  if (he != hipSuccess) {
    ntt_plan_free(plan);
    if (he == hipErrorInvalidValue) return fail(LCPC_ERR_UNSUPPORTED, "length beyond the NTT range");
    HIP_TRY(he);
  }
  struct PlanGuard {
    NttPlan &p;
    hipStream_t s;
    ~PlanGuard() {
      (void)hipStreamSynchronize(s);
      ntt_plan_free(p);
    }
  } guard{plan, lease.s};
  DBuf a, b;
  if ((st = upload(dev, a, rows, n_rows * len * wb))) return st;
  HIP_TRY(b.alloc(dev, n_rows * len * wb));
  uint32_t inv[8] = {0};
  inv_pow2_canon(f, log_n, inv);
  // ifft_oi = reorder the evaluations to natural order (bit-reversed ones: include/
  // lcpc_fft_convention.h), DIF with the inverse root, bit-reverse back and scale by len^-1
  uint32_t *x = a.as<uint32_t>(), *y = b.as<uint32_t>();
  if (LCPC_FFT_OUTPUT_BITREV) {
    HIP_TRY(bitrev_scale(f, x, y, log_n, n_rows, nullptr, lease.s));
    std::swap(x, y);
  }
  HIP_TRY(ntt_rows(plan, x, len, len, y, len, n_rows, lease.s));
  HIP_TRY(bitrev_scale(f, y, x, log_n, n_rows, inv, lease.s));
  HIP_TRY(hipMemcpyAsync(rows, x, n_rows * len * wb, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_open_columns(const lcpc_commit *c, const uint64_t *idx, size_t n, uint64_t *cols_out,
                              uint8_t *paths_out) {
  // open_column (lcpc-2d/src/lib.rs:818-855) for n columns at once (PoS server_retreive_columns,
  // lcpc_online.rs:241-247)
  if (!c || (!idx && n)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  for (size_t k = 0; k < n; k++)
    if (idx[k] >= c->n_cols) return fail(LCPC_PROVER_COLUMN_NUMBER, "ProverError::ColumnNumber");
  if (!n) return LCPC_OK;
  Device *dev = c->dev;
  Lease lease(dev, POOL_HIGH);
  HIP_TRY(hipSetDevice(dev->id));
  const size_t path_len = log2_np2(c->n_cols);
  const int wb = field_bytes(c->fid);
  DBuf didx, dcol, dpath;
  lcpc_status st;
  if ((st = upload(dev, didx, idx, n * 8))) return st;
  HIP_TRY(dcol.alloc(dev, n * c->n_rows * wb));
  HIP_TRY(dpath.alloc(dev, n * path_len * 32 + 32));
  HIP_TRY(gather_columns(c->fid, c->comm.as<uint32_t>(), c->n_rows, c->n_cols, didx.as<uint64_t>(), n,
                         dcol.as<uint32_t>(), lease.s, c->col_major, c->canon));
  HIP_TRY(gather_paths(c->hashes.as<uint8_t>(), c->n_hashes, didx.as<uint64_t>(), n, path_len,
                       dpath.as<uint8_t>(), lease.s));
  if (cols_out) HIP_TRY(d2h_staged(cols_out, dcol.p, n * c->n_rows * wb, lease.s));
  if (paths_out && path_len)
    HIP_TRY(d2h_staged(paths_out, dpath.p, n * path_len * 32, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_pos_columns(const lcpc_encoding *e, const uint64_t *elems, size_t len,
                             const uint64_t *idx, size_t n, uint64_t *cols_out, uint8_t *leaves_out) {
  // CommitRequestType::ColumnsWithoutPath / Leaves (lcpc_online.rs:144-224): encode the file,
  // then return the requested columns and / or their BLAKE3 leaf digests -- no Merkle tree
  if (!e || !elems || len == 0 || (!idx && n)) return fail(LCPC_ERR_INVALID_ARG, "arguments");
  for (size_t k = 0; k < n; k++)
    if (idx[k] >= e->n_cols) return fail(LCPC_PROVER_COLUMN_NUMBER, "ProverError::ColumnNumber");
  Device *dev = e->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf comm, didx, dcol, dleaves, scratch;
  size_t n_rows = 0;
  lcpc_status st = encode_matrix(e, elems, len, comm, &n_rows, lease.s);
  if (st) return st;
  if (!n) return LCPC_OK;
  const int wb = field_bytes(e->fid);
  if ((st = upload(dev, didx, idx, n * 8))) return st;
  HIP_TRY(dcol.alloc(dev, n * n_rows * wb));
  HIP_TRY(gather_columns(e->fid, comm.as<uint32_t>(), n_rows, e->n_cols, didx.as<uint64_t>(), n,
                         dcol.as<uint32_t>(), lease.s));
  if (leaves_out) {
    HIP_TRY(dleaves.alloc(dev, n * 32));
    HIP_TRY(scratch.alloc(dev, leaf_hash_scratch_bytes(e->fid, n_rows, n)));
    HIP_TRY(leaf_hashes_cols(e->fid, dcol.as<uint32_t>(), n_rows, n, dleaves.as<uint8_t>(), scratch.p,
                             lease.s));
    HIP_TRY(hipMemcpyAsync(leaves_out, dleaves.p, n * 32, hipMemcpyDeviceToHost, lease.s));
  }
  if (cols_out) HIP_TRY(hipMemcpyAsync(cols_out, dcol.p, n * n_rows * wb, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

}  // extern "C"

// ================================================================= row shards (multi-GPU commit)
// One GPU's share of a Ligero commitment whose rows are split across processes:
// the shard encodes its rows, computes the BLAKE3 chunk chaining values of the leaf-message
// chunks its rows cover, its partial row combinations and its rows of opened columns.  The
// exchanges between shards (chaining values by column block, subtree roots, partial sums,
// challenge broadcasts) are the caller's (lcpc_proof_of_storage_amd/shard.py, RCCL through
// torch.distributed); together they reproduce commit / prove bit for bit.
struct lcpc_shard {
  const lcpc_encoding *e = nullptr;
  size_t row0 = 0, n_rows = 0, n_rows_total = 0;
  DBuf coeffs, comm;
};

extern "C" {

size_t lcpc_leaf_n_chunks(lcpc_field f, size_t n_rows) {
  return valid_field(f) ? leaf_n_chunks(f, n_rows) : 0;
}

size_t lcpc_leaf_chunk_first_row(lcpc_field f, size_t chunk) {
  // first row of the leaf message at or after byte 1024 * chunk (32-byte zero prefix)
  if (!valid_field(f) || chunk == 0) return 0;
  const size_t wb = (size_t)field_bytes(f);
  return (1024 * chunk - 32 + wb - 1) / wb;
}

static lcpc_status shard_new_impl(const lcpc_encoding *e, const void *coeffs, bool on_device, size_t row0,
                                  size_t n_shard_rows, size_t n_rows_total, lcpc_shard **out);

lcpc_status lcpc_shard_new(const lcpc_encoding *e, const uint64_t *coeffs, size_t row0,
                           size_t n_shard_rows, size_t n_rows_total, lcpc_shard **out) {
  return shard_new_impl(e, coeffs, false, row0, n_shard_rows, n_rows_total, out);
}

lcpc_status lcpc_shard_new_device(const lcpc_encoding *e, const void *d_coeffs, size_t row0,
                                  size_t n_shard_rows, size_t n_rows_total, lcpc_shard **out) {
  return shard_new_impl(e, d_coeffs, true, row0, n_shard_rows, n_rows_total, out);
}

static lcpc_status shard_new_impl(const lcpc_encoding *e, const void *coeffs, bool on_device, size_t row0,
                                  size_t n_shard_rows, size_t n_rows_total, lcpc_shard **out) {
  if (!e || !out || (!coeffs && n_shard_rows)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (e->kind != KIND_RS) return fail(LCPC_ERR_UNSUPPORTED, "row shards: Ligero / R-S encodings only");
  if (row0 + n_shard_rows > n_rows_total) return fail(LCPC_ERR_INVALID_ARG, "shard rows out of range");
  Device *dev = e->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  auto sh = std::make_unique<lcpc_shard>();
  sh->e = e;
  sh->row0 = row0;
  sh->n_rows = n_shard_rows;
  sh->n_rows_total = n_rows_total;
  const size_t np = e->n_per_row, nc = e->n_cols;
  const int wb = field_bytes(e->fid);
  HIP_TRY(sh->coeffs.alloc(dev, n_shard_rows * np * wb + 16));
  HIP_TRY(sh->comm.alloc(dev, n_shard_rows * nc * wb + 16));
  if (n_shard_rows && on_device) {  // encode straight from the caller's rows; pass A copies them
    HIP_TRY(ntt_rows(e->plan, (const uint32_t *)coeffs, np, np, sh->comm.as<uint32_t>(), nc, n_shard_rows,
                     lease.s, sh->coeffs.as<uint32_t>(), np, true));
  } else if (n_shard_rows) {
    HIP_TRY(hipMemcpyAsync(sh->coeffs.p, coeffs, n_shard_rows * np * wb, hipMemcpyHostToDevice, lease.s));
    HIP_TRY(ntt_rows(e->plan, sh->coeffs.as<uint32_t>(), np, np, sh->comm.as<uint32_t>(), nc, n_shard_rows,
                     lease.s, nullptr, 0, true));
  }
  HIP_TRY(hipStreamSynchronize(lease.s));
  sh->coeffs.settle();
  sh->comm.settle();
  *out = sh.release();
  return LCPC_OK;
}

void lcpc_shard_free(lcpc_shard *s) {
  if (!s) return;
  Lease lease(s->e->dev);
  (void)hipStreamSynchronize(lease.s);
  delete s;
}

lcpc_status lcpc_shard_chunk_cvs(const lcpc_shard *s, size_t chunk_lo, size_t chunk_hi,
                                 uint8_t *out) {
  if (!s || (!out && chunk_hi > chunk_lo)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  const int fid = s->e->fid;
  const size_t nc = s->e->n_cols;
  if (chunk_hi > leaf_n_chunks(fid, s->n_rows_total) || chunk_lo > chunk_hi)
    return fail(LCPC_ERR_INVALID_ARG, "chunk range");
  // every row the chunks read must be in the shard
  const size_t need_lo = lcpc_leaf_chunk_first_row((lcpc_field)fid, chunk_lo);
  const size_t need_hi = chunk_hi >= leaf_n_chunks(fid, s->n_rows_total)
                             ? s->n_rows_total
                             : lcpc_leaf_chunk_first_row((lcpc_field)fid, chunk_hi);
  if (chunk_hi > chunk_lo && (need_lo < s->row0 || need_hi > s->row0 + s->n_rows))
    return fail(LCPC_ERR_INVALID_ARG, "the shard does not hold every row of those chunks");
  if (chunk_hi == chunk_lo) return LCPC_OK;
  Device *dev = s->e->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf cvs;
  HIP_TRY(cvs.alloc(dev, (chunk_hi - chunk_lo) * nc * 32));
  HIP_TRY(leaf_chunk_cvs(fid, s->comm.as<uint32_t>(), s->row0, s->n_rows_total, nc, nc, chunk_lo, chunk_hi,
                         cvs.as<uint32_t>(), lease.s, true));
  HIP_TRY(hipMemcpyAsync(out, cvs.p, (chunk_hi - chunk_lo) * nc * 32, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_leaves_from_cvs(const uint8_t *cvs, size_t n_chunks, size_t n_cols, uint8_t *leaves) {
  if ((!cvs || !leaves) && n_cols) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (n_chunks == 0) return fail(LCPC_ERR_INVALID_ARG, "n_chunks");
  if (!n_cols) return LCPC_OK;
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf dc, dl;
  if ((st = upload(dev, dc, cvs, n_chunks * n_cols * 32))) return st;
  HIP_TRY(dl.alloc(dev, n_cols * 32));
  HIP_TRY(leaves_from_cvs(dc.as<uint32_t>(), n_cols, (int)n_chunks, dl.as<uint8_t>(), lease.s));
  HIP_TRY(hipMemcpyAsync(leaves, dl.p, n_cols * 32, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_shard_collapse(const lcpc_shard *s, const uint64_t *tensors, size_t n_tensors,
                                uint64_t *out) {
  // partial collapse_columns over the shard's rows: out[t][c] = sum_{r in shard} t[r] coeffs[r][c]
  if (!s || !out || (!tensors && s->n_rows)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (n_tensors < 1 || n_tensors > 4) return fail(LCPC_ERR_INVALID_ARG, "1..4 tensors");
  const int fid = s->e->fid, wb = field_bytes(fid);
  const size_t np = s->e->n_per_row;
  Device *dev = s->e->dev;
  Lease lease(dev, POOL_HIGH);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf dt, dout, scratch;
  lcpc_status st;
  HIP_TRY(dout.alloc(dev, n_tensors * np * wb));
  if (s->n_rows == 0) {
    HIP_TRY(hipMemsetAsync(dout.p, 0, n_tensors * np * wb, lease.s));
  } else {
    if ((st = upload(dev, dt, tensors, n_tensors * s->n_rows * wb))) return st;
    HIP_TRY(scratch.alloc(dev, collapse_scratch_bytes(fid, s->n_rows, np, (int)n_tensors)));
    HIP_TRY(collapse_rows(fid, s->coeffs.as<uint32_t>(), s->n_rows, np, dt.as<uint32_t>(), (int)n_tensors,
                          dout.as<uint32_t>(), scratch.p, lease.s));
  }
  HIP_TRY(hipMemcpyAsync(out, dout.p, n_tensors * np * wb, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_shard_gather_columns(const lcpc_shard *s, const uint64_t *idx, size_t n, uint64_t *out) {
  if (!s || (!idx && n) || (!out && n)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  const size_t nc = s->e->n_cols;
  for (size_t k = 0; k < n; k++)
    if (idx[k] >= nc) return fail(LCPC_PROVER_COLUMN_NUMBER, "ProverError::ColumnNumber");
  if (!n || !s->n_rows) return LCPC_OK;
  const int fid = s->e->fid, wb = field_bytes(fid);
  Device *dev = s->e->dev;
  Lease lease(dev, POOL_HIGH);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf didx, dcol;
  lcpc_status st;
  if ((st = upload(dev, didx, idx, n * 8))) return st;
  HIP_TRY(dcol.alloc(dev, n * s->n_rows * wb));
  HIP_TRY(gather_columns(fid, s->comm.as<uint32_t>(), s->n_rows, nc, didx.as<uint64_t>(), n,
                         dcol.as<uint32_t>(), lease.s, false, true));
  HIP_TRY(hipMemcpyAsync(out, dcol.p, n * s->n_rows * wb, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_field_sum(lcpc_field f, const uint64_t *vecs, size_t n_vecs, size_t len, uint64_t *out) {
  // out[i] = sum_k vecs[k][i] mod p (folds the shards' partial row combinations)
  if (!valid_field(f) || (!vecs && n_vecs * len) || (!out && len)) return fail(LCPC_ERR_INVALID_ARG, "arguments");
  if (!len) return LCPC_OK;
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  const int wb = field_bytes(f);
  DBuf dv, dout;
  if (n_vecs == 0) {
    std::memset(out, 0, len * wb);
    return LCPC_OK;
  }
  if ((st = upload(dev, dv, vecs, n_vecs * len * wb))) return st;
  HIP_TRY(dout.alloc(dev, len * wb));
  // the fold kernel of collapse: partial[split][t][c] with T = 1
  HIP_TRY(collapse_fold_rows(f, dv.as<uint32_t>(), n_vecs, len, dout.as<uint32_t>(), lease.s));
  HIP_TRY(hipMemcpyAsync(out, dout.p, len * wb, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

// ---- device-resident exchanges: the same steps with the exchanged buffers in device memory
// (torch tensors that RCCL moves over xGMI), so nothing crosses PCIe but the transcript inputs.
// Each call runs on a leased library stream and returns once its results are in memory.
lcpc_status lcpc_shard_chunk_cvs_device(const lcpc_shard *s, size_t chunk_lo, size_t chunk_hi, void *d_out) {
  if (!s || (!d_out && chunk_hi > chunk_lo)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  const int fid = s->e->fid;
  const size_t nc = s->e->n_cols;
  if (chunk_hi > leaf_n_chunks(fid, s->n_rows_total) || chunk_lo > chunk_hi)
    return fail(LCPC_ERR_INVALID_ARG, "chunk range");
  const size_t need_lo = lcpc_leaf_chunk_first_row((lcpc_field)fid, chunk_lo);
  const size_t need_hi = chunk_hi >= leaf_n_chunks(fid, s->n_rows_total)
                             ? s->n_rows_total
                             : lcpc_leaf_chunk_first_row((lcpc_field)fid, chunk_hi);
  if (chunk_hi > chunk_lo && (need_lo < s->row0 || need_hi > s->row0 + s->n_rows))
    return fail(LCPC_ERR_INVALID_ARG, "the shard does not hold every row of those chunks");
  if (chunk_hi == chunk_lo) return LCPC_OK;
  Device *dev = s->e->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  HIP_TRY(leaf_chunk_cvs(fid, s->comm.as<uint32_t>(), s->row0, s->n_rows_total, nc, nc, chunk_lo, chunk_hi,
                         (uint32_t *)d_out, lease.s, true));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_leaves_tree_device(void *d_cvs, size_t n_chunks, size_t n_cols, void *d_hashes) {
  // d_cvs [chunk][col][32] (consumed as scratch) -> d_hashes = leaves || merkle levels || root
  if ((!d_cvs || !d_hashes) && n_cols) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (n_chunks == 0 || n_cols == 0 || (n_cols & (n_cols - 1)))
    return fail(LCPC_ERR_INVALID_ARG, "n_chunks >= 1, n_cols a power of two");
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  HIP_TRY(leaves_from_cvs((uint32_t *)d_cvs, n_cols, (int)n_chunks, (uint8_t *)d_hashes, lease.s));
  if (n_cols > 1) HIP_TRY(merkle_tree((uint8_t *)d_hashes, n_cols, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_shard_collapse_device(const lcpc_shard *s, const void *d_tensors, size_t n_tensors, void *d_out) {
  if (!s || !d_out || (!d_tensors && s->n_rows)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (n_tensors < 1 || n_tensors > 4) return fail(LCPC_ERR_INVALID_ARG, "1..4 tensors");
  const int fid = s->e->fid, wb = field_bytes(fid);
  const size_t np = s->e->n_per_row;
  Device *dev = s->e->dev;
  Lease lease(dev, POOL_HIGH);
  HIP_TRY(hipSetDevice(dev->id));
  if (s->n_rows == 0) {
    HIP_TRY(hipMemsetAsync(d_out, 0, n_tensors * np * wb, lease.s));
  } else {
    DBuf scratch;
    HIP_TRY(scratch.alloc(dev, collapse_scratch_bytes(fid, s->n_rows, np, (int)n_tensors)));
    HIP_TRY(collapse_rows(fid, s->coeffs.as<uint32_t>(), s->n_rows, np, (const uint32_t *)d_tensors,
                          (int)n_tensors, (uint32_t *)d_out, scratch.p, lease.s));
  }
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_shard_gather_columns_device(const lcpc_shard *s, const uint64_t *idx, size_t n, void *d_out) {
  if (!s || (!idx && n) || (!d_out && n)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  const size_t nc = s->e->n_cols;
  for (size_t k = 0; k < n; k++)
    if (idx[k] >= nc) return fail(LCPC_PROVER_COLUMN_NUMBER, "ProverError::ColumnNumber");
  if (!n || !s->n_rows) return LCPC_OK;
  const int fid = s->e->fid;
  Device *dev = s->e->dev;
  Lease lease(dev, POOL_HIGH);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf didx;
  lcpc_status st;
  if ((st = upload(dev, didx, idx, n * 8))) return st;
  HIP_TRY(gather_columns(fid, s->comm.as<uint32_t>(), s->n_rows, nc, didx.as<uint64_t>(), n, (uint32_t *)d_out,
                         lease.s, false, true));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_field_sum_device(lcpc_field f, const void *d_vecs, size_t n_vecs, size_t len, uint64_t *out) {
  if (!valid_field(f) || (!d_vecs && n_vecs * len) || (!out && len)) return fail(LCPC_ERR_INVALID_ARG, "arguments");
  if (!len) return LCPC_OK;
  const int wb = field_bytes(f);
  if (n_vecs == 0) {
    std::memset(out, 0, len * wb);
    return LCPC_OK;
  }
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  DBuf dout;
  HIP_TRY(dout.alloc(dev, len * wb));
  HIP_TRY(collapse_fold_rows(f, (const uint32_t *)d_vecs, n_vecs, len, dout.as<uint32_t>(), lease.s));
  HIP_TRY(hipMemcpyAsync(out, dout.p, len * wb, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

lcpc_status lcpc_challenge_tensor(lcpc_transcript *tr, lcpc_field f, size_t n, uint64_t *out) {
  // prove / verify degree-test tensor (lcpc-2d/src/lib.rs:1056-1062, 899-907)
  if (!tr || !valid_field(f) || (!out && n)) return fail(LCPC_ERR_INVALID_ARG, "arguments");
  std::vector<uint64_t> t;
  challenge_tensor(*tr, f, n, t);
  if (n) std::memcpy(out, t.data(), t.size() * 8);
  return transcript_status(tr);
}

lcpc_status lcpc_challenge_columns(lcpc_transcript *tr, size_t n_cols, size_t n, uint64_t *out) {
  // column choice (lcpc-2d/src/lib.rs:1101-1110, 932-941)
  if (!tr || !n_cols || (!out && n)) return fail(LCPC_ERR_INVALID_ARG, "arguments");
  std::vector<uint64_t> idx;
  challenge_columns(*tr, n_cols, n, idx);
  if (n) std::memcpy(out, idx.data(), n * 8);
  return transcript_status(tr);
}

lcpc_status lcpc_transcript_append_field_elems(lcpc_transcript *tr, const uint8_t *label, size_t ln,
                                               lcpc_field f, const uint64_t *elems, size_t n) {
  // append_message(label, to_repr(e)) for every e (lcpc-2d/src/lib.rs:1075-1077, 1096-1098)
  if (!tr || !valid_field(f) || (!elems && n)) return fail(LCPC_ERR_INVALID_ARG, "arguments");
  if (!n) return LCPC_OK;
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev, POOL_HIGH);
  HIP_TRY(hipSetDevice(dev->id));
  const int wb = field_bytes(f);
  DBuf de;
  if ((st = upload(dev, de, elems, n * wb))) return st;
  const uint8_t *repr = nullptr;
  if ((st = to_repr_host(dev, f, de.as<uint32_t>(), n, &repr))) return st;
  tr->append_messages(label, ln, repr, wb, n);
  return transcript_status(tr);
}

}  // extern "C"

// ================================================================= PoS encoded files
// The `.porenc` / `.portree` formats of proof-of-storage/src/lcpc_online.
// The whole data path (byte packing, Ligero encode, canonical conversion + transpose to the
// column-major file layout, BLAKE3 column digests, Merkle tree) runs on the GPU in row batches
// that end on BLAKE3 chunk boundaries of the column messages, so each batch contributes whole
// chunk chaining values and the file streams through bounded device memory.  The host only
// moves bytes between the caller's buffers (typically mmaps of the files) and page-locked
// staging, with the copies of one batch overlapping the GPU work of the next.
namespace {

constexpr int POS_FID = LCPC_FT63;  // WriteableFt63: Ft63's modulus (writable_ft63.rs:8-12)
constexpr size_t POS_WB = 8;        // F::WRITTEN_BYTES_WIDTH = size_of::<F>() (data_field.rs:24)
constexpr size_t POS_DB = 7;        // F::DATA_BYTE_CAPACITY (data_field.rs:22)
constexpr size_t POS_STAGE_BYTES = (size_t)256 << 20;  // encoded bytes per pipelined batch

template <class Fn>
void parallel_for(size_t n, Fn fn) {
  const size_t hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t T = std::min<size_t>(n, std::min<size_t>(16, hw));
  if (T <= 1) {
    for (size_t i = 0; i < n; i++) fn(i);
    return;
  }
  std::atomic<size_t> next{0};
  const size_t grain = std::max<size_t>(1, n / (T * 8));
  std::vector<std::thread> th;
  for (size_t t = 0; t < T; t++)
    th.emplace_back([&] {
      for (;;) {
        const size_t i0 = next.fetch_add(grain);
        if (i0 >= n) break;
        const size_t i1 = std::min(n, i0 + grain);
        for (size_t i = i0; i < i1; i++) fn(i);
      }
    });
  for (auto &t : th) t.join();
}

// large memcpy split over host threads
void par_memcpy(uint8_t *dst, const uint8_t *src, size_t n) {
  constexpr size_t BLK = (size_t)8 << 20;
  if (n <= BLK) {
    if (n) std::memcpy(dst, src, n);
    return;
  }
  parallel_for((n + BLK - 1) / BLK, [&](size_t i) {
    const size_t o = i * BLK;
    std::memcpy(dst + o, src + o, std::min(BLK, n - o));
  });
}

// a page-locked block from the device's pool, returned at scope exit
struct Pinned {
  Device *d = nullptr;
  void *p = nullptr;
  size_t n = 0;
  Pinned() = default;
  Pinned(const Pinned &) = delete;
  Pinned &operator=(const Pinned &) = delete;
  ~Pinned() { reset(); }
  void reset() {
    if (d && p) d->pinned_put(p);
    p = nullptr;
    n = 0;
  }
  bool get(Device *dev, size_t bytes) {
    reset();
    d = dev;
    p = dev->pinned_get(bytes);
    n = p ? bytes : 0;
    return p != nullptr;
  }
  uint8_t *b() const { return (uint8_t *)p; }
};

// events destroyed at scope exit
struct Events {
  hipEvent_t e[2] = {nullptr, nullptr};
  ~Events() {
    for (auto &x : e)
      if (x) (void)hipEventDestroy(x);
  }
  hipError_t init() {
    for (auto &x : e)
      if (!x) {
        hipError_t r = hipEventCreateWithFlags(&x, hipEventDisableTiming);
        if (r != hipSuccess) return r;
      }
    return hipSuccess;
  }
};

lcpc_status pos_dims_check(size_t pre, size_t enc) {
  // EncodedFileWriter::convert_unencoded_file / new (encoded_file_writer.rs:53-67, 146-163)
  if (pre < 1) return fail(LCPC_ERR_INVALID_ARG, "Number of pre-encoded columns must be greater than 0");
  if (enc < 2 || (enc & (enc - 1)))
    return fail(LCPC_ERR_INVALID_ARG, "Number of encoded columns must be a power of 2 (>= 2)");
  if (enc <= pre)
    return fail(LCPC_ERR_INVALID_ARG, "Number of encoded columns must be greater than the number of columns");
  if ((int)log2_np2(enc) > field_info(POS_FID).s) return fail(LCPC_FFT_TOO_BIG, "FFTError::TooBig");
  return LCPC_OK;
}

}  // namespace

// EncodedFileWriter (encoded_file_writer.rs:24-38): bytes arrive in pushes; whole batches of
// rows are encoded once the data provably continues past them (so no chunk they close can be
// a column message's last chunk), the rest at finalize when the row count is known.
struct lcpc_pos_writer {
  std::unique_ptr<lcpc_encoding> e;
  size_t pre = 0, enc = 0, row_capacity = 0;
  uint8_t *porenc = nullptr;
  size_t cpb = 1, bmax = 1;        // chunks per batch, rows per batch (at most)
  size_t rows_done = 0, chunks_done = 0, bytes_received = 0;
  bool finalized = false;
  Pinned pend;                     // data bytes from row rows_done on (page-locked)
  size_t pend_len = 0;
  std::vector<uint8_t> cvs;        // [chunk][column] chaining values of the chunks done
  size_t buf_rows = 0;             // rows the batch buffers below hold (grown on demand)
  DBuf dbytes, coeffs, comm, dout, dcv;
  Pinned stg[2];
  Events ev;
};

namespace {

size_t pos_row_bytes(const lcpc_pos_writer *w) { return w->pre * POS_DB; }

lcpc_status writer_append(lcpc_pos_writer *w, const uint8_t *bytes, size_t n) {
  if (!n) return LCPC_OK;
  if (w->pend_len + n > w->pend.n) {
    Pinned bigger;
    if (!bigger.get(w->e->dev, std::max(w->pend_len + n, std::max<size_t>(1 << 20, 2 * w->pend.n))))
      return fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
    par_memcpy(bigger.b(), w->pend.b(), w->pend_len);
    std::swap(w->pend.p, bigger.p);
    std::swap(w->pend.n, bigger.n);
    std::swap(w->pend.d, bigger.d);
  }
  par_memcpy(w->pend.b() + w->pend_len, bytes, n);
  w->pend_len += n;
  return LCPC_OK;
}

// Encode chunks [chunks_done, c_end) (rows from pend), n_rows_cv = the row count the chunk
// chaining values are computed for (exact at finalize; any larger-than-covered count before).
lcpc_status writer_run(lcpc_pos_writer *w, size_t c_end, size_t n_rows_cv, size_t n_rows_max) {
  if (c_end <= w->chunks_done) return LCPC_OK;
  const int fid = POS_FID;
  const size_t pre = w->pre, enc = w->enc, rb = pos_row_bytes(w);
  Device *dev = w->e->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  hipStream_t s = lease.s;
  for (auto *b : {&w->dbytes, &w->coeffs, &w->comm, &w->dout, &w->dcv}) b->s = s;
  lcpc_status st;
  struct Pending {
    int slot = -1;
    size_t r0 = 0, rows = 0;
  } pend;
  auto scatter = [&](const Pending &p) -> lcpc_status {
    if (p.slot < 0) return LCPC_OK;
    HIP_TRY(hipEventSynchronize(w->ev.e[p.slot]));
    const uint8_t *src = w->stg[p.slot].b();
    uint8_t *dst = w->porenc;
    const size_t cap = w->row_capacity;
    parallel_for(enc, [&](size_t c) {
      std::memcpy(dst + (c * cap + p.r0) * POS_WB, src + c * p.rows * POS_WB, p.rows * POS_WB);
    });
    return LCPC_OK;
  };
  const size_t pend_row0 = w->rows_done;
  // batch buffers sized for the largest batch of this run (small files stay small)
  const size_t need_rows = std::min(w->bmax, std::max<size_t>(1, n_rows_max - std::min(n_rows_max, pend_row0)));
  if (need_rows > w->buf_rows) {
    HIP_TRY(w->dbytes.alloc(dev, need_rows * pre * POS_DB + 64));
    HIP_TRY(w->coeffs.alloc(dev, need_rows * pre * POS_WB));
    HIP_TRY(w->comm.alloc(dev, need_rows * enc * POS_WB));
    HIP_TRY(w->dout.alloc(dev, need_rows * enc * POS_WB));
    for (auto &x : w->stg)
      if (!x.get(dev, need_rows * enc * POS_WB)) return fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
    w->buf_rows = need_rows;
  }
  // chaining values land in w->cvs by async copies: no reallocation while they are queued
  w->cvs.reserve(c_end * w->enc * 32);
  int k = 0;
  for (size_t c_lo = w->chunks_done; c_lo < c_end; c_lo += w->cpb, k++) {
    const size_t c_hi = std::min(c_end, c_lo + w->cpb);
    const size_t r0 = std::min(n_rows_max, lcpc_leaf_chunk_first_row((lcpc_field)fid, c_lo));
    const size_t r1 = std::min(n_rows_max, lcpc_leaf_chunk_first_row((lcpc_field)fid, c_hi));
    const size_t rr1 = c_hi == leaf_n_chunks(fid, n_rows_cv) ? n_rows_max : r1;
    const size_t B = rr1 - r0;
    if (B > w->buf_rows) return fail(LCPC_ERR_INVALID_ARG, "internal: batch larger than its buffers");
    if (B) {
      if (w->porenc && r0 + B > w->row_capacity) return fail(LCPC_ERR_INVALID_ARG, "row capacity exceeded");
      // rows r0..r0+B are data bytes [rb (r0 - pend_row0), ...) of pend (the last may be short)
      const size_t b0 = (r0 - pend_row0) * rb;
      const size_t b1 = std::min(w->pend_len, b0 + B * rb);
      const size_t ne = (b1 - b0 + POS_DB - 1) / POS_DB;
      HIP_TRY(hipMemcpyAsync(w->dbytes.p, w->pend.b() + b0, b1 - b0, hipMemcpyHostToDevice, s));
      if (B * pre > ne)
        HIP_TRY(hipMemsetAsync(w->coeffs.as<uint8_t>() + ne * POS_WB, 0, (B * pre - ne) * POS_WB, s));
      HIP_TRY(pos_pack7(w->dbytes.as<uint8_t>(), b1 - b0, w->coeffs.as<uint64_t>(), s));
      // canonical codeword: the file's repr words and the leaves' input without conversion
      HIP_TRY(ntt_rows(w->e->plan, w->coeffs.as<uint32_t>(), pre, pre, w->comm.as<uint32_t>(), enc, B, s,
                       nullptr, 0, true));
      if (w->porenc)  // (digest-only writers keep no image)
        HIP_TRY(transpose_elems(fid, w->comm.as<uint32_t>(), B, enc, enc, enc, w->dout.as<uint32_t>(), B, s));
    }
    // column-digest chunks of these rows (ColumnDigestAccumulator::update, :62-87)
    HIP_TRY(leaf_chunk_cvs(fid, w->comm.as<uint32_t>(), r0, n_rows_cv, enc, enc, c_lo, c_hi,
                           w->dcv.as<uint32_t>(), s, true));
    const size_t cv_bytes = (c_hi - c_lo) * enc * 32;
    const size_t cv_off = w->cvs.size();
    w->cvs.resize(cv_off + cv_bytes);
    HIP_TRY(hipMemcpyAsync(w->cvs.data() + cv_off, w->dcv.p, cv_bytes, hipMemcpyDeviceToHost, s));
    if (B && w->porenc) {
      const int slot = k & 1;
      HIP_TRY(hipMemcpyAsync(w->stg[slot].p, w->dout.p, B * enc * POS_WB, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipEventRecord(w->ev.e[slot], s));
      if ((st = scatter(pend))) return st;  // overlaps this batch's GPU work
      pend = Pending{slot, r0, B};
    }
    w->chunks_done = c_hi;
    w->rows_done = rr1;
  }
  if ((st = scatter(pend))) return st;
  HIP_TRY(hipStreamSynchronize(s));
  for (auto *b : {&w->dbytes, &w->coeffs, &w->comm, &w->dout, &w->dcv}) b->settle();
  const size_t used = std::min(w->pend_len, (w->rows_done - pend_row0) * rb);
  std::memmove(w->pend.b(), w->pend.b() + used, w->pend_len - used);
  w->pend_len -= used;
  return LCPC_OK;
}

}  // namespace

extern "C" {

lcpc_status lcpc_pos_writer_new(size_t pre, size_t enc, uint8_t *porenc, size_t row_capacity,
                                size_t batch_rows, lcpc_pos_writer **out) {
  lcpc_status st = pos_dims_check(pre, enc);
  if (st) return st;
  if (!out || (!porenc && row_capacity)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  lcpc_encoding *ep = nullptr;
  if ((st = make_rs_encoding(POS_FID, pre, enc, 0, 0, &ep))) return st;
  auto w = std::make_unique<lcpc_pos_writer>();
  w->e.reset(ep);
  w->pre = pre;
  w->enc = enc;
  w->porenc = porenc;
  w->row_capacity = row_capacity;
  const size_t rows_per_chunk = 1024 / POS_WB;
  size_t want = batch_rows;
  if (!want) want = std::max<size_t>(rows_per_chunk, POS_STAGE_BYTES / (enc * POS_WB));
  w->cpb = std::max<size_t>(1, want / rows_per_chunk);
  w->bmax = w->cpb * rows_per_chunk;
  Device *dev = w->e->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  HIP_TRY(w->dcv.alloc(dev, w->cpb * enc * 32));
  HIP_TRY(w->ev.init());
  HIP_TRY(hipStreamSynchronize(lease.s));
  for (auto *b : {&w->dbytes, &w->coeffs, &w->comm, &w->dout, &w->dcv}) b->settle();
  *out = w.release();
  return LCPC_OK;
}

void lcpc_pos_writer_free(lcpc_pos_writer *w) { delete w; }

lcpc_status lcpc_pos_writer_set_target(lcpc_pos_writer *w, uint8_t *porenc, size_t row_capacity) {
  // after the caller grew the file (EncodedFileReader::set_new_capacity layout, :348-381)
  if (!w || (!porenc && row_capacity)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (row_capacity < w->rows_done) return fail(LCPC_ERR_INVALID_ARG, "row_capacity < rows written");
  w->porenc = porenc;
  w->row_capacity = row_capacity;
  return LCPC_OK;
}

size_t lcpc_pos_writer_rows_written(const lcpc_pos_writer *w) { return w ? w->rows_done : 0; }

lcpc_status lcpc_pos_writer_push_bytes(lcpc_pos_writer *w, const uint8_t *bytes, size_t n) {
  // push_bytes (encoded_file_writer.rs:233-262)
  if (!w || (!bytes && n)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (w->finalized) return fail(LCPC_ERR_INVALID_ARG, "writer already finalized");
  lcpc_status st;
  const size_t rb = pos_row_bytes(w);
  // large pushes are taken a batch at a time, so the staging stays about a batch
  const size_t step = std::max<size_t>(1, w->bmax * rb);
  for (size_t off = 0; off < n || (n == 0 && off == 0); off += step) {
    const size_t m = std::min(step, n - off);
    if ((st = writer_append(w, bytes + off, m))) return st;
    w->bytes_received += m;
    // whole batches whose rows are followed by at least one more full row
    const size_t full_rows = w->rows_done + w->pend_len / rb;
    size_t c_end = w->chunks_done;
    while (lcpc_leaf_chunk_first_row(LCPC_FT63, c_end + w->cpb) < full_rows) c_end += w->cpb;
    if (c_end > w->chunks_done &&
        (st = writer_run(w, c_end, full_rows, lcpc_leaf_chunk_first_row(LCPC_FT63, c_end))))
      return st;
    if (n == 0) break;
  }
  return LCPC_OK;
}

lcpc_status lcpc_pos_writer_finalize(lcpc_pos_writer *w, uint8_t *digests, uint8_t *tree,
                                     size_t *rows_written, size_t *bytes_of_data) {
  // finalize_to_column_digest / _to_commit / _to_merkle_tree (encoded_file_writer.rs:452-501):
  // digests = the enc column digests, tree = MerkleTree::to_bytes (2 enc - 1 digests); either
  // may be NULL
  if (!w) return fail(LCPC_ERR_INVALID_ARG, "null writer");
  if (w->finalized) return fail(LCPC_ERR_INVALID_ARG, "writer already finalized");
  const size_t rb = pos_row_bytes(w);
  const size_t n_rows = w->rows_done + (w->pend_len + rb - 1) / rb;
  if (w->porenc && n_rows > w->row_capacity) return fail(LCPC_ERR_INVALID_ARG, "row capacity exceeded");
  const int fid = POS_FID;
  const size_t n_chunks = leaf_n_chunks(fid, n_rows);
  lcpc_status st = writer_run(w, n_chunks, n_rows, n_rows);
  if (st) return st;
  w->finalized = true;
  const size_t enc = w->enc;
  Device *dev = w->e->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  hipStream_t s = lease.s;
  DBuf dc, hashes;
  if ((st = upload(dev, dc, w->cvs.data(), w->cvs.size()))) return st;
  HIP_TRY(hashes.alloc(dev, (2 * enc - 1) * 32));
  HIP_TRY(leaves_from_cvs(dc.as<uint32_t>(), enc, (int)n_chunks, hashes.as<uint8_t>(), s));
  if (tree) {
    HIP_TRY(merkle_tree(hashes.as<uint8_t>(), enc, s));
    HIP_TRY(hipMemcpyAsync(tree, hashes.p, (2 * enc - 1) * 32, hipMemcpyDeviceToHost, s));
  }
  if (digests) HIP_TRY(hipMemcpyAsync(digests, hashes.p, enc * 32, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (rows_written) *rows_written = w->rows_done;
  if (bytes_of_data) *bytes_of_data = w->bytes_received;
  return LCPC_OK;
}

lcpc_status lcpc_pos_encode_file_batched(const uint8_t *data, size_t n_bytes, size_t pre, size_t enc,
                                         size_t row_capacity, uint8_t *porenc, uint8_t *tree,
                                         size_t *rows_written, size_t batch_rows) {
  lcpc_status st = pos_dims_check(pre, enc);
  if (st) return st;
  if (!tree || (!data && n_bytes)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  const size_t n_rows = ((n_bytes + POS_DB - 1) / POS_DB + pre - 1) / pre;
  if (rows_written) *rows_written = n_rows;
  if (row_capacity < n_rows) return fail(LCPC_ERR_INVALID_ARG, "row_capacity < rows to write");
  lcpc_pos_writer *w = nullptr;
  if ((st = lcpc_pos_writer_new(pre, enc, porenc, row_capacity, batch_rows, &w))) return st;
  std::unique_ptr<lcpc_pos_writer> guard(w);
  if ((st = lcpc_pos_writer_push_bytes(w, data, n_bytes))) return st;
  return lcpc_pos_writer_finalize(w, nullptr, tree, rows_written, nullptr);
}

lcpc_status lcpc_pos_encode_file(const uint8_t *data, size_t n_bytes, size_t pre, size_t enc,
                                 size_t row_capacity, uint8_t *porenc, uint8_t *tree,
                                 size_t *rows_written) {
  return lcpc_pos_encode_file_batched(data, n_bytes, pre, enc, row_capacity, porenc, tree, rows_written, 0);
}

lcpc_status lcpc_pos_reencode_rows(const uint8_t *bytes, size_t n_bytes, size_t pre, size_t enc,
                                   size_t row_lo, uint8_t *porenc, size_t row_capacity) {
  // FileHandler::reencode_row / EncodedFileReader::replace_row_with_decoded_bytes +
  // replace_encoded_row (file_handler.rs:380-402, encoded_file_reader.rs:196-315) for the rows
  // [row_lo, row_lo + ceil(n_bytes / (7 pre))): pack each row's bytes (the last row may be
  // short: zero-padded), encode, and write the canonical repr into the column-major image at
  // column stride row_capacity.  Batches of rows go through the GPU like the writer's.
  lcpc_status st = pos_dims_check(pre, enc);
  if (st) return st;
  if ((!bytes || !porenc) && n_bytes) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  const size_t rb = pre * POS_DB;
  const size_t n_rows = (n_bytes + rb - 1) / rb;
  if (!n_rows) return LCPC_OK;
  if (row_lo + n_rows > row_capacity) return fail(LCPC_ERR_INVALID_ARG, "rows beyond row_capacity");
  lcpc_encoding *ep = nullptr;
  if ((st = make_rs_encoding(POS_FID, pre, enc, 0, 0, &ep))) return st;
  std::unique_ptr<lcpc_encoding> eg(ep);
  Device *dev = ep->dev;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  hipStream_t s = lease.s;
  const size_t bmax = std::min(n_rows, std::max<size_t>(1, POS_STAGE_BYTES / (enc * POS_WB)));
  DBuf dbytes, coeffs, comm, dout;
  for (auto *b : {&dbytes, &coeffs, &comm, &dout}) b->s = s;
  HIP_TRY(dbytes.alloc(dev, bmax * rb + 64));
  HIP_TRY(coeffs.alloc(dev, bmax * pre * POS_WB));
  HIP_TRY(comm.alloc(dev, bmax * enc * POS_WB));
  HIP_TRY(dout.alloc(dev, bmax * enc * POS_WB));
  Pinned stg;
  if (!stg.get(dev, bmax * enc * POS_WB)) return fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
  for (size_t r0 = 0; r0 < n_rows; r0 += bmax) {
    const size_t B = std::min(bmax, n_rows - r0);
    const size_t b0 = r0 * rb, b1 = std::min(n_bytes, b0 + B * rb);
    const size_t ne = (b1 - b0 + POS_DB - 1) / POS_DB;
    HIP_TRY(hipMemcpyAsync(dbytes.p, bytes + b0, b1 - b0, hipMemcpyHostToDevice, s));
    if (B * pre > ne) HIP_TRY(hipMemsetAsync(coeffs.as<uint8_t>() + ne * POS_WB, 0, (B * pre - ne) * POS_WB, s));
    HIP_TRY(pos_pack7(dbytes.as<uint8_t>(), b1 - b0, coeffs.as<uint64_t>(), s));
    HIP_TRY(ntt_rows(ep->plan, coeffs.as<uint32_t>(), pre, pre, comm.as<uint32_t>(), enc, B, s, nullptr, 0, true));
    HIP_TRY(transpose_elems(POS_FID, comm.as<uint32_t>(), B, enc, enc, enc, dout.as<uint32_t>(), B, s));
    HIP_TRY(hipMemcpyAsync(stg.p, dout.p, B * enc * POS_WB, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const uint8_t *src = stg.b();
    parallel_for(enc, [&](size_t c) {
      std::memcpy(porenc + (c * row_capacity + row_lo + r0) * POS_WB, src + c * B * POS_WB, B * POS_WB);
    });
  }
  for (auto *b : {&dbytes, &coeffs, &comm, &dout}) b->settle();
  return LCPC_OK;
}

lcpc_status lcpc_pos_porenc_tree(const uint8_t *porenc, size_t enc, size_t rows_written,
                                 size_t row_capacity, uint8_t *tree) {
  // EncodedFileReader::process_file_to_merkle_tree (encoded_file_reader.rs:328-346): every
  // column's first rows_written elements, hashed after the 32-byte zero block
  if (enc < 2 || (enc & (enc - 1))) return fail(LCPC_ERR_INVALID_ARG, "encoded width must be a power of 2 (>= 2)");
  if (!tree || (!porenc && rows_written)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (rows_written > row_capacity) return fail(LCPC_ERR_INVALID_ARG, "rows_written > row_capacity");
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  hipStream_t s = lease.s;
  const int fid = POS_FID;
  const size_t col_bytes = rows_written * POS_WB;
  const size_t cpb = col_bytes ? std::max<size_t>(1, std::min(enc, POS_STAGE_BYTES / col_bytes)) : enc;
  DBuf hashes, dcols[2], scratch[2], dbad;
  HIP_TRY(hashes.alloc(dev, (2 * enc - 1) * 32));
  for (int i = 0; i < 2; i++) {
    HIP_TRY(dcols[i].alloc(dev, cpb * col_bytes));
    HIP_TRY(scratch[i].alloc(dev, leaf_hash_scratch_bytes(fid, rows_written, cpb)));
  }
  HIP_TRY(dbad.alloc(dev, 4));
  HIP_TRY(hipMemsetAsync(dbad.p, 0, 4, s));
  Pinned stg[2];
  Events ev;
  HIP_TRY(ev.init());
  if (col_bytes)
    for (auto &x : stg)
      if (!x.get(dev, cpb * col_bytes)) return fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
  int k = 0;
  for (size_t c0 = 0; c0 < enc; c0 += cpb, k++) {
    const size_t nc = std::min(enc, c0 + cpb) - c0;
    const int slot = k & 1;
    if (col_bytes) {
      if (k >= 2) HIP_TRY(hipEventSynchronize(ev.e[slot]));  // its last upload has left it
      parallel_for(nc, [&](size_t c) {
        std::memcpy(stg[slot].b() + c * col_bytes, porenc + (c0 + c) * row_capacity * POS_WB, col_bytes);
      });
      HIP_TRY(hipMemcpyAsync(dcols[slot].p, stg[slot].p, nc * col_bytes, hipMemcpyHostToDevice, s));
      HIP_TRY(hipEventRecord(ev.e[slot], s));
      // raw_bytes_to_field_vec: from_repr(..).unwrap() (data_field.rs:72-81)
      HIP_TRY(convert(fid, dcols[slot].as<uint32_t>(), dcols[slot].as<uint32_t>(), nc * rows_written, true, s,
                      dbad.as<uint32_t>()));
    }
    HIP_TRY(leaf_hashes_cols(fid, dcols[slot].as<uint32_t>(), rows_written, nc, hashes.as<uint8_t>() + c0 * 32,
                             scratch[slot].p, s));
  }
  HIP_TRY(merkle_tree(hashes.as<uint8_t>(), enc, s));
  uint32_t bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, dbad.p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(tree, hashes.p, (2 * enc - 1) * 32, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (bad) return fail(LCPC_ERR_INVALID_ARG, "encoded file holds a non-canonical element (from_repr fails)");
  return LCPC_OK;
}

lcpc_status lcpc_pos_decode_porenc(const uint8_t *porenc, size_t pre, size_t enc, size_t row_capacity,
                                   size_t row_lo, size_t row_hi, uint8_t *out) {
  // EncodedFileReader::get_unencoded_row_bytes / decode_to_target_file (encoded_file_reader.rs:
  // 59-91): gather each row's enc elements from the columns, decode_row (ifft_oi), keep the
  // first pre coefficients, 7 data bytes each
  lcpc_status st = pos_dims_check(pre, enc);
  if (st) return st;
  if (row_lo > row_hi || row_hi > row_capacity) return fail(LCPC_ERR_INVALID_ARG, "row range");
  const size_t n = row_hi - row_lo;
  if (!n) return LCPC_OK;
  if (!porenc || !out) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  Device *dev = current_device(&st);
  if (!dev) return st;
  Lease lease(dev);
  HIP_TRY(hipSetDevice(dev->id));
  hipStream_t s = lease.s;
  const int fid = POS_FID;
  const int log_n = (int)log2_np2(enc);
  NttPlan plan;
  hipError_t he = ntt_plan_init(plan, fid, log_n, true, s);
  if (he != hipSuccess) {
    ntt_plan_free(plan);
    if (he == hipErrorInvalidValue) return fail(LCPC_ERR_UNSUPPORTED, "length beyond the NTT range");
    HIP_TRY(he);
  }
  struct PlanGuard {
    NttPlan &p;
    hipStream_t s;
    ~PlanGuard() {
      (void)hipStreamSynchronize(s);
      ntt_plan_free(p);
    }
  } guard{plan, s};
  uint32_t inv[8] = {0};
  inv_pow2_canon(fid, log_n, inv);
  const size_t bmax = std::max<size_t>(1, std::min(n, POS_STAGE_BYTES / (enc * POS_WB)));
  DBuf a, b, dbytes, dbad;
  HIP_TRY(a.alloc(dev, bmax * enc * POS_WB));
  HIP_TRY(b.alloc(dev, bmax * enc * POS_WB));
  HIP_TRY(dbytes.alloc(dev, bmax * pre * POS_DB + 64));
  HIP_TRY(dbad.alloc(dev, 4));
  HIP_TRY(hipMemsetAsync(dbad.p, 0, 4, s));
  Pinned stg[2], ostg[2];
  Events in_ev, out_ev;
  HIP_TRY(in_ev.init());
  HIP_TRY(out_ev.init());
  for (int i = 0; i < 2; i++)
    if (!stg[i].get(dev, bmax * enc * POS_WB) || !ostg[i].get(dev, bmax * pre * POS_DB))
      return fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
  struct Done {
    int slot = -1;
    size_t r0 = 0, rows = 0;
  } done;
  auto copy_out = [&](const Done &d) -> lcpc_status {
    if (d.slot < 0) return LCPC_OK;
    HIP_TRY(hipEventSynchronize(out_ev.e[d.slot]));
    par_memcpy(out + (d.r0 - row_lo) * pre * POS_DB, ostg[d.slot].b(), d.rows * pre * POS_DB);
    return LCPC_OK;
  };
  int k = 0;
  for (size_t r0 = row_lo; r0 < row_hi; r0 += bmax, k++) {
    const size_t B = std::min(row_hi, r0 + bmax) - r0;
    const int slot = k & 1;
    if (k >= 2) HIP_TRY(hipEventSynchronize(in_ev.e[slot]));  // its last upload has left it
    parallel_for(enc, [&](size_t c) {
      std::memcpy(stg[slot].b() + c * B * POS_WB, porenc + (c * row_capacity + r0) * POS_WB, B * POS_WB);
    });
    HIP_TRY(hipMemcpyAsync(a.p, stg[slot].p, enc * B * POS_WB, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(in_ev.e[slot], s));
    // [enc][B] canonical -> [B][enc] Montgomery (get_encoded_row + raw_bytes_to_field_vec)
    HIP_TRY(transpose_elems(fid, a.as<uint32_t>(), enc, B, B, B, b.as<uint32_t>(), enc, s, TR_TO_MONT,
                            dbad.as<uint32_t>()));
    // ifft_oi (see lcpc_ifft_oi_rows): the decoded rows end in x, y is free
    uint32_t *x = b.as<uint32_t>(), *y = a.as<uint32_t>();
    if (LCPC_FFT_OUTPUT_BITREV) {
      HIP_TRY(bitrev_scale(fid, x, y, log_n, B, nullptr, s));
      std::swap(x, y);
    }
    HIP_TRY(ntt_rows(plan, x, enc, enc, y, enc, B, s));
    HIP_TRY(bitrev_scale(fid, y, x, log_n, B, inv, s));
    // decoded_row.drain(pre..) then field_vec_to_byte_vec
    HIP_TRY(hipMemcpy2DAsync(y, pre * POS_WB, x, enc * POS_WB, pre * POS_WB, B, hipMemcpyDeviceToDevice, s));
    HIP_TRY(pos_unpack7(reinterpret_cast<const uint64_t *>(y), B * pre, dbytes.as<uint8_t>(), B * pre * POS_DB, s));
    if (k >= 2) HIP_TRY(hipEventSynchronize(out_ev.e[slot]));
    HIP_TRY(hipMemcpyAsync(ostg[slot].p, dbytes.p, B * pre * POS_DB, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(out_ev.e[slot], s));
    if ((st = copy_out(done))) return st;  // overlaps this batch's GPU work
    done = Done{slot, r0, B};
  }
  if ((st = copy_out(done))) return st;
  uint32_t bad = 0;
  HIP_TRY(hipMemcpyAsync(&bad, dbad.p, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  if (bad) return fail(LCPC_ERR_INVALID_ARG, "encoded file holds a non-canonical element (from_repr fails)");
  return LCPC_OK;
}

}  // extern "C"

// ColumnDigestAccumulator<Blake3, F> with ColumnsToCareAbout::All (column_digest_accumulator.rs:
// 17-118): encoded rows pushed one batch at a time; every column's message is the 32 zero bytes
// then the repr of its elements, hashed in 1-KiB BLAKE3 chunks on the GPU as soon as a chunk is
// complete and the message is known to continue past it (so no chunk is hashed as the only one).
struct lcpc_column_digests {
  Device *dev = nullptr;
  int fid = 0;
  size_t width = 0, chunks_done = 0, rows_in = 0, batch_rows = 0;
  std::vector<uint64_t> pend;  // rows from leaf_chunk_first_row(chunks_done) on
  std::vector<uint8_t> cvs;    // [chunk][column] chaining values of the chunks done
  bool finalized = false;
};

namespace {

constexpr size_t ACC_BATCH_BYTES = (size_t)256 << 20;  // default rows per GPU pass: about this much input

// hash chunks [a->chunks_done, c_end) of messages n_rows_cv rows long (exact, or any count past
// the covered rows while the message continues) from the pending rows
lcpc_status acc_run(lcpc_column_digests *a, size_t c_end, size_t n_rows_cv) {
  if (c_end <= a->chunks_done) return LCPC_OK;
  const int fid = a->fid;
  const size_t nl = (size_t)field_bytes(fid) / 8, w = a->width;
  const size_t r0 = lcpc_leaf_chunk_first_row((lcpc_field)fid, a->chunks_done);
  const size_t r1 = std::min(a->rows_in, lcpc_leaf_chunk_first_row((lcpc_field)fid, c_end));
  Lease lease(a->dev);
  HIP_TRY(hipSetDevice(a->dev->id));
  DBuf drows, dcv;
  lcpc_status st;
  if ((st = upload(a->dev, drows, a->pend.data(), (r1 - r0) * w * nl * 8))) return st;
  HIP_TRY(dcv.alloc(a->dev, (c_end - a->chunks_done) * w * 32));
  HIP_TRY(leaf_chunk_cvs(fid, drows.as<uint32_t>(), r0, n_rows_cv, w, w, a->chunks_done, c_end,
                         dcv.as<uint32_t>(), lease.s));
  const size_t off = a->cvs.size();
  a->cvs.resize(off + (c_end - a->chunks_done) * w * 32);
  HIP_TRY(hipMemcpyAsync(a->cvs.data() + off, dcv.p, (c_end - a->chunks_done) * w * 32, hipMemcpyDeviceToHost,
                         lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  a->pend.erase(a->pend.begin(), a->pend.begin() + (r1 - r0) * w * nl);
  a->chunks_done = c_end;
  return LCPC_OK;
}

}  // namespace

extern "C" {

lcpc_status lcpc_column_digests_new(lcpc_field f, size_t width, size_t batch_rows, lcpc_column_digests **out) {
  if (!out) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (!valid_field(f) || !field_gpu_supported(f)) return fail(LCPC_ERR_UNSUPPORTED, "field");
  if (992 % field_bytes(f)) return fail(LCPC_ERR_UNSUPPORTED, "elements that straddle BLAKE3 chunks (Ft191)");
  if (!width) return fail(LCPC_ERR_INVALID_ARG, "width must be > 0");
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  auto a = std::make_unique<lcpc_column_digests>();
  a->dev = dev;
  a->fid = f;
  a->width = width;
  a->batch_rows = batch_rows ? batch_rows : std::max<size_t>(1, ACC_BATCH_BYTES / (width * field_bytes(f)));
  *out = a.release();
  return LCPC_OK;
}

void lcpc_column_digests_free(lcpc_column_digests *a) { delete a; }

size_t lcpc_column_digests_width(const lcpc_column_digests *a) { return a ? a->width : 0; }

lcpc_status lcpc_column_digests_update(lcpc_column_digests *a, const uint64_t *rows, size_t n_rows) {
  // update (:62-87), for n_rows encoded rows of `width` elements at once
  if (!a || (!rows && n_rows)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (a->finalized) return fail(LCPC_ERR_INVALID_ARG, "accumulator already finalized");
  const size_t nl = (size_t)field_bytes(a->fid) / 8, w = a->width;
  a->pend.insert(a->pend.end(), rows, rows + n_rows * w * nl);
  a->rows_in += n_rows;
  // chunks that end at or before the last row but one: complete, and not their column's last
  size_t c_end = a->chunks_done;
  while (lcpc_leaf_chunk_first_row((lcpc_field)a->fid, c_end + 1) < a->rows_in) c_end++;
  const size_t r0 = lcpc_leaf_chunk_first_row((lcpc_field)a->fid, a->chunks_done);
  if (lcpc_leaf_chunk_first_row((lcpc_field)a->fid, c_end) - r0 < a->batch_rows) return LCPC_OK;  // keep buffering
  return acc_run(a, c_end, a->rows_in);
}

lcpc_status lcpc_column_digests_finalize(lcpc_column_digests *a, uint8_t *digests, uint8_t *tree) {
  // get_column_digests (:89-96) into digests (width x 32 B), and / or finalize_to_merkle_tree
  // (:109-118) into tree (MerkleTree::to_bytes: 2 width - 1 digests, root last; width a power
  // of two >= 2, MerkleTree::new's requirement); either may be NULL
  if (!a) return fail(LCPC_ERR_INVALID_ARG, "null accumulator");
  if (a->finalized) return fail(LCPC_ERR_INVALID_ARG, "accumulator already finalized");
  const size_t w = a->width;
  if (tree && (w < 2 || (w & (w - 1)))) return fail(LCPC_ERR_INVALID_ARG, "Input needs to be a power of two, at least two.");
  const size_t n_chunks = leaf_n_chunks(a->fid, a->rows_in);
  lcpc_status st = acc_run(a, n_chunks, a->rows_in);
  if (st) return st;
  a->finalized = true;
  Lease lease(a->dev);
  HIP_TRY(hipSetDevice(a->dev->id));
  DBuf dc, hashes;
  if ((st = upload(a->dev, dc, a->cvs.data(), a->cvs.size()))) return st;
  HIP_TRY(hashes.alloc(a->dev, (2 * w - 1) * 32));
  HIP_TRY(leaves_from_cvs(dc.as<uint32_t>(), w, (int)n_chunks, hashes.as<uint8_t>(), lease.s));
  if (tree) {
    HIP_TRY(merkle_tree(hashes.as<uint8_t>(), w, lease.s));
    HIP_TRY(hipMemcpyAsync(tree, hashes.p, (2 * w - 1) * 32, hipMemcpyDeviceToHost, lease.s));
  }
  if (digests) HIP_TRY(hipMemcpyAsync(digests, hashes.p, w * 32, hipMemcpyDeviceToHost, lease.s));
  HIP_TRY(hipStreamSynchronize(lease.s));
  return LCPC_OK;
}

}  // extern "C"
