// host_internal.hpp -- shared host-side machinery of liblcpc_mi.so (per-device stream pools and
// caching allocator, pinned staging, handle layouts, Fiat-Shamir helpers).  Internal: included by
// lcpc_host.cpp and shard_native.cpp; one definition of every pool / thread-local across them.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <new>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lcpc_mi.h"
#include "field.hpp"
#include "kernels.hpp"
#include "pos.hpp"
#include "pool.hpp"
#include "prof.hpp"
#include "sdig.hpp"
#include "transcript.hpp"

namespace lcpc_host {
using namespace lcpc;

inline thread_local std::string g_err;
inline thread_local int g_device = 0;

inline lcpc_status fail(lcpc_status st, const std::string &msg) {
  g_err = msg;
  return st;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e__ = (expr);                                                           \
    if (e__ != hipSuccess)                                                             \
      return fail(e__ == hipErrorOutOfMemory ? LCPC_ERR_OUT_OF_MEMORY : LCPC_ERR_DEVICE, \
                  std::string(#expr) + ": " + hipGetErrorString(e__));               \
  } while (0)

inline const uint8_t LABEL_DT[] = {'$', 'l', '/', '/', 'D', 'T'};  // lcpc-2d/src/macros.rs:29-36:
inline const uint8_t LABEL_PR[] = {'$', 'l', '/', '/', 'P', 'R'};  // b"$l//DT" is a byte-string
inline const uint8_t LABEL_PE[] = {'$', 'l', '/', '/', 'P', 'E'};  // literal, which macro_rules!
inline const uint8_t LABEL_CO[] = {'$', 'l', '/', '/', 'C', 'O'};  // never substitutes into.

struct FieldInfo {
  int limbs, num_bits, s;
  uint64_t p[4];
};

inline FieldInfo field_info(int fid) {
  return dispatch_field(fid, []<class F>() {
    FieldInfo fi{};
    fi.limbs = F::N / 2;
    fi.num_bits = F::NUM_BITS;
    fi.s = F::S;
    for (int i = 0; i < F::N / 2; i++)
      fi.p[i] = (uint64_t)F::P[2 * i] | ((uint64_t)F::P[2 * i + 1] << 32);
    return fi;
  });
}

inline bool valid_field(int f) { return f >= 0 && f <= 4; }

// ---------------------------------------------------------------- per-device context
// The stream-ordered block pool's HIP backend (pool.hpp).
struct HipPoolBackend {
  using Stream = hipStream_t;
  using Event = hipEvent_t;
  Event event_new() {
    hipEvent_t e = nullptr;
    return hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess ? e : nullptr;
  }
  void event_free(Event e) { (void)hipEventDestroy(e); }
  bool record(Event e, Stream s) { return hipEventRecord(e, s) == hipSuccess; }
  bool done(Event e) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipErrorNotReady) (void)hipGetLastError();
    return r == hipSuccess;
  }
  bool wait(Stream s, Event e) { return hipStreamWaitEvent(s, e, 0) == hipSuccess; }
  bool sync(Event e) { return hipEventSynchronize(e) == hipSuccess; }
  void drain(Stream s) { (void)hipStreamSynchronize(s); }
};

// The stream pools of a device (a scoped enum: a stray `true` / `false` no longer selects one).
enum class StreamPool : int { Bulk = 0, High = 1, Prover = 2 };
constexpr StreamPool POOL_BULK = StreamPool::Bulk, POOL_HIGH = StreamPool::High, POOL_PROVER = StreamPool::Prover;

// A pool of HIP streams and a caching allocator per device.  Every API call leases its own
// stream, so independent commitments run concurrently (their CPU-side Fiat-Shamir work
// overlaps another commitment's kernels); only pool bookkeeping is locked.
struct Device {
  int id = 0;
  bool ok = false;
  std::string init_err;
  std::mutex mu;  // guards the pools below
  // [POOL_BULK] commit / encode, [POOL_HIGH] the latency-side calls (verify, openings, the sharded
  // driver), [POOL_PROVER] lcpc_prove's row combinations and gathers.  (Confining the prover's
  // streams to a quarter or eighth of the CUs, so that its kernels never hold CUs the encodes
  // need, changed the K = 20 line by less than its spread: profiles/r05_k20_prover_cu_mask_ab.json.)
  std::vector<hipStream_t> idle_streams[3];
  // device blocks: cached by exact size, each ordered after a fence on the streams that used it
  // (pool.hpp); sizes = every block this device allocated
  HipPoolBackend pool_backend;
  lcpc_pool::OrderedPool<HipPoolBackend> blocks{pool_backend};
  std::map<void *, size_t> sizes;

  // (all pools' streams run at one priority by default: see stream_priority below)
  hipStream_t shared_stream = nullptr;  // LCPC_STREAM_MODE=serial: every call on one stream

  static bool serial_mode() {
    static const bool v = [] {
      const char *m = getenv("LCPC_STREAM_MODE");
      return m && std::string(m) == "serial";
    }();
    return v;
  }

  hipStream_t acquire_stream(StreamPool pool) {
    if (serial_mode()) {
      std::lock_guard<std::mutex> lk(mu);
      if (!shared_stream) {
        (void)hipSetDevice(id);
        if (hipStreamCreateWithFlags(&shared_stream, hipStreamNonBlocking) != hipSuccess)
          shared_stream = nullptr;
      }
      return shared_stream;
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      auto &idle = idle_streams[(int)pool];
      if (!idle.empty()) {
        hipStream_t s = idle.back();
        idle.pop_back();
        return s;
      }
    }
    prof::HostScope hs("rt_stream_create");
    hipStream_t s = nullptr;
    (void)hipSetDevice(id);
    if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, stream_priority(pool != POOL_BULK)) != hipSuccess)
      return nullptr;
    return s;
  }
  // Every stream at ONE priority (round 5): mixed priorities are the one condition under which a
  // wrong commitment was ever observed (eight ranks on one GPU), and a high-priority
  // prover bought nothing measurable (profiles/r04_k20_stream_priority_ab.json).  The two stream
  // pools stay separate so that LCPC_PRIORITY_STREAMS=1 can still put the prover's streams (and the
  // sharded driver's) above the bulk ones for A/B runs.
  static bool priority_streams() {
    static const bool v = [] {
      const char *e = getenv("LCPC_PRIORITY_STREAMS");
      return e && e[0] == '1';
    }();
    return v;
  }
  static int stream_priority(bool high) {
    int lo = 0, hi = 0;
    if (!priority_streams() || hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return 0;
    return high ? hi : lo;
  }
  void release_stream(hipStream_t s, StreamPool pool) {
    if (serial_mode()) return;
    std::lock_guard<std::mutex> lk(mu);
    idle_streams[(int)pool].push_back(s);
  }
  static size_t round_bytes(size_t bytes) { return ((bytes ? bytes : 16) + 255) & ~(size_t)255; }
  // a block of at least `bytes`, ordered after every earlier use of it: on stream `s` when given
  // (device-side waits), on the host otherwise
  hipError_t alloc(void **p, size_t bytes, hipStream_t s = nullptr) {
    bytes = round_bytes(bytes);
    if ((*p = blocks.take(bytes, s))) return hipSuccess;
    prof::HostScope hs("rt_hipMalloc");
    // a pool thread's current device is whatever it last set (GPU 0 for a fresh thread): the
    // block must come from THIS device, so make it current before allocating
    hipError_t e = hipSetDevice(id);
    if (e != hipSuccess) return e;
    e = hipMalloc(p, bytes);
    if (e == hipErrorOutOfMemory) {
      (void)hipGetLastError();
      trim();
      e = hipMalloc(p, bytes);
    }
    if (e == hipSuccess) {
      std::lock_guard<std::mutex> lk(mu);
      sizes[*p] = bytes;
    }
    return e;
  }
  // back to the pool; the streams ss[0..n) may still have work queued on it (a fence is recorded
  // on each), none if the caller knows every use has completed
  void release(void *p, const hipStream_t *ss = nullptr, int n = 0) {
    if (!p) return;
    size_t bytes;
    {
      std::lock_guard<std::mutex> lk(mu);
      auto it = sizes.find(p);
      if (it == sizes.end()) return;
      bytes = it->second;
    }
    blocks.put(p, bytes, ss, n);
  }
  // page-locked host blocks for the file paths' staging (pinning is slow: blocks are reused)
  std::multimap<size_t, void *> pinned_free;
  std::map<void *, size_t> pinned_sizes;
  void *pinned_get(size_t bytes) {
    // blocks are whole 2 MiB multiples; a cached block up to twice the rounded size is reused
    const size_t want = (std::max<size_t>(bytes, 1) + ((size_t)2 << 20) - 1) & ~(((size_t)2 << 20) - 1);
    {
      std::lock_guard<std::mutex> lk(mu);
      auto it = pinned_free.lower_bound(want);
      if (it != pinned_free.end() && it->first <= 2 * want) {
        void *p = it->second;
        pinned_free.erase(it);
        return p;
      }
    }
    prof::HostScope hs("rt_hipHostMalloc_pool");
    void *p = nullptr;
    (void)hipSetDevice(id);
    if (hipHostMalloc(&p, want, hipHostMallocPortable) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(mu);
    pinned_sizes[p] = want;
    return p;
  }
  void pinned_put(void *p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu);
    auto it = pinned_sizes.find(p);
    if (it != pinned_sizes.end()) pinned_free.emplace(it->second, p);
  }
  void trim() {
    (void)hipSetDevice(id);
    (void)hipDeviceSynchronize();
    std::vector<void *> gone;
    blocks.drain([&](void *p) { gone.push_back(p); });
    std::lock_guard<std::mutex> lk(mu);
    for (void *p : gone) {
      sizes.erase(p);
      (void)hipFree(p);
    }
  }
};

inline std::mutex g_devices_mu;
inline std::map<int, std::unique_ptr<Device>> g_devices;

inline Device *get_device(int id, lcpc_status *st) {
  std::lock_guard<std::mutex> lk(g_devices_mu);
  auto &slot = g_devices[id];
  if (!slot) {
    slot = std::make_unique<Device>();
    slot->id = id;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= id) {
      slot->init_err = "no HIP device available (liblcpc_mi has no CPU fallback)";
    } else if ((e = hipSetDevice(id)) != hipSuccess) {
      slot->init_err = std::string("HIP init failed: ") + hipGetErrorString(e);
    } else {
      slot->ok = true;
      // how host threads wait for the GPU (LCPC_HOST_WAIT=spin|yield|blocking; unset = the
      // runtime's default).  A spinning wait burns a core of the process's CPU share.
      if (const char *w = std::getenv("LCPC_HOST_WAIT")) {
        const std::string m(w);
        const unsigned f = m == "spin"       ? hipDeviceScheduleSpin
                           : m == "yield"    ? hipDeviceScheduleYield
                           : m == "blocking" ? hipDeviceScheduleBlockingSync
                                             : hipDeviceScheduleAuto;
        e = hipSetDeviceFlags(f);
        if (e != hipSuccess) fprintf(stderr, "liblcpc_mi: hipSetDeviceFlags(%s): %s\n", w, hipGetErrorString(e));
      }
    }
  }
  if (!slot->ok) {
    *st = fail(LCPC_ERR_NO_DEVICE, slot->init_err);
    return nullptr;
  }
  *st = LCPC_OK;
  return slot.get();
}

inline thread_local hipStream_t t_stream = nullptr;  // stream of the innermost live Lease

// this thread's completion event for device `id` (created on first use; the calling thread has
// made that device current)
inline hipEvent_t t_event(int id) {
  thread_local struct Events {
    hipEvent_t e[64] = {};
    ~Events() {
      for (hipEvent_t x : e)
        if (x) (void)hipEventDestroy(x);
    }
  } te;
  if (id < 0 || id >= 64) return nullptr;
  if (!te.e[id] && hipEventCreateWithFlags(&te.e[id], hipEventDisableTiming) != hipSuccess) te.e[id] = nullptr;
  return te.e[id];
}

// A stream leased for the duration of one API call (also makes the device current).
struct Lease {
  Device *d;
  hipStream_t s;
  hipStream_t prev;
  StreamPool pool;
  explicit Lease(Device *dev, StreamPool stream_pool = POOL_BULK) : d(dev), s(nullptr), prev(t_stream), pool(stream_pool) {
    (void)hipSetDevice(dev->id);
    s = dev->acquire_stream(pool);
    t_stream = s;
  }
  ~Lease() {
    if (s) {
      (void)hipStreamSynchronize(s);
      d->release_stream(s, pool);
    }
    t_stream = prev;
  }
  Lease(const Lease &) = delete;
  Lease &operator=(const Lease &) = delete;
};

// For a scope whose work runs on a caller's stream: the DBufs it allocates are taken (and
// fenced at release) on that stream instead of the scope's lease stream
struct StreamAs {
  hipStream_t prev;
  explicit StreamAs(hipStream_t x) : prev(t_stream) { t_stream = x; }
  ~StreamAs() { t_stream = prev; }
  StreamAs(const StreamAs &) = delete;
  StreamAs &operator=(const StreamAs &) = delete;
};

// RAII device buffer from the stream-ordered pool.  It remembers the streams that use it -- the
// one current when it was allocated (t_stream) and any added with use() -- and returns its block
// with a fence on each (pool.hpp): the block's next owner is ordered after every write still
// queued here, with no host drain.  settle() / settle(s) say that all / s's uses have completed
// (the fence is then skipped), an optimisation only: an unsettled buffer is always safe.
struct DBuf {
  static constexpr int MAXS = lcpc_pool::OrderedPool<HipPoolBackend>::MAX_STREAMS;
  Device *d = nullptr;
  void *p = nullptr;
  size_t n = 0;
  hipStream_t s = nullptr;      // the stream current at allocation (its first user)
  hipStream_t xs[MAXS - 1] = {};  // further streams that use it (use())
  int nx = 0;
  DBuf() = default;
  DBuf(const DBuf &) = delete;
  DBuf &operator=(const DBuf &) = delete;
  DBuf(DBuf &&o) noexcept : d(o.d), p(o.p), n(o.n), s(o.s), nx(o.nx) {
    for (int i = 0; i < nx; i++) xs[i] = o.xs[i];
    o.p = nullptr;
    o.nx = 0;
  }
  DBuf &operator=(DBuf &&o) noexcept {
    reset();
    d = o.d; p = o.p; n = o.n; s = o.s; nx = o.nx;
    for (int i = 0; i < nx; i++) xs[i] = o.xs[i];
    o.p = nullptr;
    o.nx = 0;
    return *this;
  }
  ~DBuf() { reset(); }
  void reset() {
    if (p && d) {
      hipStream_t ss[MAXS];
      int k = 0;
      if (s) ss[k++] = s;
      for (int i = 0; i < nx; i++) ss[k++] = xs[i];
      d->release(p, ss, k);
    }
    p = nullptr;
    s = nullptr;
    nx = 0;
  }
  // another stream works on this buffer (its work is fenced at release)
  void use(hipStream_t x) {
    if (!x || x == s) return;
    for (int i = 0; i < nx; i++)
      if (xs[i] == x) return;
    if (nx < MAXS - 1) {
      xs[nx++] = x;
    } else {  // (never in the library: at most three streams touch a buffer) drain it instead
      (void)hipStreamSynchronize(x);
    }
  }
  // every queued use of this buffer has completed (no fence needed at release)
  void settle() {
    s = nullptr;
    nx = 0;
  }
  // stream x has drained: its uses need no fence
  void settle(hipStream_t x) {
    if (x && s == x) s = nullptr;
    for (int i = 0; i < nx; i++)
      if (xs[i] == x) xs[i--] = xs[--nx];
  }
  hipError_t alloc(Device *dev, size_t bytes) {
    reset();
    d = dev;
    n = bytes;
    s = t_stream;
    return dev->alloc(&p, bytes, t_stream);
  }
  template <class T>
  T *as() const { return reinterpret_cast<T *>(p); }
};

// Thread-local pinned (page-locked) host staging buffers: device<->host copies of proof-sized
// vectors go through these so they are true async DMA (pageable copies are staged and
// serialize concurrent commitments).  Slots are grown on demand and reused across calls.
struct PinnedSlot {
  void *p = nullptr;
  size_t cap = 0;
  ~PinnedSlot() {
    if (p) (void)hipHostFree(p);
  }
  void *get(size_t n) {
    if (n > cap) {
      prof::HostScope hs("rt_pinned_slot_grow");
      if (p) (void)hipHostFree(p);
      p = nullptr;
      cap = 0;
      size_t want = n < 4096 ? 4096 : n + n / 4;
      if (hipHostMalloc(&p, want, hipHostMallocPortable) != hipSuccess) return nullptr;
      cap = want;
    }
    return p;
  }
};
enum { PIN_REPR = 0, PIN_PRANDOM, PIN_PEVAL, PIN_COLS, PIN_PATHS, PIN_TENSOR, PIN_OUTER, PIN_STAGE, PIN_STAGE2, PIN_N };
inline thread_local PinnedSlot t_pin[PIN_N];
// lcpc_prove: the evaluation's repr bytes, converted with the first degree test's (host memory)
inline thread_local std::vector<uint8_t> t_eval_repr;

inline size_t next_pow2(size_t v) {
  size_t p = 1;
  while (p < v) p <<= 1;
  return p;
}
inline size_t log2_np2(size_t v) {  // lcpc-2d log2 (:857-859)
  size_t p = next_pow2(v), l = 0;
  while (((size_t)1 << l) < p) l++;
  return l;
}

}  // namespace lcpc_host

using namespace lcpc;
using namespace lcpc_host;

// ---------------------------------------------------------------- handles
enum { KIND_RS = 0, KIND_SDIG = 1 };

struct lcpc_encoding {
  int fid = 1;
  int kind = KIND_RS;  // R-S / fft_io (Ligero) or SDIG expander code (Brakedown)
  int code = 0;        // SdigCode id
  uint64_t seed = 0;
  size_t n_per_row = 0, n_cols = 0, n_col_opens = 0, n_degree_tests = 0;
  Device *dev = nullptr;
  NttPlan plan;
  SdigPlan sdig;
  ~lcpc_encoding() {
    if (dev) {
      Lease lease(dev);
      (void)hipSetDevice(dev->id);
      (void)hipStreamSynchronize(lease.s);
      ntt_plan_free(plan);
      sdig_plan_free(sdig);
    }
  }
};

struct lcpc_commit {
  int fid = 1;
  Device *dev = nullptr;
  size_t n_rows = 0, n_cols = 0, n_per_row = 0, n_hashes = 0;
  bool col_major = false;  // comm stored [n_cols][n_rows] (SDIG) instead of [n_rows][n_cols]
  bool canon = false;      // comm holds canonical values (R-S: ntt_rows canon_out), not Montgomery
  DBuf coeffs, comm, hashes;
  uint8_t root[32];
};

// Page-locked host memory for proofs: prove's device -> host copies land in the proof itself
// (no staging slot and no host memcpy: ~23 MB per Brakedown proof at cfg4), and verify uploads
// from it by DMA.  Blocks of >= 64 KiB come from a process-wide reuse pool (pinning is slow);
// smaller ones, and any when the HIP runtime cannot pin (a host-only process), are heap memory.  Elements are default-initialised (resize does not zero).
struct PinnedHeap {
  std::mutex mu;
  std::multimap<size_t, void *> free_;
  std::map<void *, size_t> size_;
  std::atomic<bool> no_pin{false};
  size_t cached = 0;  // bytes on the free list
  static constexpr size_t MIN = (size_t)64 << 10;
  // the free list keeps at most this much page-locked memory; blocks returned beyond it are
  // unpinned (varied proof sizes would otherwise grow the pool without bound)
  static constexpr size_t CAP = (size_t)4 << 30;
  void *get(size_t bytes) {
    const size_t want = (bytes + MIN - 1) & ~(MIN - 1);
    {
      std::lock_guard<std::mutex> lk(mu);
      auto it = free_.lower_bound(want);
      if (it != free_.end() && it->first <= 2 * want) {
        void *p = it->second;
        cached -= it->first;
        free_.erase(it);
        return p;
      }
    }
    if (no_pin.load(std::memory_order_relaxed)) return nullptr;
    prof::HostScope hs("rt_hipHostMalloc_proof");
    void *p = nullptr;
    if (hipHostMalloc(&p, want, hipHostMallocPortable) != hipSuccess) {
      (void)hipGetLastError();
      // latch heap memory only when there is no HIP runtime at all (a host-only process); a
      // transient failure (e.g. the page-locked limit) falls back for this block alone
      int n = 0;
      if (hipGetDeviceCount(&n) != hipSuccess || n == 0) no_pin.store(true, std::memory_order_relaxed);
      return nullptr;
    }
    std::lock_guard<std::mutex> lk(mu);
    size_[p] = want;
    return p;
  }
  // false if p is not one of ours (heap memory)
  bool put(void *p) {
    std::lock_guard<std::mutex> lk(mu);
    auto it = size_.find(p);
    if (it == size_.end()) return false;
    if (cached + it->second > CAP) {
      size_.erase(it);
      (void)hipHostFree(p);
      return true;
    }
    cached += it->second;
    free_.emplace(it->second, p);
    return true;
  }
};
// never destroyed: proofs freed during interpreter teardown still return their blocks safely
inline PinnedHeap &g_pinned_heap = *new PinnedHeap;

template <class T>
struct PinnedAlloc {
  using value_type = T;
  PinnedAlloc() = default;
  template <class U>
  PinnedAlloc(const PinnedAlloc<U> &) {}
  T *allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    void *p = bytes >= PinnedHeap::MIN ? g_pinned_heap.get(bytes) : nullptr;
    if (!p) p = std::malloc(bytes ? bytes : 1);  // small, or no HIP runtime (host-only use)
    if (!p) throw std::bad_alloc();
    return static_cast<T *>(p);
  }
  void deallocate(T *p, size_t) {
    if (!g_pinned_heap.put(p)) std::free(p);
  }
  template <class U>
  void construct(U *p) noexcept {
    ::new ((void *)p) U;  // default-initialise: the buffers are filled by DMA or memcpy
  }
  template <class U, class... A>
  void construct(U *p, A &&...a) {
    ::new ((void *)p) U(std::forward<A>(a)...);
  }
  template <class U>
  bool operator==(const PinnedAlloc<U> &) const { return true; }
  template <class U>
  bool operator!=(const PinnedAlloc<U> &) const { return false; }
};
template <class T>
using pinned_vector = std::vector<T, PinnedAlloc<T>>;

struct lcpc_proof {
  int fid = 1;
  size_t n_cols = 0, n_per_row = 0, n_rows = 0, ndt = 0, nco = 0, path_len = 0;
  pinned_vector<uint64_t> p_eval, p_random, cols;
  std::vector<uint64_t> col_idx;
  pinned_vector<uint8_t> paths;
};

// A merlin::Transcript as prove / verify see it: the library's own restatement (t), or the
// caller's transcript behind lcpc_transcript_ops (lcpc_transcript_from_ops), every absorb and
// squeeze forwarded.  The reference threads the caller's `&mut Transcript` through prove / verify
// (lcpc-2d/src/lib.rs:319-326, 547-556); ops let a caller that owns one keep it.
struct lcpc_transcript {
  Transcript t;
  lcpc_transcript_ops ops{};
  bool external = false;
  int cb_status = 0;  // first non-zero return of an ops callback (the call then fails)
  explicit lcpc_transcript(const uint8_t *l, size_t n) : t(l, n) {}
  explicit lcpc_transcript(const lcpc_transcript_ops &o)
      : t(reinterpret_cast<const uint8_t *>(""), 0), ops(o), external(true) {}
  void append_message(const uint8_t *label, size_t ln, const uint8_t *msg, size_t mn) {
    if (!external) return t.append_message(label, ln, msg, mn);
    if (!cb_status) cb_status = ops.append_message(ops.ctx, label, ln, msg, mn);
  }
  // append_message(label, msgs + i * ml) for i < n: one callback when the caller batches
  void append_messages(const uint8_t *label, size_t ln, const uint8_t *msgs, size_t ml, size_t n) {
    if (!external) return t.append_messages(label, ln, msgs, ml, n);
    if (cb_status) return;
    if (ops.append_messages) {
      cb_status = ops.append_messages(ops.ctx, label, ln, msgs, ml, n);
      return;
    }
    for (size_t i = 0; i < n && !cb_status; i++) cb_status = ops.append_message(ops.ctx, label, ln, msgs + i * ml, ml);
  }
  void challenge_bytes(const uint8_t *label, size_t ln, uint8_t *dst, size_t n) {
    if (!external) return t.challenge_bytes(label, ln, dst, n);
    if (!cb_status) cb_status = ops.challenge_bytes(ops.ctx, label, ln, dst, n);
    if (cb_status) std::memset(dst, 0, n);  // (the call fails; keep the bytes defined)
  }
};

namespace lcpc_host {
inline lcpc_status encoding_dims_ok(const lcpc_encoding *e, size_t n_per_row, size_t n_cols) {
  if (e->kind == KIND_SDIG)  // SdigEncodingS::dims_ok (lcpc-brakedown-pc/src/lib.rs:157-164)
    return (n_per_row < n_cols && n_per_row == e->n_per_row && n_cols == e->n_cols)
               ? LCPC_OK
               : LCPC_ERR_INVALID_ARG;
  // LigeroEncodingRho::dims_ok (lcpc-ligero-pc/src/lib.rs:171-177)
  const bool pow = n_cols && !(n_cols & (n_cols - 1));
  return (n_per_row < n_cols && pow && n_per_row == e->n_per_row && n_cols == e->n_cols) ? LCPC_OK
                                                                                       : LCPC_ERR_INVALID_ARG;
}

// Encode n_rows row-major rows: row r reads n_valid leading coefficients at src + r * ss (the
// rest of its message zero) and writes n_cols elements at dst + r * ds.  Runs on stream s
// (normally the caller's lease); scratch comes from the pool.
inline lcpc_status encode_rows_any(const lcpc_encoding *e, const uint32_t *src, size_t ss, size_t nv,
                            uint32_t *dst, size_t ds, size_t n_rows, hipStream_t s) {
  if (n_rows == 0) return LCPC_OK;
  if (e->kind == KIND_RS) {
    HIP_TRY(ntt_rows(e->plan, src, ss, nv, dst, ds, n_rows, s));
    return LCPC_OK;
  }
  // SDIG: element-major working codeword, then back to rows.  The code is systematic (the
  // codeword starts with the message, encode.rs:36-94), so the input transpose also writes the
  // zero-padded message row-major into dst as it reads it, and only the parity part [np, nc) is
  // transposed back (an in-place call with a full message has its message part in place already)
  const size_t nc = e->n_cols, np = e->n_per_row;
  const int wb = field_bytes(e->fid), nw = wb / 4;
  DBuf cw, tmp;
  HIP_TRY(cw.alloc(e->dev, nc * n_rows * wb));
  HIP_TRY(tmp.alloc(e->dev, e->sdig.tmp_elems * n_rows * wb));
  const bool in_place = (const void *)src == (const void *)dst && ss == ds && nv >= np;
  HIP_TRY(transpose_elems(e->fid, src, n_rows, np, ss, nv < np ? nv : np, cw.as<uint32_t>(), n_rows, s, TR_PLAIN,
                          nullptr, SIZE_MAX, in_place ? nullptr : dst, ds));
  HIP_TRY(sdig_encode_cm(e->sdig, cw.as<uint32_t>(), n_rows, tmp.as<uint32_t>(), s));
  HIP_TRY(transpose_elems(e->fid, cw.as<uint32_t>() + np * n_rows * nw, nc - np, n_rows, n_rows, n_rows,
                          dst + np * nw, ds, s));
  return LCPC_OK;  // (cw / tmp go back to the pool fenced on s: no drain here)
}

// Device address of page-locked (hipHostMalloc'd) host memory, or nullptr for pageable memory.
// Every page-locked block of this library is allocated hipHostMallocPortable, so it is mapped
// for every device a thread may switch to.
inline void *host_dev_ptr(const void *h) {
  if (!h) return nullptr;
  void *d = nullptr;
  if (hipHostGetDevicePointer(&d, const_cast<void *>(h), 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return d;
}
// Small prover transfers between device buffers and page-locked host memory go through a copy
// kernel on the caller's stream (the kernel stores to / loads from the mapped host memory), so
// they are ordered like any other launch: a copy-engine transfer queued behind kernels can hold
// the issuing thread until other streams' work drains (measured: 20-60 ms per K = 20 bench run
// in the row-combination rounds).  Pageable memory still takes hipMemcpyAsync.
inline hipError_t d2h(void *h, const void *d, size_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  if (void *hd = host_dev_ptr(h); hd && !(((uintptr_t)hd | (uintptr_t)d | bytes) & 7)) return copy_words(hd, d, bytes, s);
  return hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s);
}
inline hipError_t h2d(void *d, const void *h, size_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  if (void *hd = host_dev_ptr(h); hd && !(((uintptr_t)hd | (uintptr_t)d | bytes) & 7)) return copy_words(d, hd, bytes, s);
  return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
}

// Device -> any host memory.  Mapped page-locked memory: the copy kernel, asynchronous.
// Pageable memory: pieces of at most 4 MiB go through this thread's two page-locked staging
// slots by the copy kernel, double-buffered (the next piece's kernel runs while the host copies
// the previous one out); returns once the data is in place.
struct StageEvents {
  hipEvent_t e[2] = {nullptr, nullptr};
  int dev = -1;  // events belong to the device current when they were created
  ~StageEvents() { reset(); }
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
    for (hipEvent_t &x : e) {
      if (!x && hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) {
        x = nullptr;
        return false;
      }
    }
    return true;
  }
};
inline thread_local StageEvents t_stage_ev;
inline hipError_t d2h_staged(void *h, const void *d, size_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  if (host_dev_ptr(h) || (((uintptr_t)d | bytes) & 7)) return d2h(h, d, bytes, s);
  constexpr size_t PIECE = (size_t)4 << 20;
  const size_t first = std::min(bytes, PIECE);
  uint8_t *stg[2] = {(uint8_t *)t_pin[PIN_STAGE].get(first), (uint8_t *)t_pin[PIN_STAGE2].get(first)};
  void *sd[2] = {host_dev_ptr(stg[0]), host_dev_ptr(stg[1])};
  if (!sd[0] || !sd[1] || !t_stage_ev.ready()) return hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s);
  const size_t n_pieces = (bytes + PIECE - 1) / PIECE;
  auto issue = [&](size_t k) -> hipError_t {
    const size_t off = k * PIECE, n = std::min(PIECE, bytes - off);
    hipError_t e = copy_words(sd[k & 1], (const uint8_t *)d + off, n, s);
    return e == hipSuccess ? hipEventRecord(t_stage_ev.e[k & 1], s) : e;
  };
  hipError_t e = issue(0);
  for (size_t k = 0; e == hipSuccess && k < n_pieces; k++) {
    if (k + 1 < n_pieces) e = issue(k + 1);  // its slot was copied out in the previous iteration
    if (e == hipSuccess) e = hipEventSynchronize(t_stage_ev.e[k & 1]);
    if (e == hipSuccess) std::memcpy((uint8_t *)h + k * PIECE, stg[k & 1], std::min(PIECE, bytes - k * PIECE));
  }
  return e;
}

inline hipError_t d2d(void *dst, const void *src, size_t bytes, hipStream_t s) {
  if (!bytes) return hipSuccess;
  if (!(((uintptr_t)dst | (uintptr_t)src | bytes) & 7)) return copy_words(dst, src, bytes, s, false);
  return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s);
}

// upload host -> device (pool buffer)
inline lcpc_status upload(Device *dev, DBuf &b, const void *h, size_t bytes) {
  HIP_TRY(b.alloc(dev, bytes));
  if (bytes) HIP_TRY(h2d(b.p, h, bytes, t_stream));  // page-locked sources (a proof's vectors): copy kernel
  return LCPC_OK;
}

// field elements -> canonical repr bytes (device convert, D2H into a pinned slot, host byte
// order); *out points into thread-local pinned memory valid until the next call.
inline lcpc_status to_repr_host(Device *dev, int fid, const uint32_t *d_elems, size_t n,
                         const uint8_t **out) {
  const int wb = field_bytes(fid);
  uint8_t *h = (uint8_t *)t_pin[PIN_REPR].get(n * wb);
  if (!h) return fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
  if (void *hd = host_dev_ptr(h)) {  // the conversion kernel writes the pinned slot itself
    HIP_TRY(convert(fid, d_elems, (uint32_t *)hd, n, false, t_stream));
  } else {
    DBuf canon;
    HIP_TRY(canon.alloc(dev, n * wb));
    HIP_TRY(convert(fid, d_elems, canon.as<uint32_t>(), n, false, t_stream));
    if (n) HIP_TRY(hipMemcpyAsync(h, canon.p, n * wb, hipMemcpyDeviceToHost, t_stream));
  }
  HIP_TRY(hipStreamSynchronize(t_stream));
  if (fid == LCPC_FT253_192) {  // PrimeFieldReprEndianness = "big" (ft253_192.rs:9)
    for (size_t i = 0; i < n; i++) std::reverse(h + i * wb, h + (i + 1) * wb);
  }
  *out = h;
  return LCPC_OK;
}

inline void challenge_tensor(lcpc_transcript &tr, int fid, size_t n_rows, std::vector<uint64_t> &out) {
  // lcpc-2d/src/lib.rs:1056-1062 (prove) / :899-907 (verify)
  uint8_t key[32];
  tr.challenge_bytes(LABEL_DT, 6, key, 32);
  ChaCha20Rng rng(key);
  const FieldInfo fi = field_info(fid);
  out.resize(n_rows * fi.limbs);
  field_random(rng, fi.limbs, fi.num_bits, fi.p, out.data(), n_rows);
}

inline void challenge_columns(lcpc_transcript &tr, size_t n_cols, size_t nco, std::vector<uint64_t> &idx) {
  // lcpc-2d/src/lib.rs:1103-1110 (prove) / :932-941 (verify)
  uint8_t key[32];
  tr.challenge_bytes(LABEL_CO, 6, key, 32);
  ChaCha20Rng rng(key);
  idx.resize(nco);
  for (size_t i = 0; i < nco; i++) idx[i] = uniform_usize(rng, 0, n_cols);
}

inline Device *current_device(lcpc_status *st) { return get_device(g_device, st); }

// a caller-owned transcript's callback failed during the call: its state is no longer the
// reference's, so the proof / verdict is void
inline lcpc_status transcript_status(const lcpc_transcript *tr) {
  if (!tr || !tr->cb_status) return LCPC_OK;
  return fail(LCPC_ERR_TRANSCRIPT, "a caller transcript callback failed (status " + std::to_string(tr->cb_status) + ")");
}
}  // namespace lcpc_host

