// shard_native.cpp -- row-sharded Ligero commit / prove across GPUs behind the C ABI
// (include/lcpc_mi.h, "communicators" and "row-sharded commitments").
//
// One process per GPU.  A commitment's n_rows rows are cut at BLAKE3 chunk boundaries of the
// leaf message (32 zero bytes || column, lcpc-2d/src/lib.rs:736-775), so rank g can encode its
// rows and compute the chaining values of its chunks of every column by itself.  The exchanges
// (all on device buffers; with RCCL they are device-side sends / receives over xGMI):
//   commit (lib.rs:651-815)
//     A  all-to-all by column block: rank k receives every rank's chaining values of block k
//        (at cfg3 x 8 GPUs 2.4 MB per rank, instead of the 64 MiB codeword shard), merges them
//        into the block's leaves and builds the block's subtree;
//     B  all-gather of the subtrees: every rank assembles the whole tree (the bytes the
//        single-GPU commit holds) and the root;
//   prove (lib.rs:1034-1123), the Merlin transcript on one root rank
//     BC_r  broadcast of degree-test tensor r (then the column indices) from the root,
//     G_r   gather of the partial row combinations to the root, which folds them mod p and
//           absorbs the sum (RCCL has no mod-p reduction),
//     G_c   gather of the opened columns' row pieces; the root reads the paths off its tree.
// Every step's exchanges are one op kind of a generic "exchange group"; the pipelined driver
// (lcpc_sharded_commit_prove_many) puts the ops of several polynomials in flight into one group
// per tick, in a schedule fixed at launch so that every rank issues identical groups in identical
// order on one comm stream (RCCL ops that wait on peers therefore never deadlock against each
// other), while each polynomial's compute runs on its own stream and the root ranks' transcript
// absorption runs on host threads.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <array>
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <optional>

#include "host_internal.hpp"

using namespace lcpc;
using namespace lcpc_host;

namespace {

// ---------------------------------------------------------------- RCCL, loaded at first use
// (no link-time dependency: a process that never shards never loads it; a process where torch
// already loaded its librccl.so.1 shares that copy, same SONAME)
struct Rccl {
  bool ok = false;
  std::string err;
  decltype(&::ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&::ncclCommInitRank) CommInitRank = nullptr;
  decltype(&::ncclCommDestroy) CommDestroy = nullptr;
  decltype(&::ncclGetErrorString) GetErrorString = nullptr;
  decltype(&::ncclSend) Send = nullptr;
  decltype(&::ncclRecv) Recv = nullptr;
  decltype(&::ncclGroupStart) GroupStart = nullptr;
  decltype(&::ncclGroupEnd) GroupEnd = nullptr;
};

Rccl &rccl() {
  static Rccl r = [] {
    Rccl x;
    const char *name = getenv("LCPC_RCCL_LIB");
    void *h = dlopen(name && *name ? name : "librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      x.err = std::string("cannot load librccl.so.1: ") + dlerror();
      return x;
    }
#define SYM(f)                                                   \
  x.f = reinterpret_cast<decltype(x.f)>(dlsym(h, "nccl" #f));    \
  if (!x.f) {                                                    \
    x.err = "librccl.so.1 lacks nccl" #f;                        \
    return x;                                                    \
  }
    SYM(GetUniqueId) SYM(CommInitRank) SYM(CommDestroy) SYM(GetErrorString) SYM(Send) SYM(Recv)
    SYM(GroupStart) SYM(GroupEnd)
#undef SYM
    x.ok = true;
    return x;
  }();
  return r;
}

#define NCCL_TRY(expr)                                                                   \
  do {                                                                                   \
    ncclResult_t r__ = (expr);                                                           \
    if (r__ != ncclSuccess)                                                              \
      return fail(LCPC_ERR_DEVICE, std::string(#expr) + ": " + rccl().GetErrorString(r__)); \
  } while (0)

// ---------------------------------------------------------------- a small host task pool
// (the root rank's transcript work for several polynomials in flight)
class TaskPool {
 public:
  // dev >= 0: every worker makes that device current before its first task (a fresh thread's
  // current device is GPU 0, and the stages allocate from the device pool and launch there)
  explicit TaskPool(size_t n, int dev = -1) {
    for (size_t i = 0; i < n; i++)
      th_.emplace_back([this, dev] {
        if (dev >= 0) (void)hipSetDevice(dev);
        run();
      });
  }
  ~TaskPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : th_) t.join();
  }
  std::future<lcpc_status> submit(std::function<lcpc_status()> fn) {
    auto task = std::make_shared<std::packaged_task<lcpc_status()>>(std::move(fn));
    auto fut = task->get_future();
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.emplace_back([task] { (*task)(); });
    }
    cv_.notify_one();
    return fut;
  }

 private:
  void run() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      job();
    }
  }
  std::vector<std::thread> th_;
  std::deque<std::function<void()>> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

}  // namespace

// ---------------------------------------------------------------- the communicator
// What a communicator shares with its sharded commitments, refcounted so that either may be freed
// first: the comm stream (a commitment freed while an exchange of it is still queued fences its
// buffers on it) and the free list of per-(polynomial, stage) events.
struct CommShared {
  hipStream_t cs = nullptr;  // the comm stream: every exchange, in issue order
  std::mutex ev_mu;
  std::vector<hipEvent_t> ev_free;
  ~CommShared() {
    if (cs) {
      (void)hipStreamSynchronize(cs);
      (void)hipStreamDestroy(cs);
    }
    for (hipEvent_t e : ev_free) (void)hipEventDestroy(e);
  }
};

struct lcpc_comm {
  int nranks = 1, rank = 0;
  bool is_rccl = false;
  ncclComm_t nc = nullptr;
  lcpc_comm_ops ops{};
  Device *dev = nullptr;
  hipStream_t cs = nullptr;  // = shared->cs (owned by shared)
  std::shared_ptr<CommShared> shared = std::make_shared<CommShared>();
  std::mutex mu;             // one sharded call at a time
  // the pipelined driver's host threads (transcripts and proofs, compute launches, encodes),
  // started on its first call and kept across calls: idle between calls, joined last
  std::unique_ptr<TaskPool> pool, launch, encoder;
  ~lcpc_comm() {
    if (cs) (void)hipStreamSynchronize(cs);
    if (nc) rccl().CommDestroy(nc);
    // the stream and the event free list go with the last holder of `shared`
  }
};

namespace {

// One exchange of a group.  Device buffers; `ready` (optional) marks the device work that
// produces the send data.
struct Xop {
  enum Kind { ALL_GATHER, ALL_TO_ALL, BROADCAST } kind;
  const uint8_t *send = nullptr;
  uint8_t *recv = nullptr;  // BROADCAST: the buffer (send data on the root)
  size_t bytes = 0;         // ALL_GATHER: per rank; BROADCAST: total
  std::vector<size_t> sb, rb;  // ALL_TO_ALL: bytes to / from each rank
  int root = 0;
  hipEvent_t ready = nullptr;
  hipStream_t s = nullptr;  // the producing polynomial's compute stream
};

// One point-to-point transfer of an exchange group on rank `me` (G > 1).  RCCL matches the
// sends p -> q and the receives on q from p of one group in issue order, so a group is
// deadlock-free and moves the right bytes iff, for every ordered pair (p, q), p's sends to q and
// q's receives from p form the same sequence of sizes.  This list is the single source of the
// RCCL calls (run_group) and of the host-only schedule check (lcpc_sharded_p2p_schedule).
struct P2p {
  bool send;
  int peer;
  size_t op;  // index of the exchange in the group
  const uint8_t *sbuf;
  uint8_t *rbuf;
  size_t bytes;
};

std::vector<P2p> p2p_plan(int G, int me, const std::vector<Xop> &ops) {
  std::vector<P2p> v;
  for (size_t i = 0; i < ops.size(); i++) {
    const Xop &op = ops[i];
    switch (op.kind) {
      case Xop::ALL_GATHER:
        if (!op.bytes) break;
        for (int p = 0; p < G; p++) {
          if (p == me) continue;
          v.push_back({true, p, i, op.send, nullptr, op.bytes});
          v.push_back({false, p, i, nullptr, op.recv + (size_t)p * op.bytes, op.bytes});
        }
        break;
      case Xop::ALL_TO_ALL: {
        size_t so = 0, ro = 0;
        for (int p = 0; p < G; p++) {
          if (p != me) {
            if (op.sb[p]) v.push_back({true, p, i, op.send + so, nullptr, op.sb[p]});
            if (op.rb[p]) v.push_back({false, p, i, nullptr, op.recv + ro, op.rb[p]});
          }
          so += op.sb[p];
          ro += op.rb[p];
        }
        break;
      }
      case Xop::BROADCAST:
        if (!op.bytes) break;
        if (me == op.root) {
          for (int p = 0; p < G; p++)
            if (p != me) v.push_back({true, p, i, op.recv, nullptr, op.bytes});
        } else {
          v.push_back({false, op.root, i, nullptr, op.recv, op.bytes});
        }
        break;
    }
  }
  return v;
}

// Issues one group of exchanges on the comm stream; `done` events are recorded after it.
lcpc_status run_group(lcpc_comm *c, std::vector<Xop> &ops, const std::vector<hipEvent_t> &done) {
  const int G = c->nranks, me = c->rank;
  hipStream_t cs = c->cs;
  if (G == 1) {
    // one rank: nothing crosses a process, so each exchange is its own-piece copy on the
    // polynomial's stream (no comm stream: polynomials in flight do not wait for each other)
    // (an exchange whose receive buffer is its send buffer moves nothing)
    for (size_t i = 0; i < ops.size(); i++) {
      const Xop &op = ops[i];
      if (op.ready) HIP_TRY(hipStreamWaitEvent(op.s, op.ready, 0));
      if (op.kind == Xop::ALL_GATHER && op.bytes && op.recv != op.send)
        HIP_TRY(d2d(op.recv, op.send, op.bytes, op.s));
      if (op.kind == Xop::ALL_TO_ALL && op.rb[0] && op.recv != op.send)
        HIP_TRY(d2d(op.recv, op.send, op.rb[0], op.s));
      if (i < done.size()) HIP_TRY(hipEventRecord(done[i], op.s));
    }
    return LCPC_OK;
  }
  if (c->is_rccl) {
    for (auto &op : ops)
      if (op.ready) HIP_TRY(hipStreamWaitEvent(cs, op.ready, 0));
    // own pieces: device copies on the comm stream
    for (auto &op : ops) {
      if (op.kind == Xop::ALL_GATHER && op.bytes)
        HIP_TRY(d2d(op.recv + (size_t)me * op.bytes, op.send, op.bytes, cs));
      if (op.kind == Xop::ALL_TO_ALL && op.rb[me]) {
        size_t so = 0, ro = 0;
        for (int k = 0; k < me; k++) so += op.sb[k], ro += op.rb[k];
        HIP_TRY(d2d(op.recv + ro, op.send + so, op.rb[me], cs));
      }
    }
    Rccl &R = rccl();
    NCCL_TRY(R.GroupStart());
    {
      // an error between GroupStart and GroupEnd still closes the group (an open group on this
      // thread would swallow the next sharded call's exchanges)
      struct GroupGuard {
        Rccl &R;
        bool open = true;
        ~GroupGuard() {
          if (open) (void)R.GroupEnd();
        }
      } guard{R};
      for (const P2p &x : p2p_plan(G, me, ops)) {
        if (x.send) NCCL_TRY(R.Send(x.sbuf, x.bytes, ncclUint8, x.peer, c->nc, cs));
        else NCCL_TRY(R.Recv(x.rbuf, x.bytes, ncclUint8, x.peer, c->nc, cs));
      }
      guard.open = false;
      NCCL_TRY(R.GroupEnd());
    }
  } else {
    // caller-supplied collectives: synchronous on drained buffers
    for (auto &op : ops)
      if (op.ready) HIP_TRY(hipEventSynchronize(op.ready));
    HIP_TRY(hipStreamSynchronize(cs));
    for (auto &op : ops) {
      int rc = 0;
      switch (op.kind) {
        case Xop::ALL_GATHER:
          rc = c->ops.all_gather(c->ops.user, op.send, op.recv, op.bytes);
          break;
        case Xop::ALL_TO_ALL:
          rc = c->ops.all_to_all_v(c->ops.user, op.send, op.sb.data(), op.recv, op.rb.data());
          break;
        case Xop::BROADCAST:
          rc = c->ops.broadcast(c->ops.user, op.recv, op.bytes, op.root);
          break;
      }
      if (rc) return fail(LCPC_ERR_DEVICE, "caller-supplied collective failed (" + std::to_string(rc) + ")");
    }
  }
  for (hipEvent_t e : done) HIP_TRY(hipEventRecord(e, cs));
  return LCPC_OK;
}

// ---------------------------------------------------------------- partition
struct Part {
  size_t c_lo, c_hi, r_lo, r_hi;
};

size_t chunk_first_row(int fid, size_t chunk, size_t n_chunks, size_t n_rows) {
  if (chunk == 0) return 0;
  if (chunk >= n_chunks) return n_rows;
  const size_t wb = (size_t)field_bytes(fid);
  return std::min(n_rows, (1024 * chunk - 32 + wb - 1) / wb);
}

// A rank boundary must fall on a chunk boundary that is also an element boundary, so that every
// element of a rank's chunks is its own: chunk c (message byte 1024 c) qualifies iff
// (1024 c - 32) is a multiple of the element size -- every chunk for 8/16/32-byte elements, one
// chunk in three for Ft191's 24 bytes (c = 2 mod 3).  The qualifying boundaries cut the message
// into units that are dealt to the ranks evenly.
std::vector<Part> partition(int fid, size_t n_rows, int G) {
  const size_t nch = leaf_n_chunks(fid, n_rows), wb = (size_t)field_bytes(fid);
  std::vector<size_t> cuts{0};
  for (size_t c = 1; c < nch; c++)
    if ((1024 * c - 32) % wb == 0) cuts.push_back(c);
  cuts.push_back(nch);
  const size_t units = cuts.size() - 1;
  std::vector<Part> p(G);
  for (int g = 0; g < G; g++) {
    p[g].c_lo = cuts[(size_t)g * units / G];
    p[g].c_hi = cuts[(size_t)(g + 1) * units / G];
    p[g].r_lo = chunk_first_row(fid, p[g].c_lo, nch, n_rows);
    p[g].r_hi = chunk_first_row(fid, p[g].c_hi, nch, n_rows);
  }
  return p;
}

// pinned host block from the device pool
struct HostBuf {
  Device *d = nullptr;
  uint8_t *p = nullptr;
  HostBuf() = default;
  HostBuf(const HostBuf &) = delete;
  HostBuf &operator=(const HostBuf &) = delete;
  ~HostBuf() {
    if (p) d->pinned_put(p);
  }
  lcpc_status get(Device *dev, size_t n) {  // (any previous block: its copies have completed)
    if (p) d->pinned_put(p);
    d = dev;
    p = (uint8_t *)dev->pinned_get(n);
    return p ? LCPC_OK : fail(LCPC_ERR_OUT_OF_MEMORY, "pinned host staging");
  }
};

}  // namespace

// ---------------------------------------------------------------- one polynomial's shard state
// stages of one polynomial: 0 chaining values, 1 subtrees, 2 + 2r / 3 + 2r round r's tensor
// broadcast / partial gather, then the column indices and the column gather (make_sched); the
// proof-of-storage request's two gathers take the last two slots
constexpr size_t kMaxStages = 64;
enum EvKind { EV_READY = 0, EV_DONE = 1, EV_HOST = 2 };
constexpr size_t kPosEvalStage = kMaxStages - 2, kPosColsStage = kMaxStages - 1;
enum { S_CV = 0, S_SUB = 1, S_R0 = 2 };
constexpr size_t st_bcast(size_t r) { return S_R0 + 2 * r; }
constexpr size_t st_gather(size_t r) { return S_R0 + 2 * r + 1; }

struct lcpc_sharded_commit {
  const lcpc_encoding *e = nullptr;
  lcpc_comm *comm = nullptr;              // (only during the calls that take it)
  std::shared_ptr<CommShared> shared;     // its comm stream and event free list (outlive it if need be)
  Device *dev = nullptr;
  int fid = 1, wb = 16, G = 1, me = 0;
  bool sdig = false;  // Brakedown: element-major shard [n_cols][nr] (canonical codeword, as Ligero's)
  size_t n_rows = 0, np = 0, nc = 0, np2 = 0, B = 0, n_chunks = 0, nr = 0;  // np2 leaves, B = np2 / G
  std::vector<Part> part;
  hipStream_t s = nullptr;        // this polynomial's encode stream (shared, in order, by the
                                  // pipelined driver's polynomials: encodes finish first come first)
  bool own_s = true;              // s is this polynomial's own (released with it)
  hipStream_t sp = nullptr;       // its exchange-side and prove stream (short kernels, beside the encodes)
  // One event per (stage, edge), recorded at most once per call: EV_READY = the stage's send data
  // written (producer stream -> comm stream), EV_DONE = the stage's exchange completed (comm
  // stream -> consumer stream), EV_HOST = the stage's device -> host copies landed.  No event is
  // re-recorded while a wait on an earlier record of it may still be queued (the pattern the
  // round-3 eight-rank wrong-root failure pointed at; DESIGN.md §6, "Hand-offs").  Created when a
  // call first needs a stage (ev_need), returned to the communicator's free list with the
  // polynomial once every wait on them has retired (ev_quiet), destroyed otherwise.
  std::array<hipEvent_t, 3 * kMaxStages> ev{};
  bool ev_quiet = true;  // no exchange of this polynomial is outstanding on the comm stream
  DBuf coeffs, comm_rows, hashes;  // kept for prove
  DBuf cv_send, cv_recv, sub, subs, sdig_tmp;  // commit scratch
  uint8_t root[32] = {0};
  const void *d_rows = nullptr;  // the caller's rows (LCPC_SHARD_DEBUG's recomputation)
  uint64_t rows_fnv = 0;         // (LCPC_SHARD_DEBUG) their digest when the encode was issued
  size_t poly = 0;               // index in a pipelined call (LCPC_SHARD_DEBUG)
  // prove state
  int root_rank = 0;
  size_t ndt = 0, nco = 0, rounds = 0;
  lcpc_transcript *tr = nullptr;
  bool own_tr = false;
  DBuf bt, tens, part_d, allpart, sum, canon, didx, mycols, allcols, dpaths, scratch;
  HostBuf h_root, h_t, h_sum, h_repr, h_repr_eval, h_idx, h_cols, h_paths, h_outer;
  std::vector<uint64_t> p_random, p_eval, col_idx;
  std::future<lcpc_status> next;  // root rank: the next challenge vector is in h_t / h_idx
  ~lcpc_sharded_commit() {
    if (s && own_s) (void)hipStreamSynchronize(s);
    if (sp && sp != s) (void)hipStreamSynchronize(sp);
    if (own_tr) delete tr;
    std::vector<hipEvent_t> mine;
    for (hipEvent_t &x : ev)
      if (x) mine.push_back(x), x = nullptr;
    if (!mine.empty()) {
      if (shared && ev_quiet) {
        std::lock_guard<std::mutex> lk(shared->ev_mu);
        shared->ev_free.insert(shared->ev_free.end(), mine.begin(), mine.end());
      } else {
        for (hipEvent_t x : mine) (void)hipEventDestroy(x);  // (HIP keeps a queued wait's marker alive)
      }
    }
    // DBufs drain s in their destructors (declared after s, destroyed before it is released)
  }
};

namespace {

// Each polynomial's exchange-side and prove kernels run on a stream of their own beside the
// shared in-order encode stream and the comm stream, ordered against them by cross-stream event
// waits alone.  All three are at ONE priority (the device's, Device::stream_priority).  With
// high-priority prove streams over normal-priority encode / comm streams (round 3's mode 2) eight
// ranks sharing one GPU produced a wrong commitment root for one of the later polynomials in about
// one run in four (tests/test_gpu_shard_native.py::test_native_pipeline_world8_rccl_one_gpu); at
// one priority it never did.  Round 5 removed the mixed mode.
bool shard_prio_streams() { return true; }
// encode streams of the pipelined driver, taken in turn by polynomial: with two, consecutive
// polynomials' encode kernels overlap each other's tails (one-rank K = 20: 11.1 / 11.5 against
// 11.0 / 11.3 G/s with one, interleaved runs, profiles/r04_sharded_bulk_streams_ab.json) while the
// roots still arrive nearly in order
// (LCPC_SHARD_BULK_STREAMS=1..4 overrides the count for A/B runs)
constexpr size_t SHARD_BULK_STREAMS = 2, SHARD_BULK_MAX = 4;
size_t shard_bulk_streams() {
  static const size_t v = [] {
    const char *e = getenv("LCPC_SHARD_BULK_STREAMS");
    const long n = e ? strtol(e, nullptr, 10) : 0;
    return (n >= 1 && n <= (long)SHARD_BULK_MAX) ? (size_t)n : SHARD_BULK_STREAMS;
  }();
  return v;
}
// the pool every stream of the sharded driver comes from (Device::acquire_stream): the
// latency-side pool POOL_HIGH (verify, openings, this driver), apart from lcpc_prove's POOL_PROVER;
// its priority equals the bulk pool's unless LCPC_PRIORITY_STREAMS=1
constexpr StreamPool kShardPool = POOL_HIGH;

struct ShardDeleter {
  void operator()(lcpc_sharded_commit *c) const {
    if (!c) return;
    hipStream_t s = c->own_s ? c->s : nullptr, sp = c->sp != c->s ? c->sp : nullptr;
    Device *d = c->dev;
    c->s = nullptr;
    c->sp = nullptr;
    if (s) (void)hipStreamSynchronize(s);
    if (sp) (void)hipStreamSynchronize(sp);
    // s and sp have drained: their uses need no fence.  An exchange of this polynomial may still
    // be queued on the comm stream when it is torn down early (an error path: !ev_quiet), so then
    // every buffer is fenced on that stream: the pool orders the block's next owner after it
    // (pool.hpp) without blocking here.
    hipStream_t cs = !c->ev_quiet && c->shared ? c->shared->cs : nullptr;
    for (DBuf *b : {&c->coeffs, &c->comm_rows, &c->hashes, &c->cv_send, &c->cv_recv, &c->sub, &c->subs, &c->sdig_tmp,
                    &c->bt, &c->tens, &c->part_d, &c->allpart, &c->sum, &c->canon, &c->didx, &c->mycols,
                    &c->allcols, &c->dpaths, &c->scratch}) {
      b->settle();
      if (cs) b->use(cs);
    }
    delete c;
    if (s) d->release_stream(s, kShardPool);
    if (sp) d->release_stream(sp, kShardPool);
  }
};
using ShardPtr = std::unique_ptr<lcpc_sharded_commit, ShardDeleter>;

// the shape conditions of a row-sharded commitment (no device needed)
lcpc_status check_geom(int fid, int kind, size_t n_cols, int G, size_t n_rows) {
  if (kind != KIND_RS && kind != KIND_SDIG) return fail(LCPC_ERR_UNSUPPORTED, "row shards: unknown encoding");
  if (G < 1 || (G & (G - 1)) || next_pow2(n_cols) % (size_t)G)
    return fail(LCPC_ERR_UNSUPPORTED, "row shards need a power-of-two rank count of at most next_pow2(n_cols)");
  if (n_rows == 0) return fail(LCPC_ERR_INVALID_ARG, "n_rows");
  return LCPC_OK;
}

lcpc_status check_shardable(const lcpc_encoding *e, lcpc_comm *comm, size_t n_rows) {
  if (!e || !comm) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  lcpc_status st = check_geom(e->fid, e->kind, e->n_cols, comm->nranks, n_rows);
  if (st) return st;
  if (comm->dev != e->dev) return fail(LCPC_ERR_INVALID_ARG, "comm and encoding on different devices");
  return LCPC_OK;
}

// the partition and sizes every exchange descriptor reads (host only)
void shard_geom(lcpc_sharded_commit *c, int fid, size_t np, size_t nc, size_t n_rows, int G, int me,
                bool sdig = false) {
  c->sdig = sdig;
  c->fid = fid;
  c->wb = field_bytes(fid);
  c->G = G;
  c->me = me;
  c->n_rows = n_rows;
  c->np = np;
  c->nc = nc;
  c->np2 = next_pow2(nc);  // the Merkle tree's leaves: columns, then zero digests (SDIG)
  c->B = c->np2 / G;
  c->n_chunks = leaf_n_chunks(fid, n_rows);
  c->part = partition(fid, n_rows, G);
  c->nr = c->part[me].r_hi - c->part[me].r_lo;
}

// the prove-side sizes (n_degree_tests / n_col_opens of the encoding passed to prove,
// lcpc-2d/src/lib.rs:1053,1101)
void prove_geom(lcpc_sharded_commit *c, size_t ndt, size_t nco, int root_rank) {
  c->root_rank = root_rank;
  c->ndt = ndt;
  c->nco = nco;
  c->rounds = std::max<size_t>(ndt, 1);
}

// bulk: a stream the caller owns for the encode (the pipelined driver's shared one), or null for
// a stream of this commitment's own
lcpc_status ev_need(lcpc_sharded_commit *c, size_t s0, size_t s1);

lcpc_status shard_init(const lcpc_encoding *e, lcpc_comm *comm, size_t n_rows, ShardPtr &out,
                       hipStream_t bulk = nullptr) {
  ShardPtr c(new lcpc_sharded_commit());
  c->e = e;
  c->comm = comm;
  c->shared = comm->shared;
  c->dev = e->dev;
  shard_geom(c.get(), e->fid, e->n_per_row, e->n_cols, n_rows, comm->nranks, comm->rank, e->kind == KIND_SDIG);
  HIP_TRY(hipSetDevice(c->dev->id));
  c->own_s = bulk == nullptr;
  c->s = bulk ? bulk : c->dev->acquire_stream(kShardPool);
  if (!c->s) return fail(LCPC_ERR_DEVICE, "no HIP stream");
  c->sp = shard_prio_streams() ? c->dev->acquire_stream(kShardPool) : c->s;
  if (!c->sp) return fail(LCPC_ERR_DEVICE, "no HIP stream");
  out = std::move(c);
  return ev_need(out.get(), 0, 2);  // (the commit's stages: chaining values, subtrees)
}

// DBuf allocations drain the polynomial's stream (not the caller's lease) when released: the
// commit stream for the commit's buffers, the prove stream for the prove's
hipError_t salloc_on(lcpc_sharded_commit *c, DBuf &b, size_t bytes, hipStream_t s) {
  hipStream_t prev = t_stream;
  t_stream = s;
  hipError_t e = b.alloc(c->dev, bytes);
  t_stream = prev;
  return e;
}
hipError_t salloc(lcpc_sharded_commit *c, DBuf &b, size_t bytes) { return salloc_on(c, b, bytes, c->s); }
hipError_t salloc_p(lcpc_sharded_commit *c, DBuf &b, size_t bytes) { return salloc_on(c, b, bytes, c->sp); }

// ---- per-(stage, edge) events
// the event of stage s's edge `k` (created by ev_need before the call's first use)
hipEvent_t EV(const lcpc_sharded_commit *c, EvKind k, size_t s) { return c->ev[3 * s + k]; }

// make sure the three events of stages [s0, s1) exist (from the communicator's free list first)
lcpc_status ev_need(lcpc_sharded_commit *c, size_t s0, size_t s1) {
  if (s1 > kMaxStages) return fail(LCPC_ERR_UNSUPPORTED, "row shards: too many prove stages");
  for (size_t i = 3 * s0; i < 3 * s1; i++) {
    if (c->ev[i]) continue;
    {
      std::lock_guard<std::mutex> lk(c->shared->ev_mu);
      if (!c->shared->ev_free.empty()) {
        c->ev[i] = c->shared->ev_free.back();
        c->shared->ev_free.pop_back();
        continue;
      }
    }
    HIP_TRY(hipEventCreateWithFlags(&c->ev[i], hipEventDisableTiming));
  }
  return LCPC_OK;
}

// ---- commit
// encode this rank's rows (the first NTT pass writes the commitment's own coefficient copy),
// chaining values of its chunks of every column, laid out [dest rank][chunk][block col]
bool shard_debug();
uint64_t debug_fnv_device(const void *d, size_t n);

lcpc_status stage_pre_commit(lcpc_sharded_commit *c, const void *d_rows) {
  const Part &pm = c->part[c->me];
  const size_t nch = pm.c_hi - pm.c_lo, wb = c->wb;
  HIP_TRY(salloc(c, c->coeffs, c->nr * c->np * wb + 16));
  HIP_TRY(salloc(c, c->comm_rows, c->nr * c->nc * wb + 16));
  HIP_TRY(salloc(c, c->cv_send, nch * c->np2 * 32 + 16));
  if (c->G > 1) HIP_TRY(salloc(c, c->cv_recv, c->n_chunks * c->B * 32 + 16));  // (one rank: cv_send itself)
  if (c->nr && !d_rows) return fail(LCPC_ERR_INVALID_ARG, "null rows");
  c->d_rows = d_rows;
  if (shard_debug() && c->nr) c->rows_fnv = debug_fnv_device(d_rows, c->nr * c->np * c->wb);
  if (c->nr && c->sdig) {
    // Brakedown rows (lcpc-brakedown-pc/src/encode.rs:36-94, independent per row): this rank's
    // rows transposed to the element-major shard [n_cols][nr] as canonical values (one pass also
    // writes the padded row-major Montgomery coefficient copy), then the expander levels on those
    // rows -- canonical in, canonical out, as the single-GPU commit (csrc/lcpc_host.cpp)
    HIP_TRY(transpose_elems(c->fid, (const uint32_t *)d_rows, c->nr, c->np, c->np, c->np,
                            c->comm_rows.as<uint32_t>(), c->nr, c->s, TR_FROM_MONT, nullptr, c->nr * c->np,
                            c->coeffs.as<uint32_t>(), c->np));
    HIP_TRY(salloc(c, c->sdig_tmp, c->e->sdig.tmp_elems * c->nr * wb + 16));
    HIP_TRY(sdig_encode_cm(c->e->sdig, c->comm_rows.as<uint32_t>(), c->nr, c->sdig_tmp.as<uint32_t>(), c->s));
  } else if (c->nr) {
    HIP_TRY(ntt_rows(c->e->plan, (const uint32_t *)d_rows, c->np, c->np, c->comm_rows.as<uint32_t>(), c->nc, c->nr,
                     c->s, c->coeffs.as<uint32_t>(), c->np, true));
  }
  if (nch)  // chaining values straight into the exchange layout [dest rank][chunk][block col]
    HIP_TRY(leaf_chunk_cvs(c->fid, c->comm_rows.as<uint32_t>(), pm.r_lo, c->n_rows, c->nc, c->sdig ? 1 : c->nc,
                           pm.c_lo, pm.c_hi, c->cv_send.as<uint32_t>(), c->s, true, c->B,
                           c->sdig ? c->nr : 1));
  HIP_TRY(hipEventRecord(EV(c, EV_READY, S_CV), c->s));
  return LCPC_OK;
}

Xop op_cv_exchange(lcpc_sharded_commit *c) {
  Xop op{Xop::ALL_TO_ALL};
  const size_t nch_me = c->part[c->me].c_hi - c->part[c->me].c_lo;
  op.send = c->cv_send.as<uint8_t>();
  op.recv = c->G > 1 ? c->cv_recv.as<uint8_t>() : c->cv_send.as<uint8_t>();
  op.sb.assign(c->G, nch_me * c->B * 32);
  op.rb.resize(c->G);
  for (int k = 0; k < c->G; k++) op.rb[k] = (c->part[k].c_hi - c->part[k].c_lo) * c->B * 32;
  op.ready = EV(c, EV_READY, S_CV);
  op.s = c->sp;  // (one rank: where the post stage waits for the encode)
  return op;
}

// leaves of my column block from all chunks' chaining values, and the block's subtree (the
// commit's short latency-critical kernels go on the prove stream, ahead of bulk encodes)
lcpc_status stage_post_cv(lcpc_sharded_commit *c) {
  HIP_TRY(hipStreamWaitEvent(c->sp, EV(c, EV_DONE, S_CV), 0));
  HIP_TRY(salloc_p(c, c->sub, (2 * c->B - 1) * 32));
  uint32_t *cvs = (c->G > 1 ? c->cv_recv : c->cv_send).as<uint32_t>();
  HIP_TRY(leaves_from_cvs(cvs, c->B, (int)c->n_chunks, c->sub.as<uint8_t>(), c->sp));
  // leaves past n_cols are zero digests (lcpc-2d/src/lib.rs:685-697; SDIG's n_cols is no power of 2)
  const size_t b0 = (size_t)c->me * c->B, valid = c->nc > b0 ? std::min(c->B, c->nc - b0) : 0;
  if (valid < c->B) HIP_TRY(hipMemsetAsync(c->sub.as<uint8_t>() + valid * 32, 0, (c->B - valid) * 32, c->sp));
  if (c->B > 1) HIP_TRY(merkle_tree(c->sub.as<uint8_t>(), c->B, c->sp));
  if (c->G > 1) HIP_TRY(salloc_p(c, c->subs, (size_t)c->G * (2 * c->B - 1) * 32));  // (one rank: sub itself)
  HIP_TRY(hipEventRecord(EV(c, EV_READY, S_SUB), c->sp));
  return LCPC_OK;
}

Xop op_subtree_exchange(lcpc_sharded_commit *c) {
  Xop op{Xop::ALL_GATHER};
  op.send = c->sub.as<uint8_t>();
  op.recv = (c->G > 1 ? c->subs : c->sub).as<uint8_t>();
  op.bytes = (2 * c->B - 1) * 32;
  op.ready = EV(c, EV_READY, S_SUB);
  op.s = c->sp;
  return op;
}

// every rank: the whole tree [leaves | level 1 | ... | root] from the G subtrees + top levels
lcpc_status stage_post_subtrees(lcpc_sharded_commit *c) {
  HIP_TRY(hipStreamWaitEvent(c->sp, EV(c, EV_DONE, S_SUB), 0));
  const size_t nc = c->np2, B = c->B, G = c->G;  // (the tree's leaf count)
  HIP_TRY(salloc_p(c, c->hashes, (2 * nc - 1) * 32));
  uint8_t *h = c->hashes.as<uint8_t>();
  HIP_TRY(assemble_subtrees((G > 1 ? c->subs : c->sub).as<uint8_t>(), B, G, h, c->sp));  // one launch, every level
  if (G > 1) HIP_TRY(merkle_tree_io(h + (2 * nc - 2 * G) * 32, G, h + (2 * nc - G) * 32, c->sp));
  lcpc_status st = c->h_root.get(c->dev, 32);
  if (st) return st;
  HIP_TRY(d2h(c->h_root.p, h + (2 * nc - 2) * 32, 32, c->sp));
  HIP_TRY(hipEventRecord(EV(c, EV_HOST, S_SUB), c->sp));
  return LCPC_OK;
}

// LCPC_SHARD_DEBUG=1 (diagnostic runs only): once a commitment's root is on the host, recompute
// this rank's encode and chunk chaining values from its rows on a private stream and print, per
// (rank, polynomial), whether the codeword shard and the sent chaining values match, with the
// first words of this rank's subtree root and of every gathered subtree: localises a wrong root
// to the encode, the chaining values, the exchange, or the subtree stage.
bool shard_debug() {
  static const bool v = [] {
    const char *e = getenv("LCPC_SHARD_DEBUG");
    return e && e[0] == '1';
  }();
  return v;
}

uint64_t debug_fnv(const uint8_t *p, size_t n) {
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

uint64_t debug_fnv_device(const void *d, size_t n) {
  std::vector<uint8_t> h(n);
  if (n) (void)hipMemcpy(h.data(), d, n, hipMemcpyDeviceToHost);
  return debug_fnv(h.data(), n);
}

void debug_commit(lcpc_sharded_commit *c) {
  if (c->sdig || c->G == 1) return;
  auto fetch = [](const void *d, size_t n) {
    std::vector<uint8_t> h(n);
    if (n) (void)hipMemcpy(h.data(), d, n, hipMemcpyDeviceToHost);
    return h;
  };
  const Part &pm = c->part[c->me];
  const size_t nch = pm.c_hi - pm.c_lo, wb = c->wb;
  const size_t cvb = nch * c->np2 * 32;
  hipStream_t ds = nullptr;
  (void)hipStreamCreateWithFlags(&ds, hipStreamNonBlocking);
  void *tc = nullptr, *tk = nullptr, *tv = nullptr;
  (void)hipMalloc(&tc, c->nr * c->nc * wb + 16);
  (void)hipMalloc(&tk, c->nr * c->np * wb + 16);
  (void)hipMalloc(&tv, cvb + 16);
  if (c->nr)
    (void)ntt_rows(c->e->plan, (const uint32_t *)c->d_rows, c->np, c->np, (uint32_t *)tc, c->nc, c->nr, ds,
                   (uint32_t *)tk, c->np, true);
  if (nch)
    (void)leaf_chunk_cvs(c->fid, (const uint32_t *)tc, pm.r_lo, c->n_rows, c->nc, c->nc, pm.c_lo, pm.c_hi,
                         (uint32_t *)tv, ds, true, c->B, 1);
  (void)hipStreamSynchronize(ds);
  const auto rows = fetch(c->comm_rows.p, c->nr * c->nc * wb), rows2 = fetch(tc, c->nr * c->nc * wb);
  // a second recomputation, and the input rows' digest against the one taken at issue time
  if (c->nr) {
    (void)hipMemsetAsync(tc, 0, c->nr * c->nc * wb, ds);
    (void)ntt_rows(c->e->plan, (const uint32_t *)c->d_rows, c->np, c->np, (uint32_t *)tc, c->nc, c->nr, ds,
                   (uint32_t *)tk, c->np, true);
    (void)hipStreamSynchronize(ds);
  }
  const auto rows3 = fetch(tc, c->nr * c->nc * wb);
  const bool input_same = !c->nr || debug_fnv_device(c->d_rows, c->nr * c->np * wb) == c->rows_fnv;
  // where the production codeword differs: element count, rows touched, first / last (row, col)
  std::string where;
  if (rows != rows2) {
    size_t cnt = 0, first = SIZE_MAX, last = 0, nrows_hit = 0, prev_row = SIZE_MAX;
    for (size_t i = 0; i < c->nr * c->nc; i++)
      if (std::memcmp(rows.data() + i * wb, rows2.data() + i * wb, wb)) {
        cnt++;
        first = std::min(first, i);
        last = i;
        if (i / c->nc != prev_row) nrows_hit++, prev_row = i / c->nc;
      }
    char b[200];
    snprintf(b, sizeof b, " [%zu elements differ in %zu rows, first (%zu,%zu) last (%zu,%zu)]", cnt, nrows_hit,
             first / c->nc, first % c->nc, last / c->nc, last % c->nc);
    where = b;
  }
  const auto cvs = fetch(c->cv_send.p, cvb), cvs2 = fetch(tv, cvb);
  const auto sub = fetch(c->sub.p, (2 * c->B - 1) * 32);
  const auto subs = fetch(c->subs.p, (size_t)c->G * (2 * c->B - 1) * 32);
  std::string per_dest;
  for (int q = 0; q < c->G; q++) {
    const size_t o = (size_t)q * nch * c->B * 32, n = nch * c->B * 32;
    per_dest += std::memcmp(cvs.data() + o, cvs2.data() + o, n) ? "X" : ".";
  }
  auto w4 = [](const uint8_t *p) {
    char b[9];
    snprintf(b, sizeof b, "%02x%02x%02x%02x", p[0], p[1], p[2], p[3]);
    return std::string(b);
  };
  std::string gathered;
  for (int q = 0; q < c->G; q++) gathered += " " + w4(subs.data() + ((size_t)q * (2 * c->B - 1) + 2 * c->B - 2) * 32);
  fprintf(stderr,
          "liblcpc_mi dbg: rank %d poly %zu rows %s%s cv_send %s (per dest %s) recompute2 %s input %s sub %s "
          "gathered%s root %s\n",
          c->me, c->poly, rows == rows2 ? "ok" : "DIFF", where.c_str(), cvs == cvs2 ? "ok" : "DIFF", per_dest.c_str(),
          rows3 == rows2 ? "same" : "DIFFERS", input_same ? "unchanged" : "CHANGED",
          w4(sub.data() + (2 * c->B - 2) * 32).c_str(), gathered.c_str(), w4(c->root).c_str());
  fflush(stderr);
  (void)hipFree(tc);
  (void)hipFree(tk);
  (void)hipFree(tv);
  (void)hipStreamDestroy(ds);
}

// commit scratch no longer needed once the root is known
lcpc_status finish_commit(lcpc_sharded_commit *c) {
  HIP_TRY(hipEventSynchronize(EV(c, EV_HOST, S_SUB)));
  c->ev_quiet = true;  // (every exchange of the commit precedes it)
  std::memcpy(c->root, c->h_root.p, 32);
  if (shard_debug()) debug_commit(c);
  // every use of the commit scratch precedes the subtree stage's EV_HOST: no drain on release
  for (DBuf *b : {&c->cv_send, &c->cv_recv, &c->sub, &c->subs, &c->sdig_tmp}) b->settle();
  c->sdig_tmp.reset();
  c->cv_send.reset();
  c->cv_recv.reset();
  c->sub.reset();
  c->subs.reset();
  return LCPC_OK;
}

// ---- prove
// buffers, pinned staging and this rank's slice of the outer tensor (no transcript needed: the
// pipelined driver does this on a launch worker while the commit is still running)
lcpc_status prove_alloc(lcpc_sharded_commit *c, const uint64_t *outer, int root_rank, const lcpc_encoding *pe) {
  prove_geom(c, pe->n_degree_tests, pe->n_col_opens, root_rank);
  const size_t wb = c->wb, np = c->np;
  lcpc_status st;
  if ((st = ev_need(c, S_R0, S_R0 + 2 * c->rounds + 2))) return st;
  HIP_TRY(salloc_p(c, c->bt, c->n_rows * wb));
  HIP_TRY(salloc_p(c, c->tens, 2 * std::max<size_t>(c->nr, 1) * wb));
  HIP_TRY(salloc_p(c, c->part_d, 2 * np * wb));
  HIP_TRY(salloc_p(c, c->scratch, collapse_scratch_bytes(c->fid, std::max<size_t>(c->nr, 1), np, 2)));
  HIP_TRY(salloc_p(c, c->didx, std::max<size_t>(c->nco, 1) * 8));
  HIP_TRY(salloc_p(c, c->mycols, std::max<size_t>(c->nco * c->nr, 1) * wb));
  // the outer tensor's slice (host -> device once per proof)
  if ((st = c->h_t.get(c->dev, c->n_rows * wb))) return st;
  if ((st = c->h_idx.get(c->dev, std::max<size_t>(c->nco, 1) * 8))) return st;
  if (c->nr) {  // (h_outer lives until the proof is released, so the copy needs no drain here)
    if ((st = c->h_outer.get(c->dev, c->nr * wb))) return st;
    std::memcpy(c->h_outer.p, (const uint8_t *)outer + c->part[c->me].r_lo * wb, c->nr * wb);
    HIP_TRY(h2d(c->tens.as<uint8_t>() + c->nr * wb, c->h_outer.p, c->nr * wb, c->sp));
  }
  if (c->me == root_rank) {
    HIP_TRY(salloc_p(c, c->allpart, (size_t)c->G * 2 * np * wb));
    HIP_TRY(salloc_p(c, c->sum, 2 * np * wb));
    HIP_TRY(salloc_p(c, c->canon, 2 * np * wb));
    size_t all_rows = c->n_rows;
    HIP_TRY(salloc_p(c, c->allcols, std::max<size_t>(c->nco * all_rows, 1) * wb));
    HIP_TRY(salloc_p(c, c->dpaths, std::max<size_t>(c->nco * log2_np2(c->nc), 1) * 32));
    if ((st = c->h_sum.get(c->dev, 2 * np * wb))) return st;
    if ((st = c->h_repr.get(c->dev, 2 * np * wb))) return st;
    if ((st = c->h_repr_eval.get(c->dev, np * wb))) return st;
    if ((st = c->h_cols.get(c->dev, std::max<size_t>(c->nco * all_rows, 1) * wb))) return st;
    if ((st = c->h_paths.get(c->dev, std::max<size_t>(c->nco * log2_np2(c->nc), 1) * 32))) return st;
    c->p_random.resize(c->ndt * np * (wb / 8));
    c->p_eval.resize(np * (wb / 8));
  }
  // The buffers above were taken on sp: a reused pool block's fence wait is queued there.  Two of
  // them are first written on the comm stream instead -- bt (the root's challenge upload and the
  // tensor broadcast) and didx (the index upload and broadcast) -- so those writes wait on this
  // record, which follows every take (the ordering lcpc_sharded_pos_request gets by taking its
  // gather buffer before its READY record)
  HIP_TRY(hipEventRecord(EV(c, EV_READY, st_bcast(0)), c->sp));
  return LCPC_OK;
}

// the comm-stream writers of bt / didx wait for the prove buffers' takes (prove_alloc)
hipEvent_t prove_taken(lcpc_sharded_commit *c) { return EV(c, EV_READY, st_bcast(0)); }

lcpc_status prove_init(lcpc_sharded_commit *c, const uint64_t *outer, int root_rank, const lcpc_encoding *pe,
                       lcpc_transcript *tr, bool own_tr) {
  c->tr = tr;
  c->own_tr = own_tr;
  return prove_alloc(c, outer, root_rank, pe);
}

// root rank, host: the first challenge (degree-test tensor 0, or the column choice if there
// are no degree tests and no... -- with n_degree_tests = 0 round 0 is the evaluation alone)
lcpc_status challenge_first(lcpc_sharded_commit *c) {
  if (c->ndt) {
    std::vector<uint64_t> t;
    challenge_tensor(*c->tr, c->fid, c->n_rows, t);
    std::memcpy(c->h_t.p, t.data(), c->n_rows * c->wb);
  }
  return LCPC_OK;
}

int round_tensors(const lcpc_sharded_commit *c, size_t r) { return (r == 0 && c->ndt) ? 2 : 1; }

Xop op_tensor_bcast(lcpc_sharded_commit *c, size_t r) {
  // round r's challenge vector (round 0 without degree tests has none: a zero-byte broadcast)
  Xop op{Xop::BROADCAST};
  op.recv = c->bt.as<uint8_t>();
  op.bytes = (r < c->ndt) ? c->n_rows * c->wb : 0;
  op.root = c->root_rank;
  op.s = c->sp;
  op.ready = prove_taken(c);
  return op;
}

// the root's host -> device challenge copies go on the stream its exchanges run on
hipStream_t upload_stream(const lcpc_sharded_commit *c) { return c->G == 1 ? c->sp : c->comm->cs; }

// root: the challenge vector onto the comm stream before the exchange group is issued
lcpc_status stage_tensor_upload(lcpc_sharded_commit *c, size_t r) {
  if (c->me != c->root_rank || r >= c->ndt) return LCPC_OK;
  HIP_TRY(hipStreamWaitEvent(upload_stream(c), prove_taken(c), 0));
  HIP_TRY(h2d(c->bt.p, c->h_t.p, c->n_rows * c->wb, upload_stream(c)));
  return LCPC_OK;
}

// partial row combinations over my rows: [t_r slice | outer slice] (round 0) or t_r slice
lcpc_status stage_collapse(lcpc_sharded_commit *c, size_t r) {
  HIP_TRY(hipStreamWaitEvent(c->sp, EV(c, EV_DONE, st_bcast(r)), 0));
  const size_t wb = c->wb, np = c->np, nr = c->nr;
  const int nt = round_tensors(c, r);
  const bool eval_only = c->ndt == 0;  // round 0 = the evaluation tensor alone
  if (nr == 0) {
    HIP_TRY(hipMemsetAsync(c->part_d.p, 0, nt * np * wb, c->sp));
  } else {
    const uint32_t *tens = c->tens.as<uint32_t>();
    if (!eval_only) {
      HIP_TRY(d2d(c->tens.p, c->bt.as<uint8_t>() + c->part[c->me].r_lo * wb, nr * wb, c->sp));
    } else {
      tens = (const uint32_t *)(c->tens.as<uint8_t>() + nr * wb);
    }
    HIP_TRY(collapse_rows(c->fid, c->coeffs.as<uint32_t>(), nr, np, tens, nt, c->part_d.as<uint32_t>(), c->scratch.p,
                          c->sp));
  }
  HIP_TRY(hipEventRecord(EV(c, EV_READY, st_gather(r)), c->sp));
  return LCPC_OK;
}

Xop op_partial_gather(lcpc_sharded_commit *c, size_t r) {
  Xop op{Xop::ALL_TO_ALL};
  const size_t bytes = (size_t)round_tensors(c, r) * c->np * c->wb;
  op.send = c->part_d.as<uint8_t>();
  op.recv = c->me == c->root_rank ? c->allpart.as<uint8_t>() : nullptr;
  op.sb.assign(c->G, 0);
  op.rb.assign(c->G, 0);
  op.sb[c->root_rank] = bytes;
  if (c->me == c->root_rank) op.rb.assign(c->G, bytes);
  op.ready = EV(c, EV_READY, st_gather(r));
  op.s = c->sp;
  return op;
}

// root: fold the G partials mod p; Montgomery sums (the proof) and canonical reprs (the
// transcript) to the host
lcpc_status stage_fold(lcpc_sharded_commit *c, size_t r) {
  if (c->me != c->root_rank) return LCPC_OK;
  HIP_TRY(hipStreamWaitEvent(c->sp, EV(c, EV_DONE, st_gather(r)), 0));
  const size_t wb = c->wb, np = c->np;
  const size_t len = (size_t)round_tensors(c, r) * np;
  HIP_TRY(collapse_fold_rows(c->fid, c->allpart.as<uint32_t>(), c->G, len, c->sum.as<uint32_t>(), c->sp));
  HIP_TRY(convert(c->fid, c->sum.as<uint32_t>(), c->canon.as<uint32_t>(), len, false, c->sp));
  HIP_TRY(d2h(c->h_sum.p, c->sum.p, len * wb, c->sp));
  HIP_TRY(d2h(c->h_repr.p, c->canon.p, len * wb, c->sp));
  HIP_TRY(hipEventRecord(EV(c, EV_HOST, st_gather(r)), c->sp));
  return LCPC_OK;
}

void repr_order(int fid, uint8_t *h, size_t n, int wb) {
  if (fid == LCPC_FT253_192)  // PrimeFieldReprEndianness = "big" (ft253_192.rs:9)
    for (size_t i = 0; i < n; i++) std::reverse(h + i * wb, h + (i + 1) * wb);
}

// root, host: absorb round r's row combination(s) (lib.rs:1075-1077, 1096-1098) and draw the
// next challenge: tensor r + 1 (:1056-1062) or, after the last round, the columns (:1101-1110)
lcpc_status host_absorb(lcpc_sharded_commit *c, size_t r) {
  {
    prof::HostScope hs("host_absorb_wait");
    HIP_TRY(hipEventSynchronize(EV(c, EV_HOST, st_gather(r))));
  }
  const size_t wb = c->wb, np = c->np, limbs = wb / 8;
  uint8_t *repr = c->h_repr.p;
  repr_order(c->fid, repr, (size_t)round_tensors(c, r) * np, (int)wb);
  if (c->ndt == 0) {  // the evaluation round
    std::memcpy(c->p_eval.data(), c->h_sum.p, np * wb);
    std::memcpy(c->h_repr_eval.p, repr, np * wb);
  } else {
    std::memcpy(c->p_random.data() + r * np * limbs, c->h_sum.p, np * wb);
    if (r == 0) {
      std::memcpy(c->p_eval.data(), c->h_sum.p + np * wb, np * wb);
      std::memcpy(c->h_repr_eval.p, repr + np * wb, np * wb);
    }
    prof::HostScope hs("host_prove_transcript");
    c->tr->append_messages(LABEL_PR, 6, repr, wb, np);
  }
  if (r + 1 < c->rounds) {
    std::vector<uint64_t> t;
    challenge_tensor(*c->tr, c->fid, c->n_rows, t);
    std::memcpy(c->h_t.p, t.data(), c->n_rows * wb);
    return LCPC_OK;
  }
  {
    prof::HostScope hs("host_prove_transcript");
    c->tr->append_messages(LABEL_PE, 6, c->h_repr_eval.p, wb, np);
  }
  challenge_columns(*c->tr, c->nc, c->nco, c->col_idx);
  std::memcpy(c->h_idx.p, c->col_idx.data(), c->nco * 8);
  return LCPC_OK;
}

Xop op_idx_bcast(lcpc_sharded_commit *c) {
  Xop op{Xop::BROADCAST};
  op.recv = c->didx.as<uint8_t>();
  op.bytes = c->nco * 8;
  op.root = c->root_rank;
  op.s = c->sp;
  op.ready = prove_taken(c);
  return op;
}

lcpc_status stage_idx_upload(lcpc_sharded_commit *c) {
  if (c->me != c->root_rank || !c->nco) return LCPC_OK;
  HIP_TRY(hipStreamWaitEvent(upload_stream(c), prove_taken(c), 0));
  HIP_TRY(h2d(c->didx.p, c->h_idx.p, c->nco * 8, upload_stream(c)));
  return LCPC_OK;
}

// my rows of the opened columns (open_column, :818-855): [col][my rows], Montgomery
size_t st_idx(const lcpc_sharded_commit *c) { return S_R0 + 2 * c->rounds; }
size_t st_cols(const lcpc_sharded_commit *c) { return S_R0 + 2 * c->rounds + 1; }

lcpc_status stage_gather_cols(lcpc_sharded_commit *c) {
  HIP_TRY(hipStreamWaitEvent(c->sp, EV(c, EV_DONE, st_idx(c)), 0));
  if (c->nco && c->nr)
    HIP_TRY(gather_columns(c->fid, c->comm_rows.as<uint32_t>(), c->nr, c->nc, c->didx.as<uint64_t>(), c->nco,
                           c->mycols.as<uint32_t>(), c->sp, c->sdig, true));
  HIP_TRY(hipEventRecord(EV(c, EV_READY, st_cols(c)), c->sp));
  return LCPC_OK;
}

Xop op_cols_gather(lcpc_sharded_commit *c) {
  Xop op{Xop::ALL_TO_ALL};
  op.send = c->mycols.as<uint8_t>();
  op.recv = c->me == c->root_rank ? c->allcols.as<uint8_t>() : nullptr;
  op.sb.assign(c->G, 0);
  op.rb.assign(c->G, 0);
  op.sb[c->root_rank] = c->nco * c->nr * c->wb;
  if (c->me == c->root_rank)
    for (int k = 0; k < c->G; k++) op.rb[k] = c->nco * (c->part[k].r_hi - c->part[k].r_lo) * c->wb;
  op.ready = EV(c, EV_READY, st_cols(c));
  op.s = c->sp;
  return op;
}

// root: Merkle paths off the whole tree, everything to the host
lcpc_status stage_paths(lcpc_sharded_commit *c) {
  HIP_TRY(hipStreamWaitEvent(c->sp, EV(c, EV_DONE, st_cols(c)), 0));
  if (c->me != c->root_rank) {
    HIP_TRY(hipEventRecord(EV(c, EV_HOST, st_cols(c)), c->sp));
    return LCPC_OK;
  }
  const size_t pl = log2_np2(c->nc);
  if (c->nco) {
    HIP_TRY(gather_paths(c->hashes.as<uint8_t>(), 2 * c->np2 - 1, c->didx.as<uint64_t>(), c->nco, pl,
                         c->dpaths.as<uint8_t>(), c->sp));
    HIP_TRY(d2h(c->h_cols.p, c->allcols.p, c->nco * c->n_rows * c->wb, c->sp));
    if (pl) HIP_TRY(d2h(c->h_paths.p, c->dpaths.p, c->nco * pl * 32, c->sp));
  }
  HIP_TRY(hipEventRecord(EV(c, EV_HOST, st_cols(c)), c->sp));
  return LCPC_OK;
}

// root, host: the LcEvalProof (:1117-1122); columns reassembled from the ranks' row pieces
lcpc_status host_proof(lcpc_sharded_commit *c, lcpc_proof **out) {
  prof::HostScope hs("host_final_proof");
  HIP_TRY(hipEventSynchronize(EV(c, EV_HOST, st_cols(c))));
  c->ev_quiet = true;  // (every exchange of the proof precedes it)
  if (c->me != c->root_rank) {
    if (out) *out = nullptr;
    return LCPC_OK;
  }
  // a caller-owned transcript whose callback failed: every exchange still ran (no rank is left
  // waiting), but the proof is void
  if (lcpc_status st = transcript_status(c->tr)) {
    if (out) *out = nullptr;
    return st;
  }
  auto p = std::make_unique<lcpc_proof>();
  const size_t wb = c->wb, nco = c->nco, n_rows = c->n_rows;
  p->fid = c->fid;
  p->n_cols = c->nc;
  p->n_per_row = c->np;
  p->n_rows = n_rows;
  p->ndt = c->ndt;
  p->nco = nco;
  p->path_len = log2_np2(c->nc);
  p->p_eval.assign(c->p_eval.begin(), c->p_eval.end());
  p->p_random.assign(c->p_random.begin(), c->p_random.end());
  p->col_idx = c->col_idx;
  p->cols.resize(nco * n_rows * (wb / 8));
  uint8_t *dst = (uint8_t *)p->cols.data();
  const uint8_t *src = c->h_cols.p;
  for (int k = 0; k < c->G; k++) {
    const size_t r0 = c->part[k].r_lo, nr = c->part[k].r_hi - r0;
    for (size_t j = 0; j < nco; j++) std::memcpy(dst + (j * n_rows + r0) * wb, src + j * nr * wb, nr * wb);
    src += nco * nr * wb;
  }
  p->paths.assign(c->h_paths.p, c->h_paths.p + nco * p->path_len * 32);
  if (out) *out = p.release();
  return LCPC_OK;
}

void prove_release(lcpc_sharded_commit *c) {
  for (DBuf *b : {&c->bt, &c->tens, &c->part_d, &c->allpart, &c->sum, &c->canon, &c->didx, &c->mycols,
                  &c->allcols, &c->dpaths, &c->scratch})
    b->reset();
  if (c->own_tr) delete c->tr;
  c->tr = nullptr;
  c->own_tr = false;
}

// ---- the pipelined schedule (lcpc_sharded_commit_prove_many)
// Stages of polynomial k: 0 = chaining-value all-to-all, 1 = subtree all-gather, then for each
// round r a tensor broadcast and a partial-sum gather, then the column-index broadcast and the
// column gather.  Stage s of polynomial k goes out in tick k + off[s]; off[] leaves `lag` ticks
// wherever the root rank absorbs one row combination before the next exchange needs its
// challenge.  Every rank computes the same schedule, so the exchange groups match.
struct Sched {
  size_t ndt = 0, rounds = 1, n_stages = 0, s_idx = 0, s_cols = 0, n_ticks = 0, lag = 1;
  std::vector<size_t> off;
  // the polynomial whose stage s goes out in tick t, or SIZE_MAX
  size_t poly(size_t t, size_t s, size_t n_polys) const {
    return (t < off[s] || t - off[s] >= n_polys) ? SIZE_MAX : t - off[s];
  }
};

Sched make_sched(size_t ndt, int G, size_t lag, size_t n_polys) {
  Sched sc;
  // ~1.2 ms of absorption per round (cfg3) over ~1.05 ms / G per tick, plus the fold's trip to
  // the host, plus slack.  One rank at K = 20 (profiles/r03_sharded_lag_sweep.json), two groups
  // per tick: 10.0-10.7 G/s at lag 3, 10.7-10.8 at 4, 11.0-11.2 at 5 (four runs), 9.4-11.0 at 6;
  // one group per tick: 9.6-9.9 at lag 2, 10.1-10.5 at 3, 10.7-10.9 at 4.  More hardware queues
  // (GPU_MAX_HW_QUEUES 8, 16) were slower at every lag.
  sc.lag = lag ? lag : std::max<size_t>(5, 2 + (size_t)G);
  sc.ndt = ndt;
  sc.rounds = std::max<size_t>(ndt, 1);
  sc.n_stages = 2 + 2 * sc.rounds + 2;
  sc.off.assign(sc.n_stages, 0);
  sc.off[S_CV] = 0;
  sc.off[S_SUB] = 1;
  sc.off[S_R0] = 3;  // the root rank needs the root on the host and the first challenge
  sc.off[S_R0 + 1] = sc.off[S_R0] + 1;
  for (size_t r = 1; r < sc.rounds; r++) {
    sc.off[S_R0 + 2 * r] = sc.off[S_R0 + 2 * r - 1] + sc.lag;
    sc.off[S_R0 + 2 * r + 1] = sc.off[S_R0 + 2 * r] + 1;
  }
  sc.s_idx = S_R0 + 2 * sc.rounds;
  sc.s_cols = sc.s_idx + 1;
  sc.off[sc.s_idx] = sc.off[sc.s_idx - 1] + (ndt ? 2 : 1) * sc.lag;
  sc.off[sc.s_cols] = sc.off[sc.s_idx] + 1;
  sc.n_ticks = n_polys + sc.off[sc.s_cols];
  return sc;
}

// the exchange of stage s (pure: descriptors only; the stage's host work happens before)
Xop stage_op(lcpc_sharded_commit *c, const Sched &sc, size_t s) {
  if (s == S_CV) return op_cv_exchange(c);
  if (s == S_SUB) return op_subtree_exchange(c);
  if (s == sc.s_idx) return op_idx_bcast(c);
  if (s == sc.s_cols) return op_cols_gather(c);
  const size_t r = (s - S_R0) / 2;
  return (s - S_R0) % 2 == 0 ? op_tensor_bcast(c, r) : op_partial_gather(c, r);
}

// A stage whose host work waits on the transcript rank: the tensor broadcasts (round 0: the
// commitment root; later rounds: the previous round's absorb) and the column-index broadcast.  A
// tick issues its other stages as one exchange group before these, so no polynomial's partial
// gather and fold -- whose absorb is the next link of that polynomial's serial chain -- queues
// behind another polynomial's transcript (with one group per tick, every lag-th polynomial's
// absorbs chained through the drain: K = 20 at one rank lost 2-3 ms there).
bool stage_waits(const Sched &sc, size_t s) {
  return s == sc.s_idx || (s >= S_R0 && s < sc.s_idx && (s - S_R0) % 2 == 0);
}

const char *stage_name(const Sched &sc, size_t s) {
  if (s == S_CV) return "chaining-value all-to-all";
  if (s == S_SUB) return "subtree all-gather";
  if (s == sc.s_idx) return "column-index broadcast";
  if (s == sc.s_cols) return "opened-column gather";
  return (s - S_R0) % 2 == 0 ? "challenge-tensor broadcast" : "partial-combination gather";
}

// ---- watchdog
// A sharded call whose exchanges never complete (a peer that issued a different group, a dead
// rank) would block forever in a stream or event wait.  The watchdog thread watches a progress
// mark the calling thread moves at every tick and wait; when it has not moved for
// LCPC_SHARD_WATCHDOG_S seconds it prints the tick, the stage and the peers on stderr and ends the
// process with status 75 (no re-exec, no further GPU call).  Off unless that variable is set (a
// library must not end its host process by default: a peer may legitimately reach an exchange
// late); bench.py and the tests set it.
class Watchdog {
 public:
  Watchdog(int G, int me) : G_(G), me_(me) {
    const char *v = getenv("LCPC_SHARD_WATCHDOG_S");
    limit_ = v ? atof(v) : 0.0;
    if (limit_ > 0) th_ = std::thread([this] { run(); });
  }
  ~Watchdog() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  bool enabled() const { return limit_ > 0; }
  // what the calling thread is about to wait for
  void mark(size_t tick, size_t n_ticks, const char *what, const std::string &group = std::string()) {
    std::lock_guard<std::mutex> lk(mu_);
    tick_ = tick;
    n_ticks_ = n_ticks;
    what_ = what;
    if (!group.empty()) group_ = group;
    last_ = std::chrono::steady_clock::now();
  }

 private:
  void run() {
    std::unique_lock<std::mutex> lk(mu_);
    while (!stop_) {
      cv_.wait_for(lk, std::chrono::milliseconds(500));
      if (stop_) return;
      const double idle = std::chrono::duration<double>(std::chrono::steady_clock::now() - last_).count();
      if (idle > limit_) {
        fprintf(stderr,
                "liblcpc_mi watchdog: rank %d of %d made no progress for %.0f s at tick %zu of %zu, waiting on %s;"
                " the tick's exchange group (poly:stage -> peers): %s\n",
                me_, G_, idle, tick_, n_ticks_, what_, group_.c_str());
        fflush(stderr);
        std::_Exit(75);
      }
    }
  }
  int G_, me_;
  double limit_ = 0;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  size_t tick_ = 0, n_ticks_ = 0;
  const char *what_ = "start";
  std::string group_ = "-";
  std::chrono::steady_clock::time_point last_ = std::chrono::steady_clock::now();
};

std::string describe_group(const std::vector<std::pair<size_t, size_t>> &items, const std::vector<Xop> &ops,
                           const Sched &sc, int G, int me) {
  std::string g;
  for (size_t i = 0; i < items.size(); i++) {
    std::string peers;
    for (const P2p &x : p2p_plan(G, me, {ops[i]}))
      peers += (x.send ? " >" : " <") + std::to_string(x.peer);
    g += "[" + std::to_string(items[i].first) + ":" + stage_name(sc, items[i].second) + (peers.empty() ? " -" : peers) +
         "] ";
  }
  return g.empty() ? "-" : g;
}

// one exchange of stage `stage` as its own group (the serial entry points)
lcpc_status one_group(lcpc_sharded_commit *c, Xop op, size_t stage, Watchdog *wd = nullptr, size_t step = 0,
                      const char *what = "") {
  std::vector<Xop> ops{std::move(op)};
  if (wd) wd->mark(step, 0, what);
  c->ev_quiet = false;
  return run_group(c->comm, ops, {EV(c, EV_DONE, stage)});
}

// a gather of per-rank byte counts to one rank (an all-to-all with only the root receiving)
Xop gather_to_root(const lcpc_sharded_commit *c, const uint8_t *send, uint8_t *recv, int root,
                   const std::vector<size_t> &bytes_of_rank, size_t stage) {
  Xop op{Xop::ALL_TO_ALL};
  op.send = send;
  op.recv = c->me == root ? recv : nullptr;
  op.sb.assign(c->G, 0);
  op.rb.assign(c->G, 0);
  op.sb[root] = bytes_of_rank[c->me];
  if (c->me == root) op.rb = bytes_of_rank;
  op.ready = EV(c, EV_READY, stage);
  op.s = c->s;
  return op;
}

}  // namespace

// ================================================================= C ABI
extern "C" {

lcpc_status lcpc_comm_rccl_unique_id(uint8_t id[LCPC_COMM_UNIQUE_ID_BYTES]) {
  if (!id) return fail(LCPC_ERR_INVALID_ARG, "null id");
  Rccl &R = rccl();
  if (!R.ok) return fail(LCPC_ERR_UNSUPPORTED, R.err);
  ncclUniqueId u;
  NCCL_TRY(R.GetUniqueId(&u));
  std::memcpy(id, u.internal, LCPC_COMM_UNIQUE_ID_BYTES);
  return LCPC_OK;
}

static lcpc_status comm_common(lcpc_comm *c) {
  lcpc_status st;
  c->dev = current_device(&st);
  if (!c->dev) return st;
  HIP_TRY(hipSetDevice(c->dev->id));
  // the comm stream at the priority of the driver's other streams (one priority unless
  // LCPC_PRIORITY_STREAMS=1 asks for the A/B split, Device::stream_priority)
  HIP_TRY(hipStreamCreateWithPriority(&c->cs, hipStreamNonBlocking, Device::stream_priority(kShardPool != POOL_BULK)));
  c->shared->cs = c->cs;
  return LCPC_OK;
}

lcpc_status lcpc_comm_rccl_new(const uint8_t id[LCPC_COMM_UNIQUE_ID_BYTES], int nranks, int rank, lcpc_comm **out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return fail(LCPC_ERR_INVALID_ARG, "arguments");
  Rccl &R = rccl();
  if (!R.ok) return fail(LCPC_ERR_UNSUPPORTED, R.err);
  auto c = std::make_unique<lcpc_comm>();
  c->nranks = nranks;
  c->rank = rank;
  c->is_rccl = true;
  lcpc_status st = comm_common(c.get());
  if (st) return st;
  ncclUniqueId u;
  std::memcpy(u.internal, id, LCPC_COMM_UNIQUE_ID_BYTES);
  NCCL_TRY(R.CommInitRank(&c->nc, nranks, u, rank));
  *out = c.release();
  return LCPC_OK;
}

lcpc_status lcpc_comm_from_ops(const lcpc_comm_ops *ops, int nranks, int rank, lcpc_comm **out) {
  if (!ops || !out || nranks < 1 || rank < 0 || rank >= nranks) return fail(LCPC_ERR_INVALID_ARG, "arguments");
  if (nranks > 1 && (!ops->all_gather || !ops->all_to_all_v || !ops->broadcast))
    return fail(LCPC_ERR_INVALID_ARG, "every collective must be supplied");
  auto c = std::make_unique<lcpc_comm>();
  c->nranks = nranks;
  c->rank = rank;
  c->ops = *ops;
  lcpc_status st = comm_common(c.get());
  if (st) return st;
  *out = c.release();
  return LCPC_OK;
}

int lcpc_comm_nranks(const lcpc_comm *c) { return c ? c->nranks : 0; }
int lcpc_comm_rank(const lcpc_comm *c) { return c ? c->rank : -1; }
int lcpc_comm_is_rccl(const lcpc_comm *c) { return c && c->is_rccl ? 1 : 0; }
void lcpc_comm_free(lcpc_comm *c) { delete c; }

lcpc_status lcpc_sharded_rows(lcpc_field f, size_t n_rows, int nranks, int rank, size_t *row0, size_t *n_shard_rows) {
  if (!valid_field(f) || nranks < 1 || rank < 0 || rank >= nranks || !row0 || !n_shard_rows)
    return fail(LCPC_ERR_INVALID_ARG, "arguments");
  const Part p = partition(f, n_rows, nranks)[rank];
  *row0 = p.r_lo;
  *n_shard_rows = p.r_hi - p.r_lo;
  return LCPC_OK;
}

lcpc_status lcpc_sharded_commit_new_device(const lcpc_encoding *e, const void *d_rows, size_t n_rows, lcpc_comm *comm,
                                           lcpc_sharded_commit **out) {
  prof::HostScope hs_total("host_sharded_commit_total");
  lcpc_status st = check_shardable(e, comm, n_rows);
  if (st) return st;
  if (!out) return fail(LCPC_ERR_INVALID_ARG, "null out");
  std::lock_guard<std::mutex> lk(comm->mu);
  ShardPtr c;
  if ((st = shard_init(e, comm, n_rows, c))) return st;
  Watchdog wd(comm->nranks, comm->rank);
  if ((st = stage_pre_commit(c.get(), d_rows))) return st;
  if ((st = one_group(c.get(), op_cv_exchange(c.get()), S_CV, &wd, 0, "chaining-value all-to-all"))) return st;
  if ((st = stage_post_cv(c.get()))) return st;
  if ((st = one_group(c.get(), op_subtree_exchange(c.get()), S_SUB, &wd, 1, "subtree all-gather"))) return st;
  if ((st = stage_post_subtrees(c.get()))) return st;
  wd.mark(2, 0, "the commitment root");
  if ((st = finish_commit(c.get()))) return st;
  *out = c.release();
  return LCPC_OK;
}

void lcpc_sharded_commit_free(lcpc_sharded_commit *c) { ShardDeleter()(c); }

lcpc_status lcpc_sharded_commit_get_root(const lcpc_sharded_commit *c, uint8_t root[32]) {
  if (!c || !root) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  std::memcpy(root, c->root, 32);
  return LCPC_OK;
}

size_t lcpc_sharded_commit_n_hashes(const lcpc_sharded_commit *c) { return c ? 2 * c->np2 - 1 : 0; }

lcpc_status lcpc_sharded_commit_copy_hashes(const lcpc_sharded_commit *c, uint8_t *out) {
  if (!c || !out) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  HIP_TRY(hipSetDevice(c->dev->id));
  HIP_TRY(d2h(out, c->hashes.p, (2 * c->np2 - 1) * 32, c->s));
  HIP_TRY(hipStreamSynchronize(c->s));
  return LCPC_OK;
}

lcpc_status lcpc_sharded_prove(lcpc_sharded_commit *c, const uint64_t *outer, size_t outer_len, const lcpc_encoding *e,
                               lcpc_transcript *tr, int root, lcpc_proof **out) {
  prof::HostScope hs_total("host_sharded_prove_total");
  if (!c || !e || !out || (!outer && outer_len)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  if (e != c->e && (e->n_per_row != c->np || e->n_cols != c->nc || e->fid != c->fid))
    return fail(LCPC_PROVER_COMMIT, "ProverError::Commit");
  if (outer_len != c->n_rows) return fail(LCPC_PROVER_OUTER_TENSOR, "ProverError::OuterTensor");
  if (root < 0 || root >= c->G) return fail(LCPC_ERR_INVALID_ARG, "root rank");
  if (c->me == root && !tr) return fail(LCPC_ERR_INVALID_ARG, "the root rank needs the transcript");
  std::lock_guard<std::mutex> lk(c->comm->mu);
  HIP_TRY(hipSetDevice(c->dev->id));
  lcpc_status st;
  struct Cleanup {
    lcpc_sharded_commit *c;
    ~Cleanup() { prove_release(c); }
  } cleanup{c};
  if ((st = prove_init(c, outer, root, e, c->me == root ? tr : nullptr, false))) return st;
  Watchdog wd(c->G, c->me);
  if (c->me == root && (st = challenge_first(c))) return st;
  for (size_t r = 0; r < c->rounds; r++) {
    if ((st = stage_tensor_upload(c, r))) return st;
    if ((st = one_group(c, op_tensor_bcast(c, r), st_bcast(r), &wd, 2 * r, "challenge-tensor broadcast"))) return st;
    if ((st = stage_collapse(c, r))) return st;
    if ((st = one_group(c, op_partial_gather(c, r), st_gather(r), &wd, 2 * r + 1, "partial-combination gather")))
      return st;
    if ((st = stage_fold(c, r))) return st;
    wd.mark(2 * r + 1, 0, "the folded row combination");
    if (c->me == root && (st = host_absorb(c, r))) return st;
  }
  if ((st = stage_idx_upload(c))) return st;
  if ((st = one_group(c, op_idx_bcast(c), st_idx(c), &wd, 2 * c->rounds, "column-index broadcast"))) return st;
  if ((st = stage_gather_cols(c))) return st;
  if ((st = one_group(c, op_cols_gather(c), st_cols(c), &wd, 2 * c->rounds + 1, "opened-column gather"))) return st;
  if ((st = stage_paths(c))) return st;
  wd.mark(2 * c->rounds + 2, 0, "the opened columns and paths");
  return host_proof(c, out);
}

// ---------------------------------------------------------------- proof-of-storage request
// networking/server.rs:652-737 on a row-sharded file commitment: verifiable_polynomial_evaluation
// (lcpc_online.rs:454-484, u^T Enc(M) over the ENCODED matrix) from the ranks' partial sums over
// their rows, gathered at `root` and folded mod p, and the client's columns (open_column,
// lcpc-2d/src/lib.rs:818-855) from the ranks' row pieces, with paths off the whole tree.

lcpc_status lcpc_sharded_pos_request(lcpc_sharded_commit *c, const uint64_t *left, size_t n_rows,
                                                const uint64_t *idx, size_t n_open, int root, uint64_t *eval_out,
                                                uint64_t *cols_out, uint8_t *paths_out) {
  prof::HostScope hs_total("host_sharded_pos_request");
  if (!c || !left || (!idx && n_open)) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (n_rows != c->n_rows) return fail(LCPC_ERR_INVALID_ARG, "left vector length != n_rows");
  if (root < 0 || root >= c->G) return fail(LCPC_ERR_INVALID_ARG, "root rank");
  if (c->sdig) return fail(LCPC_ERR_UNSUPPORTED, "proof-of-storage requests: Ligero file commitments only");
  for (size_t k = 0; k < n_open; k++)
    if (idx[k] >= c->nc) return fail(LCPC_PROVER_COLUMN_NUMBER, "ProverError::ColumnNumber");
  std::lock_guard<std::mutex> lk(c->comm->mu);
  HIP_TRY(hipSetDevice(c->dev->id));
  Watchdog wd(c->G, c->me);
  const size_t wb = c->wb, nc = c->nc, nr = c->nr, r0 = c->part[c->me].r_lo;
  const bool am_root = c->me == root;
  lcpc_status st;
  DBuf tens, part, scratch, all, sum, didx, mycols, allcols, dpaths;
  HostBuf h_left, h_idx;
  if ((st = ev_need(c, kPosEvalStage, kPosColsStage + 1))) return st;
  // (declared after the buffers, so destroyed first) on an early return once a gather is on the
  // comm stream, RCCL may still read `part` / `mycols` or write `all` / `allcols`: drain the comm
  // stream before the buffers go back to the pool
  struct CommDrain {
    lcpc_sharded_commit *c;
    ~CommDrain() {
      if (!c->ev_quiet) {
        (void)hipStreamSynchronize(c->comm->cs);
        (void)hipStreamSynchronize(c->s);
        c->ev_quiet = true;
      }
    }
  } comm_drain{c};
  // this rank's partial u^T Enc(M) over its rows.  The codeword holds canonical values (ntt_rows
  // canon_out), so the Montgomery products sum_r u_r R * m_rj R^-1 come out canonical.
  HIP_TRY(salloc(c, part, nc * wb));
  if (nr) {
    if ((st = h_left.get(c->dev, nr * wb))) return st;
    std::memcpy(h_left.p, (const uint8_t *)left + r0 * wb, nr * wb);
    HIP_TRY(salloc(c, tens, nr * wb));
    HIP_TRY(salloc(c, scratch, collapse_scratch_bytes(c->fid, nr, nc, 1)));
    HIP_TRY(h2d(tens.p, h_left.p, nr * wb, c->s));
    HIP_TRY(collapse_rows(c->fid, c->comm_rows.as<uint32_t>(), nr, nc, tens.as<uint32_t>(), 1, part.as<uint32_t>(),
                          scratch.p, c->s));
  } else {
    HIP_TRY(hipMemsetAsync(part.p, 0, nc * wb, c->s));
  }
  // the gather's receive buffer is taken BEFORE the READY record: a reused pool block's fence wait
  // is queued on c->s by the take, and the comm stream's wait on READY then orders RCCL's writes
  // into `all` after it (taken after the record, the gather could race the block's last owner)
  if (am_root) HIP_TRY(salloc(c, all, (size_t)c->G * nc * wb));
  HIP_TRY(hipEventRecord(EV(c, EV_READY, kPosEvalStage), c->s));
  if ((st = one_group(c, gather_to_root(c, part.as<uint8_t>(), all.as<uint8_t>(), root,
                                        std::vector<size_t>(c->G, nc * wb), kPosEvalStage),
                      kPosEvalStage, &wd, 0, "partial u^T Enc(M) gather")))
    return st;
  // my rows of the requested columns
  if (n_open) {
    if ((st = h_idx.get(c->dev, n_open * 8))) return st;
    std::memcpy(h_idx.p, idx, n_open * 8);
    HIP_TRY(salloc(c, didx, n_open * 8));
    HIP_TRY(h2d(didx.p, h_idx.p, n_open * 8, c->s));
  }
  HIP_TRY(hipStreamWaitEvent(c->s, EV(c, EV_DONE, kPosEvalStage), 0));
  HIP_TRY(salloc(c, mycols, std::max<size_t>(n_open * nr, 1) * wb));
  if (n_open && nr)
    HIP_TRY(gather_columns(c->fid, c->comm_rows.as<uint32_t>(), nr, nc, didx.as<uint64_t>(), n_open,
                           mycols.as<uint32_t>(), c->s, false, true));
  if (am_root) {
    // fold the partials; canonical sums -> Montgomery words (the ABI's element layout)
    HIP_TRY(salloc(c, sum, nc * wb));
    HIP_TRY(collapse_fold_rows(c->fid, all.as<uint32_t>(), c->G, nc, sum.as<uint32_t>(), c->s));
    HIP_TRY(convert(c->fid, sum.as<uint32_t>(), sum.as<uint32_t>(), nc, true, c->s));
    HIP_TRY(salloc(c, allcols, std::max<size_t>(n_open * c->n_rows, 1) * wb));
  }
  HIP_TRY(hipEventRecord(EV(c, EV_READY, kPosColsStage), c->s));
  std::vector<size_t> col_bytes(c->G);
  for (int k = 0; k < c->G; k++) col_bytes[k] = n_open * (c->part[k].r_hi - c->part[k].r_lo) * wb;
  if ((st = one_group(c, gather_to_root(c, mycols.as<uint8_t>(), allcols.as<uint8_t>(), root, col_bytes,
                                        kPosColsStage),
                      kPosColsStage, &wd, 1, "requested-column gather")))
    return st;
  HIP_TRY(hipStreamWaitEvent(c->s, EV(c, EV_DONE, kPosColsStage), 0));
  if (am_root) {
    const size_t pl = log2_np2(nc);
    HIP_TRY(salloc(c, dpaths, std::max<size_t>(n_open * pl, 1) * 32));
    if (n_open && pl)
      HIP_TRY(gather_paths(c->hashes.as<uint8_t>(), 2 * nc - 1, didx.as<uint64_t>(), n_open, pl,
                           dpaths.as<uint8_t>(), c->s));
    if (eval_out) HIP_TRY(d2h_staged(eval_out, sum.p, nc * wb, c->s));
    // columns arrive as [rank][col][rank's rows]: reassemble [col][all rows] on the host
    std::vector<uint8_t> h_cols(std::max<size_t>(n_open * c->n_rows, 1) * wb);
    if (n_open) HIP_TRY(d2h_staged(h_cols.data(), allcols.p, n_open * c->n_rows * wb, c->s));
    if (paths_out && n_open && pl) HIP_TRY(d2h_staged(paths_out, dpaths.p, n_open * pl * 32, c->s));
    wd.mark(2, 0, "the request's results");
    HIP_TRY(hipStreamSynchronize(c->s));
    c->ev_quiet = true;
    if (cols_out) {
      const uint8_t *src = h_cols.data();
      uint8_t *dst = (uint8_t *)cols_out;
      for (int k = 0; k < c->G; k++) {
        const size_t kr0 = c->part[k].r_lo, knr = c->part[k].r_hi - kr0;
        for (size_t j = 0; j < n_open; j++) std::memcpy(dst + (j * c->n_rows + kr0) * wb, src + j * knr * wb, knr * wb);
        src += n_open * knr * wb;
      }
    }
  } else {
    wd.mark(2, 0, "the request's exchanges");
    HIP_TRY(hipStreamSynchronize(c->s));
    c->ev_quiet = true;
  }
  return LCPC_OK;
}

// ---------------------------------------------------------------- the pipelined driver
// (the schedule: make_sched above)
lcpc_status lcpc_sharded_commit_prove_many(const lcpc_encoding *e, const void *const *d_rows, size_t n_polys,
                                           size_t n_rows, const uint64_t *outer, lcpc_comm *comm,
                                           lcpc_make_transcript_fn make_transcript, void *user, size_t lag,
                                           lcpc_proof **proofs, uint8_t *roots) {
  lcpc_status st = check_shardable(e, comm, n_rows);
  if (st) return st;
  if (!d_rows || !outer || !make_transcript) return fail(LCPC_ERR_INVALID_ARG, "null argument");
  if (proofs)
    for (size_t i = 0; i < n_polys; i++) proofs[i] = nullptr;
  if (n_polys == 0) return LCPC_OK;
  prof::HostScope hs_all("many_total");
  std::optional<prof::HostScope> hs_setup(std::in_place, "many_setup");
  std::lock_guard<std::mutex> lk(comm->mu);
  HIP_TRY(hipSetDevice(e->dev->id));
  const int G = comm->nranks, me = comm->rank;
  const Sched sc = make_sched(e->n_degree_tests, G, lag, n_polys);
  const size_t n_stages = sc.n_stages, S_IDX = sc.s_idx, S_COLS = sc.s_cols, n_ticks = sc.n_ticks;
  Watchdog wd(G, me);

  // Host threads: the main thread issues the exchange groups in schedule order; each
  // polynomial's compute launches after an exchange (and its first encode) run on `launch`
  // workers, one task per polynomial at a time (a task's launches precede that polynomial's next
  // exchange: the main thread settles it first), so the main thread's tick is the group plus the
  // waits; the root rank's transcript absorptions and the final proofs run on `pool`.
  // (every task of a call has finished when it returns, error paths included: fail_all)
  if (!comm->pool) {
    const size_t hw = std::max(2u, std::thread::hardware_concurrency());
    comm->pool = std::make_unique<TaskPool>(std::min<size_t>(16, hw), e->dev->id);
    comm->launch = std::make_unique<TaskPool>(std::min<size_t>(4, hw), e->dev->id);
    // every polynomial's encode goes on one stream, issued in polynomial order by one thread:
    // the encodes finish first come first (on streams of their own they ran side by side and
    // each commitment's root arrived late), while the short exchange-side and prove kernels run
    // on each polynomial's own (prove) stream
    comm->encoder = std::make_unique<TaskPool>(1, e->dev->id);
  }
  TaskPool &pool = *comm->pool, &launch = *comm->launch, &encoder = *comm->encoder;
  // the encode streams (shard_bulk_streams(), taken in turn by polynomial)
  const size_t n_bulk = shard_bulk_streams();
  hipStream_t bulks[SHARD_BULK_MAX] = {};
  struct BulkRelease {  // (destroyed after cs: returns the streams to the pool)
    Device *d;
    hipStream_t *s;
    ~BulkRelease() {
      for (size_t i = 0; i < SHARD_BULK_MAX; i++)
        if (s[i]) d->release_stream(s[i], kShardPool);
    }
  } bulk_release{e->dev, bulks};
  for (size_t i = 0; i < n_bulk; i++)
    if (!(bulks[i] = e->dev->acquire_stream(kShardPool))) return fail(LCPC_ERR_DEVICE, "no HIP stream");
  std::vector<ShardPtr> cs(n_polys);
  struct BulkDrain {  // (destroyed before cs: no polynomial is torn down under its running encode)
    hipStream_t *s;
    ~BulkDrain() {
      for (size_t i = 0; i < SHARD_BULK_MAX; i++)
        if (s[i]) (void)hipStreamSynchronize(s[i]);
    }
  } bulk_drain{bulks};
  std::vector<std::future<lcpc_status>> pending(n_polys);  // the polynomial's outstanding launch task
  std::deque<std::pair<size_t, std::future<lcpc_status>>> finals;  // (poly, host_proof)
  std::vector<size_t> to_finalize;
  std::mutex err_mu;
  std::string err_msg;  // the first failing worker's message (g_err is per thread)
  auto wrap = [&](std::function<lcpc_status()> fn) {
    return [fn = std::move(fn), &err_mu, &err_msg]() -> lcpc_status {
      const lcpc_status s2 = fn();
      if (s2) {
        std::lock_guard<std::mutex> l2(err_mu);
        if (err_msg.empty()) err_msg = g_err;
      }
      return s2;
    };
  };
  auto settle = [&](size_t k) -> lcpc_status { return pending[k].valid() ? pending[k].get() : LCPC_OK; };
  auto fail_all = [&](lcpc_status s2) {
    std::string msg = g_err;
    for (auto &f : pending)
      if (f.valid()) f.wait();
    for (auto &f : finals) f.second.wait();  // (their tasks reset cs[k])
    for (auto &c : cs)
      if (c && c->next.valid()) c->next.wait();
    {
      std::lock_guard<std::mutex> l2(err_mu);
      if (!err_msg.empty()) msg = err_msg;
    }
    return fail(s2, msg);
  };
  auto submit_final = [&](size_t k) {
    lcpc_sharded_commit *c = cs[k].get();
    lcpc_proof **dst = proofs ? proofs + k : nullptr;
    // the proof and the polynomial's teardown on the pool: nothing else touches cs[k] any more
    finals.emplace_back(k, pool.submit(wrap([c, dst, &cs, k]() -> lcpc_status {
                          lcpc_proof *p = nullptr;
                          const lcpc_status s2 = host_proof(c, &p);
                          if (dst) *dst = p;
                          else delete p;
                          cs[k].reset();
                          return s2;
                        })));
  };
  auto start = [&](size_t k) {
    pending[k] = encoder.submit(wrap([&, k]() -> lcpc_status {
      lcpc_status s2 = shard_init(e, comm, n_rows, cs[k], bulks[k % n_bulk]);
      if (s2) return s2;
      cs[k]->poly = k;
      return stage_pre_commit(cs[k].get(), d_rows[k]);
    }));
  };
  // polynomial k's encode is launched AHEAD ticks before its chaining-value exchange, so a tick's
  // exchange group (which waits for every producer in it) does not wait on a just-launched encode
  // and the encode stream stays fed while a tick waits on the host
  // (look-ahead 3: a sweep of 1-6 was within the run-to-run spread, profiles/r04_sharded_ahead_sweep.json)
  constexpr size_t AHEAD = 3;
  for (size_t k = 0; k < std::min(AHEAD, n_polys); k++) start(k);
  hs_setup.reset();
  for (size_t t = 0; t < n_ticks; t++) {
    prof::HostScope hs_tick("tick_total");
    wd.mark(t, n_ticks, "the previous tick's launches");
    // last tick's final stages: the proofs go to the pool; finished polynomials free their buffers
    for (size_t k : to_finalize) {
      if ((st = settle(k))) return fail_all(st);
      submit_final(k);
    }
    to_finalize.clear();
    while (!finals.empty() && finals.front().second.wait_for(std::chrono::seconds(0)) == std::future_status::ready) {
      if ((st = finals.front().second.get())) return fail_all(st);
      finals.pop_front();
    }
    // two exchange groups per tick: the stages with no host wait first, their compute submitted at
    // once, then the stages that wait on a transcript (see stage_waits)
    for (int pass = 0; pass < 2; pass++) {
      std::vector<Xop> ops;
      std::vector<hipEvent_t> done;
      std::vector<std::pair<size_t, size_t>> items;  // (poly, stage)
      for (size_t s = 0; s < n_stages; s++) {
        const size_t k = sc.poly(t, s, n_polys);
        if (k == SIZE_MAX || stage_waits(sc, s) != (pass == 1)) continue;
        {
          prof::HostScope hs("tick_wait_launch");
          wd.mark(t, n_ticks, "a polynomial's compute launches");
          if ((st = settle(k))) return fail_all(st);
        }
        lcpc_sharded_commit *c = cs[k].get();
        // the stage's host work before its exchange
        if (s == S_IDX) {
          if (c->me == c->root_rank) {
            prof::HostScope hs("tick_wait_challenge");
            wd.mark(t, n_ticks, "the root rank's transcript (column challenge)");
            if ((st = c->next.get())) return fail_all(st);
          }
          if ((st = stage_idx_upload(c))) return fail_all(st);
        } else if (s >= S_R0 && s < S_IDX && (s - S_R0) % 2 == 0) {
          const size_t r = (s - S_R0) / 2;
          {
            if (r == 0) {
              // the commit is complete (root on the host) and the transcript exists
              {
                prof::HostScope hs("tick_wait_root");
                wd.mark(t, n_ticks, "the commitment root (subtree exchange)");
                if ((st = finish_commit(c))) return fail_all(st);
              }
              if (roots) std::memcpy(roots + 32 * k, c->root, 32);
              lcpc_transcript *tr = nullptr;
              if (me == (int)(k % G)) {
                prof::HostScope hs2("tick_make_transcript");
                tr = make_transcript(user, k, c->root);
                if (!tr) return fail_all(fail(LCPC_ERR_INVALID_ARG, "make_transcript returned NULL"));
              }
              prof::HostScope hs("tick_prove_init");
              c->tr = tr;  // (the buffers: prove_alloc, with the subtree stage's launches)
              c->own_tr = true;
              if (me == c->root_rank && (st = challenge_first(c))) return fail_all(st);
            } else if (c->me == c->root_rank) {
              prof::HostScope hs("tick_wait_challenge");
              wd.mark(t, n_ticks, "the root rank's transcript (challenge tensor)");
              if ((st = c->next.get())) return fail_all(st);
            }
            if ((st = stage_tensor_upload(c, r))) return fail_all(st);
          }
        }
        ops.push_back(stage_op(c, sc, s));
        done.push_back(EV(c, EV_DONE, s));
        c->ev_quiet = false;
        items.emplace_back(k, s);
      }
      if (!ops.empty()) {
        prof::HostScope hs("tick_run_group");
        // (the group's text only feeds the watchdog's message: not built when it is off)
        wd.mark(t, n_ticks, "issuing the exchange group",
                G > 1 && wd.enabled() ? describe_group(items, ops, sc, G, me) : std::string());
        if ((st = run_group(comm, ops, done))) return fail_all(st);
      }
      // the compute each exchange feeds, on the polynomials' own streams (launch workers)
      prof::HostScope hs_sub("tick_submit");
      for (auto [k, s] : items) {
        lcpc_sharded_commit *c = cs[k].get();
        pending[k] = launch.submit(wrap([&pool, c, s = s, k = k, S_IDX, S_COLS, outer, G, e]() -> lcpc_status {
          if (s == S_CV) return stage_post_cv(c);
          if (s == S_SUB) {
            const lcpc_status s2 = stage_post_subtrees(c);
            return s2 ? s2 : prove_alloc(c, outer, (int)(k % G), e);
          }
          if (s == S_IDX) return stage_gather_cols(c);
          if (s == S_COLS) return stage_paths(c);
          const size_t r = (s - S_R0) / 2;
          if ((s - S_R0) % 2 == 0) return stage_collapse(c, r);
          const lcpc_status s2 = stage_fold(c, r);
          if (s2) return s2;
          if (c->me == c->root_rank) c->next = pool.submit([c, r] { return host_absorb(c, r); });
          return LCPC_OK;
        }));
        if (s == S_COLS) to_finalize.push_back(k);
      }
    }
    if (t + AHEAD < n_polys) start(t + AHEAD);
  }
  wd.mark(n_ticks, n_ticks, "the last proofs");
  for (size_t k : to_finalize) {
    if ((st = settle(k))) return fail_all(st);
    submit_final(k);
  }
  lcpc_status first = LCPC_OK;
  std::string msg;
  while (!finals.empty()) {
    const lcpc_status s2 = finals.front().second.get();
    if (s2 && !first) first = s2;
    finals.pop_front();
  }
  if (first) {
    std::lock_guard<std::mutex> l2(err_mu);
    msg = err_msg;
  }
  HIP_TRY(hipStreamSynchronize(comm->cs));
  return first ? fail(first, msg) : LCPC_OK;
}

lcpc_status lcpc_sharded_reserve(const lcpc_encoding *e, size_t n_rows, lcpc_comm *comm, size_t n_polys,
                                 size_t lag) {
  lcpc_status st = check_shardable(e, comm, n_rows);
  if (st) return st;
  if (n_polys == 0) return LCPC_OK;
  Device *dev = e->dev;
  HIP_TRY(hipSetDevice(dev->id));
  const int G = comm->nranks, me = comm->rank;
  const Sched sc = make_sched(e->n_degree_tests, G, lag, n_polys);
  // polynomials alive at once: launched AHEAD ticks early, released a tick after their last stage
  const size_t depth = std::min(n_polys, sc.off[sc.s_cols] + 4);
  lcpc_sharded_commit g;  // descriptor only: the sizes the stages ask of the pools
  shard_geom(&g, e->fid, e->n_per_row, e->n_cols, n_rows, G, me, e->kind == KIND_SDIG);
  const size_t wb = g.wb, np = g.np, nc = g.nc, nr = g.nr, B = g.B, nco = e->n_col_opens;
  const size_t nch = g.part[me].c_hi - g.part[me].c_lo, pl = log2_np2(nc);
  // (the expressions of stage_pre_commit, stage_post_cv, stage_post_subtrees and prove_alloc)
  std::vector<size_t> dsz = {nr * np * wb + 16, nr * nc * wb + 16, nch * g.np2 * 32 + 16, (2 * B - 1) * 32,
                             (2 * g.np2 - 1) * 32, n_rows * wb, 2 * std::max<size_t>(nr, 1) * wb, 2 * np * wb,
                             collapse_scratch_bytes(e->fid, std::max<size_t>(nr, 1), np, 2),
                             std::max<size_t>(nco, 1) * 8, std::max<size_t>(nco * nr, 1) * wb};
  if (g.sdig && nr) dsz.push_back(e->sdig.tmp_elems * nr * wb + 16);
  if (G > 1) {  // (one rank exchanges in place)
    dsz.push_back(g.n_chunks * B * 32 + 16);
    dsz.push_back((size_t)G * (2 * B - 1) * 32);
  }
  std::vector<size_t> psz = {32, n_rows * wb, std::max<size_t>(nco, 1) * 8};
  if (nr) psz.push_back(nr * wb);
  // the transcript rank of polynomial k is k % G: its share of the depth
  const size_t root_depth = (depth + G - 1) / G;
  std::vector<size_t> rdsz = {(size_t)G * 2 * np * wb, 2 * np * wb, 2 * np * wb,
                              std::max<size_t>(nco * n_rows, 1) * wb, std::max<size_t>(nco * pl, 1) * 32};
  std::vector<size_t> rpsz = {2 * np * wb, 2 * np * wb, np * wb, std::max<size_t>(nco * n_rows, 1) * wb,
                              std::max<size_t>(nco * pl, 1) * 32};
  std::vector<void *> blocks, pins;
  auto take = [&](const std::vector<size_t> &d, const std::vector<size_t> &h, size_t count) -> lcpc_status {
    for (size_t k = 0; k < count; k++) {
      for (size_t b : d) {
        void *p = nullptr;
        if (dev->alloc(&p, b) != hipSuccess) return fail(LCPC_ERR_OUT_OF_MEMORY, "reserve: device pool");
        blocks.push_back(p);
      }
      for (size_t b : h) {
        void *p = dev->pinned_get(b);
        if (!p) return fail(LCPC_ERR_OUT_OF_MEMORY, "reserve: pinned staging");
        pins.push_back(p);
      }
    }
    return LCPC_OK;
  };
  st = take(dsz, psz, depth);
  if (!st) st = take(rdsz, rpsz, root_depth);
  for (void *p : blocks) dev->release(p);
  for (void *p : pins) dev->pinned_put(p);
  // the streams lcpc_sharded_commit_prove_many acquires: the shared (bulk) encode streams, and a
  // prove stream per polynomial in flight
  std::vector<hipStream_t> lo, hi;
  for (size_t i = 0; i < shard_bulk_streams(); i++) lo.push_back(dev->acquire_stream(kShardPool));
  for (size_t k = 0; k < depth && shard_prio_streams(); k++) hi.push_back(dev->acquire_stream(kShardPool));
  for (hipStream_t x : lo)
    if (x) dev->release_stream(x, kShardPool);
  for (hipStream_t x : hi)
    if (x) dev->release_stream(x, kShardPool);
  // the page-locked blocks of the proofs this rank assembles (host_proof: p_random, p_eval,
  // columns, paths), one set per polynomial it is the transcript rank of: every proof of a call
  // is alive until the call returns, so a call at a new depth would otherwise pin them inside it
  if (!st) {
    const size_t own = me < (int)n_polys ? (n_polys - (size_t)me + G - 1) / G : 0;
    const size_t ndt = e->n_degree_tests;
    std::vector<void *> proof_pins;
    for (size_t k = 0; k < own; k++)
      for (size_t b : {ndt * np * wb, np * wb, nco * n_rows * wb, nco * pl * 32})
        if (b >= PinnedHeap::MIN)
          if (void *p = g_pinned_heap.get(b)) proof_pins.push_back(p);
    for (void *p : proof_pins) g_pinned_heap.put(p);
  }
  return st;
}

lcpc_status lcpc_sharded_p2p_schedule(lcpc_field f, size_t n_rows, size_t n_per_row, size_t n_cols,
                                      size_t n_degree_tests, size_t n_col_opens, int nranks, int rank,
                                      size_t n_polys, size_t lag, lcpc_p2p_record *out, size_t cap,
                                      size_t *n_out) {
  if (!valid_field(f) || nranks < 1 || rank < 0 || rank >= nranks || !n_out || (cap && !out))
    return fail(LCPC_ERR_INVALID_ARG, "arguments");
  lcpc_status st = check_geom(f, KIND_RS, n_cols, nranks, n_rows);
  if (st) return st;
  const Sched sc = make_sched(n_degree_tests, nranks, lag, n_polys);
  // one descriptor-only shard state per polynomial (no device buffers: offsets from null)
  std::vector<std::unique_ptr<lcpc_sharded_commit>> cs(n_polys);
  for (size_t k = 0; k < n_polys; k++) {
    cs[k] = std::make_unique<lcpc_sharded_commit>();
    shard_geom(cs[k].get(), f, n_per_row, n_cols, n_rows, nranks, rank);
    prove_geom(cs[k].get(), n_degree_tests, n_col_opens, (int)(k % nranks));
  }
  size_t n = 0;
  for (size_t grp = 0; grp < 2 * sc.n_ticks; grp++) {  // (the driver's two groups per tick)
    const size_t t = grp / 2;
    std::vector<Xop> ops;
    std::vector<std::pair<size_t, size_t>> items;
    for (size_t s = 0; s < sc.n_stages; s++) {
      const size_t k = sc.poly(t, s, n_polys);
      if (k == SIZE_MAX || stage_waits(sc, s) != (grp % 2 == 1)) continue;
      ops.push_back(stage_op(cs[k].get(), sc, s));
      items.emplace_back(k, s);
    }
    uint32_t pos = 0;
    for (const P2p &x : p2p_plan(nranks, rank, ops)) {
      if (n < cap) {
        lcpc_p2p_record &r = out[n];
        r.tick = (uint32_t)grp;
        r.pos = pos;
        r.poly = (uint32_t)items[x.op].first;
        r.stage = (uint32_t)items[x.op].second;
        r.is_send = x.send ? 1 : 0;
        r.peer = x.peer;
        r.bytes = x.bytes;
      }
      n++;
      pos++;
    }
  }
  *n_out = n;
  return n > cap ? fail(LCPC_ERR_INVALID_ARG, "cap") : LCPC_OK;
}

}  // extern "C"
