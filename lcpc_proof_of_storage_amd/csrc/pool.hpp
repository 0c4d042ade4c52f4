// pool.hpp -- stream-ordered caching pool of device blocks (host logic only, no HIP types).
//
// A block handed back to the pool carries a FENCE: one event recorded on every stream that used
// it, at the moment it was released.  Whoever takes the block next is ordered after that fence:
//   * a taker with a stream makes the stream wait on each pending event (device side; the host
//     does not block),
//   * a taker without a stream (host code that will hand the block to a stream of its choosing
//     later) waits on the host.
// So a write still queued on ANY stream that used the block -- a late exchange on the
// communicator's stream, an error path that returned early -- completes before the next owner's
// first use, without each caller proving its own drain (the round-4 review's "late writer into a
// recycled block" class).  Events whose record has completed are skipped and recycled at once;
// events a stream was made to wait on go through a retiring list and are reused only once their
// record has completed.
//
// The pool is templated on a backend so that its ordering logic is testable without a GPU
// (tests/cpp/test_pool.cpp drives it with a simulated-stream backend).  Backend:
//   using Stream, Event;                  (Stream{} / Event{} are "none")
//   Event event_new();                    a fresh event, or Event{} on failure
//   void event_free(Event);
//   bool record(Event, Stream);           event := completion of the work queued on the stream so far
//   bool done(Event);                     its record has completed
//   bool wait(Stream, Event);             the stream's later work waits for the record (device side)
//   bool sync(Event);                     the host waits for the record
//   void drain(Stream);                   the host waits for the stream (fallback when no event)
#pragma once
#include <cstddef>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

namespace lcpc_pool {

template <class B>
class OrderedPool {
 public:
  using Stream = typename B::Stream;
  using Event = typename B::Event;
  static constexpr int MAX_STREAMS = 4;  // streams a block can carry a fence for

  explicit OrderedPool(B &backend) : b_(backend) {}
  OrderedPool(const OrderedPool &) = delete;
  OrderedPool &operator=(const OrderedPool &) = delete;

  // A cached block of exactly `bytes`, ordered after its fence on `s` (on the host when s is
  // none), or nullptr when none is cached.
  void *take(size_t bytes, Stream s) {
    Entry e;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = free_.find(bytes);
      if (it == free_.end()) return nullptr;
      e = std::move(it->second);
      free_.erase(it);
    }
    order_after(e, s);  // (device-side waits, or a host wait, outside the lock)
    return e.p;
  }

  // Return a block of `bytes` that the streams ss[0..n) may still use: a fence is recorded on
  // each of them (none: the caller knows every use has completed).
  void put(void *p, size_t bytes, const Stream *ss, int n) {
    if (!p) return;
    Entry e;
    e.p = p;
    Stream to_drain[MAX_STREAMS];
    int nd = 0;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (int i = 0; i < n && i < MAX_STREAMS; i++) {
        if (ss[i] == Stream{}) continue;
        bool dup = false;
        for (int k = 0; k < i; k++) dup |= ss[k] == ss[i];
        if (dup) continue;
        Event ev = event_get();
        if (ev == Event{} || !b_.record(ev, ss[i])) {
          // no event: order the release on the host instead (rare: event creation failed)
          if (ev != Event{}) b_.event_free(ev);
          to_drain[nd++] = ss[i];
          continue;
        }
        e.st[e.n] = ss[i];
        e.ev[e.n++] = ev;
      }
      if (!nd) {
        free_.emplace(bytes, std::move(e));
        return;
      }
    }
    // host waits outside the lock (other threads' take / put do not queue behind unrelated GPU
    // work); the block joins the free list only once they are done
    for (int i = 0; i < nd; i++) b_.drain(to_drain[i]);
    std::lock_guard<std::mutex> lk(mu_);
    syncs_ += nd;
    free_.emplace(bytes, std::move(e));
  }

  // Every cached block (for trimming or teardown), each freed only after its fence has completed
  // on the host: a block released by another thread after the caller's device drain may still
  // have work queued on it.
  template <class FreeFn>
  void drain(FreeFn &&free_block) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto &kv : free_) {
      for (int i = 0; i < kv.second.n; i++) {
        if (!b_.done(kv.second.ev[i])) {
          b_.sync(kv.second.ev[i]);
          syncs_++;
        }
        recycle(kv.second.ev[i]);
      }
      free_block(kv.second.p);
    }
    free_.clear();
    for (Event e : retiring_)
      if (!b_.done(e)) b_.sync(e);
    reap(true);
  }

  // (tests) counters
  size_t cached() {
    std::lock_guard<std::mutex> lk(mu_);
    return free_.size();
  }
  size_t events_idle() {
    std::lock_guard<std::mutex> lk(mu_);
    return idle_.size();
  }
  size_t events_retiring() {
    std::lock_guard<std::mutex> lk(mu_);
    return retiring_.size();
  }
  size_t waits_issued() {
    std::lock_guard<std::mutex> lk(mu_);
    return waits_;
  }
  size_t host_syncs() {
    std::lock_guard<std::mutex> lk(mu_);
    return syncs_;
  }
  size_t same_stream() {
    std::lock_guard<std::mutex> lk(mu_);
    return same_;
  }

  ~OrderedPool() {
    for (Event e : idle_) b_.event_free(e);
    for (Event e : retiring_) b_.event_free(e);  // (a queued wait keeps its own reference)
    for (auto &kv : free_)
      for (int i = 0; i < kv.second.n; i++) b_.event_free(kv.second.ev[i]);
  }

 private:
  struct Entry {
    void *p = nullptr;
    Event ev[MAX_STREAMS] = {};
    Stream st[MAX_STREAMS] = {};  // the stream each event was recorded on
    int n = 0;
  };

  void order_after(Entry &e, Stream s) {
    Event to_retire[MAX_STREAMS], to_idle[MAX_STREAMS];
    int nr = 0, ni = 0;
    size_t waits = 0, syncs = 0, same = 0;
    for (int i = 0; i < e.n; i++) {
      Event ev = e.ev[i];
      if (s != Stream{} && s == e.st[i]) {
        to_retire[nr++] = ev;  // the taker's own stream: already ordered after the fence
        same++;
      } else if (b_.done(ev)) {
        to_idle[ni++] = ev;
      } else if (s != Stream{} && b_.wait(s, ev)) {
        waits++;
        to_retire[nr++] = ev;
      } else {
        b_.sync(ev);
        syncs++;
        to_idle[ni++] = ev;
      }
    }
    e.n = 0;
    std::lock_guard<std::mutex> lk(mu_);
    for (int i = 0; i < nr; i++) retiring_.push_back(to_retire[i]);
    for (int i = 0; i < ni; i++) recycle(to_idle[i]);
    waits_ += waits;
    syncs_ += syncs;
    same_ += same;
    reap(false);
  }

  Event event_get() {
    reap(false);
    if (!idle_.empty()) {
      Event e = idle_.back();
      idle_.pop_back();
      return e;
    }
    return b_.event_new();
  }
  void recycle(Event e) {
    if (idle_.size() < 256)
      idle_.push_back(e);
    else
      b_.event_free(e);
  }
  // retiring events whose record has completed become reusable
  void reap(bool all) {
    size_t k = 0;
    for (Event e : retiring_) {
      if (all || b_.done(e))
        recycle(e);
      else
        retiring_[k++] = e;
    }
    retiring_.resize(k);
  }
  B &b_;
  std::mutex mu_;
  std::multimap<size_t, Entry> free_;
  std::vector<Event> idle_, retiring_;
  size_t waits_ = 0, syncs_ = 0, same_ = 0;  // (under mu_)
};

}  // namespace lcpc_pool
