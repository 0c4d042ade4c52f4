// prof.cpp -- see prof.hpp.
#include "prof.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lcpc_mi.h"

namespace lcpc {
namespace prof {

namespace {
struct Rec {
  const char *name;
  hipEvent_t a, b;
};
std::mutex mu;
bool on = false;
std::vector<Rec> pending;
std::vector<hipEvent_t> spare;
std::map<std::string, std::pair<double, uint64_t>> totals;
// LCPC_PROF_TIMELINE=<path>: every host phase as (name, start, end, thread), appended to <path> as
// CSV (steady-clock ms, the clock rocprofv3's kernel timestamps use) when profiling is switched off
struct Span {
  const char *name;
  double t0, t1;
  size_t tid;
};
std::vector<Span> spans;
const char *timeline_path() {
  static const char *p = getenv("LCPC_PROF_TIMELINE");
  return p && p[0] ? p : nullptr;
}
void flush_timeline() {  // caller holds mu
  if (spans.empty() || !timeline_path()) return;
  if (FILE *f = fopen(timeline_path(), "a")) {
    for (auto &s : spans) fprintf(f, "%s,%.4f,%.4f,%zu\n", s.name, s.t0, s.t1, s.tid);
    fclose(f);
  }
  spans.clear();
}

hipEvent_t get_event() {
  if (!spare.empty()) {
    hipEvent_t e = spare.back();
    spare.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

void resolve() {  // caller holds mu
  for (auto &r : pending) {
    (void)hipEventSynchronize(r.b);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
      auto &t = totals[r.name];
      t.first += ms;
      t.second += 1;
    }
    spare.push_back(r.a);
    spare.push_back(r.b);
  }
  pending.clear();
}
}  // namespace

bool enabled() { return on; }

// LCPC_PROF_HOST_ONLY=1: record the host phases only (no event pair per launch)
static bool host_only() {
  static const bool v = [] {
    const char *e = getenv("LCPC_PROF_HOST_ONLY");
    return e && e[0] == '1';
  }();
  return v;
}

Scope::Scope(const char *name, hipStream_t s) : name_(name), s_(s) {
  if (!on || host_only()) return;
  {
    std::lock_guard<std::mutex> lk(mu);
    a_ = get_event();
    b_ = get_event();
  }
  (void)hipEventRecord(a_, s);
}

Scope::~Scope() {
  if (!a_) return;
  (void)hipEventRecord(b_, s_);
  std::lock_guard<std::mutex> lk(mu);
  pending.push_back(Rec{name_, a_, b_});
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

HostScope::HostScope(const char *name) : name_(name) {
  if (on) t0_ = now_ms();
}

HostScope::~HostScope() {
  if (t0_ < 0) return;
  const double dt = now_ms() - t0_;
  std::lock_guard<std::mutex> lk(mu);
  auto &t = totals[name_];
  t.first += dt;
  t.second += 1;
  if (timeline_path())
    spans.push_back(Span{name_, t0_, t0_ + dt, std::hash<std::thread::id>{}(std::this_thread::get_id()) % 100000});
}

}  // namespace prof
}  // namespace lcpc

extern "C" {

void lcpc_prof_enable(int enable) {
  std::lock_guard<std::mutex> lk(lcpc::prof::mu);
  lcpc::prof::on = enable != 0;
  if (!enable) lcpc::prof::flush_timeline();
}

void lcpc_prof_reset(void) {
  std::lock_guard<std::mutex> lk(lcpc::prof::mu);
  lcpc::prof::resolve();
  lcpc::prof::totals.clear();
}

int lcpc_prof_get(const char *name, double *total_ms, uint64_t *count) {
  std::lock_guard<std::mutex> lk(lcpc::prof::mu);
  lcpc::prof::resolve();
  auto it = lcpc::prof::totals.find(name);
  if (it == lcpc::prof::totals.end()) {
    *total_ms = 0;
    *count = 0;
    return 0;
  }
  *total_ms = it->second.first;
  *count = it->second.second;
  return 1;
}

size_t lcpc_prof_names(char *buf, size_t cap) {
  std::lock_guard<std::mutex> lk(lcpc::prof::mu);
  lcpc::prof::resolve();
  std::string all;
  for (auto &kv : lcpc::prof::totals) {
    all += kv.first;
    all += '\n';
  }
  if (buf && cap) {
    const size_t n = all.size() < cap - 1 ? all.size() : cap - 1;
    std::memcpy(buf, all.data(), n);
    buf[n] = 0;
  }
  return all.size();
}

}  // extern "C"
