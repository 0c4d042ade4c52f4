// prof.hpp -- optional per-kernel timing with HIP events on the launching stream.
// Enabled by lcpc_prof_enable(1); every launch wrapped in prof::Scope records a start/stop
// event pair; lcpc_prof_get() synchronizes and accumulates durations per kernel name.
#pragma once
#include <hip/hip_runtime.h>

namespace lcpc {
namespace prof {

bool enabled();
// record one event pair around the launches issued while the scope is alive
class Scope {
 public:
  Scope(const char *name, hipStream_t s);
  ~Scope();

 private:
  const char *name_;
  hipEvent_t a_ = nullptr, b_ = nullptr;
  hipStream_t s_;
};

// wall time of a host-side phase (accumulated under `name`, same table as the kernels)
class HostScope {
 public:
  explicit HostScope(const char *name);
  ~HostScope();

 private:
  const char *name_;
  double t0_ = -1.0;
};

}  // namespace prof
}  // namespace lcpc
