// selftest.cpp -- on-device check of the stream-ordered pool's fences (pool.hpp, DBuf).
//
// A block released while a slow writer on another stream still owns it must not be overwritten
// by that writer after its next owner's first kernel: each round queues a writer that spins
// ~spin_us before storing X, releases the block (fence on the writer's stream), takes the same
// block on a third stream and stores Y there at once, then reads it back.  With the fence every
// word reads Y; without it (the unfenced control: the buffer is settle()d before release, the
// fast store runs first) the late writer leaves X behind.  This replaces nothing in the
// reference (whose buffers are host Vecs, lcpc-2d/src/lib.rs:659-690); it is the device-side
// evidence for the pool that the commit / prove / shard paths share.
#include "host_internal.hpp"

#include <vector>

namespace lcpc_host {
namespace {

__global__ __launch_bounds__(256) void k_late_fill(uint32_t *__restrict__ p, size_t n, uint32_t v, uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

__global__ __launch_bounds__(256) void k_fill(uint32_t *__restrict__ p, size_t n, uint32_t v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

constexpr size_t WORDS = (1 << 18) + 37;
constexpr unsigned BLOCKS = 1024;

// one round: the block is allocated on `a`, the writer runs on `w` (a itself, or a second stream
// marked with use()), the next owner on `b`; adds the words not reading Y to *bad
lcpc_status pool_round(Device *dev, hipStream_t a, hipStream_t w, hipStream_t b, bool fenced, uint64_t ticks,
                       uint32_t x, uint32_t y, uint64_t *bad, uint64_t *reused) {
  struct Restore {
    hipStream_t prev = t_stream;
    ~Restore() { t_stream = prev; }
  } restore;
  void *first = nullptr;
  {
    t_stream = a;
    DBuf buf;
    HIP_TRY(buf.alloc(dev, WORDS * 4));
    first = buf.p;
    buf.use(w);
    hipLaunchKernelGGL(k_late_fill, dim3(BLOCKS), dim3(256), 0, w, (uint32_t *)buf.p, WORDS, x, ticks);
    HIP_TRY(hipGetLastError());
    if (!fenced) buf.settle();  // the control: claim the writer is done while it still spins
  }  // released here, fenced on a and w unless settled
  std::vector<uint32_t> host(WORDS);
  {
    t_stream = b;
    DBuf nxt;
    HIP_TRY(nxt.alloc(dev, WORDS * 4));
    if (nxt.p == first) ++*reused;
    hipLaunchKernelGGL(k_fill, dim3(BLOCKS), dim3(256), 0, b, (uint32_t *)nxt.p, WORDS, y);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(b));
    HIP_TRY(hipStreamSynchronize(w));  // the late writer has finished either way
    HIP_TRY(hipStreamSynchronize(a));
    HIP_TRY(hipMemcpy(host.data(), nxt.p, WORDS * 4, hipMemcpyDeviceToHost));
    nxt.settle();
  }
  for (size_t i = 0; i < WORDS; i++) *bad += host[i] != y;
  return LCPC_OK;
}

}  // namespace
}  // namespace lcpc_host

using namespace lcpc_host;

extern "C" lcpc_status lcpc_selftest_pool_ordering(int rounds, uint32_t spin_us, uint64_t *violations,
                                                   uint64_t *control_violations, uint64_t *reused) {
  if (rounds < 1 || !violations || !control_violations || !reused || spin_us > 100000)
    return fail(LCPC_ERR_INVALID_ARG, "rounds / outputs / spin_us");
  lcpc_status st;
  Device *dev = current_device(&st);
  if (!dev) return st;
  *violations = *control_violations = *reused = 0;
  const uint64_t ticks = (uint64_t)spin_us * 100;  // wall_clock64 runs at 100 MHz on gfx950
  // blocks of the test's size that earlier calls left cached are held aside for the run (a
  // host-ordered take), so that every take below can only return the block just released
  const size_t rb = Device::round_bytes(WORDS * 4);
  std::vector<void *> held;
  while (void *q = dev->blocks.take(rb, hipStream_t{})) held.push_back(q);
  Lease la(dev, POOL_BULK);
  const hipStream_t a = la.s;
  hipStream_t w = dev->acquire_stream(POOL_HIGH);
  hipStream_t b = dev->acquire_stream(POOL_PROVER);
  lcpc_status rc = LCPC_OK;
  for (int r = 0; r < rounds && rc == LCPC_OK; r++) {
    const uint32_t x = 0x5a000000u + 2 * r, y = x + 1;
    // fenced: the writer on the allocating stream, then on a use()d second stream
    if ((rc = pool_round(dev, a, a, b, true, ticks, x, y, violations, reused)) != LCPC_OK) break;
    if ((rc = pool_round(dev, a, w, b, true, ticks, x, y, violations, reused)) != LCPC_OK) break;
    rc = pool_round(dev, a, w, b, false, ticks, x, y, control_violations, reused);
  }
  (void)hipStreamSynchronize(w);
  (void)hipStreamSynchronize(b);
  dev->release_stream(w, POOL_HIGH);
  dev->release_stream(b, POOL_PROVER);
  for (void *q : held) dev->blocks.put(q, rb, nullptr, 0);
  return rc;
}
