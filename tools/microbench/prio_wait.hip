// prio_wait.hip -- do cross-stream event waits hold between streams of different priority?
//
// Each iteration: a producer stream writes generation g into a 64 MiB buffer (a kernel long
// enough to still run when the consumer is enqueued) and records event E; the consumer stream
// waits on E and counts words that are not g.  The same event object is re-recorded every
// iteration (as the sharded driver's per-polynomial events are), and a third stream keeps the
// GPU busy with unrelated work.  Any nonzero count means a wait did not hold.
//
// Second pattern (rerecord, the round-3 review's hypothesis for the sharded driver's wrong root):
// record E on A after the slow fill, enqueue B's wait on E, then at once re-record the SAME E on a
// third stream C that is idle (its record completes at once) -- before B's wait can have retired.
// A runtime that resolved B's wait against E's latest record instead of the record current at the
// wait call would let B's check run before the fill: stale words.  Every combination of the three
// streams' priorities, at the default 4 hardware queues per priority.
// Build: hipcc -O3 --offload-arch=gfx950 prio_wait.hip -o prio_wait
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void k_fill(unsigned *x, size_t n, unsigned g) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    x[i] = g;
}
__global__ void k_check(const unsigned *x, size_t n, unsigned g, unsigned *bad) {
  unsigned b = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b += x[i] != g;
  if (b) atomicAdd(bad, b);
}
__global__ void k_busy(unsigned *y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = y[i] * 1664525u + 1013904223u;
}

int run(int prod_high, int cons_high, int iters) {
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t sp, sc, sb;
  CK(hipStreamCreateWithPriority(&sp, hipStreamNonBlocking, prod_high ? hi : lo));
  CK(hipStreamCreateWithPriority(&sc, hipStreamNonBlocking, cons_high ? hi : lo));
  CK(hipStreamCreateWithPriority(&sb, hipStreamNonBlocking, lo));
  const size_t n = (size_t)16 << 20;  // 64 MiB
  unsigned *x, *y, *bad;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  CK(hipMemset(x, 0xff, n * 4));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipDeviceSynchronize());
  for (int g = 0; g < iters; g++) {
    hipLaunchKernelGGL(k_busy, dim3(512), dim3(256), 0, sb, y, n);
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, sp, x, n, (unsigned)g);  // few blocks: slow
    CK(hipEventRecord(ev, sp));
    CK(hipStreamWaitEvent(sc, ev, 0));
    hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, sc, x, n, (unsigned)g, bad);
    // the producer must not overwrite x before the check has read it
    CK(hipEventRecord(ev, sc));
    CK(hipStreamWaitEvent(sp, ev, 0));
  }
  CK(hipDeviceSynchronize());
  unsigned h = 0;
  CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
  printf("producer %s, consumer %s: %d iterations, %u stale words%s\n", prod_high ? "high" : "normal",
         cons_high ? "high" : "normal", iters, h, h ? "  <-- a wait did not hold" : "");
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(bad));
  CK(hipEventDestroy(ev));
  CK(hipStreamDestroy(sp));
  CK(hipStreamDestroy(sc));
  CK(hipStreamDestroy(sb));
  return h != 0;
}

int run_rerecord(int a_high, int b_high, int c_high, int iters) {
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t A, B, Cs, busy;
  CK(hipStreamCreateWithPriority(&A, hipStreamNonBlocking, a_high ? hi : lo));
  CK(hipStreamCreateWithPriority(&B, hipStreamNonBlocking, b_high ? hi : lo));
  CK(hipStreamCreateWithPriority(&Cs, hipStreamNonBlocking, c_high ? hi : lo));
  CK(hipStreamCreateWithPriority(&busy, hipStreamNonBlocking, lo));
  const size_t n = (size_t)16 << 20;  // 64 MiB
  unsigned *x, *y, *bad;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  CK(hipMemset(x, 0xff, n * 4));
  hipEvent_t E, back;
  CK(hipEventCreateWithFlags(&E, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&back, hipEventDisableTiming));
  CK(hipDeviceSynchronize());
  for (int g = 0; g < iters; g++) {
    hipLaunchKernelGGL(k_busy, dim3(512), dim3(256), 0, busy, y, n);
    hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, A, x, n, (unsigned)g);  // few blocks: slow
    CK(hipEventRecord(E, A));
    CK(hipStreamWaitEvent(B, E, 0));
    CK(hipEventRecord(E, Cs));  // the re-record, on an idle stream, before B's wait retires
    hipLaunchKernelGGL(k_check, dim3(1024), dim3(256), 0, B, x, n, (unsigned)g, bad);
    CK(hipEventRecord(back, B));  // (a separate event: the next fill waits for this check)
    CK(hipStreamWaitEvent(A, back, 0));
  }
  CK(hipDeviceSynchronize());
  unsigned h = 0;
  CK(hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost));
  printf("rerecord: A %s, B %s, C %s: %d iterations, %u stale words%s\n", a_high ? "high" : "normal",
         b_high ? "high" : "normal", c_high ? "high" : "normal", iters, h, h ? "  <-- a wait did not hold" : "");
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(bad));
  CK(hipEventDestroy(E));
  CK(hipEventDestroy(back));
  for (hipStream_t s : {A, B, Cs, busy}) CK(hipStreamDestroy(s));
  return h != 0;
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 300;
  int bad = 0;
  bad |= run(0, 0, iters);
  bad |= run(0, 1, iters);
  bad |= run(1, 0, iters);
  bad |= run(1, 1, iters);
  for (int m = 0; m < 8; m++) bad |= run_rerecord(m & 1, (m >> 1) & 1, (m >> 2) & 1, iters);
  return bad;
}
