// hipHostGetDevicePointer on interior pointers of page-locked blocks (hipHostMalloc, Default and
// Portable): is the returned device address base + offset?  And does a kernel's store into the
// mapped block read back on the host after hipStreamSynchronize?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k_fill(uint64_t *p, size_t n, uint64_t v) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) p[i] = v + i;
}
int main() {
  int bad = 0;
  for (unsigned flags : {hipHostMallocDefault, hipHostMallocPortable}) {
    void *h = nullptr;
    if (hipHostMalloc(&h, 1 << 20, flags) != hipSuccess) { printf("alloc failed\n"); return 1; }
    void *d0 = nullptr, *d1 = nullptr;
    hipError_t e0 = hipHostGetDevicePointer(&d0, h, 0);
    hipError_t e1 = hipHostGetDevicePointer(&d1, (char *)h + 4104, 0);
    printf("flags %u base h=%p d=%p (%d) interior d=%p (%d) diff %ld same_va %d\n", flags, h, d0, (int)e0, d1, (int)e1,
           (long)((char *)d1 - (char *)d0), d0 == h);
    if (e1 != hipSuccess || (char *)d1 - (char *)d0 != 4104) bad++;
    hipStream_t s;
    hipStreamCreate(&s);
    uint64_t *dp = (uint64_t *)((char *)d0 + 8192);
    hipLaunchKernelGGL(k_fill, dim3(4), dim3(256), 0, s, dp, 1000, 77);
    hipStreamSynchronize(s);
    uint64_t *hp = (uint64_t *)((char *)h + 8192);
    for (int i = 0; i < 1000; i++) if (hp[i] != 77 + (uint64_t)i) { bad++; break; }
    hipStreamDestroy(s);
    hipHostFree(h);
  }
  void *m = malloc(1 << 16), *dm = nullptr;
  hipError_t em = hipHostGetDevicePointer(&dm, m, 0);
  printf("pageable: err %d d=%p\n", (int)em, dm);
  if (em == hipSuccess) bad++;
  printf("bad %d\n", bad);
  return bad != 0;
}
