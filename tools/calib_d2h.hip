// Which engine moves a device -> pinned-host copy, and what it costs a
// concurrent HBM-bound kernel (the step worker's drain).
// For each host allocation flavour: a 64 MiB hipMemcpyAsync D2H alone, a
// streaming kernel alone, and both at once on two streams; times from HIP
// events.  Under rocprofv3 --kernel-trace --memory-copy-trace a blit shows
// as __amd_rocclr_copyBuffer, an SDMA copy as MEMORY_COPY_DEVICE_TO_HOST.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_bin/calib_d2h tools/calib_d2h.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

// a read + write stream over a large buffer (HBM-bound)
__global__ void k_stream(const uint4 *a, uint4 *b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    uint4 x = a[i];
    x.x += 1;
    b[i] = x;
  }
}

int main() {
  const size_t B = 64ull << 20, S = 1ull << 30;  // copy, stream bytes
  void *dsrc, *sa, *sb;
  CK(hipMalloc(&dsrc, B));
  CK(hipMalloc(&sa, S));
  CK(hipMalloc(&sb, S));
  CK(hipMemset(dsrc, 1, B));
  CK(hipMemset(sa, 2, S));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a0, a1, b0, b1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  struct {
    const char *name;
    unsigned flags;
    int reg;  // 1: malloc + hipHostRegister
  } kinds[] = {{"hostmalloc_default", hipHostMallocDefault, 0},
               {"hostmalloc_mapped", hipHostMallocMapped, 0},
               {"hostmalloc_noncoherent", hipHostMallocNonCoherent, 0},
               {"hostmalloc_coherent", hipHostMallocCoherent, 0},
               {"malloc_registered", 0, 1}};
  const unsigned grid = 2048;
  for (auto &k : kinds) {
    void *h = nullptr;
    if (k.reg) {
      h = aligned_alloc(4096, B);
      CK(hipHostRegister(h, B, hipHostRegisterDefault));
    } else {
      CK(hipHostMalloc(&h, B, k.flags));
    }
    float tc = 0, tk = 0, tc2 = 0, tk2 = 0;
    for (int rep = 0; rep < 3; ++rep) {
      // copy alone
      CK(hipEventRecord(a0, s1));
      CK(hipMemcpyAsync(h, dsrc, B, hipMemcpyDeviceToHost, s1));
      CK(hipEventRecord(a1, s1));
      CK(hipEventSynchronize(a1));
      CK(hipEventElapsedTime(&tc, a0, a1));
      // kernel alone
      CK(hipEventRecord(b0, s2));
      k_stream<<<grid, 256, 0, s2>>>((const uint4 *)sa, (uint4 *)sb, S / 16);
      CK(hipEventRecord(b1, s2));
      CK(hipEventSynchronize(b1));
      CK(hipEventElapsedTime(&tk, b0, b1));
      // both at once
      CK(hipEventRecord(b0, s2));
      k_stream<<<grid, 256, 0, s2>>>((const uint4 *)sa, (uint4 *)sb, S / 16);
      CK(hipEventRecord(b1, s2));
      CK(hipEventRecord(a0, s1));
      CK(hipMemcpyAsync(h, dsrc, B, hipMemcpyDeviceToHost, s1));
      CK(hipEventRecord(a1, s1));
      CK(hipDeviceSynchronize());
      CK(hipEventElapsedTime(&tc2, a0, a1));
      CK(hipEventElapsedTime(&tk2, b0, b1));
    }
    printf("%-24s copy %.3f ms (%.1f GB/s)  kernel %.3f ms  together: "
           "copy %.3f kernel %.3f ms\n",
           k.name, tc, B / tc / 1e6, tk, tc2, tk2);
    if (k.reg) {
      CK(hipHostUnregister(h));
      free(h);
    } else {
      CK(hipHostFree(h));
    }
  }
  return 0;
}
