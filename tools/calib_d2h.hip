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

#include <thread>

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
  // the step worker's situation: pinned mapped host buffers, several
  // streams, an H2D upload in flight, copies issued from another thread
  {
    void *h, *hu;
    CK(hipHostMalloc(&h, B, hipHostMallocMapped));
    CK(hipHostMalloc(&hu, B, hipHostMallocDefault));
    void *du;
    CK(hipMalloc(&du, B));
    hipStream_t ss[4];
    for (auto &x : ss) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    for (int nstr : {1, 2, 4}) {
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a0, ss[0]));
        for (int q = 1; q < nstr; ++q) CK(hipStreamWaitEvent(ss[q], a0, 0));
        const size_t part = B / nstr;
        for (int q = 0; q < nstr; ++q)
          CK(hipMemcpyAsync((char *)h + q * part, (char *)dsrc + q * part,
                            part, hipMemcpyDeviceToHost, ss[q]));
        for (int q = 1; q < nstr; ++q) {
          CK(hipEventRecord(b0, ss[q]));
          CK(hipStreamWaitEvent(ss[0], b0, 0));
        }
        CK(hipEventRecord(a1, ss[0]));
        CK(hipEventSynchronize(a1));
        float t;
        CK(hipEventElapsedTime(&t, a0, a1));
        if (rep == 2)
          printf("d2h on %d streams: %.3f ms (%.1f GB/s)\n", nstr, t,
                 B / t / 1e6);
      }
    }
    // with a 64 MiB H2D on another stream at the same time
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a0, ss[0]));
      CK(hipStreamWaitEvent(ss[1], a0, 0));
      CK(hipMemcpyAsync(du, hu, B, hipMemcpyHostToDevice, ss[1]));
      CK(hipMemcpyAsync(h, dsrc, B, hipMemcpyDeviceToHost, ss[0]));
      CK(hipEventRecord(a1, ss[0]));
      CK(hipEventRecord(b1, ss[1]));
      CK(hipDeviceSynchronize());
      float t1, t2;
      CK(hipEventElapsedTime(&t1, a0, a1));
      CK(hipEventElapsedTime(&t2, a0, b1));
      if (rep == 2)
        printf("d2h beside h2d: d2h %.3f ms, h2d done at %.3f ms\n", t1, t2);
    }
    // issued from another host thread
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipDeviceSynchronize());
      float t = 0;
      std::thread th([&]() {
        CK(hipSetDevice(0));
        CK(hipEventRecord(a0, ss[2]));
        CK(hipMemcpyAsync(h, dsrc, B, hipMemcpyDeviceToHost, ss[2]));
        CK(hipEventRecord(a1, ss[2]));
        CK(hipEventSynchronize(a1));
        CK(hipEventElapsedTime(&t, a0, a1));
      });
      th.join();
      if (rep == 2) printf("d2h from another thread: %.3f ms\n", t);
    }
  }
  return 0;
}
