// Device -> pinned-host copies on chosen SDMA engines
// (hsa_amd_memory_async_copy_on_engine): what one engine moves, whether
// engines run side by side, and what they cost a concurrent HBM-bound
// kernel (the step worker's drain).  hipMemcpyAsync D2H puts
// every copy on one engine (tools/calib_d2h: ~29 GB/s however many streams).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_bin/calib_sdma tools/calib_sdma.hip -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdio.h>
#include <stdlib.h>

#include <numaif.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <chrono>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      exit(1);                                                         \
    }                                                                  \
  } while (0)
#define HK(x)                                                          \
  do {                                                                 \
    hsa_status_t s_ = (x);                                             \
    if (s_ != HSA_STATUS_SUCCESS) {                                    \
      fprintf(stderr, "%s: hsa status 0x%x\n", #x, (unsigned)s_);      \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

__global__ void k_stream(const uint4 *a, uint4 *b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    uint4 x = a[i];
    x.x += 1;
    b[i] = x;
  }
}

static hsa_agent_t g_cpu, g_gpu;
static bool have_cpu = false, have_gpu = false;

static hsa_status_t pick(hsa_agent_t a, void *) {
  hsa_device_type_t t;
  HK(hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t));
  if (t == HSA_DEVICE_TYPE_CPU && !have_cpu) g_cpu = a, have_cpu = true;
  if (t == HSA_DEVICE_TYPE_GPU && !have_gpu) g_gpu = a, have_gpu = true;
  return HSA_STATUS_SUCCESS;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main() {
  const size_t B = 64ull << 20, S = 1ull << 30;
  void *dsrc, *sa, *sb, *h;
  CK(hipMalloc(&dsrc, B));
  CK(hipMalloc(&sa, S));
  CK(hipMalloc(&sb, S));
  CK(hipMemset(dsrc, 1, B));
  CK(hipMemset(sa, 2, S));
  CK(hipHostMalloc(&h, B, hipHostMallocMapped));
  CK(hipDeviceSynchronize());
  {
    // NUMA placement: the GPU's node, the nodes of the CPUs this process
    // may run on, and the node of the pinned buffer's first page
    int bus = 0, devn = 0, dom = 0;
    CK(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, 0));
    CK(hipDeviceGetAttribute(&devn, hipDeviceAttributePciDeviceId, 0));
    CK(hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, 0));
    char path[128];
    snprintf(path, sizeof(path), "/sys/bus/pci/devices/%04x:%02x:%02x.0/numa_node",
             dom, bus, devn);
    int gnode = -9;
    if (FILE *f = fopen(path, "r")) {
      if (fscanf(f, "%d", &gnode) != 1) gnode = -8;
      fclose(f);
    }
    cpu_set_t cs;
    CPU_ZERO(&cs);
    sched_getaffinity(0, sizeof(cs), &cs);
    int counts[8] = {0};
    for (int c = 0; c < CPU_SETSIZE; ++c) {
      if (!CPU_ISSET(c, &cs)) continue;
      for (int n = 0; n < 8; ++n) {
        snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/node%d", c, n);
        if (access(path, F_OK) == 0) counts[n]++;
      }
    }
    void *pg = h;
    int status = -99;
    syscall(SYS_move_pages, 0, 1UL, &pg, nullptr, &status, 0);
    printf("numa: gpu node %d; allowed cpus per node:", gnode);
    for (int n = 0; n < 8; ++n)
      if (counts[n]) printf(" n%d=%d", n, counts[n]);
    printf("; pinned buffer page on node %d\n", status);
  }
  HK(hsa_init());
  HK(hsa_iterate_agents(pick, nullptr));
  if (!have_cpu || !have_gpu) return 1;
  uint32_t mask = 0, pref = 0;
  HK(hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &mask));
  (void)hsa_amd_memory_get_preferred_copy_engine(g_cpu, g_gpu, &pref);
  printf("D2H engines available 0x%x preferred 0x%x\n", mask, pref);
  std::vector<int> eng;
  for (int i = 0; i < 16; ++i)
    if (mask & (1u << i)) eng.push_back(i);
  std::vector<hsa_signal_t> sig(16);
  for (auto &s : sig) HK(hsa_signal_create(1, 0, nullptr, &s));
  hipStream_t s2;
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t b0, b1;
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  // copy B bytes split over the first n engines; ms from the host clock
  auto copy = [&](int n) {
    const size_t part = (B / n + 4095) & ~(size_t)4095;
    const double t0 = now_ms();
    for (int q = 0; q < n; ++q) {
      const size_t o = q * part, len = o < B ? std::min(part, B - o) : 0;
      hsa_signal_store_relaxed(sig[q], 1);
      HK(hsa_amd_memory_async_copy_on_engine(
          (char *)h + o, g_cpu, (const char *)dsrc + o, g_gpu, len, 0,
          nullptr, sig[q], (hsa_amd_sdma_engine_id_t)(1u << eng[q]), true));
    }
    for (int q = 0; q < n; ++q)
      while (hsa_signal_wait_scacquire(sig[q], HSA_SIGNAL_CONDITION_LT, 1,
                                       UINT64_MAX, HSA_WAIT_STATE_ACTIVE))
        ;
    return now_ms() - t0;
  };
  for (int n = 1; n <= (int)eng.size() && n <= 8; n *= 2) {
    double t = 0;
    for (int rep = 0; rep < 4; ++rep) t = copy(n);
    printf("d2h over %d engine(s): %.3f ms (%.1f GB/s)\n", n, t, B / t / 1e6);
  }
  for (size_t i = 0; i < eng.size(); ++i) {
    // each engine alone, to see that they differ
    std::swap(eng[0], eng[i]);
    double t = 0;
    for (int rep = 0; rep < 3; ++rep) t = copy(1);
    printf("  engine %d alone: %.3f ms (%.1f GB/s)\n", eng[0], t, B / t / 1e6);
    std::swap(eng[0], eng[i]);
  }
  // beside an HBM-bound kernel
  for (int n = 1; n <= (int)eng.size() && n <= 4; n *= 2) {
    float tk = 0, tk2 = 0;
    double tc = 0;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(b0, s2));
      k_stream<<<2048, 256, 0, s2>>>((const uint4 *)sa, (uint4 *)sb, S / 16);
      CK(hipEventRecord(b1, s2));
      CK(hipEventSynchronize(b1));
      CK(hipEventElapsedTime(&tk, b0, b1));
      CK(hipEventRecord(b0, s2));
      k_stream<<<2048, 256, 0, s2>>>((const uint4 *)sa, (uint4 *)sb, S / 16);
      CK(hipEventRecord(b1, s2));
      tc = copy(n);
      CK(hipEventSynchronize(b1));
      CK(hipEventElapsedTime(&tk2, b0, b1));
    }
    printf("beside the kernel, %d engine(s): copy %.3f ms, kernel %.3f ms "
           "(alone %.3f)\n", n, tc, tk2, tk);
  }
  // a hipMemcpyAsync H2D (the staged proposals' upload) beside a D2H on
  // each of the first engines: does HIP's engine choice collide with it?
  {
    void *hu, *du;
    CK(hipHostMalloc(&hu, B, hipHostMallocDefault));
    CK(hipMalloc(&du, B));
    const double tu0 = now_ms();
    CK(hipMemcpyAsync(du, hu, B, hipMemcpyHostToDevice, s2));
    CK(hipStreamSynchronize(s2));
    printf("h2d alone: %.3f ms\n", now_ms() - tu0);
    for (size_t i = 0; i < eng.size() && i < 4; ++i) {
      std::swap(eng[0], eng[i]);
      double tc = 0, tu = 0;
      for (int rep = 0; rep < 3; ++rep) {
        const double t0 = now_ms();
        hsa_signal_store_relaxed(sig[0], 1);
        HK(hsa_amd_memory_async_copy_on_engine(
            h, g_cpu, dsrc, g_gpu, B, 0, nullptr, sig[0],
            (hsa_amd_sdma_engine_id_t)(1u << eng[0]), true));
        CK(hipMemcpyAsync(du, hu, B, hipMemcpyHostToDevice, s2));
        CK(hipStreamSynchronize(s2));
        tu = now_ms() - t0;
        while (hsa_signal_wait_scacquire(sig[0], HSA_SIGNAL_CONDITION_LT, 1,
                                         UINT64_MAX, HSA_WAIT_STATE_ACTIVE))
          ;
        tc = now_ms() - t0;
      }
      printf("d2h on engine %d beside a hip h2d: d2h done %.3f ms, h2d done "
             "%.3f ms\n", eng[0], tc, tu);
      std::swap(eng[0], eng[i]);
    }
  }
  for (auto &s : sig) hsa_signal_destroy(s);
  HK(hsa_shut_down());
  return 0;
}
