// calib_hbm.hip -- calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE and the
// achievable rate for the access shapes the step kernel uses:
//   u64 coalesced (8 B/lane), uint4 coalesced (16 B/lane), and 16 B
//   random slots in a table larger than the Infinity Cache (KV apply).
// Build: hipcc --offload-arch=gfx950 -O3 -o calib tools/calib_hbm.hip
// Run under: rocprofv3 --pmc FETCH_SIZE -- ./calib   (and WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void rd_u64(const uint64_t *p, uint64_t n, uint64_t *sink) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t s = 0;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) s += p[i];
  if (s == 0x123456789ull) *sink = s;
}
__global__ void rd_u4(const uint4 *p, uint64_t n, uint64_t *sink) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t s = 0;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 q = p[i];
    s += q.x ^ q.w;
  }
  if (s == 0x12345679u) *sink = s;
}
__global__ void wr_u64(uint64_t *p, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) p[i] = i;
}
__global__ void wr_u4(uint4 *p, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__device__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// one random 16 B slot per lane in a table of `slots` uint4 (read+write)
__global__ void rmw_rand(uint4 *p, uint64_t slots, uint64_t n, uint32_t salt) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t s = mix(i ^ ((uint64_t)salt << 40)) % slots;
  uint4 q = p[s];
  q.x += 1;
  p[s] = q;
}
__global__ void rd_rand(const uint4 *p, uint64_t slots, uint64_t n,
                        uint32_t salt, uint64_t *sink) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t s = mix(i ^ ((uint64_t)salt << 40)) % slots;
  uint4 q = p[s];
  if (q.x == 0x12345679u) *sink = q.y;
}

typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__device__ uint4 ld_nt(const uint4 *p) {
  u4v v = __builtin_nontemporal_load((const u4v *)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ void st_nt(uint4 *p, uint4 q) {
  u4v v = {q.x, q.y, q.z, q.w};
  __builtin_nontemporal_store(v, (u4v *)p);
}
// 8 independent random 16 B reads per lane (memory-level parallelism);
// NT: the loads carry the nontemporal hint (streaming, no L2 reuse)
template <bool NT>
__global__ void rd_rand8(const uint4 *p, uint64_t slots, uint64_t n,
                         uint32_t salt, uint64_t *sink) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint4 q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint64_t s = mix((i * 8 + k) ^ ((uint64_t)salt << 40)) % slots;
    q[k] = NT ? ld_nt(p + s) : p[s];
  }
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= q[k].x + q[k].w;
  if (x == 0x12345679u) *sink = x;
}
// 8 random 8 B reads per lane
__global__ void rd_rand8_u2(const uint2 *p, uint64_t slots, uint64_t n,
                            uint32_t salt, uint64_t *sink) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint2 q[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint64_t s = mix((i * 8 + k) ^ ((uint64_t)salt << 40)) % slots;
    q[k] = p[s];
  }
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= q[k].x + q[k].y;
  if (x == 0x12345679u) *sink = x;
}
// random 16 B RMW with a nontemporal store
__global__ void rmw_rand_nt(uint4 *p, uint64_t slots, uint64_t n,
                            uint32_t salt) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t s = mix(i ^ ((uint64_t)salt << 40)) % slots;
  uint4 q = ld_nt(p + s);
  q.x += 1;
  st_nt(p + s, q);
}

int main() {
  const uint64_t bytes = 4ull << 30;  // 4 GiB streams (>> 256 MiB L3)
  void *buf;
  uint64_t *sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 8));
  CK(hipMemset(buf, 0, bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = 256 * 8 * 4, blk = 256;
  float ms;
#define TIME(name, nbytes, launch)                                        \
  for (int rep = 0; rep < 3; ++rep) {                                     \
    CK(hipEventRecord(a));                                                \
    launch;                                                               \
    CK(hipEventRecord(b));                                                \
    CK(hipEventSynchronize(b));                                           \
    CK(hipEventElapsedTime(&ms, a, b));                                   \
    printf("%-10s rep %d: %.3f ms  %.1f GB/s (of %.0f MB)\n", name, rep,  \
           ms, (double)(nbytes) / ms / 1e6, (double)(nbytes) / 1e6);      \
  }
  TIME("rd_u64", bytes, (rd_u64<<<grid, blk>>>((uint64_t *)buf, bytes / 8, sink)));
  TIME("rd_u4", bytes, (rd_u4<<<grid, blk>>>((uint4 *)buf, bytes / 16, sink)));
  TIME("wr_u64", bytes, (wr_u64<<<grid, blk>>>((uint64_t *)buf, bytes / 8)));
  TIME("wr_u4", bytes, (wr_u4<<<grid, blk>>>((uint4 *)buf, bytes / 16)));
  const uint64_t n = 1ull << 24, slots = bytes / 16;  // 16M random slots
  TIME("rd_rand16", n * 16, (rd_rand<<<(unsigned)(n / 256), 256>>>((uint4 *)buf, slots, n, rep, sink)));
  TIME("rmw_rand16", n * 32, (rmw_rand<<<(unsigned)(n / 256), 256>>>((uint4 *)buf, slots, n, rep)));
  const uint64_t n8 = 1ull << 24;  // 16M lanes x 8 reads
  TIME("rd_rand8", n8 * 128, (rd_rand8<false><<<(unsigned)(n8 / 256), 256>>>((uint4 *)buf, slots, n8, rep, sink)));
  TIME("rd_rand8nt", n8 * 128, (rd_rand8<true><<<(unsigned)(n8 / 256), 256>>>((uint4 *)buf, slots, n8, rep, sink)));
  TIME("rd_rand8u2", n8 * 64, (rd_rand8_u2<<<(unsigned)(n8 / 256), 256>>>((uint2 *)buf, slots * 2, n8, rep, sink)));
  TIME("rmw_randnt", n * 32, (rmw_rand_nt<<<(unsigned)(n / 256), 256>>>((uint4 *)buf, slots, n, rep)));
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
