// drb_worker.hpp -- a step worker's round outputs for the host
// (drb_worker_export / drb_worker_wait, include/drb_engine.h), included at
// the end of drb_engine.hip.
//
// engine.processSteps (engine.go:1304-1364) hands each node's Update to the
// host every round: the ReadyToReads (node.processReadyToRead, node.go:1081),
// the reads served behind them (pendingReadIndex.applied, request.go:
// 930-953) and the applied entries (pendingProposals.applied, node.go:
// 243-257).  Here one export covers every group of a replica slot:
//   1. on the engine stream, behind the round: per lane the three record
//      counts, one exclusive scan of {ReadyToReads, values, deferred}
//      (hipCUB), and a compaction of the lean records (include/drb_engine.h:
//      a word per lane -- its applied count included --, a 4 B ctx tag per
//      ReadyToRead, 4 B + 2 bits per served read, 8 B per ReadyToRead whose
//      reads were not served) into device staging[parity]; the totals go
//      straight to mapped host memory;
//   2. the engine's drain thread waits for that compaction and copies
//      exactly those bytes into the caller's pinned buffers on the
//      engine's download SDMA engine (drb_hsa.hpp: a completion signal per
//      buffer set): the transfer overlaps the next rounds at PCIe rate
//      (~56 GB/s) and takes no CU, and the staged proposals go up on
//      another engine.  Measured (tools/calib_sdma, tools/calib_d2h,
//      profiles/r05_worker): a drain kernel writing host memory from 256
//      workgroups slowed the concurrent leader kernel from 0.72 to 1.76 ms;
//      hipMemcpyAsync D2H runs either on one SDMA queue at ~29 GB/s or,
//      inside a PyTorch process, as __amd_rocclr_copyBuffer blit kernels
//      that take CUs from the round; one engine moves 56 GB/s beside an
//      HBM-bound kernel without slowing it, and an upload and a download on
//      the same engine run one after the other.
// No host synchronisation in the caller until drb_worker_wait.
#pragma once

#include <condition_variable>
#include <deque>
#include <thread>

// staging sets: an export takes a free one and holds it until its wait
// (two per step worker, one per partition and parity)
constexpr int kWorkerSets = 16;

struct WorkerSet {
  hipEvent_t ev_staged = nullptr, ev_drained = nullptr;
  uint32_t *lanes = nullptr;  // [G]
  uint32_t *rd = nullptr;     // ctx tags
  uint32_t *val = nullptr;
  uint32_t *meta = nullptr;   // 2-bit codes, 16 per word
  uint64_t *dfr = nullptr;    // deferred ReadyToReads' Index
  uint64_t cap_rd = 0, cap_val = 0, cap_df = 0;  // staging capacity
  // the buffers of the export in flight (waited for or not)
  const drb_worker_bufs *owner = nullptr;
  bool issued = false;  // the copies of its job issued
  int err = 0;          // a failed copy (reported and cleared by its wait)
  hsa_signal_t done{0};  // copies outstanding (HSA)
};

struct WorkerState {
  hipStream_t sx = nullptr;  // the drain thread's copies
  WorkerSet set[kWorkerSets];
  uint4 *cnt = nullptr, *off = nullptr;  // [G + 1]
  void *tmp = nullptr;
  size_t tmp_bytes = 0;
  unsigned long long *hdr = nullptr;      // pinned, mapped [sets][4]: totals
  unsigned long long *hdr_dev = nullptr;  // ... its device address
  // the drain thread: one job per export, in order
  struct Job {
    int k;
    drb_worker_bufs b;  // (the pointers and capacities at export time)
    uint64_t np;        // lanes exported
  };
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Job> jobs;
  bool stop = false;
  // the copies on the engine's download SDMA engine (drb_hsa.hpp;
  // hipMemcpyAsync on sx when HSA is unavailable)
  bool hsa = false;
};

// until the copies of staging set k are done
static void worker_wait_copies(WorkerState &w, int k) {
  // (a set never used has no signal yet: nothing to wait for)
  if (!w.hsa || !w.set[k].done.handle) return;
  while (hsa_signal_wait_scacquire(w.set[k].done, HSA_SIGNAL_CONDITION_LT, 1,
                                   UINT64_MAX, HSA_WAIT_STATE_BLOCKED) >= 1) {
  }
}

// every export's copies issued and done (the drain thread idle)
static void worker_quiesce(WorkerState &w) {
  {
    std::unique_lock<std::mutex> g(w.mu);
    w.cv.wait(g, [&] {
      if (!w.jobs.empty()) return false;
      for (const WorkerSet &s : w.set)
        if (s.owner && !s.issued) return false;
      return true;
    });
  }
  for (int k = 0; k < kWorkerSets; ++k) worker_wait_copies(w, k);
}

namespace {

struct U4Sum {
  __host__ __device__ uint4 operator()(const uint4 &a, const uint4 &b) const {
    return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
};

// the applied range (applied_index, sm_index] of the round a replica last
// ran, as drb_apply_results reads it (k_apply_results)
__device__ inline void worker_apply_range(const View &v, uint32_t slot,
                                          uint64_t g, uint64_t *lo,
                                          uint64_t *hi) {
  *lo = *hi = 0;
  const uint32_t fl = v.u32[u32_ix(v, W_FLAGS, slot, g)];
  const bool frozen =
      (fl & (DRB_F_FALLBACK | DRB_F_ERROR)) && !(fl & DRB_F_APPLY_STOPPED);
  if ((fl & DRB_F_HOSTED) && !frozen) {
    *lo = pk_field(v, slot, g, PI_APPLIED_INDEX);
    *hi = pk_field(v, slot, g, PI_SM_INDEX);
  }
}

// the host's own entries among the applied ones (include/drb_engine.h):
// those of its registered session client (sess), else every entry with a
// ClientID -- raft's own empty entries have none (statemachine.go:939)
__device__ inline uint32_t worker_applied(const View &v, uint32_t slot,
                                          uint64_t g, const uint64_t *sess) {
  uint64_t lo, hi;
  worker_apply_range(v, slot, g, &lo, &hi);
  const uint64_t sc = sess ? sess[g] : 0ull;
  uint32_t n = 0;
  for (uint64_t idx = lo + 1; idx <= hi; ++idx) {
    const uint64_t client = lo64(v.ring[ring_ix(v, slot, idx, 1, g)]);
    n += client != 0 && (sess == nullptr || client == sc);
  }
  return min(n, 0xffffu);
}

// lanes g0, g0 + stride, ... (np of them): one step worker's partition
__global__ void k_worker_count(const View v, uint32_t slot, uint32_t n_reads,
                               uint64_t g0, uint64_t stride, uint64_t np,
                               uint4 *cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > np) return;
  const uint64_t g = g0 + i * stride;
  uint4 c = make_uint4(0, 0, 0, 0);
  if (i < np) {
    const uint32_t nr = min(v.rtr_count[ix(v, slot, g)], (uint32_t)RTR_CAP);
    const uint32_t m =
        nr && n_reads ? v.read_served[ix(v, slot, g)] & ((1u << nr) - 1u) : 0u;
    c.x = nr;
    c.y = (uint32_t)__popc(m) * n_reads;
    c.z = nr - (uint32_t)__popc(m);
  }
  cnt[i] = c;  // cnt[np] = 0: the scan's last element is the total
}

// a served read's 2-bit code and value word (include/drb_engine.h):
// read_res.y is vlen | found << 31 (serve_reads_lane), .x the value's first
// 4 bytes
__device__ inline uint32_t worker_code(uint2 w, uint32_t *word) {
  *word = w.x;
  if (!(w.y >> 31)) {
    *word = 0;
    return DRB_WORKER_MISS;
  }
  const uint32_t vlen = w.y & 0x7fffffffu;
  if (vlen == 4) return DRB_WORKER_V4;
  if (vlen > 4) return DRB_WORKER_LONG;
  *word = (w.x & ((1u << (8 * vlen)) - 1u)) | (vlen << 24);
  return DRB_WORKER_SHORT;
}

__global__ void k_worker_compact(const View v, uint32_t slot,
                                 uint32_t n_reads, uint64_t g0,
                                 uint64_t stride, uint64_t np,
                                 const uint64_t *sess, const uint4 *off,
                                 uint32_t *lanes, uint32_t *rd,
                                 uint64_t cap_rd, uint32_t *val,
                                 uint32_t *meta, uint64_t cap_val,
                                 uint64_t *dfr, uint64_t cap_df,
                                 unsigned long long *tot) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == np) {  // the totals, into mapped host memory
    tot[0] = off[i].x;
    tot[1] = off[i].y;
    tot[2] = off[i].z;
    __threadfence_system();
  }
  if (i >= np) return;
  const uint64_t g = g0 + i * stride;
  const uint4 o = off[i];
  const uint32_t nr = min(v.rtr_count[ix(v, slot, g)], (uint32_t)RTR_CAP);
  const uint32_t m =
      nr && n_reads ? v.read_served[ix(v, slot, g)] & ((1u << nr) - 1u) : 0u;
  const uint32_t na = worker_applied(v, slot, g, sess);
  lanes[i] = nr | (m << 4) | (na << 12);
  uint64_t vo = o.y, di = o.z;
  // the codes of this lane's reads, one word (16 codes) at a time; the
  // first and last words may be shared with the neighbouring lanes (the
  // staging words start zeroed, shared ones take an atomicOr)
  uint32_t word = 0;
  uint64_t wi = vo / 16;
  auto flush = [&](bool last) {
    if (!word) return;
    const uint64_t first_w = o.y / 16;
    const bool shared = wi == first_w || last;
    if (wi * 16 < cap_val) {
      if (shared)
        atomicOr(&meta[wi], word);
      else
        meta[wi] = word;
    }
    word = 0;
  };
  for (uint32_t k = 0; k < nr; ++k) {
    const uint4 c0 = v.rtr[rtr_ix(v, slot, k, 0, g)];
    if (o.x + k < cap_rd) rd[o.x + k] = c0.z;  // the ctx tag: Low's low word
    if (!((m >> k) & 1u)) {  // not served: the host needs its Index
      if (di < cap_df) dfr[di] = (uint64_t)c0.x | ((uint64_t)c0.y << 32);
      ++di;
      continue;
    }
    for (uint32_t j = 0; j < n_reads; ++j, ++vo) {
      uint32_t x;
      const uint32_t code =
          worker_code(v.read_res[rres_ix(v, slot, k, j, g)], &x);
      if (vo < cap_val) val[vo] = x;
      if (vo / 16 != wi) {
        flush(false);
        wi = vo / 16;
      }
      word |= code << (2 * (vo & 15));
    }
  }
  flush(true);
}

}  // namespace

static void worker_free(drb_engine *e) {
  WorkerState *w = e->worker;
  if (!w) return;
  if (w->th.joinable()) {
    {
      std::lock_guard<std::mutex> g(w->mu);
      w->stop = true;
    }
    w->cv.notify_all();
    w->th.join();
  }
  if (w->sx) (void)hipStreamSynchronize(w->sx);
  for (int k = 0; k < kWorkerSets; ++k) {
    WorkerSet &s = w->set[k];
    if (w->hsa) {
      worker_wait_copies(*w, k);
      if (s.done.handle) (void)hsa_signal_destroy(s.done);
    }
    if (s.ev_staged) (void)hipEventDestroy(s.ev_staged);
    if (s.ev_drained) (void)hipEventDestroy(s.ev_drained);
    if (s.lanes) (void)hipFree(s.lanes);
    if (s.rd) (void)hipFree(s.rd);
    if (s.val) (void)hipFree(s.val);
    if (s.meta) (void)hipFree(s.meta);
    if (s.dfr) (void)hipFree(s.dfr);
  }
  if (w->cnt) (void)hipFree(w->cnt);
  if (w->off) (void)hipFree(w->off);
  if (w->tmp) (void)hipFree(w->tmp);
  if (w->hdr) (void)hipHostFree(w->hdr);
  if (w->sx) (void)hipStreamDestroy(w->sx);
  delete w;
  e->worker = nullptr;
}

// the drain thread's copies of one export: exactly the compacted bytes
// (totals from the mapped header, capped by the caller's capacities)
static hipError_t worker_copy(drb_engine *e, WorkerState &w,
                              const WorkerState::Job &j) {
  const int k = j.k;
  WorkerSet &s = w.set[k];
  hipError_t r = hipEventSynchronize(s.ev_staged);
  if (r != hipSuccess) return r;
  const unsigned long long *t = w.hdr + 4 * k;
  const uint64_t nrd = std::min<uint64_t>(t[0], j.b.reads_cap);
  const uint64_t nval = std::min<uint64_t>(t[1], j.b.values_cap);
  const uint64_t ndf = std::min<uint64_t>(t[2], j.b.deferred_cap);
  struct {
    void *dst;
    const void *src;
    size_t n;
  } cp[5] = {{j.b.lanes, s.lanes, (size_t)j.np * 4},
             {j.b.reads, s.rd, nrd * 4},
             {j.b.values, s.val, nval * 4},
             {j.b.value_meta, s.meta, (nval + 3) / 4},
             {j.b.deferred, s.dfr, ndf * 8}};
  if (w.hsa) {
    const HsaXfer &x = e->xfer;
    int n = 0;
    for (auto &c : cp) n += c.n && c.dst;
    hsa_signal_store_screlease(s.done, n);
    for (auto &c : cp) {
      if (!(c.n && c.dst)) continue;
      if (hsa_amd_memory_async_copy_on_engine(
              c.dst, x.cpu, c.src, x.gpu, c.n, 0, nullptr, s.done,
              (hsa_amd_sdma_engine_id_t)x.down, true) != HSA_STATUS_SUCCESS) {
        hsa_signal_subtract_screlease(s.done, 1);
        r = hipErrorUnknown;
      }
    }
    return r;
  }
  for (auto &c : cp)
    if (c.n && c.dst && r == hipSuccess)
      r = hipMemcpyAsync(c.dst, c.src, c.n, hipMemcpyDeviceToHost, w.sx);
  if (r == hipSuccess) r = hipEventRecord(s.ev_drained, w.sx);
  return r;
}

static void worker_thread(drb_engine *e) {
  WorkerState &w = *e->worker;
  (void)hipSetDevice(e->cfg.device);  // (the current device is per thread)
  for (;;) {
    WorkerState::Job j;
    {
      std::unique_lock<std::mutex> g(w.mu);
      w.cv.wait(g, [&] { return w.stop || !w.jobs.empty(); });
      if (w.jobs.empty()) return;  // stop, nothing left
      j = w.jobs.front();
      w.jobs.pop_front();
    }
    const hipError_t r = worker_copy(e, w, j);
    {
      std::lock_guard<std::mutex> g(w.mu);
      if (r != hipSuccess) w.set[j.k].err = DRB_EDEVICE;
      w.set[j.k].issued = true;
    }
    w.cv.notify_all();
  }
}

// the 2-bit code words of cval reads (+ slack for the last shared word)
static uint64_t worker_meta_words(uint64_t cval) {
  return std::max<uint64_t>(cval, 1) / 16 + 2;
}

// staging set k (free: no export holds it, its copies done) of at least
// these capacities (grow-only)
static int worker_reserve(drb_engine *e, int k, uint64_t crd, uint64_t cval,
                          uint64_t cdf) {
  WorkerSet &s = e->worker->set[k];
  if (!s.ev_staged)
    HIPCHK(hipEventCreateWithFlags(&s.ev_staged, hipEventDisableTiming));
  if (!s.ev_drained)
    HIPCHK(hipEventCreateWithFlags(&s.ev_drained, hipEventDisableTiming));
  if (!s.lanes)
    HIPCHK(hipMalloc(&s.lanes, std::max<uint64_t>(e->v.G, 1) * 4 + 16));
  if (e->worker->hsa && !s.done.handle &&
      hsa_signal_create(0, 0, nullptr, &s.done) != HSA_STATUS_SUCCESS) {
    s.done.handle = 0;
    return DRB_EDEVICE;
  }
  if (s.rd && crd <= s.cap_rd && cval <= s.cap_val && cdf <= s.cap_df)
    return DRB_OK;
  // (the engine stream's earlier exports may still read the old staging)
  HIPCHK(hipStreamSynchronize(e->stream));
  crd = std::max(crd, s.cap_rd);
  cval = std::max(cval, s.cap_val);
  cdf = std::max(cdf, s.cap_df);
  if (s.rd) HIPCHK(hipFree(s.rd));
  if (s.val) HIPCHK(hipFree(s.val));
  if (s.meta) HIPCHK(hipFree(s.meta));
  if (s.dfr) HIPCHK(hipFree(s.dfr));
  s.rd = nullptr;
  s.val = nullptr;
  s.meta = nullptr;
  s.dfr = nullptr;
  HIPCHK(hipMalloc(&s.rd, std::max<uint64_t>(crd, 1) * 4 + 16));
  HIPCHK(hipMalloc(&s.val, std::max<uint64_t>(cval, 1) * 4 + 16));
  HIPCHK(hipMalloc(&s.meta, worker_meta_words(cval) * 4));
  HIPCHK(hipMalloc(&s.dfr, std::max<uint64_t>(cdf, 1) * 8 + 16));
  s.cap_rd = crd;
  s.cap_val = cval;
  s.cap_df = cdf;
  return DRB_OK;
}

static int worker_init(drb_engine *e) {
  if (e->worker) return DRB_OK;
  WorkerState *w = new WorkerState();
  e->worker = w;
  const uint64_t G = e->v.G;
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(hipStreamCreateWithFlags(&w->sx, hipStreamNonBlocking));
  HIPCHK(hipMalloc(&w->cnt, (G + 1) * sizeof(uint4)));
  HIPCHK(hipMalloc(&w->off, (G + 1) * sizeof(uint4)));
  HIPCHK(hipcub::DeviceScan::ExclusiveScan(nullptr, w->tmp_bytes, w->cnt,
                                           w->off, U4Sum(),
                                           make_uint4(0, 0, 0, 0),
                                           (int)(G + 1), e->stream));
  HIPCHK(hipMalloc(&w->tmp, std::max<size_t>(w->tmp_bytes, 16)));
  const size_t hb = 4 * kWorkerSets * sizeof(unsigned long long);
  HIPCHK(hipHostMalloc((void **)&w->hdr, hb, hipHostMallocMapped));
  memset(w->hdr, 0, hb);
  HIPCHK(hipHostGetDevicePointer((void **)&w->hdr_dev, w->hdr, 0));
  // the copies on the engine's download SDMA engine (drb_hsa.hpp)
  w->hsa = hsa_xfer_init(e->cfg.device, &e->xfer);
  w->th = std::thread(worker_thread, e);
  return DRB_OK;
}

extern "C" int drb_host_alloc(drb_engine *e, size_t bytes, void **p) {
  if (!e || !p || !bytes) return DRB_EINVAL;
  *p = nullptr;
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(hipHostMalloc(p, bytes, hipHostMallocMapped));
  return DRB_OK;
}

extern "C" int drb_host_free(drb_engine *e, void *p) {
  if (!e) return DRB_EINVAL;
  if (p) {
    if (WorkerState *w = e->worker) {
      // no copy of an export in flight may still write into it
      worker_quiesce(*w);
      if (w->sx) HIPCHK(hipStreamSynchronize(w->sx));
    }
    HIPCHK(hipHostFree(p));
  }
  return DRB_OK;
}

// the SDMA engine writes the caller's buffers directly: every byte of each
// must be pinned host memory (its first and its last byte checked, as
// drb_stage_proposals_packed checks its upload)
static bool worker_pinned(const void *p, uint64_t bytes) {
  if (!p || !bytes) return true;
  return hsa_host_pinned(p) &&
         hsa_host_pinned((const uint8_t *)p + (bytes - 1));
}

extern "C" int drb_worker_export_part(drb_engine *e, uint32_t slot,
                                      uint32_t n_parts, uint32_t part,
                                      const drb_worker_bufs *b) {
  if (!e || !b || slot >= e->v.R || !n_parts || part >= n_parts)
    return DRB_EINVAL;
  const View &v = e->v;
  // the partition's lanes: ShardID % n_parts == part (FixedPartitioner,
  // internal/server/partition.go:38), i.e. every n_parts-th lane from g0
  // (co-resident placement: lane g is ShardID first_shard_id + g)
  if (n_parts > 1 && v.place_world > 1) return DRB_EINVAL;
  const uint64_t g0 =
      (part + n_parts - (uint32_t)(e->cfg.first_shard_id % n_parts)) % n_parts;
  const uint64_t np = v.G > g0 ? (v.G - g0 + n_parts - 1) / n_parts : 0;
  if (!b->lanes || b->lanes_cap < np || (b->reads_cap && !b->reads) ||
      (b->values_cap && (!b->values || !b->value_meta)) ||
      (b->deferred_cap && !b->deferred))
    return DRB_EINVAL;
  if (!worker_pinned(b->lanes, np * 4) ||
      !worker_pinned(b->reads, b->reads_cap * 4) ||
      !worker_pinned(b->values, b->values_cap * 4) ||
      !worker_pinned(b->value_meta, (b->values_cap + 3) / 4) ||
      !worker_pinned(b->deferred, b->deferred_cap * 8))
    return DRB_EINVAL;
  if (int rc = worker_init(e)) return rc;
  WorkerState &w = *e->worker;
  int k = -1;
  {
    // one export in flight per buffer set, and a free staging set (its
    // last export waited for: its copies are done)
    std::lock_guard<std::mutex> g(w.mu);
    for (int q = 0; q < kWorkerSets; ++q) {
      if (w.set[q].owner == b) return DRB_EAGAIN;
      if (k < 0 && !w.set[q].owner) k = q;
    }
    if (k < 0) return DRB_EAGAIN;
    w.set[k].owner = b;  // (held from here; released on failure below)
    w.set[k].issued = false;
  }
  auto release = [&](int rc) {
    std::lock_guard<std::mutex> g(w.mu);
    w.set[k].owner = nullptr;
    return rc;
  };
  WorkerSet &s = w.set[k];
  if (int rc = worker_reserve(e, k, b->reads_cap, b->values_cap,
                              b->deferred_cap))
    return release(rc);
  // the reads of the last round, if it served them with results
  const uint32_t n_reads =
      v.read_res && e->reads_round == e->round ? e->reads_n : 0u;
  const unsigned blocks = (unsigned)((np + 1 + 255) / 256);
  k_worker_count<<<blocks, 256, 0, e->stream>>>(v, slot, n_reads, g0,
                                                n_parts, np, w.cnt);
  size_t tb = w.tmp_bytes;
  if (hipGetLastError() != hipSuccess ||
      hipcub::DeviceScan::ExclusiveScan(w.tmp, tb, w.cnt, w.off, U4Sum(),
                                        make_uint4(0, 0, 0, 0), (int)(np + 1),
                                        e->stream) != hipSuccess ||
      hipMemsetAsync(s.meta, 0, worker_meta_words(s.cap_val) * 4,
                     e->stream) != hipSuccess)
    return release(DRB_EDEVICE);
  k_worker_compact<<<blocks, 256, 0, e->stream>>>(
      v, slot, n_reads, g0, n_parts, np, e->sess_client, w.off, s.lanes, s.rd,
      b->reads_cap, s.val, s.meta, b->values_cap, s.dfr, b->deferred_cap,
      w.hdr_dev + 4 * k);
  if (hipGetLastError() != hipSuccess ||
      hipEventRecord(s.ev_staged, e->stream) != hipSuccess)
    return release(DRB_EDEVICE);
  {
    std::lock_guard<std::mutex> g(w.mu);
    w.jobs.push_back(WorkerState::Job{k, *b, np});
  }
  w.cv.notify_all();
  return DRB_OK;
}

extern "C" int drb_worker_export(drb_engine *e, uint32_t slot,
                                 const drb_worker_bufs *b) {
  return drb_worker_export_part(e, slot, 1, 0, b);
}

extern "C" int drb_worker_wait(drb_engine *e, drb_worker_bufs *b) {
  if (!e || !b || !e->worker) return DRB_EINVAL;
  WorkerState &w = *e->worker;
  int k = -1;
  {
    std::unique_lock<std::mutex> g(w.mu);
    for (int q = 0; q < kWorkerSets; ++q)
      if (w.set[q].owner == b) k = q;
    if (k < 0) return DRB_EINVAL;
    w.cv.wait(g, [&] { return w.set[k].issued; });
  }
  WorkerSet &s = w.set[k];
  // (the copies that were issued finish before the set is released)
  hipError_t r = hipSuccess;
  if (w.hsa)
    worker_wait_copies(w, k);
  else
    r = hipEventSynchronize(s.ev_drained);
  {
    std::lock_guard<std::mutex> g(w.mu);
    const int err = s.err ? s.err : r != hipSuccess ? DRB_EDEVICE : 0;
    if (err) {  // reported once; the buffer set and the staging are free
      s.err = 0;
      s.owner = nullptr;
      return err;
    }
  }
  b->n_reads = w.hdr[4 * k];
  b->n_values = w.hdr[4 * k + 1];
  b->n_deferred = w.hdr[4 * k + 2];
  {
    std::lock_guard<std::mutex> g(w.mu);
    s.owner = nullptr;
  }
  return b->n_reads > b->reads_cap || b->n_values > b->values_cap ||
                 b->n_deferred > b->deferred_cap
             ? DRB_ERANGE
             : DRB_OK;
}
