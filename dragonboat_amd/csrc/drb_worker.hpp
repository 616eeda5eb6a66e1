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
//      counts, one exclusive scan of {reads, values, applied} (hipCUB), and
//      a compaction of the lean records (include/drb_engine.h: a word per
//      lane, 16 B per ReadyToRead, 4 B + a nibble per served read, 4 B per
//      applied entry) into device staging[parity]; the totals go straight
//      to mapped host memory;
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

struct WorkerState {
  hipStream_t sx = nullptr;  // the drain thread's copies
  hipEvent_t ev_staged[2] = {nullptr, nullptr};
  hipEvent_t ev_drained[2] = {nullptr, nullptr};
  uint32_t *lanes[2] = {nullptr, nullptr};  // [G]
  drb_worker_read *rd[2] = {nullptr, nullptr};
  uint32_t *val[2] = {nullptr, nullptr};
  uint32_t *meta[2] = {nullptr, nullptr};  // nibbles, 8 per word
  uint32_t *ap[2] = {nullptr, nullptr};
  uint64_t cap_rd = 0, cap_val = 0, cap_ap = 0;  // staging capacity
  uint4 *cnt = nullptr, *off = nullptr;          // [G + 1]
  void *tmp = nullptr;
  size_t tmp_bytes = 0;
  unsigned long long *hdr = nullptr;      // pinned, mapped [2][4]: totals
  unsigned long long *hdr_dev = nullptr;  // ... its device address
  // the buffers of the exports in flight (waited for or not), by parity
  const drb_worker_bufs *owner[2] = {nullptr, nullptr};
  uint64_t seq = 0;
  // the drain thread: one job per export, in order
  struct Job {
    int k;
    drb_worker_bufs b;  // (the pointers and capacities at export time)
  };
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Job> jobs;
  bool issued[2] = {false, false};  // the copies of its job issued
  int err = 0;                      // a failed copy (reported by wait)
  bool stop = false;
  // the copies on the engine's download SDMA engine (drb_hsa.hpp;
  // hipMemcpyAsync on sx when HSA is unavailable)
  bool hsa = false;
  hsa_signal_t done[2] = {{0}, {0}};  // copies outstanding, by parity
};

// until the copies of buffer set k are done
static void worker_wait_copies(WorkerState &w, int k) {
  if (!w.hsa) return;
  while (hsa_signal_wait_scacquire(w.done[k], HSA_SIGNAL_CONDITION_LT, 1,
                                   UINT64_MAX, HSA_WAIT_STATE_BLOCKED) >= 1) {
  }
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

__global__ void k_worker_count(const View v, uint32_t slot, uint32_t n_reads,
                               uint4 *cnt) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g > v.G) return;
  uint4 c = make_uint4(0, 0, 0, 0);
  if (g < v.G) {
    const uint32_t nr = min(v.rtr_count[ix(v, slot, g)], (uint32_t)RTR_CAP);
    c.x = nr;
    if (nr && n_reads) {
      const uint32_t m = v.read_served[ix(v, slot, g)] & ((1u << nr) - 1u);
      c.y = (uint32_t)__popc(m) * n_reads;
    }
    uint64_t lo, hi;
    worker_apply_range(v, slot, g, &lo, &hi);
    c.z = hi > lo ? (uint32_t)min(hi - lo, (uint64_t)0xffffu) : 0u;
  }
  cnt[g] = c;  // cnt[G] = 0: the scan's last element is the total
}

// a served read's value-meta nibble (include/drb_engine.h): read_res.y is
// vlen | found << 31 (serve_reads_lane)
__device__ inline uint32_t worker_nibble(uint32_t y) {
  if (!(y >> 31)) return 0u;
  const uint32_t vlen = y & 0x7fffffffu;
  return DRB_WORKER_FOUND | (vlen > 4 ? (uint32_t)DRB_WORKER_LONG : vlen);
}

__global__ void k_worker_compact(const View v, uint32_t slot,
                                 uint32_t n_reads, const uint4 *off,
                                 uint32_t *lanes, drb_worker_read *rd,
                                 uint64_t cap_rd, uint32_t *val,
                                 uint32_t *meta, uint64_t cap_val,
                                 uint32_t *ap, uint64_t cap_ap,
                                 unsigned long long *tot) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g == v.G) {  // the totals, into mapped host memory
    tot[0] = off[g].x;
    tot[1] = off[g].y;
    tot[2] = off[g].z;
    __threadfence_system();
  }
  if (g >= v.G) return;
  const uint4 o = off[g];
  const uint32_t nr = min(v.rtr_count[ix(v, slot, g)], (uint32_t)RTR_CAP);
  const uint32_t m =
      nr && n_reads ? v.read_served[ix(v, slot, g)] & ((1u << nr) - 1u) : 0u;
  uint64_t lo, hi;
  worker_apply_range(v, slot, g, &lo, &hi);
  const uint32_t na = hi > lo ? (uint32_t)min(hi - lo, (uint64_t)0xffffu) : 0u;
  lanes[g] = nr | (m << 4) | (na << 12);
  uint64_t vo = o.y;
  // the nibbles of this lane's reads, one word (8 nibbles) at a time; the
  // first and last words may be shared with the neighbouring lanes (the
  // staging words start zeroed, shared ones take an atomicOr)
  uint32_t word = 0;
  uint64_t wi = vo / 8;
  auto flush = [&](bool last) {
    if (!word) return;
    const uint64_t first_w = o.y / 8;
    const bool shared = wi == first_w || last;
    if (wi * 8 < cap_val) {
      if (shared)
        atomicOr(&meta[wi], word);
      else
        meta[wi] = word;
    }
    word = 0;
  };
  for (uint32_t k = 0; k < nr; ++k) {
    if (o.x + k < cap_rd) {
      const uint4 c0 = v.rtr[rtr_ix(v, slot, k, 0, g)];
      drb_worker_read r;
      r.index = (uint64_t)c0.x | ((uint64_t)c0.y << 32);
      r.ctx_low = (uint64_t)c0.z | ((uint64_t)c0.w << 32);
      rd[o.x + k] = r;
    }
    if (!((m >> k) & 1u)) continue;
    for (uint32_t j = 0; j < n_reads; ++j, ++vo) {
      const uint2 w = v.read_res[rres_ix(v, slot, k, j, g)];
      if (vo < cap_val) val[vo] = w.x;
      if (vo / 8 != wi) {
        flush(false);
        wi = vo / 8;
      }
      word |= worker_nibble(w.y) << (4 * (vo & 7));
    }
  }
  flush(true);
  for (uint64_t idx = lo + 1, a = o.z; idx <= hi && a < cap_ap; ++idx, ++a) {
    const uint4 m1 = v.ring[ring_ix(v, slot, idx, 1, g)];
    const uint4 m2 = v.ring[ring_ix(v, slot, idx, 2, g)];
    const uint64_t client = lo64(m1);
    const uint32_t type = m2.z, clen = m2.w;
    // KVTest.Update's Result.Value: the payload length (kvtest.go:161); an
    // empty no-op entry is ignored by the rsm (statemachine.go:939)
    ap[a] = client == 0 ? DRB_WORKER_IGNORED
                        : (type == DRB_ENTRY_ENCODED && clen ? clen - 1 : clen);
  }
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
  if (w->hsa)
    for (int k = 0; k < 2; ++k) {
      worker_wait_copies(*w, k);
      (void)hsa_signal_destroy(w->done[k]);
    }
  for (int k = 0; k < 2; ++k) {
    if (w->ev_staged[k]) (void)hipEventDestroy(w->ev_staged[k]);
    if (w->ev_drained[k]) (void)hipEventDestroy(w->ev_drained[k]);
    if (w->lanes[k]) (void)hipFree(w->lanes[k]);
    if (w->rd[k]) (void)hipFree(w->rd[k]);
    if (w->val[k]) (void)hipFree(w->val[k]);
    if (w->meta[k]) (void)hipFree(w->meta[k]);
    if (w->ap[k]) (void)hipFree(w->ap[k]);
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
  hipError_t r = hipEventSynchronize(w.ev_staged[k]);
  if (r != hipSuccess) return r;
  const unsigned long long *t = w.hdr + 4 * k;
  const uint64_t nrd = std::min<uint64_t>(t[0], j.b.reads_cap);
  const uint64_t nval = std::min<uint64_t>(t[1], j.b.values_cap);
  const uint64_t nap = std::min<uint64_t>(t[2], j.b.applied_cap);
  struct {
    void *dst;
    const void *src;
    size_t n;
  } cp[5] = {{j.b.lanes, w.lanes[k], (size_t)e->v.G * 4},
             {j.b.reads, w.rd[k], nrd * sizeof(drb_worker_read)},
             {j.b.values, w.val[k], nval * 4},
             {j.b.value_meta, w.meta[k], (nval + 1) / 2},
             {j.b.applied, w.ap[k], nap * 4}};
  if (w.hsa) {
    const HsaXfer &x = e->xfer;
    int n = 0;
    for (auto &c : cp) n += c.n && c.dst;
    hsa_signal_store_screlease(w.done[k], n);
    for (auto &c : cp) {
      if (!(c.n && c.dst)) continue;
      if (hsa_amd_memory_async_copy_on_engine(
              c.dst, x.cpu, c.src, x.gpu, c.n, 0, nullptr, w.done[k],
              (hsa_amd_sdma_engine_id_t)x.down, true) != HSA_STATUS_SUCCESS) {
        hsa_signal_subtract_screlease(w.done[k], 1);
        r = hipErrorUnknown;
      }
    }
    return r;
  }
  for (auto &c : cp)
    if (c.n && c.dst && r == hipSuccess)
      r = hipMemcpyAsync(c.dst, c.src, c.n, hipMemcpyDeviceToHost, w.sx);
  if (r == hipSuccess) r = hipEventRecord(w.ev_drained[k], w.sx);
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
      if (r != hipSuccess) w.err = DRB_EDEVICE;
      w.issued[j.k] = true;
    }
    w.cv.notify_all();
  }
}

// device staging of at least these capacities (grow-only; growing waits
// for the exports in flight)
static int worker_reserve(drb_engine *e, uint64_t crd, uint64_t cval,
                          uint64_t cap) {
  WorkerState &w = *e->worker;
  if (crd <= w.cap_rd && cval <= w.cap_val && cap <= w.cap_ap) return DRB_OK;
  {
    // every export's copies issued (the drain thread done with its jobs)
    std::unique_lock<std::mutex> g(w.mu);
    w.cv.wait(g, [&] {
      return w.jobs.empty() && (!w.owner[0] || w.issued[0]) &&
             (!w.owner[1] || w.issued[1]);
    });
  }
  for (int k = 0; k < 2; ++k) worker_wait_copies(w, k);
  HIPCHK(hipStreamSynchronize(w.sx));
  HIPCHK(hipStreamSynchronize(e->stream));
  crd = std::max(crd, w.cap_rd);
  cval = std::max(cval, w.cap_val);
  cap = std::max(cap, w.cap_ap);
  for (int k = 0; k < 2; ++k) {
    if (w.rd[k]) HIPCHK(hipFree(w.rd[k]));
    if (w.val[k]) HIPCHK(hipFree(w.val[k]));
    if (w.meta[k]) HIPCHK(hipFree(w.meta[k]));
    if (w.ap[k]) HIPCHK(hipFree(w.ap[k]));
    w.rd[k] = nullptr;
    w.val[k] = nullptr;
    w.meta[k] = nullptr;
    w.ap[k] = nullptr;
    HIPCHK(hipMalloc(&w.rd[k], std::max<uint64_t>(crd, 1) *
                                   sizeof(drb_worker_read)));
    HIPCHK(hipMalloc(&w.val[k], std::max<uint64_t>(cval, 1) * 4 + 16));
    HIPCHK(hipMalloc(&w.meta[k], (std::max<uint64_t>(cval, 1) / 8 + 2) * 4));
    HIPCHK(hipMalloc(&w.ap[k], std::max<uint64_t>(cap, 1) * 4 + 16));
  }
  w.cap_rd = crd;
  w.cap_val = cval;
  w.cap_ap = cap;
  return DRB_OK;
}

static int worker_init(drb_engine *e) {
  if (e->worker) return DRB_OK;
  WorkerState *w = new WorkerState();
  e->worker = w;
  const uint64_t G = e->v.G;
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(hipStreamCreateWithFlags(&w->sx, hipStreamNonBlocking));
  for (int k = 0; k < 2; ++k) {
    HIPCHK(hipEventCreateWithFlags(&w->ev_staged[k], hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&w->ev_drained[k], hipEventDisableTiming));
  }
  for (int k = 0; k < 2; ++k)
    HIPCHK(hipMalloc(&w->lanes[k], std::max<uint64_t>(G, 1) * 4 + 16));
  HIPCHK(hipMalloc(&w->cnt, (G + 1) * sizeof(uint4)));
  HIPCHK(hipMalloc(&w->off, (G + 1) * sizeof(uint4)));
  HIPCHK(hipcub::DeviceScan::ExclusiveScan(nullptr, w->tmp_bytes, w->cnt,
                                           w->off, U4Sum(),
                                           make_uint4(0, 0, 0, 0),
                                           (int)(G + 1), e->stream));
  HIPCHK(hipMalloc(&w->tmp, std::max<size_t>(w->tmp_bytes, 16)));
  HIPCHK(hipHostMalloc((void **)&w->hdr, 8 * sizeof(unsigned long long),
                       hipHostMallocMapped));
  memset(w->hdr, 0, 8 * sizeof(unsigned long long));
  HIPCHK(hipHostGetDevicePointer((void **)&w->hdr_dev, w->hdr, 0));
  // the copies on the engine's download SDMA engine (drb_hsa.hpp)
  if (hsa_xfer_init(e->cfg.device, &e->xfer)) {
    w->hsa = hsa_signal_create(0, 0, nullptr, &w->done[0]) ==
             HSA_STATUS_SUCCESS;
    if (w->hsa && hsa_signal_create(0, 0, nullptr, &w->done[1]) !=
                      HSA_STATUS_SUCCESS) {
      (void)hsa_signal_destroy(w->done[0]);
      w->hsa = false;
    }
  }
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
      {
        std::unique_lock<std::mutex> g(w->mu);
        w->cv.wait(g, [&] {
          return w->jobs.empty() && (!w->owner[0] || w->issued[0]) &&
                 (!w->owner[1] || w->issued[1]);
        });
      }
      for (int k = 0; k < 2; ++k) worker_wait_copies(*w, k);
      if (w->sx) HIPCHK(hipStreamSynchronize(w->sx));
    }
    HIPCHK(hipHostFree(p));
  }
  return DRB_OK;
}

static int worker_dev_ptr(void *h, void **d) {
  *d = nullptr;
  if (!h) return DRB_OK;
  HIPCHK(hipHostGetDevicePointer(d, h, 0));
  return DRB_OK;
}

extern "C" int drb_worker_export(drb_engine *e, uint32_t slot,
                                 const drb_worker_bufs *b) {
  if (!e || !b || slot >= e->v.R) return DRB_EINVAL;
  if (!b->lanes || b->lanes_cap < e->v.G || (b->reads_cap && !b->reads) ||
      (b->values_cap && (!b->values || !b->value_meta)) ||
      (b->applied_cap && !b->applied))
    return DRB_EINVAL;
  if (int rc = worker_init(e)) return rc;
  WorkerState &w = *e->worker;
  const int k = (int)(w.seq & 1);
  {
    // one export in flight per buffer set, and staging[k] free (its
    // export, two back, waited for: its copies are done)
    std::lock_guard<std::mutex> g(w.mu);
    if (w.owner[0] == b || w.owner[1] == b || w.owner[k]) return DRB_EAGAIN;
  }
  if (int rc = worker_reserve(e, b->reads_cap, b->values_cap, b->applied_cap))
    return rc;
  const View &v = e->v;
  // the reads of the last round, if it served them with results
  const uint32_t n_reads =
      v.read_res && e->reads_round == e->round ? e->reads_n : 0u;
  const unsigned blocks = (unsigned)((v.G + 1 + 255) / 256);
  k_worker_count<<<blocks, 256, 0, e->stream>>>(v, slot, n_reads, w.cnt);
  HIPCHK(hipGetLastError());
  size_t tb = w.tmp_bytes;
  HIPCHK(hipcub::DeviceScan::ExclusiveScan(w.tmp, tb, w.cnt, w.off, U4Sum(),
                                           make_uint4(0, 0, 0, 0),
                                           (int)(v.G + 1), e->stream));
  HIPCHK(hipMemsetAsync(w.meta[k], 0,
                        (std::max<uint64_t>(w.cap_val, 1) / 8 + 2) * 4,
                        e->stream));
  k_worker_compact<<<blocks, 256, 0, e->stream>>>(
      v, slot, n_reads, w.off, w.lanes[k], w.rd[k], b->reads_cap, w.val[k],
      w.meta[k], b->values_cap, w.ap[k], b->applied_cap, w.hdr_dev + 4 * k);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(w.ev_staged[k], e->stream));
  {
    std::lock_guard<std::mutex> g(w.mu);
    w.owner[k] = b;
    w.issued[k] = false;
    w.jobs.push_back(WorkerState::Job{k, *b});
  }
  w.cv.notify_all();
  w.seq++;
  return DRB_OK;
}

extern "C" int drb_worker_wait(drb_engine *e, drb_worker_bufs *b) {
  if (!e || !b || !e->worker) return DRB_EINVAL;
  WorkerState &w = *e->worker;
  int k = -1;
  {
    std::unique_lock<std::mutex> g(w.mu);
    for (int q = 0; q < 2; ++q)
      if (w.owner[q] == b) k = q;
    if (k < 0) return DRB_EINVAL;
    w.cv.wait(g, [&] { return w.issued[k]; });
    if (w.err) return w.err;
  }
  if (w.hsa)
    worker_wait_copies(w, k);
  else
    HIPCHK(hipEventSynchronize(w.ev_drained[k]));
  b->n_reads = w.hdr[4 * k];
  b->n_values = w.hdr[4 * k + 1];
  b->n_applied = w.hdr[4 * k + 2];
  {
    std::lock_guard<std::mutex> g(w.mu);
    w.owner[k] = nullptr;
  }
  return b->n_reads > b->reads_cap || b->n_values > b->values_cap ||
                 b->n_applied > b->applied_cap
             ? DRB_ERANGE
             : DRB_OK;
}
