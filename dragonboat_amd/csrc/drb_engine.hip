// drb_engine.hip -- host side of the C ABI (include/drb_engine.h) and the
// auxiliary device kernels (initialisation, input generation, state
// movement, CRC32).  The step round itself is drb_step.hpp.
//
// Written for gfx950 (MI355X) only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <unordered_map>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "../../include/drb_engine.h"
#include "drb_layout.hpp"
#include "drb_msg.hpp"
#include "drb_step.hpp"
#include "drb_launch.hpp"
#include "drb_hsa.hpp"

using namespace drb;

#define HIPCHK(x)                                                        \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      fprintf(stderr, "drb_engine: %s failed: %s (%s:%d)\n", #x,          \
              hipGetErrorString(e_), __FILE__, __LINE__);                \
      return DRB_EDEVICE;                                                \
    }                                                                    \
  } while (0)

struct drb_engine {
  drb_config cfg;
  View v;
  View *dview;  // device copy of v (kernels read it with scalar loads)
  hipStream_t stream;
  hipStream_t stream2;            // the follower kernel of a round
  hipEvent_t ev_fork, ev_join;    // stream -> stream2 -> stream
  hipStream_t stream_h2d;         // drb_stage_proposals uploads
  HsaXfer xfer;  // the engine's own SDMA transfers (drb_hsa.hpp)
  // sticky: a multi-round call failed after some of its rounds were
  // enqueued, so the device ran rounds the host did not account for (round
  // tags, mailbox parity); every later step call returns it
  int failed = 0;
  // drb_set_session_clients: per lane the ClientID of the host's NoOP
  // session of its group ([G], null until set)
  uint64_t *sess_client = nullptr;
  // the lean kernel of listed rounds off (drb_config.no_lean: A/B only)
  bool no_lean = false;
  // drb_exchange_local_bind: the engines of the group, this one included,
  // and per rank their outbox planes (host copy; v.peers the device one)
  std::vector<drb_engine *> bound;
  std::vector<PeerPlanes> peers_host;
  hipEvent_t ev_staged;           // upload done -> layout kernel
  hipEvent_t ev_stage_free;       // layout kernel done -> next upload
  hipEvent_t ev_uploaded;         // packed upload done -> host arrays free
  // drb_exchange_local: this engine's round done (its outbox planes may be
  // copied), and the copies into its inbound planes done (its senders'
  // next rounds may overwrite their outbox planes)
  hipEvent_t ev_xsend = nullptr, ev_xrecv = nullptr;
  // the last round whose remote planes were exchanged (or enqueued, drb_
  // exchange_mark): ingest into remote planes waits for it (DRB_EAGAIN)
  uint64_t exchanged_round = 0;
  // per proposal slot: the engine-stream work that last read or wrote it
  // (drb_step_round_async, the generators, drb_stage_proposals), so that
  // drb_stage_proposals_packed lays a slot out on the copy stream while
  // rounds on other slots run
  std::vector<hipEvent_t> ev_prop;
  uint64_t round;
  uint64_t ticks;  // LocalTicks delivered so far (RoundParams.tick_no)
  uint64_t committed_round = 0;  // drb_commit_round (durable_log)
  uint64_t bytes;
  std::vector<void *> allocs;
  uint64_t ctr_rows = 0;                     // workgroup counter rows
  uint32_t *xcount = nullptr;                // [R][R] plane summaries
  uint32_t role_slots[2] = {0, 0};           // role map (launch_step)
  uint32_t *role_dev = nullptr;
  unsigned long long *ctr_total = nullptr;   // their sum (read_counters)
  void *scratch;
  size_t scratch_bytes;
  void *stage_buf = nullptr;  // drb_stage_proposals upload (grow-only)
  size_t stage_bytes = 0;
  struct WireState *wire = nullptr;          // drb_encode_wire (drb_wire.hpp)
  struct IngestState *ingest = nullptr;      // drb_ingest_wire (drb_ingest.hpp)
  struct WorkerState *worker = nullptr;      // drb_worker_export (drb_worker.hpp)
  std::mutex ingest_mu;  // drb_ingest: concurrent transport threads
  bool crc_tab_ready = false;  // c_crc_tab uploaded on this engine's device
  uint64_t tan_blocks = 0;                   // k_tan_select grid (save_tan)
  uint64_t tan_wblocks = 0;                  // k_tan_write grid
  uint32_t *tan_list = nullptr;              // replicas with a record
  uint32_t *tan_n = nullptr;                 // their counts, 256 B apart
  uint32_t tan_per_list = 0;
  unsigned long long *tan_total = nullptr;   // its counter rows summed
  // the last round whose reads were served (in-round or drb_serve_reads),
  // their count per ctx and key space (drb_export_read_results)
  uint64_t reads_round = ~0ull;
  uint32_t reads_n = 0, reads_ks = 0;
  void *xout = nullptr;  // batch exports' device output (grow-only)
  size_t xout_bytes = 0;
  // drb_exchange_bytes: inbound plane bytes of the device pull (a device
  // counter) and of region copies (host-side sum)
  unsigned long long *xpull_bytes = nullptr;
  uint64_t xcopy_bytes = 0;
  // drb_plane_counts has read the plane summaries (xrows): the rounds clear
  // them from then on
  bool xrows_used = false;
};

static void wire_free(drb_engine *e);
static void ingest_free(struct IngestState *st);
static void worker_free(drb_engine *e);
static bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }
static int refresh_roles(drb_engine *e);
static int launch_tan(drb_engine *e, uint32_t round);  // drb_tan.hpp
static int read_tan_counters(drb_engine *e, unsigned long long *t4,
                             int reset);

template <typename T>
static int dalloc(drb_engine *e, T **p, uint64_t count) {
  uint64_t b = count * sizeof(T);
  if (b == 0) b = 16;
  void *q = nullptr;
  HIPCHK(hipMalloc(&q, b));
  HIPCHK(hipMemsetAsync(q, 0, b, e->stream));
  e->allocs.push_back(q);
  e->bytes += b;
  *p = (T *)q;
  return DRB_OK;
}

static int scratch(drb_engine *e, size_t bytes, void **out) {
  if (bytes > e->scratch_bytes) {
    if (e->scratch) HIPCHK(hipFree(e->scratch));
    e->scratch = nullptr;
    size_t b = std::max(bytes, (size_t)1 << 20);
    HIPCHK(hipMalloc(&e->scratch, b));
    e->scratch_bytes = b;
  }
  *out = e->scratch;
  return DRB_OK;
}

// ---------------------------------------------------------------- gather
template <typename T>
__global__ void k_gather(const T *base, const uint64_t *idx, T *out,
                         uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = base[idx[i]];
}

template <typename T>
__global__ void k_scatter(T *base, const uint64_t *idx, const T *in,
                          uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) base[idx[i]] = in[i];
}

template <typename T>
static int gather(drb_engine *e, const T *base,
                  const std::vector<uint64_t> &idx, std::vector<T> &out) {
  uint64_t n = idx.size();
  out.resize(n);
  if (!n) return DRB_OK;
  void *s;
  if (scratch(e, n * (8 + sizeof(T)) + 64, &s)) return DRB_EDEVICE;
  uint64_t *didx = (uint64_t *)s;
  T *dout = (T *)((char *)s + ((n * 8 + 15) & ~15ull));
  HIPCHK(hipMemcpyAsync(didx, idx.data(), n * 8, hipMemcpyHostToDevice,
                        e->stream));
  k_gather<T><<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(base, didx,
                                                                   dout, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out.data(), dout, n * sizeof(T), hipMemcpyDeviceToHost,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

template <typename T>
static int scatter(drb_engine *e, T *base, const std::vector<uint64_t> &idx,
                   const std::vector<T> &in) {
  uint64_t n = idx.size();
  if (!n) return DRB_OK;
  void *s;
  if (scratch(e, n * (8 + sizeof(T)) + 64, &s)) return DRB_EDEVICE;
  uint64_t *didx = (uint64_t *)s;
  T *din = (T *)((char *)s + ((n * 8 + 15) & ~15ull));
  HIPCHK(hipMemcpyAsync(didx, idx.data(), n * 8, hipMemcpyHostToDevice,
                        e->stream));
  HIPCHK(hipMemcpyAsync(din, in.data(), n * sizeof(T), hipMemcpyHostToDevice,
                        e->stream));
  k_scatter<T><<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(base, didx,
                                                                    din, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

__host__ __device__ static inline uint4 mk4h(uint64_t a, uint64_t b) {
  uint4 q;
  q.x = (uint32_t)a;
  q.y = (uint32_t)(a >> 32);
  q.z = (uint32_t)b;
  q.w = (uint32_t)(b >> 32);
  return q;
}
static uint64_t lo64h(uint4 q) { return (uint64_t)q.x | ((uint64_t)q.y << 32); }
static uint64_t hi64h(uint4 q) { return (uint64_t)q.z | ((uint64_t)q.w << 32); }

__global__ void k_fill_u4(uint4 *p, uint64_t n, uint4 val) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = val;
}

__global__ void k_fill_u64(uint64_t *p, uint64_t n, uint64_t val) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = val;
}

// ---------------------------------------------------------------- create
extern "C" int drb_engine_create(const drb_config *cfg, drb_engine **out) {
  if (!cfg || !out) return DRB_EINVAL;
  *out = nullptr;
  if (cfg->num_groups == 0 || cfg->num_replicas < 1 ||
      cfg->num_replicas > DRB_MAX_REPLICAS)
    return DRB_EINVAL;
  if (!is_pow2(cfg->window) || cfg->window < 4 || cfg->window > 65535)
    return DRB_EINVAL;
  if (cfg->cmd_cap == 0 || cfg->cmd_cap % 16 || cfg->cmd_cap > 1040)
    return DRB_ENOSYS;
  if (cfg->mailbox < 4 || cfg->mailbox > MB_MAX) return DRB_EINVAL;
  if (!is_pow2(cfg->kv_slots) || cfg->kv_val_cap == 0 ||
      cfg->kv_val_cap > 1024)
    return DRB_EINVAL;
  if (cfg->max_props == 0 || cfg->prop_slots == 0 || cfg->ri_slots == 0)
    return DRB_EINVAL;
  if (cfg->save_cap % 16) return DRB_EINVAL;
  // batched records merge from the window: a batch's 47 earlier entries
  // plus the round's must be resident
  if (cfg->save_batched && (cfg->save_cap == 0 || cfg->window < 64))
    return DRB_EINVAL;
  if (cfg->save_tan && (cfg->save_cap == 0 || cfg->save_batched))
    return DRB_EINVAL;
  // PreVote runs in the raft launch
  if (cfg->pre_vote && !cfg->elections) return DRB_EINVAL;
  // the multiplexed tan: a tan option, ShardIDs of this rank's groups
  if (cfg->tan_multiplexed && (!cfg->save_tan || cfg->place_world > 1))
    return DRB_EINVAL;
  // (the tan write pass lists replicas by 32-bit lane number)
  if (cfg->save_tan && (uint64_t)cfg->num_replicas * cfg->num_groups > 0xffffffffull)
    return DRB_ERANGE;
  // entry_mbox travels as the 8-bit E of the plane summary word
  // (block_plane_summary, DRB_PLANE_E)
  if (cfg->place_world > 1 &&
      (cfg->place_rank >= cfg->place_world || cfg->entry_mbox == 0 ||
       cfg->entry_mbox > cfg->window || cfg->entry_mbox > 255))
    return DRB_EINVAL;
  if (cfg->election_rtt == 0 || cfg->heartbeat_rtt == 0) return DRB_EINVAL;
  // member kinds: a slot is one kind; some voting member remains
  if ((cfg->nonvoting_slots & cfg->witness_slots) ||
      ((cfg->nonvoting_slots | cfg->witness_slots) >> cfg->num_replicas) ||
      __builtin_popcount(cfg->nonvoting_slots | cfg->witness_slots) >=
          (int)cfg->num_replicas)
    return DRB_EINVAL;
  // forwarded proposals: a Propose's entry count travels in 4 header bits
  // (MI_NPROP); co-resident planes only
  if (cfg->forward_proposals &&
      (cfg->max_props > MAX_FWD_PROPS || cfg->place_world > 1))
    return DRB_EINVAL;
  // limitSize never binds inside the window (entryutils.go:50-63)
  if ((uint64_t)cfg->window * (128 + cfg->cmd_cap) > MAX_ENTRY_SIZE)
    return DRB_EINVAL;
  drb_engine *e = new drb_engine();
  e->cfg = *cfg;
  e->round = 0;
  e->ticks = 0;
  e->bytes = 0;
  e->scratch = nullptr;
  e->scratch_bytes = 0;
  if (cfg->host_copies > 1) {
    delete e;
    return DRB_EINVAL;
  }
  // (host_copies: HIP copies, as when the SDMA engines are unavailable)
  if (cfg->host_copies) e->xfer.state = -1;
  e->no_lean = cfg->no_lean != 0;
  if (hipSetDevice(cfg->device) != hipSuccess ||
      hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) !=
          hipSuccess ||
      hipStreamCreateWithFlags(&e->stream2, hipStreamNonBlocking) !=
          hipSuccess ||
      hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming) !=
          hipSuccess ||
      hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming) !=
          hipSuccess ||
      hipStreamCreateWithFlags(&e->stream_h2d, hipStreamNonBlocking) !=
          hipSuccess ||
      hipEventCreateWithFlags(&e->ev_staged, hipEventDisableTiming) !=
          hipSuccess ||
      hipEventCreateWithFlags(&e->ev_stage_free, hipEventDisableTiming) !=
          hipSuccess ||
      hipEventCreateWithFlags(&e->ev_uploaded, hipEventDisableTiming) !=
          hipSuccess ||
      hipEventCreateWithFlags(&e->ev_xsend, hipEventDisableTiming) !=
          hipSuccess ||
      hipEventCreateWithFlags(&e->ev_xrecv, hipEventDisableTiming) !=
          hipSuccess) {
    delete e;
    return DRB_EDEVICE;
  }
  e->ev_prop.resize(cfg->prop_slots);
  for (auto &ev : e->ev_prop)
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      delete e;
      return DRB_EDEVICE;
    }
  View &v = e->v;
  memset(&v, 0, sizeof(v));
  const uint64_t G = cfg->num_groups, R = cfg->num_replicas;
  v.G = G;
  v.R = (uint32_t)R;
  v.W = cfg->window;
  v.C16 = cfg->cmd_cap / 16;
  v.MB = cfg->mailbox;
  v.KS = cfg->kv_slots;
  v.kv_val_cap = cfg->kv_val_cap;
  v.kv_ool = cfg->kv_val_cap > 124;
  v.KVW = v.kv_ool ? 2
                   : 1 + (cfg->kv_val_cap > 4 ? (cfg->kv_val_cap - 4 + 15) / 16
                                              : 0);
  v.VB = v.kv_ool ? (cfg->kv_val_cap + 15) / 16 : 0;
  // default: a block for every slot, overflow slots included (the pool
  // never runs out before the table does); large configurations size it
  // to their key count
  v.kv_pool_blocks =
      v.kv_ool ? (cfg->kv_pool_blocks
                      ? cfg->kv_pool_blocks
                      : std::min<uint64_t>(G * R * v.KS +
                                               4 * cfg->kv_overflow_buckets,
                                           0xffffffffull))
               : 0;
  v.max_props = cfg->max_props;
  v.election_rtt = cfg->election_rtt;
  v.heartbeat_rtt = cfg->heartbeat_rtt;
  v.check_quorum = cfg->check_quorum;
  v.quiesce = cfg->quiesce ? 1u : 0u;
  v.nv_mask = cfg->nonvoting_slots;
  v.wt_mask = cfg->witness_slots;
  v.quorum = (uint32_t)(R - __builtin_popcount(v.nv_mask)) / 2 + 1;
  v.first_shard_id = cfg->first_shard_id;
  v.place_world = cfg->place_world > 1 ? cfg->place_world : 1;
  v.place_rank = v.place_world > 1 ? cfg->place_rank : 0;
  v.total_groups = cfg->total_groups ? cfg->total_groups : G * v.place_world;
  if (v.total_groups > G * v.place_world) {
    delete e;
    return DRB_EINVAL;
  }
  v.remote_mask = 0;
  if (v.place_world > 1)
    for (uint32_t a = 0; a < R; ++a)
      for (uint32_t b = 0; b < R; ++b)
        if (a != b && b % v.place_world != a % v.place_world)
          v.remote_mask |= 1ull << (a * R + b);
  v.E = v.remote_mask ? cfg->entry_mbox : 0;
  v.stage_slot = 0;
  int rc = 0;
  rc |= dalloc(e, &v.u64, (uint64_t)NUM_U64 * R * G);
  rc |= dalloc(e, &v.pk, 4ull * R * G);
  rc |= dalloc(e, &v.u32, (uint64_t)NUM_U32 * R * G);
  rc |= dalloc(e, &v.rem_match, R * R * G);
  rc |= dalloc(e, &v.rem_next, R * R * G);
  rc |= dalloc(e, &v.rem_state, R * R * G);
  rc |= dalloc(e, &v.rem_active, R * R * G);
  rc |= dalloc(e, &v.ri_ctx, R * DRB_RI_DEPTH * G);
  rc |= dalloc(e, &v.ri_idx, R * DRB_RI_DEPTH * G);
  rc |= dalloc(e, &v.ri_conf, R * DRB_RI_DEPTH * G);
  rc |= dalloc(e, &v.ring, R * v.W * (ENT_META + v.C16) * G);
  rc |= dalloc(e, &v.mbox, 2 * R * R * v.MB * MSG_CHUNKS * G);
  rc |= dalloc(e, &v.mbox_meta, 2 * R * R * G);  // uint4
  rc |= dalloc(e, &v.mbox_maxapp, 2 * R * R * G);
  rc |= dalloc(e, &v.inbox_tag, 2 * R * G);
  rc |= dalloc(e, &v.kv, R * G * v.KS * v.KVW);
  if (v.kv_ool) {
    rc |= dalloc(e, &v.kv_pool, v.kv_pool_blocks * v.VB);
    rc |= dalloc(e, &v.kv_pool_next, 1);
  }
  if (const char *ph = getenv("DRB_PHASE"))  // timing builds only
    if (ph[0] == '1') rc |= dalloc(e, &v.phase, 16);
  v.kv_ovf_cap = cfg->kv_overflow_buckets;
  if (v.kv_ovf_cap) {
    if (v.kv_ovf_cap >= 0xffffffffull) {
      delete e;
      return DRB_ERANGE;
    }
    rc |= dalloc(e, &v.kv_ovf, v.kv_ovf_cap * 4 * v.KVW);
    rc |= dalloc(e, &v.kv_ovf_next, v.kv_ovf_cap);
    rc |= dalloc(e, &v.kv_ovf_head, R * G);
    rc |= dalloc(e, &v.kv_ovf_used, 1);
  }
  v.P = cfg->prop_slots;
  v.fwd_props = cfg->forward_proposals ? 1u : 0u;
  rc |= dalloc(e, &v.props,
               ((uint64_t)cfg->prop_slots + (v.fwd_props ? 2 * R : 0)) *
                   v.max_props * (PROP_META + v.C16) * G);
  rc |= dalloc(e, &v.prop_count, (uint64_t)cfg->prop_slots * G);
  rc |= dalloc(e, &v.ri_in, (uint64_t)cfg->ri_slots * G);
  rc |= dalloc(e, &v.rtr, R * RTR_CAP * 2 * G);
  rc |= dalloc(e, &v.rtr_count, R * G);
  rc |= dalloc(e, &v.read_sum, R * G);
  v.max_reads = cfg->max_reads_per_ctx;
  if (v.max_reads) {
    rc |= dalloc(e, &v.read_res, R * RTR_CAP * (uint64_t)v.max_reads * G);
    rc |= dalloc(e, &v.read_served, R * G);
  }
  if (v.remote_mask) {  // inbound copies of the remote planes
    rc |= dalloc(e, &v.mbox_in, 2 * R * R * v.MB * MSG_CHUNKS * G);
    rc |= dalloc(e, &v.meta_in, 2 * R * R * G);
    rc |= dalloc(e, &v.maxapp_in, 2 * R * R * G);
    rc |= dalloc(e, &v.elo, 2 * R * R * G);
    rc |= dalloc(e, &v.elo_in, 2 * R * R * G);
    rc |= dalloc(e, &v.embox,
                 2 * R * R * (uint64_t)v.E * (ENT_META + v.C16) * G);
    rc |= dalloc(e, &v.embox_in,
                 2 * R * R * (uint64_t)v.E * (ENT_META + v.C16) * G);
    rc |= dalloc(e, &v.xrows, 2 * R * R * ((G + 255) / 256));
    rc |= dalloc(e, &e->xcount, R * R);
  }
  v.save_cap16 = cfg->save_cap / 16;
  if (v.save_cap16) {
    // the multiplexed tan stages each log's round in save_buf: 16 logs per
    // slot of at most tanm_J records each
    v.tan_mux = cfg->save_tan && cfg->tan_multiplexed ? 1u : 0u;
    v.tanm_J = (uint32_t)((((G + 15) / 16) + 255) & ~255ull);
    v.tanm_cap16 = (uint64_t)v.tanm_J * v.save_cap16;
    if (v.tan_mux && v.tanm_cap16 * 16 > 0xffffffffull) return DRB_ERANGE;
    rc |= dalloc(e, &v.save_buf,
                 std::max<uint64_t>(R * G, v.tan_mux ? R * 16 * v.tanm_J : 0) *
                     v.save_cap16);
    rc |= dalloc(e, &v.save_len, R * G);
    rc |= dalloc(e, &v.save_crc, R * G);
  }
  v.save_batched = cfg->save_batched ? 1u : 0u;
  if (v.save_batched) {
    rc |= dalloc(e, &v.save_rec, R * G * DRB_SAVE_RECS);
    rc |= dalloc(e, &v.save_nrec, R * G);
  }
  v.save_tan = cfg->save_tan ? 1u : 0u;
  if (v.save_tan) {
    // beyond the entries' EntryBatch bound: the Update's shard, replica,
    // State and counts (<= 63 B), zero padding (<= 6 B) and a 7-byte chunk
    // header per block the record touches
    v.save_slack = 63 + 6 + 7 * (cfg->save_cap / (32768 - 7) + 2);
    e->tan_blocks = (R * G + 255) / 256;
    rc |= dalloc(e, &v.tan_sum, 3 * R * G);
    rc |= dalloc(e, &v.tan_st, R * G);
    rc |= dalloc(e, &v.tan_rec, R * G);
    e->tan_wblocks = std::min<uint64_t>(e->tan_blocks, 4096);
    e->tan_per_list =
        (uint32_t)(((e->tan_blocks + drb::TAN_LISTS - 1) / drb::TAN_LISTS) * 256);
    rc |= dalloc(e, &v.tan_ctr, e->tan_blocks * 4);
    rc |= dalloc(e, &e->tan_list, (uint64_t)e->tan_per_list * drb::TAN_LISTS);
    rc |= dalloc(e, &e->tan_n, 64 * drb::TAN_LISTS);
    if (v.tan_mux) {
      rc |= dalloc(e, &v.tanm_len, R * 16 * v.tanm_J);
      rc |= dalloc(e, &v.tanm_pos, R * 16 * v.tanm_J);
      rc |= dalloc(e, &v.tanm_cur, R * 16);
      rc |= dalloc(e, &v.tanm_log, R * 16 * 2);
    }
    rc |= dalloc(e, &e->tan_total, 4);
  }
  v.elections = cfg->elections ? 1u : 0u;
  v.pre_vote = cfg->pre_vote ? 1u : 0u;
  if (v.elections) {
    // the raft launch's workgroups own counter rows 0.. (block_counters):
    // at most 2 per group block
    v.slow_cap = (uint32_t)std::min<uint64_t>(
        R * G, 2ull * ((G + 255) / 256) * 256);
    rc |= dalloc(e, &v.slow_list, v.slow_cap);
    rc |= dalloc(e, &v.slow_n, 1);
    rc |= dalloc(e, &v.rterm, 2ull * R * R * v.MB * G);
    rc |= dalloc(e, &v.xfer_in, (uint64_t)R * G);
    if (v.remote_mask) {
      rc |= dalloc(e, &v.rterm_in, 2ull * R * R * v.MB * G);
      rc |= dalloc(e, &v.xslow, 4ull * R * R * ((G + 255) / 256));
    }
  }
  e->ctr_rows = 2ull * R * ((G + 255) / 256);  // see block_counters
  rc |= dalloc(e, &v.counters, e->ctr_rows * NUM_COUNTERS);
  rc |= dalloc(e, &e->ctr_total, NUM_COUNTERS);
  v.flog_cap = cfg->flagged_cap ? cfg->flagged_cap : 65536;
  rc |= dalloc(e, &v.flog, v.flog_cap);
  rc |= dalloc(e, &v.flog_n, 1);
  {
    const uint64_t nb = (G + 255) / 256;
    rc |= dalloc(e, &v.act_list, 2 * R * G);
    rc |= dalloc(e, &v.act_total, 4 * R);
    rc |= dalloc(e, &v.act_cnt, 4 * R * nb);
    rc |= dalloc(e, &v.act_off, 4 * R * nb);
    rc |= dalloc(e, &v.act_mask, 4 * R * nb * 4);
    rc |= dalloc(e, &v.esc_list, 2ull * R * ESC_SPLIT * esc_seg(G));
    rc |= dalloc(e, &v.esc_n, 2ull * R * ESC_SPLIT);
  }
  rc |= dalloc(e, &e->role_dev, 2);
  rc |= dalloc(e, &e->dview, 1);
  if (!rc) {  // no Replicate in flight: ring_guard = +inf
    k_fill_u4<<<(unsigned)((R * G + 255) / 256), 256, 0, e->stream>>>(
        v.pk + pk_ix(v, 1, 0, 0), R * G, make_uint4(0, 0, 0, PK_INF16 << 16));
    if (hipGetLastError() != hipSuccess) rc = 1;
  }
  if (!rc && hipMemcpyAsync(e->dview, &e->v, sizeof(View),
                            hipMemcpyHostToDevice, e->stream) != hipSuccess)
    rc = 1;
  if (rc || hipStreamSynchronize(e->stream) != hipSuccess) {
    drb_engine_destroy(e);
    return DRB_ENOMEM;
  }
  *out = e;
  return DRB_OK;
}

extern "C" int drb_engine_destroy(drb_engine *e) {
  if (!e) return DRB_EINVAL;
  (void)hipStreamSynchronize(e->stream);
  (void)hipStreamSynchronize(e->stream2);
  // bound peers read this engine's outbox planes: their work drains first,
  // and their later rounds fail (their remote planes are gone)
  for (drb_engine *o : e->bound) {
    if (o == e) continue;
    (void)hipStreamSynchronize(o->stream);
    o->failed = DRB_EINVAL;
    o->bound.erase(std::remove(o->bound.begin(), o->bound.end(), e),
                   o->bound.end());
  }
  for (void *p : e->allocs) (void)hipFree(p);
  if (e->scratch) (void)hipFree(e->scratch);
  if (e->stage_buf) (void)hipFree(e->stage_buf);
  if (e->xout) (void)hipFree(e->xout);
  wire_free(e);
  ingest_free(e->ingest);
  worker_free(e);
  if (e->sess_client) (void)hipFree(e->sess_client);
  hsa_xfer_fini(&e->xfer);
  (void)hipEventDestroy(e->ev_fork);
  (void)hipEventDestroy(e->ev_join);
  (void)hipEventDestroy(e->ev_staged);
  (void)hipEventDestroy(e->ev_stage_free);
  (void)hipEventDestroy(e->ev_uploaded);
  if (e->ev_xsend) (void)hipEventDestroy(e->ev_xsend);
  if (e->ev_xrecv) (void)hipEventDestroy(e->ev_xrecv);
  for (auto &ev : e->ev_prop) (void)hipEventDestroy(ev);
  (void)hipStreamDestroy(e->stream_h2d);
  (void)hipStreamDestroy(e->stream2);
  (void)hipStreamDestroy(e->stream);
  delete e;
  return DRB_OK;
}

extern "C" uint64_t drb_engine_device_bytes(const drb_engine *e) {
  return e ? e->bytes : 0;
}

extern "C" void *drb_engine_stream(drb_engine *e) {
  return e ? (void *)e->stream : nullptr;
}

extern "C" int drb_engine_sync(drb_engine *e) {
  if (!e) return DRB_EINVAL;
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

extern "C" uint64_t drb_engine_round(const drb_engine *e) {
  return e ? e->round : 0;
}

// ---------------------------------------------------------------- state
static const int kU64Order[NUM_U64_EXPORTED] = {
    F_TERM,           F_VOTE,          F_LEADER_ID,       F_APPLIED,
    F_ELECTION_TICK,  F_HEARTBEAT_TICK, F_RAND_TIMEOUT,   F_TICK_COUNT,
    F_COMMITTED,      F_PROCESSED,     F_LAST_INDEX,      F_MARKER_INDEX,
    F_SAVED_TO,       F_APPLIED_TO_INDEX, F_APPLIED_TO_TERM, F_APPLIED_INDEX,
    F_CONFIRMED_INDEX, F_PUSHED_INDEX, F_PREV_TERM,       F_PREV_VOTE,
    F_PREV_COMMIT,    F_SM_INDEX,      F_SM_TERM,         F_KV_COUNT,
    F_QS_TICK,        F_QS_IDLE,       F_QS_SINCE,        F_QS_EXIT,
    F_RNG};

// drb_replica_state fields 2.. in kU64Order order (after shard/replica id)
static uint64_t *st_u64(drb_replica_state *s, int k) {
  uint64_t *base = &s->term;
  return base + k;
}

static int check_range(drb_engine *e, uint64_t first, uint64_t n) {
  if (!e || first >= e->cfg.num_groups || n > e->cfg.num_groups - first)
    return DRB_ERANGE;
  return DRB_OK;
}

// decoded field values [replica][NUM_U64] of groups [first, first + n)
// from the packed records and the u64 array (overflow, counters)
static int read_records(drb_engine *e, uint64_t first, uint64_t n,
                        std::vector<uint64_t> &vals) {
  const View &v = e->v;
  const uint32_t R = v.R;
  std::vector<uint64_t> ipk, i64;
  for (uint64_t gi = 0; gi < n; ++gi)
    for (uint32_t s = 0; s < R; ++s) {
      for (int ch = 0; ch < 4; ++ch) ipk.push_back(pk_ix(v, ch, s, first + gi));
      for (int k = 0; k < NUM_U64; ++k)
        i64.push_back(u64_ix(v, k, s, first + gi));
    }
  std::vector<uint4> pk;
  std::vector<uint64_t> over;
  if (gather(e, v.pk, ipk, pk) || gather(e, v.u64, i64, over))
    return DRB_EDEVICE;
  vals.assign(n * R * NUM_U64, 0);
  for (uint64_t q = 0; q < n * R; ++q) {
    uint32_t w[16];
    for (int ch = 0; ch < 4; ++ch) {
      const uint4 c = pk[q * 4 + ch];
      w[4 * ch] = c.x;
      w[4 * ch + 1] = c.y;
      w[4 * ch + 2] = c.z;
      w[4 * ch + 3] = c.w;
    }
    pk_decode(w, &over[q * NUM_U64], &vals[q * NUM_U64]);
  }
  return DRB_OK;
}

extern "C" int drb_import_replicas(drb_engine *e, uint64_t first_group,
                                   uint64_t n_groups,
                                   const drb_replica_state *st) {
  if (check_range(e, first_group, n_groups)) return DRB_ERANGE;
  const View &v = e->v;
  const uint32_t R = v.R;
  std::vector<uint64_t> i64, i32, irm;
  std::vector<uint64_t> d64;
  std::vector<uint32_t> d32, drs, dra;
  std::vector<uint64_t> drm, drn;
  std::vector<uint64_t> iri;
  std::vector<uint4> dric, drii;
  std::vector<uint32_t> dricf;
  // the window bounds are engine state (drb_import_log sets ring_lo): keep
  // the current ones across the re-encoding of the packed records
  std::vector<uint64_t> cur;
  if (read_records(e, first_group, n_groups, cur)) return DRB_EDEVICE;
  // a replica coming back from the CPU path has nothing in flight on the
  // device: its window guard restarts (no Replicate to keep resident)
  std::vector<uint64_t> ifl;
  std::vector<uint32_t> oldfl;
  for (uint64_t gi = 0; gi < n_groups; ++gi)
    for (uint32_t s = 0; s < R; ++s)
      ifl.push_back(u32_ix(v, W_FLAGS, s, first_group + gi));
  if (gather(e, v.u32, ifl, oldfl)) return DRB_EDEVICE;
  std::vector<uint64_t> ipk;
  std::vector<uint4> dpk;
  for (uint64_t gi = 0; gi < n_groups; ++gi) {
    uint64_t g = first_group + gi;
    for (uint32_t s = 0; s < R; ++s) {
      drb_replica_state c = st[gi * R + s];
      uint64_t vals[NUM_U64], over[NUM_U64];
      for (int k = 0; k < NUM_U64; ++k) vals[k] = over[k] = 0;
      for (int k = 0; k < NUM_U64_EXPORTED; ++k)
        vals[kU64Order[k]] = *st_u64(&c, k);
      const uint64_t *old = &cur[(gi * R + s) * NUM_U64];
      vals[F_RING_LO] = old[F_RING_LO];
      vals[F_RING_GUARD] =
          (oldfl[gi * R + s] & (DRB_F_FALLBACK | DRB_F_ERROR)) ? ~0ull
                                                             : old[F_RING_GUARD];
      vals[F_TERM_START] = c.last_index + 1;  // the term cache restarts empty
      uint32_t w[16];
      pk_encode(w, vals, over);
      for (int ch = 0; ch < 4; ++ch) {
        ipk.push_back(pk_ix(v, ch, s, g));
        dpk.push_back(make_uint4(w[4 * ch], w[4 * ch + 1], w[4 * ch + 2],
                                 w[4 * ch + 3]));
      }
      // overflow of escaped fields and the u64 counters
      // a quiesced replica's skipped ticks count from now
      vals[F_QS_BASE] = e->ticks;
      vals[F_SAVE_BASE] = 0;  // its LogDB record stream restarts
      for (int k = 0; k < NUM_U64; ++k) {
        const bool counter = k == F_TICK_COUNT || k == F_KV_COUNT ||
                             (k >= F_QS_TICK && k <= F_QS_EXIT) ||
                             k == F_RNG ||
                             k == F_QS_BASE || k == F_SAVE_BASE;
        i64.push_back(u64_ix(v, k, s, g));
        d64.push_back(counter ? vals[k] : (over[k] ? over[k] : vals[k]));
      }
      const uint32_t quiesced =
          v.quiesce && c.qs_quiesced_since > 0 ? F_QUIESCED : 0u;
      // a leader's transfer target (a pending request is not imported)
      const uint32_t xfer = c.role == DRB_LEADER && c.transfer >= 1 &&
                                    c.transfer <= R && c.transfer != s + 1
                                ? c.transfer << F_XFER_SHIFT
                                : 0u;
      const uint32_t w32[NUM_U32] = {c.role,
                                     (c.flags & F_PUBLIC) | quiesced | xfer,
                                     c.fallback_reason, c.ri_count, c.votes};
      for (int k = 0; k < NUM_U32; ++k) {
        i32.push_back(u32_ix(v, k, s, g));
        d32.push_back(w32[k]);
      }
      for (uint32_t p = 0; p < R; ++p) {
        irm.push_back(rem_ix(v, s, p, g));
        drm.push_back(c.remotes[p].match);
        drn.push_back(c.remotes[p].next);
        drs.push_back(c.remotes[p].state);
        dra.push_back(c.remotes[p].active);
      }
      for (uint32_t d = 0; d < DRB_RI_DEPTH; ++d) {
        iri.push_back(ri_ix(v, s, d, g));
        dric.push_back(mk4h(c.ri[d].ctx_low, c.ri[d].ctx_high));
        drii.push_back(mk4h(c.ri[d].index, c.ri[d].from));
        dricf.push_back(c.ri[d].confirmed);
      }
    }
  }
  int rc = 0;
  rc |= scatter(e, v.u64, i64, d64);
  rc |= scatter(e, v.pk, ipk, dpk);
  rc |= scatter(e, v.u32, i32, d32);
  rc |= scatter(e, v.rem_match, irm, drm);
  rc |= scatter(e, v.rem_next, irm, drn);
  rc |= scatter(e, v.rem_state, irm, drs);
  rc |= scatter(e, v.rem_active, irm, dra);
  rc |= scatter(e, v.ri_ctx, iri, dric);
  rc |= scatter(e, v.ri_idx, iri, drii);
  rc |= scatter(e, v.ri_conf, iri, dricf);
  if (rc) return DRB_EDEVICE;
  return refresh_roles(e);
}

extern "C" int drb_export_replicas(drb_engine *e, uint64_t first_group,
                                   uint64_t n_groups, drb_replica_state *st) {
  if (check_range(e, first_group, n_groups)) return DRB_ERANGE;
  const View &v = e->v;
  const uint32_t R = v.R;
  std::vector<uint64_t> i64, i32, irm, iri;
  for (uint64_t gi = 0; gi < n_groups; ++gi) {
    uint64_t g = first_group + gi;
    for (uint32_t s = 0; s < R; ++s) {
      for (int k = 0; k < NUM_U32; ++k) i32.push_back(u32_ix(v, k, s, g));
      for (uint32_t p = 0; p < R; ++p) irm.push_back(rem_ix(v, s, p, g));
      for (uint32_t d = 0; d < DRB_RI_DEPTH; ++d)
        iri.push_back(ri_ix(v, s, d, g));
    }
  }
  std::vector<uint64_t> d64, drm, drn;
  std::vector<uint32_t> d32, drs, dra, dricf;
  std::vector<uint4> dric, drii;
  int rc = 0;
  rc |= read_records(e, first_group, n_groups, d64);
  rc |= gather(e, v.u32, i32, d32);
  rc |= gather(e, v.rem_match, irm, drm);
  rc |= gather(e, v.rem_next, irm, drn);
  rc |= gather(e, v.rem_state, irm, drs);
  rc |= gather(e, v.rem_active, irm, dra);
  rc |= gather(e, v.ri_ctx, iri, dric);
  rc |= gather(e, v.ri_idx, iri, drii);
  rc |= gather(e, v.ri_conf, iri, dricf);
  if (rc) return DRB_EDEVICE;
  size_t a = 0, b = 0, c2 = 0, d = 0;
  for (uint64_t gi = 0; gi < n_groups; ++gi) {
    uint64_t g = first_group + gi;
    for (uint32_t s = 0; s < R; ++s) {
      drb_replica_state &o = st[gi * R + s];
      memset(&o, 0, sizeof(o));
      o.shard_id = v.first_shard_id + gid(v, s, g);
      o.replica_id = s + 1;
      for (int k = 0; k < NUM_U64_EXPORTED; ++k)
        *st_u64(&o, k) = d64[a + kU64Order[k]];
      const uint32_t fl = d32[b + 1];
      if ((fl & F_QUIESCED) && (fl & F_AT_REST) && (fl & DRB_F_HOSTED) &&
          !(fl & (DRB_F_FALLBACK | DRB_F_ERROR))) {
        // quiesced ticks not applied yet (drb_step.hpp, F_QS_BASE: stored
        // by a round that ends quiesced and at rest)
        const uint64_t owed = e->ticks - d64[a + F_QS_BASE];
        o.election_tick += owed;
        o.qs_current_tick += owed;
      }
      a += NUM_U64;
      o.role = d32[b++];
      o.flags = d32[b++] & F_PUBLIC;
      o.fallback_reason = d32[b++];
      o.ri_count = d32[b++];
      o.votes = d32[b++];
      o.transfer = (fl & F_XFER) >> F_XFER_SHIFT;
      for (uint32_t p = 0; p < R; ++p, ++c2) {
        o.remotes[p].match = drm[c2];
        o.remotes[p].next = drn[c2];
        o.remotes[p].state = drs[c2];
        o.remotes[p].active = dra[c2];
      }
      for (uint32_t q = 0; q < DRB_RI_DEPTH; ++q, ++d) {
        if (q >= o.ri_count) continue;
        o.ri[q].ctx_low = lo64h(dric[d]);
        o.ri[q].ctx_high = hi64h(dric[d]);
        o.ri[q].index = lo64h(drii[d]);
        o.ri[q].from = hi64h(drii[d]);
        o.ri[q].confirmed = dricf[d];
      }
    }
  }
  return DRB_OK;
}

// ---------------------------------------------------------------- log
static void entry_to_chunks(const View &v, const drb_entry &en,
                            const uint8_t *pool, uint4 *out /*3 + C16*/) {
  out[0] = mk4h(en.term, en.key);
  out[1] = mk4h(en.client_id, en.series_id);
  out[2] = mk4h(en.responded_to, 0);
  out[2].z = en.type;
  out[2].w = en.cmd_len;
  for (uint32_t c = 0; c < v.C16; ++c) {
    uint8_t b[16] = {0};
    for (uint32_t k = 0; k < 16; ++k) {
      uint32_t o = c * 16 + k;
      if (o < en.cmd_len) b[k] = pool[en.cmd_off + o];
    }
    memcpy(&out[ENT_META + c], b, 16);
  }
}

extern "C" int drb_import_log(drb_engine *e, uint64_t group, uint32_t slot,
                              const drb_entry *ents, size_t n,
                              const uint8_t *pool) {
  if (!e || group >= e->cfg.num_groups || slot >= e->cfg.num_replicas)
    return DRB_ERANGE;
  const View &v = e->v;
  if (n > v.W) return DRB_ERANGE;
  std::vector<uint64_t> idx;
  std::vector<uint4> val;
  std::vector<uint4> ch(ENT_META + v.C16);
  for (size_t i = 0; i < n; ++i) {
    if (ents[i].cmd_len > v.C16 * 16) return DRB_ERANGE;
    if (i && ents[i].index != ents[i - 1].index + 1) return DRB_EINVAL;
    entry_to_chunks(v, ents[i], pool, ch.data());
    for (uint32_t c = 0; c < ENT_META + v.C16; ++c) {
      idx.push_back(ring_ix(v, slot, ents[i].index, c, group));
      val.push_back(ch[c]);
    }
  }
  if (scatter(e, v.ring, idx, val)) return DRB_EDEVICE;
  if (n) {  // the window now starts at the first imported entry
    std::vector<uint64_t> cur;
    if (read_records(e, group, 1, cur)) return DRB_EDEVICE;
    uint64_t *vals = &cur[slot * NUM_U64];
    vals[F_RING_LO] = ents[0].index;
    uint64_t over[NUM_U64] = {0};
    uint32_t w[16];
    pk_encode(w, vals, over);
    std::vector<uint64_t> ipk = {pk_ix(v, 1, slot, group),
                                 pk_ix(v, 2, slot, group)};
    std::vector<uint4> dpk = {make_uint4(w[4], w[5], w[6], w[7]),
                              make_uint4(w[8], w[9], w[10], w[11])};
    std::vector<uint64_t> ri = {u64_ix(v, F_RING_LO, slot, group)};
    std::vector<uint64_t> rv = {ents[0].index};
    if (scatter(e, v.pk, ipk, dpk) || scatter(e, v.u64, ri, rv))
      return DRB_EDEVICE;
  }
  return DRB_OK;
}

extern "C" int drb_export_log(drb_engine *e, uint64_t group, uint32_t slot,
                              uint64_t lo, uint64_t hi, drb_entry *out,
                              uint8_t *pool, size_t pool_cap) {
  if (!e || group >= e->cfg.num_groups || slot >= e->cfg.num_replicas)
    return DRB_ERANGE;
  if (hi < lo) return DRB_OK;
  const View &v = e->v;
  if (hi - lo + 1 > v.W) return DRB_ERANGE;
  std::vector<uint64_t> idx;
  for (uint64_t i = lo; i <= hi; ++i)
    for (uint32_t c = 0; c < ENT_META + v.C16; ++c)
      idx.push_back(ring_ix(v, slot, i, c, group));
  std::vector<uint4> val;
  if (gather(e, v.ring, idx, val)) return DRB_EDEVICE;
  size_t used = 0, k = 0;
  for (uint64_t i = lo; i <= hi; ++i, ++k) {
    const uint4 *c = &val[k * (ENT_META + v.C16)];
    drb_entry &o = out[k];
    o.term = lo64h(c[0]);
    o.key = hi64h(c[0]);
    o.client_id = lo64h(c[1]);
    o.series_id = hi64h(c[1]);
    o.responded_to = lo64h(c[2]);
    o.type = c[2].z;
    o.cmd_len = c[2].w;
    o.index = i;
    o.cmd_off = used;
    if (o.cmd_len > v.C16 * 16 || used + o.cmd_len > pool_cap)
      return DRB_ERANGE;
    memcpy(pool + used, &c[ENT_META], o.cmd_len);
    used += o.cmd_len;
  }
  return DRB_OK;
}

// ---------------------------------------------------------------- init
// ConfigChange{AddNode, ReplicaID id, "localhost:<26000+id-1>", Initialize}
// (configchange.go:28-56, bootstrap peer.go:404-428)
__host__ __device__ static uint32_t cc_bytes(uint32_t id, uint8_t *b) {
  uint32_t i = 0;
  b[i++] = 0x08;
  b[i++] = 0;
  b[i++] = 0x10;
  b[i++] = 0;
  b[i++] = 0x18;
  b[i++] = (uint8_t)id;  // id < 128
  b[i++] = 0x22;
  b[i++] = 15;
  const char *h = "localhost:";
  for (int k = 0; k < 10; ++k) b[i++] = (uint8_t)h[k];
  uint32_t port = 26000 + id - 1;
  char d[5];
  for (int k = 4; k >= 0; --k) {
    d[k] = (char)('0' + port % 10);
    port /= 10;
  }
  for (int k = 0; k < 5; ++k) b[i++] = (uint8_t)d[k];
  b[i++] = 0x28;
  b[i++] = 1;
  return i;  // 25
}

__global__ void k_init_steady(View v, uint64_t term, uint32_t leader,
                              uint64_t seed) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t s = blockIdx.y;
  if (g >= v.G) return;
  const uint64_t R = v.R, L1 = R + 1;  // last index: R config + 1 no-op
  const bool is_leader = s == leader;
  uint64_t vals[NUM_U64], over[NUM_U64];
  for (int k = 0; k < NUM_U64; ++k) vals[k] = over[k] = 0;
#define SET(F, x) vals[F] = (x)
  SET(F_TERM, term);
  SET(F_VOTE, leader + 1);
  SET(F_LEADER_ID, leader + 1);
  SET(F_APPLIED, L1);
  SET(F_ELECTION_TICK, 0);
  SET(F_HEARTBEAT_TICK, 0);
  SET(F_RAND_TIMEOUT,
      v.election_rtt +
          mix64(seed ^ (0xE1ull << 56) ^ (gid(v, s, g) * R + s)) %
              v.election_rtt);
  SET(F_TICK_COUNT, 1);
  SET(F_COMMITTED, L1);
  SET(F_PROCESSED, L1);
  SET(F_LAST_INDEX, L1);
  SET(F_MARKER_INDEX, L1 + 1);
  SET(F_SAVED_TO, L1);
  SET(F_APPLIED_TO_INDEX, L1);
  SET(F_APPLIED_TO_TERM, term);
  SET(F_APPLIED_INDEX, L1);
  SET(F_CONFIRMED_INDEX, L1);
  SET(F_PUSHED_INDEX, L1);
  SET(F_PREV_TERM, term);
  SET(F_PREV_VOTE, leader + 1);
  SET(F_PREV_COMMIT, L1);
  SET(F_SM_INDEX, L1);
  SET(F_SM_TERM, term);
  SET(F_KV_COUNT, 0);
  SET(F_RING_LO, 1);
  SET(F_RING_GUARD, ~0ull);
  SET(F_TERM_START, L1);  // the leader's no-op opened the term
  if (v.quiesce) {
    // the election round of the setup ticked once, and its messages were
    // activity (quiesce.go:40-74)
    SET(F_QS_TICK, 1);
    SET(F_QS_IDLE, 1);
  }
#undef SET
  uint32_t w[16];
  pk_encode(w, vals, over);
  for (int k = 0; k < NUM_U64; ++k)  // escaped values (large ElectionRTT)
    if (over[k]) v.u64[u64_ix(v, k, s, g)] = over[k];
  for (int ch = 0; ch < 4; ++ch)
    v.pk[pk_ix(v, ch, s, g)] =
        make_uint4(w[4 * ch], w[4 * ch + 1], w[4 * ch + 2], w[4 * ch + 3]);
  v.u64[u64_ix(v, F_TICK_COUNT, s, g)] = vals[F_TICK_COUNT];
  v.u64[u64_ix(v, F_KV_COUNT, s, g)] = 0;
  for (int f = F_QS_TICK; f <= F_QS_EXIT; ++f) v.u64[u64_ix(v, f, s, g)] = vals[f];
  v.u64[u64_ix(v, F_QS_BASE, s, g)] = 0;
  v.u64[u64_ix(v, F_SAVE_BASE, s, g)] = 0;
  // raft.rand: restarted from a per-replica seed (the oracle's setup does
  // the same), one splitmix64 draw per randomized timeout afterwards
  v.u64[u64_ix(v, F_RNG, s, g)] =
      mix64(seed ^ (0xE2ull << 56) ^ (gid(v, s, g) * R + s));
  v.u32[u32_ix(v, W_ROLE, s, g)] = is_leader                  ? DRB_LEADER
                                  : (v.nv_mask >> s) & 1u ? DRB_NONVOTING
                                  : (v.wt_mask >> s) & 1u ? DRB_WITNESS
                                                          : DRB_FOLLOWER;
  v.u32[u32_ix(v, W_FLAGS, s, g)] =
      gid(v, s, g) < v.total_groups ? DRB_F_HOSTED : 0u;
  v.u32[u32_ix(v, W_FB_REASON, s, g)] = 0;
  v.u32[u32_ix(v, W_RI_COUNT, s, g)] = 0;
  v.u32[u32_ix(v, W_VOTES, s, g)] = 0;
  for (uint32_t p = 0; p < v.R; ++p) {
    uint64_t m, n;
    uint32_t st, act;
    if (is_leader) {  // after the no-op round trip (raft.go:1878-1908)
      m = L1;
      n = L1 + 1;
      st = p == s ? DRB_REMOTE_RETRY : DRB_REMOTE_REPLICATE;
      act = p == s ? 0 : 1;
    } else {  // becomeFollowerKE at the vote (raft.go:1088-1097)
      m = p == s ? R : 0;
      n = R + 1;
      st = DRB_REMOTE_RETRY;
      act = 0;
    }
    v.rem_match[rem_ix(v, s, p, g)] = m;
    v.rem_next[rem_ix(v, s, p, g)] = n;
    v.rem_state[rem_ix(v, s, p, g)] = st;
    v.rem_active[rem_ix(v, s, p, g)] = act;
  }
  // resident window: R config-change entries (term 1) + the no-op (term)
  for (uint64_t i = 1; i <= L1; ++i) {
    bool cc = i <= R;
    v.ring[ring_ix(v, s, i, 0, g)] = make_uint4(
        (uint32_t)(cc ? 1 : term), (uint32_t)((cc ? 1 : term) >> 32), 0, 0);
    v.ring[ring_ix(v, s, i, 1, g)] = make_uint4(0, 0, 0, 0);
    uint8_t b[32] = {0};
    uint32_t len = cc ? cc_bytes((uint32_t)i, b) : 0;
    v.ring[ring_ix(v, s, i, 2, g)] =
        make_uint4(0, 0, cc ? DRB_ENTRY_CONFIG_CHANGE : DRB_ENTRY_APPLICATION,
                   len);
    for (uint32_t c = 0; c < v.C16; ++c) {
      uint32_t w[4] = {0, 0, 0, 0};
      for (uint32_t k = 0; k < 16; ++k) {
        uint32_t o = c * 16 + k;
        if (o < 32) w[k >> 2] |= (uint32_t)b[o] << (8 * (k & 3));
      }
      v.ring[ring_ix(v, s, i, ENT_META + c, g)] =
          make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

extern "C" int drb_init_steady(drb_engine *e, uint64_t term,
                               uint32_t leader_slot, uint64_t seed) {
  if (!e || leader_slot >= e->cfg.num_replicas || term < 2) return DRB_EINVAL;
  if (((e->v.nv_mask | e->v.wt_mask) >> leader_slot) & 1u)
    return DRB_EINVAL;  // the leader is a voting member
  if (e->cfg.cmd_cap < 32 || e->v.W < e->cfg.num_replicas + 2)
    return DRB_EINVAL;
  e->v.stage_slot = leader_slot;  // staged inputs go to the leaders
  e->ticks = 0;                   // every replica's ticks start here
  dim3 grid((unsigned)((e->v.G + 255) / 256), e->v.R);
  k_init_steady<<<grid, 256, 0, e->stream>>>(e->v, term, leader_slot, seed);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(e->stream));
  return refresh_roles(e);
}

__global__ void k_host_slot(View v, uint32_t slot, uint32_t hosted) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= v.G || gid(v, slot, g) >= v.total_groups) return;
  uint32_t &f = v.u32[u32_ix(v, W_FLAGS, slot, g)];
  f = hosted ? (f | DRB_F_HOSTED) : (f & ~(DRB_F_HOSTED | F_AT_REST));
}

extern "C" int drb_host_slot(drb_engine *e, uint32_t slot, int hosted) {
  if (!e || slot >= e->v.R) return DRB_EINVAL;
  k_host_slot<<<(unsigned)((e->v.G + 255) / 256), 256, 0, e->stream>>>(
      e->v, slot, hosted ? 1u : 0u);
  HIPCHK(hipGetLastError());
  return refresh_roles(e);
}

// ---------------------------------------------------------------- inputs
// The entry queue as the host holds it (drb_entry rows + Cmd pool) is
// uploaded as-is and laid out in the staged-proposal planes on the device:
// one lane per group, entries j < counts[g] (the step reads no others).
__global__ void k_stage_props(View v, uint32_t slot, const uint32_t *counts,
                              const drb_entry *ents, const uint8_t *pool,
                              uint64_t pool_len) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= v.G) return;
  const uint32_t n = counts[g];
  v.prop_count[(uint64_t)slot * v.G + g] = n;
  for (uint32_t j = 0; j < n; ++j) {
    const drb_entry en = ents[g * v.max_props + j];
    const uint8_t *cmd = pool + en.cmd_off;
    v.props[prop_ix(v, slot, j, 0, g)] = mk4h(en.key, en.client_id);
    v.props[prop_ix(v, slot, j, 1, g)] = mk4h(en.series_id, en.responded_to);
    if (en.cmd_len > v.C16 * 16 || en.cmd_off + en.cmd_len > pool_len) {
      // a Cmd the staged planes cannot hold (or outside the pool): the
      // leader's pre-pass sends the group to the CPU path (DRB_FB_CAPACITY)
      v.props[prop_ix(v, slot, j, 2, g)] = make_uint4(en.type, ~0u, 1, 0);
      continue;
    }
    const uint32_t b0 = en.cmd_len ? cmd[0] : 0u;
    v.props[prop_ix(v, slot, j, 2, g)] = make_uint4(
        en.type, en.cmd_len,
        prop_fast(en.type, en.client_id, en.series_id, en.cmd_len, b0), 0);
    for (uint32_t c = 0; c < v.C16; ++c) {
      uint32_t w[4] = {0, 0, 0, 0};
      for (uint32_t b = 0; b < 16 && c * 16 + b < en.cmd_len; ++b)
        w[b >> 2] |= (uint32_t)cmd[c * 16 + b] << (8 * (b & 3));
      v.props[prop_ix(v, slot, j, PROP_META + c, g)] =
          make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

extern "C" int drb_stage_proposals(drb_engine *e, uint32_t slot,
                                   const uint32_t *counts,
                                   const drb_entry *ents,
                                   const uint8_t *pool, size_t pool_len) {
  if (!e || slot >= e->cfg.prop_slots) return DRB_ERANGE;
  if (!counts || !ents || (pool_len && !pool)) return DRB_EINVAL;
  const View &v = e->v;
  const uint64_t G = v.G;
  // the counts are checked here (DRB_ERANGE leaves the slot untouched);
  // each entry's Cmd extent on the device (k_stage_props)
  for (uint64_t g = 0; g < G; ++g)
    if (counts[g] > v.max_props) return DRB_ERANGE;
  const size_t ent_b = (size_t)G * v.max_props * sizeof(drb_entry);
  const size_t cnt_off = ent_b, pool_off = (cnt_off + G * 4 + 255) & ~(size_t)255;
  const size_t need = pool_off + std::max<uint64_t>(pool_len, 16);
  if (need > e->stage_bytes) {
    HIPCHK(hipStreamSynchronize(e->stream));  // the buffer may be in use
    HIPCHK(hipStreamSynchronize(e->stream_h2d));
    if (e->stage_buf) HIPCHK(hipFree(e->stage_buf));
    e->stage_buf = nullptr;
    HIPCHK(hipMalloc(&e->stage_buf, need));
    e->stage_bytes = need;
  }
  uint8_t *d = (uint8_t *)e->stage_buf;
  // The upload runs on its own stream, so it overlaps a round still
  // running on the engine stream; it starts once the previous call's layout
  // kernel has consumed the upload buffer.  The call returns when the host
  // arrays have been read (they may be reused); the layout kernel is
  // ordered on the engine stream after the upload, ahead of the round
  // that reads the slot.
  HIPCHK(hipStreamWaitEvent(e->stream_h2d, e->ev_stage_free, 0));
  HIPCHK(hipMemcpyAsync(d, ents, ent_b, hipMemcpyHostToDevice,
                        e->stream_h2d));
  HIPCHK(hipMemcpyAsync(d + cnt_off, counts, G * 4, hipMemcpyHostToDevice,
                        e->stream_h2d));
  if (pool_len)
    HIPCHK(hipMemcpyAsync(d + pool_off, pool, pool_len, hipMemcpyHostToDevice,
                          e->stream_h2d));
  HIPCHK(hipEventRecord(e->ev_staged, e->stream_h2d));
  HIPCHK(hipStreamWaitEvent(e->stream, e->ev_staged, 0));
  k_stage_props<<<(unsigned)((G + 255) / 256), 256, 0, e->stream>>>(
      v, slot, (const uint32_t *)(d + cnt_off), (const drb_entry *)d,
      d + pool_off, (uint64_t)pool_len);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e->ev_stage_free, e->stream));
  HIPCHK(hipEventRecord(e->ev_prop[slot], e->stream));
  HIPCHK(hipEventSynchronize(e->ev_staged));
  return DRB_OK;
}

// The packed form of a NoOP-session batch (drb_stage_proposals_packed):
// counts u8 per group, Key / ClientID / Cmd length per entry, the Cmd bytes
// back to back.  ent0[g] / coff[i]: exclusive scans of counts / lengths,
// read through widening iterators (no widened copies, no extra launches).
struct WidenU32 {
  __host__ __device__ uint32_t operator()(uint8_t x) const { return x; }
  __host__ __device__ uint32_t operator()(uint16_t x) const { return x; }
};
using WidenU8 = hipcub::TransformInputIterator<uint32_t, WidenU32,
                                               const uint8_t *>;
using WidenU16 = hipcub::TransformInputIterator<uint32_t, WidenU32,
                                                const uint16_t *>;

// clients null: every entry of lane g carries the group's registered
// session client, sess[g] (drb_set_session_clients)
__global__ void k_stage_packed(View v, uint32_t slot, uint32_t type,
                               const uint8_t *counts, const uint32_t *ent0,
                               const uint64_t *keys, const uint64_t *clients,
                               const uint64_t *sess, const uint16_t *lens,
                               const uint32_t *coff, const uint8_t *pool,
                               uint64_t pool_len) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= v.G) return;
  const uint32_t n = counts[g];
  v.prop_count[(uint64_t)slot * v.G + g] = n;
  const uint64_t sc = clients || !n ? 0ull : sess[g];
  for (uint32_t j = 0; j < n; ++j) {
    const uint64_t i = (uint64_t)ent0[g] + j;
    const uint64_t key = keys[i], cid = clients ? clients[i] : sc;
    const uint32_t len = lens[i];
    const uint64_t off = coff[i];
    v.props[prop_ix(v, slot, j, 0, g)] = mk4h(key, cid);
    v.props[prop_ix(v, slot, j, 1, g)] = make_uint4(0, 0, 0, 0);
    if (len > v.C16 * 16 || off + len > pool_len) {  // CAPACITY (pre-pass)
      v.props[prop_ix(v, slot, j, 2, g)] = make_uint4(type, ~0u, 1, 0);
      continue;
    }
    const uint8_t *cmd = pool + off;
    v.props[prop_ix(v, slot, j, 2, g)] = make_uint4(
        type, len, prop_fast(type, cid, 0, len, len ? cmd[0] : 0u), 0);
    for (uint32_t c = 0; c < v.C16; ++c) {
      uint32_t w[4] = {0, 0, 0, 0};
      for (uint32_t b = 0; b < 16 && c * 16 + b < len; ++b)
        w[b >> 2] |= (uint32_t)cmd[c * 16 + b] << (8 * (b & 3));
      v.props[prop_ix(v, slot, j, PROP_META + c, g)] =
          make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}

// the smallest staged upload worth the engine's own SDMA engine
constexpr size_t kSdmaMinBytes = 8u << 20;

// the packed batch's block layout (drb_stage_packed_layout): counts at 0,
// then keys, lengths, the pool and last the client ids, each 256-aligned
// (off[] = keys, client ids, lengths, pool); *bytes = the block's length.
// A batch of the registered session clients stops at the pool's end.
static void stage_layout(uint64_t G, uint64_t n, size_t pool_len,
                         uint64_t off[4], size_t *bytes) {
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const uint64_t n1 = n ? n : 1;
  off[0] = al(G);
  off[2] = off[0] + al(8 * n1);
  off[3] = off[2] + al(2 * n1);
  off[1] = al(off[3] + pool_len);
  *bytes = off[1] + 8 * n1;
}

extern "C" int drb_stage_packed_layout(const drb_engine *e, uint64_t n_entries,
                                       size_t pool_len, uint64_t *offsets,
                                       size_t *bytes) {
  if (!e || !offsets || !bytes) return DRB_EINVAL;
  stage_layout(e->v.G, n_entries, pool_len, offsets, bytes);
  return DRB_OK;
}

// drb_stage_proposals_packed(_async): `async` returns with the upload
// queued, once the previous call's upload is done (its arrays free)
static int stage_packed(drb_engine *e, uint32_t slot, uint32_t type,
                        const uint8_t *counts, uint64_t n_entries,
                        const uint64_t *keys, const uint64_t *client_ids,
                        const uint16_t *cmd_lens, const uint8_t *pool,
                        size_t pool_len, bool async) {
  if (!e || slot >= e->cfg.prop_slots) return DRB_ERANGE;
  if (!counts || (n_entries && (!keys || !cmd_lens)) || (pool_len && !pool))
    return DRB_EINVAL;
  // without client ids: the registered session clients
  if (n_entries && !client_ids && !e->sess_client) return DRB_EINVAL;
  const View &v = e->v;
  const uint64_t G = v.G, n = n_entries;
  // the counts before anything reads the entry arrays (they bound n); the
  // lengths' sum below, beside the upload (vectorised loops; on 8 host
  // threads the call measured slower: thread start-up costs more than the
  // 3 MB these read)
  uint64_t tsum = 0;
  uint32_t cmax = 0;
  for (uint64_t g = 0; g < G; ++g) {
    cmax = std::max<uint32_t>(cmax, counts[g]);
    tsum += counts[g];
  }
  if (cmax > v.max_props) return DRB_ERANGE;
  if (tsum != n) return DRB_EINVAL;
  // upload: counts | keys | lengths | pool | client ids (stage_layout),
  // then device-side the two scans and their temp storage
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const uint64_t n1 = n ? n : 1;
  size_t tb1 = 0, tb2 = 0;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(
      nullptr, tb1, WidenU8((const uint8_t *)nullptr, WidenU32()),
      (uint32_t *)nullptr, (int)G, e->stream));
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(
      nullptr, tb2, WidenU16((const uint16_t *)nullptr, WidenU32()),
      (uint32_t *)nullptr, (int)n1, e->stream));
  uint64_t lo[4];
  size_t up = 0;
  stage_layout(G, n, pool_len, lo, &up);
  const size_t o_cnt = 0, o_key = lo[0], o_cid = lo[1], o_len = lo[2],
               o_pool = lo[3];
  if (!client_ids) up = o_pool + pool_len;  // (no client region)
  const size_t o_e0 = al(std::max<size_t>(up, o_pool + 16)),
               o_off = o_e0 + al(4 * G), o_tmp = o_off + al(4 * n1),
               need = o_tmp + al(std::max(tb1, tb2));
  if (need > e->stage_bytes) {
    HIPCHK(hipStreamSynchronize(e->stream));  // the buffer may be in use
    HIPCHK(hipStreamSynchronize(e->stream_h2d));
    if (e->stage_buf) HIPCHK(hipFree(e->stage_buf));
    e->stage_buf = nullptr;
    HIPCHK(hipMalloc(&e->stage_buf, need));
    e->stage_bytes = need;
  }
  uint8_t *d = (uint8_t *)e->stage_buf;
  // the previous call's arrays are read once its upload is done
  if (async) HIPCHK(hipEventSynchronize(e->ev_uploaded));
  // the upload and the layout on the copy stream: the upload overlaps the
  // running round; the layout waits only for the engine-stream work on
  // this slot (ev_prop), so it runs beside a round that reads another
  // slot, and the engine stream waits for it before its next round
  HIPCHK(hipStreamWaitEvent(e->stream_h2d, e->ev_stage_free, 0));
  // the arrays in one block at stage_layout's offsets (a host that builds
  // its batch in place, drb_stage_packed_layout): one DMA
  const uint8_t *c8 = counts;
  const bool one_block =
      (const uint8_t *)keys == c8 + o_key &&
      (!client_ids || (const uint8_t *)client_ids == c8 + o_cid) &&
      (const uint8_t *)cmd_lens == c8 + o_len &&
      (!pool_len || pool == c8 + o_pool);
  // a large pinned one-block batch goes up on the engine's upload SDMA
  // engine (drb_hsa.hpp), the host waiting for it below, after the
  // lengths' sum; a small one (C2: 2.4 MB) as one hipMemcpyAsync, whose
  // wait the next call takes (0.238 against 0.265 ms/round at C2)
  bool sdma = false;
  if (one_block && up >= kSdmaMinBytes && hsa_host_pinned(counts) &&
      hsa_xfer_init(e->cfg.device, &e->xfer)) {
    const HsaXfer &x = e->xfer;
    HIPCHK(hipEventSynchronize(e->ev_stage_free));  // the buffer is free
    hsa_signal_store_screlease(x.up_done, 1);
    sdma = hsa_amd_memory_async_copy_on_engine(
               d, x.gpu, counts, x.cpu, up, 0, nullptr, x.up_done,
               (hsa_amd_sdma_engine_id_t)x.up, true) == HSA_STATUS_SUCCESS;
    if (!sdma) hsa_signal_store_screlease(x.up_done, 0);
  }
  if (!sdma && one_block) {
    HIPCHK(hipMemcpyAsync(d, counts, up, hipMemcpyHostToDevice,
                          e->stream_h2d));
  } else if (!sdma) {
    HIPCHK(hipMemcpyAsync(d + o_cnt, counts, G, hipMemcpyHostToDevice,
                          e->stream_h2d));
    if (n) {
      HIPCHK(hipMemcpyAsync(d + o_key, keys, 8 * n, hipMemcpyHostToDevice,
                            e->stream_h2d));
      if (client_ids)
        HIPCHK(hipMemcpyAsync(d + o_cid, client_ids, 8 * n,
                              hipMemcpyHostToDevice, e->stream_h2d));
      HIPCHK(hipMemcpyAsync(d + o_len, cmd_lens, 2 * n,
                            hipMemcpyHostToDevice, e->stream_h2d));
    }
    if (pool_len)
      HIPCHK(hipMemcpyAsync(d + o_pool, pool, pool_len,
                            hipMemcpyHostToDevice, e->stream_h2d));
  }
  HIPCHK(hipEventRecord(e->ev_uploaded, e->stream_h2d));
  // the lengths' sum while the upload runs; a batch that fails it is not
  // laid out, the slot stays as it was
  uint64_t bsum = 0;
  for (uint64_t i = 0; i < n; ++i) bsum += cmd_lens[i];
  if (sdma) hsa_wait_zero(e->xfer.up_done);  // (this call's arrays free)
  if (bsum != pool_len) {
    HIPCHK(hipEventRecord(e->ev_stage_free, e->stream_h2d));
    HIPCHK(hipEventSynchronize(e->ev_uploaded));
    return DRB_EINVAL;
  }
  HIPCHK(hipStreamWaitEvent(e->stream_h2d, e->ev_prop[slot], 0));
  hipStream_t ls = e->stream_h2d;
  uint32_t *e0 = (uint32_t *)(d + o_e0), *off = (uint32_t *)(d + o_off);
  const uint16_t *l16 = (const uint16_t *)(d + o_len);
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(
      d + o_tmp, tb1, WidenU8(d + o_cnt, WidenU32()), e0, (int)G, ls));
  if (n)
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(
        d + o_tmp, tb2, WidenU16(l16, WidenU32()), off, (int)n, ls));
  k_stage_packed<<<(unsigned)((G + 255) / 256), 256, 0, ls>>>(
      v, slot, type, d + o_cnt, e0, (const uint64_t *)(d + o_key),
      client_ids ? (const uint64_t *)(d + o_cid) : nullptr, e->sess_client,
      l16, off, d + o_pool, (uint64_t)pool_len);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(e->ev_staged, ls));
  HIPCHK(hipEventRecord(e->ev_stage_free, ls));
  HIPCHK(hipStreamWaitEvent(e->stream, e->ev_staged, 0));
  if (!async) HIPCHK(hipEventSynchronize(e->ev_uploaded));
  return DRB_OK;
}

extern "C" int drb_stage_proposals_packed(
    drb_engine *e, uint32_t slot, uint32_t type, const uint8_t *counts,
    uint64_t n_entries, const uint64_t *keys, const uint64_t *client_ids,
    const uint16_t *cmd_lens, const uint8_t *pool, size_t pool_len) {
  return stage_packed(e, slot, type, counts, n_entries, keys, client_ids,
                      cmd_lens, pool, pool_len, false);
}

extern "C" int drb_stage_proposals_packed_async(
    drb_engine *e, uint32_t slot, uint32_t type, const uint8_t *counts,
    uint64_t n_entries, const uint64_t *keys, const uint64_t *client_ids,
    const uint16_t *cmd_lens, const uint8_t *pool, size_t pool_len) {
  return stage_packed(e, slot, type, counts, n_entries, keys, client_ids,
                      cmd_lens, pool, pool_len, true);
}

extern "C" int drb_set_session_clients(drb_engine *e,
                                       const uint64_t *client_ids) {
  if (!e || !client_ids) return DRB_EINVAL;
  const uint64_t G = e->v.G;
  HIPCHK(hipSetDevice(e->cfg.device));
  if (!e->sess_client) {
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMalloc(&e->sess_client, std::max<uint64_t>(G, 1) * 8));
    e->bytes += G * 8;
  }
  // ordered before every later staging and export (both streams wait)
  HIPCHK(hipStreamSynchronize(e->stream_h2d));
  HIPCHK(hipMemcpyAsync(e->sess_client, client_ids, G * 8,
                        hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

extern "C" int drb_stage_wait_upload(drb_engine *e) {
  if (!e) return DRB_EINVAL;
  HIPCHK(hipEventSynchronize(e->ev_uploaded));
  return DRB_OK;
}

// SURVEY 8(d) synthetic writes; bit-identical to dragonboat_amd/workload.py
constexpr uint64_t ACTIVE_SALT = 0xAC71BE5EAC71BE5Eull;

// the proposals of one proposing lane
__device__ static void gen_kv_lane(const View &v, uint32_t ps, uint32_t k,
                                   uint32_t key_space, uint32_t val_len,
                                   uint64_t seed, uint64_t salt,
                                   uint64_t lane) {
  const uint64_t g = gid(v, v.stage_slot, lane);  // the seeded group
  const uint64_t cid = mix64(seed ^ 0xC11E47C11E47C11Eull ^ g) | 1;
  for (uint32_t j = 0; j < k; ++j) {
    uint64_t r0 = mix64(seed ^ (g * 0x9E3779B97F4A7C15ull) ^ (salt << 32) ^
                        ((uint64_t)j << 16));
    uint64_t r1 = mix64(r0), r2 = mix64(r1);
    uint64_t kv_key = r1 % key_space;
    // Cmd = 00 | 0a 08 <key8 LE> 12 <varint vlen> <val>, built 16 B at a
    // time; val = the LE64 words of the chain r2, mix64(r2), ...
    const uint32_t vs = val_len < 128 ? 1 : 2;
    const uint32_t hdr = 12 + vs, clen = hdr + val_len;
    uint64_t x = r2;
    uint32_t xi = 0;  // x is chain element xi
    for (uint32_t c = 0; c < v.C16; ++c) {
      uint32_t w[4] = {0, 0, 0, 0};
      for (uint32_t t = 0; t < 16; ++t) {
        const uint32_t q = c * 16 + t;
        uint32_t b = 0;
        if (q < hdr) {
          if (q == 1) b = 0x0a;
          else if (q == 2) b = 8;
          else if (q >= 3 && q < 11) b = (uint32_t)(kv_key >> (8 * (q - 3))) & 0xff;
          else if (q == 11) b = 0x12;
          else if (q == 12) b = vs == 1 ? val_len : ((val_len & 0x7f) | 0x80);
          else if (q == 13) b = val_len >> 7;
        } else if (q < clen) {
          const uint32_t pv = q - hdr;
          while (xi < pv / 8) {
            x = mix64(x);
            xi++;
          }
          b = (uint32_t)(x >> (8 * (pv % 8))) & 0xff;
        }
        w[t >> 2] |= b << (8 * (t & 3));
      }
      v.props[prop_ix(v, ps, j, PROP_META + c, lane)] =
          make_uint4(w[0], w[1], w[2], w[3]);
    }
    v.props[prop_ix(v, ps, j, 0, lane)] = mk4(r0 | 1, cid);
    v.props[prop_ix(v, ps, j, 1, lane)] = mk4(0, 0);
    v.props[prop_ix(v, ps, j, 2, lane)] = make_uint4(
        DRB_ENTRY_ENCODED, clen, prop_fast(DRB_ENTRY_ENCODED, cid, 0, clen, 0),
        0);
  }
}

// Each workgroup draws GEN_ITERS x 256 lanes, 256 at a time, writes every
// prop_count and gathers the proposing lanes in LDS; a full batch of 256
// (or the rest, at the end) is then generated one lane per thread.  At C5's
// 1 % a thread per lane left ~half the waves running the whole byte loop
// for one or two lanes (117 us a round at 4M groups).
constexpr uint32_t GEN_ITERS = 16;

__global__ __launch_bounds__(256) void k_gen_kv(
    View v, uint32_t ps, uint32_t k, uint32_t key_space, uint32_t val_len,
    uint64_t seed, uint64_t salt, uint32_t active_ppm) {
  if (active_ppm >= 1000000u) {  // every lane proposes: a thread per lane
    const uint64_t lane = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (lane >= v.G) return;
    v.prop_count[(uint64_t)ps * v.G + lane] = k;
    gen_kv_lane(v, ps, k, key_space, val_len, seed, salt, lane);
    return;
  }
  __shared__ uint32_t list[512];
  __shared__ uint32_t nlist;
  if (threadIdx.x == 0) nlist = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * GEN_ITERS * 256;
  for (uint32_t it = 0; it < GEN_ITERS; ++it) {
    const uint64_t lane = base + (uint64_t)it * 256 + threadIdx.x;
    if (lane < v.G) {
      const uint64_t g = gid(v, v.stage_slot, lane);
      const bool on =
          mix64(seed ^ ACTIVE_SALT ^ (g * 0x9E3779B97F4A7C15ull) ^
                (salt << 24)) % 1000000u < active_ppm;
      v.prop_count[(uint64_t)ps * v.G + lane] = on ? k : 0u;
      if (on) list[atomicAdd(&nlist, 1u)] = (uint32_t)(lane - base);
    }
    __syncthreads();
    const uint32_t n = nlist;
    if (n >= 256 || it + 1 == GEN_ITERS) {
      if (threadIdx.x < n && threadIdx.x < 256)
        gen_kv_lane(v, ps, k, key_space, val_len, seed, salt,
                    base + list[threadIdx.x]);
      __syncthreads();  // (the batch read before the list moves down)
      if (n > 256 && threadIdx.x < n - 256)
        list[threadIdx.x] = list[256 + threadIdx.x];
      if (threadIdx.x == 0) nlist = n > 256 ? n - 256 : 0u;
      __syncthreads();
    }
  }
  // (at most 255 left after the last batch of 256: one more pass)
  const uint32_t n = nlist;
  if (threadIdx.x < n)
    gen_kv_lane(v, ps, k, key_space, val_len, seed, salt,
                base + list[threadIdx.x]);
}

extern "C" int drb_gen_kv_proposals_active(drb_engine *e, uint32_t slot,
                                           uint32_t k, uint32_t key_space,
                                           uint32_t val_len, uint64_t seed,
                                           uint64_t salt, uint32_t active_ppm) {
  if (!e || slot >= e->cfg.prop_slots || k > e->cfg.max_props || !key_space ||
      val_len > 16383 ||
      12 + (val_len < 128 ? 1 : 2) + val_len > e->cfg.cmd_cap)
    return DRB_EINVAL;
  const uint64_t per = active_ppm >= 1000000u ? 256 : GEN_ITERS * 256;
  k_gen_kv<<<(unsigned)((e->v.G + per - 1) / per), 256, 0, e->stream>>>(
      e->v, slot, k, key_space, val_len, seed, salt, active_ppm);
  HIPCHK(hipGetLastError());  // stream-ordered before the next round
  HIPCHK(hipEventRecord(e->ev_prop[slot], e->stream));
  return DRB_OK;
}

extern "C" int drb_gen_kv_proposals(drb_engine *e, uint32_t slot, uint32_t k,
                                    uint32_t key_space, uint32_t val_len,
                                    uint64_t seed, uint64_t salt) {
  return drb_gen_kv_proposals_active(e, slot, k, key_space, val_len, seed,
                                     salt, 1000000u);
}

extern "C" int drb_stage_read_index(drb_engine *e, uint32_t slot,
                                    const uint64_t *ctx_low,
                                    const uint64_t *ctx_high) {
  if (!e || slot >= e->cfg.ri_slots) return DRB_ERANGE;
  const uint64_t G = e->v.G;
  std::vector<uint4> host(G);
  for (uint64_t g = 0; g < G; ++g) host[g] = mk4h(ctx_low[g], ctx_high[g]);
  HIPCHK(hipMemcpyAsync(e->v.ri_in + (uint64_t)slot * G, host.data(),
                        G * sizeof(uint4), hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

__global__ void k_gen_ri(View v, uint32_t rs, uint64_t seed, uint64_t salt,
                         uint64_t high) {
  const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (lane >= v.G) return;
  const uint64_t g = gid(v, v.stage_slot, lane);
  uint64_t low = mix64(seed ^ 0x5EAD1DE85EAD1DE8ull ^
                       (g * 0x9E3779B97F4A7C15ull) ^ (salt << 40)) |
                 1;
  v.ri_in[(uint64_t)rs * v.G + lane] = mk4(low, high);
}

extern "C" int drb_gen_read_index(drb_engine *e, uint32_t slot, uint64_t seed,
                                  uint64_t high) {
  if (!e || slot >= e->cfg.ri_slots) return DRB_ERANGE;
  // the ctx of batch `high` (ctx.High = the round + 30 of the reference's
  // genCtx, request.go:864-875): Low drawn from (seed, group, high), so
  // every batch staged ahead of its round has its own ctx and read keys
  k_gen_ri<<<(unsigned)((e->v.G + 255) / 256), 256, 0, e->stream>>>(
      e->v, slot, seed, high, high);
  HIPCHK(hipGetLastError());  // stream-ordered before the next round
  return DRB_OK;
}

// ------------------------------------------------------- leader transfer
// pendingLeaderTransfer.request (node.go:474-482, request.go): one pending
// target per replica -- a replica that still holds one refuses (busy)
__global__ void k_stage_xfer(View v, uint32_t slot, const uint32_t *targets,
                             unsigned long long *busy) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= v.G) return;
  const uint32_t t = targets[g];
  if (t == 0) return;
  const uint64_t fi = u32_ix(v, W_FLAGS, slot, g);
  const uint32_t f = v.u32[fi];
  if (!(f & DRB_F_HOSTED)) return;  // ErrShardNotFound at this NodeHost
  if (f & (F_XFER_REQ | DRB_F_FALLBACK | DRB_F_ERROR)) {
    atomicAdd(busy, 1ull);
    return;
  }
  v.xfer_in[ix(v, slot, g)] = (uint8_t)t;
  // the round takes it even when the replica is at rest (setStepReady,
  // nodehost.go:1249)
  v.u32[fi] = (f | F_XFER_REQ) & ~F_AT_REST;
}

extern "C" int drb_request_leader_transfer(drb_engine *e, uint32_t slot,
                                           const uint32_t *targets,
                                           uint64_t *busy) {
  if (!e || !targets) return DRB_EINVAL;
  if (slot >= e->cfg.num_replicas) return DRB_ERANGE;
  if (!e->v.elections || e->v.place_world > 1) return DRB_EINVAL;
  const uint64_t G = e->v.G;
  const uint32_t R = e->cfg.num_replicas;
  for (uint64_t g = 0; g < G; ++g)
    if (targets[g] > R) return DRB_EINVAL;
  std::lock_guard<std::mutex> lock(e->ingest_mu);  // ordered with rounds
  uint32_t *dt = nullptr;
  unsigned long long *db = nullptr;
  void *sc = nullptr;
  const size_t tb = (G * sizeof(uint32_t) + 15) & ~(size_t)15;
  if (scratch(e, tb + 16, &sc)) return DRB_EDEVICE;
  dt = (uint32_t *)sc;
  db = (unsigned long long *)((char *)sc + tb);
  HIPCHK(hipMemcpyAsync(dt, targets, G * sizeof(uint32_t),
                        hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipMemsetAsync(db, 0, sizeof(*db), e->stream));
  k_stage_xfer<<<(unsigned)((G + 255) / 256), 256, 0, e->stream>>>(e->v, slot,
                                                                   dt, db);
  HIPCHK(hipGetLastError());
  unsigned long long nb = 0;
  HIPCHK(hipMemcpyAsync(&nb, db, sizeof(nb), hipMemcpyDeviceToHost,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (busy) *busy = nb;
  return DRB_OK;
}

// ---------------------------------------------------------------- ingest
// A receiver whose inbox cannot hold a message leaves the fast path before
// its next round: DRB_F_FALLBACK with DRB_FB_CAPACITY, one flagged record
// (the first marker only; several planes of one receiver may race here).
// The message and the receiver's later ones go to the CPU path
// (include/drb_engine.h, drb_ingest_ex).
DRB_DEV void ing_flag_capacity(const View &v, uint64_t g, uint32_t slot,
                               uint64_t round) {
  const uint32_t old =
      atomicOr(&v.u32[u32_ix(v, W_FLAGS, slot, g)], DRB_F_FALLBACK);
  if (!(old & (DRB_F_FALLBACK | DRB_F_ERROR))) {
    v.u32[u32_ix(v, W_FB_REASON, slot, g)] = DRB_FB_CAPACITY;
    flag_log(v, g, slot, DRB_FB_CAPACITY, old | DRB_F_FALLBACK, round);
  }
}
// recv[i] = group << 8 | slot
__global__ void k_ing_flag(View v, const uint64_t *recv, uint64_t n,
                           uint64_t round) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ing_flag_capacity(v, recv[i] >> 8, (uint32_t)(recv[i] & 0xffu),
                               round);
}

// drb_ingest: the whole batch in a fixed number of device transfers.  The
// host decides every message's fate from one gather of the replicas'
// flags and one of the current (sender, receiver) headers; then the
// records, the Replicates' entries (into the unhosted sender's window, where
// the receiver reads them), the headers, the max-append words and the round
// tag bytes each go down in one scatter.  Messages keep their order within
// a (sender, receiver) pair (the receiver handles them in that order).
namespace {
struct InPlane {  // one (group, from, to) plane of this call
  uint64_t g;
  uint32_t from, to;
  uint4 cur;      // header: tag | quiesce, info, sender term
  uint64_t maxapp;
  bool maxapp_valid;
  bool remote;    // placement C4: the sender slot lives on another rank
  uint64_t elo;   // remote: the first entry index of the entry rows
};
}  // namespace

extern "C" int drb_ingest_ex(drb_engine *e, const drb_message *msgs, size_t n,
                             const drb_entry *ents, const uint8_t *pool,
                             uint8_t *status, uint64_t *accepted,
                             uint64_t *dropped, uint64_t *diverted) {
  if (!e || (n && !msgs)) return DRB_EINVAL;
  // a bound engine's remote planes are its peers' outboxes
  // (drb_exchange_local_bind): nothing is delivered into them
  if (!e->bound.empty()) return DRB_EINVAL;
  const View &v = e->v;
  std::lock_guard<std::mutex> lock(e->ingest_mu);
  // replicas spread over ranks: not between a round and its exchange
  if (v.remote_mask && e->exchanged_round != e->round) return DRB_EAGAIN;
  const uint32_t buf = (uint32_t)(e->round & 1);  // read by round+1
  const uint32_t tag = (uint32_t)e->round;
  uint64_t acc = 0, drop = 0, div = 0;
  // each message's fate (drb_ingest_fate); PLACED until decided otherwise
  std::vector<uint8_t> fate(n, DRB_ING_PLACED);
  // 1. shape checks, then the hosted flags of every target and sender
  std::vector<uint64_t> fidx;
  fidx.reserve(2 * n);
  std::vector<uint64_t> lane(n, 0);  // the receiver's lane (ing_target)
  for (size_t i = 0; i < n; ++i) {
    const drb_message &m = msgs[i];
    uint64_t g = 0;
    // (an unknown shard, a receiver of another rank: nodehost.go:2089-2098)
    if (!ing_target(v, m.shard_id, m.from, m.to, &g)) {
      fate[i] = DRB_ING_DROPPED;
      continue;
    }
    lane[i] = g;
    fidx.push_back(u32_ix(v, W_FLAGS, (uint32_t)(m.to - 1), g));
    fidx.push_back(u32_ix(v, W_FLAGS, (uint32_t)(m.from - 1), g));
  }
  std::vector<uint32_t> fl;
  if (gather(e, v.u32, fidx, fl)) return DRB_EDEVICE;
  // receivers flagged in this call (group * R + slot)
  std::unordered_map<uint64_t, uint8_t> flagged;
  // 2. the planes touched and their current headers
  std::unordered_map<uint64_t, uint32_t> pid;  // (g, from, to) -> plane
  std::vector<InPlane> planes;
  std::vector<uint32_t> mplane(n, ~0u);
  uint64_t last_key = ~0ull;
  uint32_t last_plane = 0;
  size_t q = 0;
  for (size_t i = 0; i < n; ++i) {
    if (fate[i] != DRB_ING_PLACED) continue;
    const drb_message &m = msgs[i];
    const uint32_t ft = fl[q++], ff = fl[q++];
    const uint32_t from = (uint32_t)(m.from - 1), to = (uint32_t)(m.to - 1);
    const uint64_t g = lane[i];
    // (a sender slot on another rank: this lane's is another group)
    const bool from_hosted = !pair_remote(v, from, to) &&
                             (ff & DRB_F_HOSTED) &&
                             !(ff & (DRB_F_FALLBACK | DRB_F_ERROR));
    if (!(ft & DRB_F_HOSTED) || from_hosted) {
      // the transport delivers remote senders to hosted replicas only
      fate[i] = DRB_ING_DROPPED;
      continue;
    }
    if (ft & (DRB_F_FALLBACK | DRB_F_ERROR)) {  // the CPU raft.Peer's
      fate[i] = DRB_ING_DIVERTED;
      continue;
    }
    const uint64_t key = (g * v.R + from) * v.R + to;
    if (key == last_key) {  // a transport batch keeps a group's messages
      mplane[i] = last_plane;  // together
      continue;
    }
    auto it = pid.find(key);
    if (it == pid.end()) {
      it = pid.emplace(key, (uint32_t)planes.size()).first;
      planes.push_back(
          InPlane{g, from, to, make_uint4(0, 0, 0, 0), 0, false, false, 0});
    }
    mplane[i] = it->second;
    last_key = key;
    last_plane = it->second;
  }
  // co-resident planes (local) and, with placement C4, planes whose sender
  // slot lives on another rank (remote: the inbound copies, entries in the
  // plane's entry rows)
  std::vector<uint64_t> hidx[2], xidx[2], lidx;
  std::vector<size_t> pidx[2];
  for (size_t p = 0; p < planes.size(); ++p) {
    const InPlane &pl = planes[p];
    const int r = pair_remote(v, pl.from, pl.to) ? 1 : 0;
    hidx[r].push_back(mmeta_ix(v, buf, pl.from, pl.to, pl.g));
    xidx[r].push_back(mmeta_ix(v, buf, pl.from, pl.to, pl.g));
    pidx[r].push_back(p);
    if (r) lidx.push_back(mmeta_ix(v, buf, pl.from, pl.to, pl.g));
  }
  std::vector<uint4> hdr[2];
  std::vector<uint64_t> mx[2], lo;
  if (gather(e, v.mbox_meta, hidx[0], hdr[0]) ||
      gather(e, v.mbox_maxapp, xidx[0], mx[0]))
    return DRB_EDEVICE;
  if (!lidx.empty() &&
      (gather(e, v.meta_in, hidx[1], hdr[1]) ||
       gather(e, v.maxapp_in, xidx[1], mx[1]) || gather(e, v.elo_in, lidx, lo)))
    return DRB_EDEVICE;
  for (int r = 0; r < 2; ++r)
    for (size_t q = 0; q < pidx[r].size(); ++q) {
      InPlane &pl = planes[pidx[r][q]];
      uint4 cur = hdr[r][q];
      if (!tag_is(cur.x, tag)) {  // nothing there yet this round
        cur = pack2(0, 0);
        cur.x = tag & MQ_TAG;
      }
      pl.cur = cur;
      pl.maxapp = mx[r][q];
      pl.maxapp_valid = mi_nrep(cur.y) > 0;
      pl.remote = r == 1;
      pl.elo = r && pl.maxapp_valid ? lo[q] : 0;
    }
  // 3. place every message in its plane, in order
  // [0] local arrays, [1] the inbound (remote) ones
  std::vector<uint64_t> ridx[2], eidx[2], tridx[2], trval[2], fwidx;
  std::vector<uint4> rval[2], eval[2], fwval;
  std::vector<uint4> ch(ENT_META + v.C16);
  for (size_t i = 0; i < n; ++i) {
    if (fate[i] != DRB_ING_PLACED) continue;
    const drb_message &m = msgs[i];
    InPlane &pl = planes[mplane[i]];
    uint4 &cur = pl.cur;
    const uint64_t rk = pl.g * v.R + pl.to;
    if (flagged.count(rk)) {  // the receiver left the fast path in this call
      fate[i] = DRB_ING_DIVERTED;
      continue;
    }
    // a GPU capacity: the receiver goes to the CPU path with this message
    auto capacity = [&]() {
      flagged.emplace(rk, 1);
      fate[i] = DRB_ING_DIVERTED;
    };
    if (m.type == DRB_MSG_QUIESCE) {  // node-level: a header bit
      cur.x |= MQ_QUIESCE;
      continue;
    }
    if (mi_count(cur.y) >= v.MB) {  // the plane's records
      capacity();
      continue;
    }
    const bool rep = m.type == DRB_MSG_REPLICATE;
    const int r = pl.remote ? 1 : 0;
    const uint32_t k = rep ? mi_nrep(cur.y)
                           : rec_pos(false, mi_noth(cur.y), v.MB);
    bool fit = true;
    for (uint64_t x = 0; fit && x < m.n_entries; ++x)
      fit = ents[m.entries_off + x].cmd_len <= v.C16 * 16;
    if (m.type == DRB_MSG_PROPOSE) {
      // handleFollowerPropose's message from another NodeHost: its entries
      // go to the sender's forward rows, one Propose per plane and round
      // (drb_config.forward_proposals)
      fit = fit && v.fwd_props && !pl.remote && !(cur.y & MI_PROP) &&
            m.n_entries <= v.max_props;
    }
    if (rep && pl.remote && m.n_entries) {
      // entry rows [elo, elo + E), elo set by the round's first Replicate
      // that carries entries (0: none yet; a commit-only Replicate needs no
      // rows)
      const uint64_t elo = pl.elo ? pl.elo : m.log_index + 1;
      fit = fit && m.log_index + 1 >= elo &&
            m.log_index + m.n_entries - elo < v.E;
      if (fit) pl.elo = elo;
    }
    if (rep && m.n_entries > v.W) fit = false;  // (the window rows)
    if (!fit) {
      capacity();
      continue;
    }
    if (m.type == DRB_MSG_PROPOSE) {
      const uint32_t fw = fwd_ps(v, buf, pl.from);
      for (uint64_t x = 0; x < m.n_entries; ++x) {
        const drb_entry &en = ents[m.entries_off + x];
        const uint8_t *cmd = pool + en.cmd_off;
        std::vector<uint4> pc(PROP_META + v.C16, make_uint4(0, 0, 0, 0));
        pc[0] = mk4h(en.key, en.client_id);
        pc[1] = mk4h(en.series_id, en.responded_to);
        pc[2] = make_uint4(en.type, en.cmd_len,
                           prop_fast(en.type, en.client_id, en.series_id,
                                     en.cmd_len, en.cmd_len ? cmd[0] : 0u),
                           0);
        if (en.cmd_len) memcpy(&pc[PROP_META], cmd, en.cmd_len);
        for (uint32_t c = 0; c < PROP_META + v.C16; ++c) {
          fwidx.push_back(prop_ix(v, fw, (uint32_t)x, c, pl.g));
          fwval.push_back(pc[c]);
        }
      }
    }
    if (rep && m.n_entries) {
      // the entries travel in the sender's (unhosted) window slot, or in the
      // plane's entry rows when the plane is remote
      for (uint64_t x = 0; x < m.n_entries; ++x) {
        drb_entry en = ents[m.entries_off + x];
        en.index = m.log_index + 1 + x;
        entry_to_chunks(v, en, pool, ch.data());
        for (uint32_t c = 0; c < ENT_META + v.C16; ++c) {
          eidx[r].push_back(
              pl.remote ? embox_ix(v, buf, pl.from, pl.to,
                                   (uint32_t)(en.index - pl.elo), c, pl.g)
                        : ring_ix(v, pl.from, en.index, c, pl.g));
          eval[r].push_back(ch[c]);
        }
      }
    }
    Msg mm;
    mm.type = m.type;
    mm.reject = m.reject ? 1 : 0;
    mm.n = (uint32_t)m.n_entries;
    mm.term = m.term;
    mm.log_index = m.log_index;
    mm.log_term = m.log_term;
    mm.commit = m.commit;
    mm.hint = m.hint;
    mm.hint_high = m.hint_high;
    uint4 c0, c1;
    msg_encode(mm, pl.to, nullptr, c0, c1);
    // the sender's term is stored once per (sender, receiver, round) in the
    // header; a record whose term differs from it makes the receiver fall
    // back (term gate, raft.go:1596-1609)
    const bool zero = (c0.x & MF_TERM_ZERO) != 0;
    bool other = false;
    if (!zero) {
      // a pre-vote record carries a term of its own (r.term + 1 or the
      // granted one): it never seeds the header's term (drb_ingest_wire
      // and the GPU's emit do the same)
      const bool pv = is_prevote_type(m.type);
      if (!pv && !(cur.y & MI_TERM)) {
        cur.z = (uint32_t)m.term;
        cur.w = (uint32_t)(m.term >> 32);
      } else if (pv || q_hi(cur) != m.term) {
        other = true;
        c0.x |= MF_TERM_OTHER;
        if (v.rterm) {  // elections: the raft launch reads it
          tridx[r].push_back(rterm_ix(v, buf, pl.from, pl.to, k, pl.g));
          trval[r].push_back(m.term);
        }
      }
    }
    ridx[r].push_back(mbox_ix(v, buf, pl.from, pl.to, k, 0, pl.g));
    rval[r].push_back(c0);
    ridx[r].push_back(mbox_ix(v, buf, pl.from, pl.to, k, 1, pl.g));
    rval[r].push_back(c1);
    const uint32_t inf =
        msg_info(m.type, zero, m.reject != 0, (uint32_t)m.n_entries) |
        (other ? MI_TERM_OTHER : 0);
    cur.y = (cur.y + (inf & MI_CNTS)) | (inf & ~MI_CNTS);
    if (rep) {
      const uint64_t ma = m.log_index + m.n_entries;
      pl.maxapp = pl.maxapp_valid ? std::max(pl.maxapp, ma) : ma;
      pl.maxapp_valid = true;
    }
  }
  for (size_t i = 0; i < n; ++i) {
    acc += fate[i] == DRB_ING_PLACED;
    drop += fate[i] == DRB_ING_DROPPED;
    div += fate[i] == DRB_ING_DIVERTED;
  }
  // 4. down: entries, records, headers, max-append, the round tag bytes
  std::vector<uint4> hval[2];
  std::vector<uint64_t> xval[2], tidx, lval;
  for (int r = 0; r < 2; ++r)
    for (size_t p : pidx[r]) {
      hval[r].push_back(planes[p].cur);
      xval[r].push_back(planes[p].maxapp);
      if (r) lval.push_back(planes[p].elo);
    }
  // tag bytes: one u64 word per (receiver, group), a byte per sender
  std::unordered_map<uint64_t, uint32_t> tw;
  std::vector<uint64_t> tmask;  // sender bytes to set per word
  std::vector<uint64_t> tbyte;  // their values (tag_byte, drb_msg.hpp)
  for (const InPlane &pl : planes) {
    if (pl.remote) continue;  // (remote planes: the header's tag alone)
    if (!(mi_count(pl.cur.y) || (pl.cur.x & MQ_QUIESCE))) continue;
    const uint64_t w = ((uint64_t)buf * v.R + pl.to) * v.G + pl.g;
    auto it = tw.find(w);
    if (it == tw.end()) {
      it = tw.emplace(w, (uint32_t)tidx.size()).first;
      tidx.push_back(w);
      tmask.push_back(0);
      tbyte.push_back(0);
    }
    tmask[it->second] |= 0xffull << (8 * pl.from);
    tbyte[it->second] |= (uint64_t)tag_byte(tag, pl.cur.y) << (8 * pl.from);
  }
  std::vector<uint64_t> tv;
  if ((v.rterm && scatter(e, v.rterm, tridx[0], trval[0])) ||
      scatter(e, v.ring, eidx[0], eval[0]) ||
      scatter(e, v.props, fwidx, fwval) ||
      scatter(e, v.mbox, ridx[0], rval[0]) ||
      scatter(e, v.mbox_meta, hidx[0], hval[0]) ||
      scatter(e, v.mbox_maxapp, xidx[0], xval[0]) ||
      gather(e, v.inbox_tag, tidx, tv))
    return DRB_EDEVICE;
  if (!pidx[1].empty() &&
      ((v.rterm_in && scatter(e, v.rterm_in, tridx[1], trval[1])) ||
       scatter(e, v.embox_in, eidx[1], eval[1]) ||
       scatter(e, v.mbox_in, ridx[1], rval[1]) ||
       scatter(e, v.meta_in, hidx[1], hval[1]) ||
       scatter(e, v.maxapp_in, xidx[1], xval[1]) ||
       scatter(e, v.elo_in, lidx, lval)))
    return DRB_EDEVICE;
  for (size_t w = 0; w < tidx.size(); ++w)
    tv[w] = (tv[w] & ~tmask[w]) | (tmask[w] & tbyte[w]);
  if (scatter(e, v.inbox_tag, tidx, tv)) return DRB_EDEVICE;
  // 5. the receivers that left the fast path in this call
  if (!flagged.empty()) {
    std::vector<uint64_t> rv;
    for (const auto &kv : flagged)
      rv.push_back(((kv.first / v.R) << 8) | (kv.first % v.R));
    uint64_t *d = nullptr;
    void *sc = nullptr;
    if (scratch(e, rv.size() * 8, &sc)) return DRB_EDEVICE;
    d = (uint64_t *)sc;
    HIPCHK(hipMemcpyAsync(d, rv.data(), rv.size() * 8, hipMemcpyHostToDevice,
                          e->stream));
    k_ing_flag<<<(unsigned)((rv.size() + 255) / 256), 256, 0, e->stream>>>(
        e->v, d, rv.size(), e->round);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(e->stream));  // (rv and the scratch)
  }
  if (status && n) memcpy(status, fate.data(), n);
  if (accepted) *accepted = acc;
  if (dropped) *dropped = drop;
  if (diverted) *diverted = div;
  return DRB_OK;
}

extern "C" int drb_ingest(drb_engine *e, const drb_message *msgs, size_t n,
                          const drb_entry *ents, const uint8_t *pool,
                          uint64_t *accepted, uint64_t *dropped) {
  uint64_t div = 0;
  const int rc = drb_ingest_ex(e, msgs, n, ents, pool, nullptr, accepted,
                               dropped, &div);
  // (a caller without the fates must not lose the diverted messages)
  return rc == DRB_OK && div ? DRB_EDIVERTED : rc;
}

// ---------------------------------------------------------------- step
// Each role's launch covers only the slots where that role occurs (the
// role map, refreshed after every host-side state change): in the steady
// state the leader kernel's grid is one slot high, not R.
static uint32_t slot_list(uint32_t mask, uint32_t *n) {
  uint32_t l = 0;
  *n = 0;
  for (uint32_t s = 0; s < 8; ++s)
    if ((mask >> s) & 1u) l |= s << (4 * (*n)++);
  return l;
}

// ---------------------------------------------------------------- active list
// A listed round (drb_round_in.listed) first lists, per (role, slot), the
// lanes whose replica has work this round -- everything the step kernel's
// idle rule (drb_step.hpp idle_round) would not skip -- in group order:
// k_active_scan ballots the rule per wave, k_active_prefix turns the
// per-block counts into offsets, k_active_scatter writes the lanes.  The
// step kernels then take 256 listed lanes per block, so a round where most
// replicas are at rest (C5 with Quiesce) runs dense waves; group order
// keeps neighbouring lanes' SoA accesses in the same lines.  Each row's
// list holds the "heavy" lanes first -- a leader with staged proposals, or
// a replica whose inbox holds a Replicate / ReplicateResp (the tag byte's
// heavy bit, drb_msg.hpp): it appends, commits, applies, saves -- then the
// light ones (ticks, heartbeats), so the long paths of a round where 1 %
// of the groups propose run in dense waves of their own instead of one
// lane in sixty-four.  Count rows: [(role * R + slot) * 2 + heavy?0:1].
template <int R>
__global__ __launch_bounds__(256) void k_active_scan(const View v,
                                                     RoundParams p) {
  // one thread per group, all R replica slots: every input of the rule
  // loaded at once (one memory round trip), the group's proposal count and
  // ReadIndex row once for all slots
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t nb = gridDim.x;
  const bool valid = g < v.G;
  const uint32_t rbuf = (uint32_t)((p.round - 1) & 1);
  uint32_t flags[R], role[R], pc = 0;
  uint64_t tags[R];
  uint4 ri = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int s = 0; s < R; ++s) {
    flags[s] = role[s] = 0;
    tags[s] = 0;
  }
  if (valid) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      flags[s] = v.u32[u32_ix(v, W_FLAGS, s, g)];
      role[s] = v.u32[u32_ix(v, W_ROLE, s, g)];
      tags[s] = v.inbox_tag[((uint64_t)rbuf * v.R + s) * v.G + g];
    }
    if (p.prop_slot != DRB_NONE)
      pc = v.prop_count[(uint64_t)p.prop_slot * v.G + g];
    if (p.ri_slot != DRB_NONE) ri = v.ri_in[(uint64_t)p.ri_slot * v.G + g];
  }
  __shared__ uint32_t c[R][4][4];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < R; ++s) {
    const bool lead = role[s] == DRB_LEADER;
    bool run = false, heavy = false;
    if (flags[s] & DRB_F_HOSTED) {
      if (flags[s] & (DRB_F_FALLBACK | DRB_F_ERROR)) {
        v.rtr_count[ix(v, s, g)] = 0;  // no round output (step kernel)
        if (p.encode_saves) v.save_len[ix(v, s, g)] = 0;
      } else {
        run = !idle_round_of<R>(v, p, s, lead, flags[s], tags[s], pc, ri);
      }
    }
    if (run) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const uint32_t b = (uint32_t)(tags[s] >> (8 * q)) & 0xffu;
        if (q != s && tag_current(b, p.round - 1) && (b & TAG_HEAVY))
          heavy = true;
      }
      if (prop_here(v, p, s, lead) && pc != 0) heavy = true;
    }
    uint64_t bal[4];
    bal[0] = __ballot(run && lead && heavy);
    bal[1] = __ballot(run && lead && !heavy);
    bal[2] = __ballot(run && !lead && heavy);
    bal[3] = __ballot(run && !lead && !heavy);
    if (lane == 0) {
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        const uint64_t row = ((uint64_t)(k >> 1) * v.R + s) * 2 + (k & 1);
        v.act_mask[(row * nb + blockIdx.x) * 4 + wave] = bal[k];
        c[s][k][wave] = (uint32_t)__popcll(bal[k]);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 4 * R) {
    const uint32_t s = threadIdx.x >> 2, k = threadIdx.x & 3;
    const uint64_t row = ((uint64_t)(k >> 1) * v.R + s) * 2 + (k & 1);
    v.act_cnt[row * nb + blockIdx.x] =
        c[s][k][0] + c[s][k][1] + c[s][k][2] + c[s][k][3];
  }
}

// exclusive scan of one row's block counts (one workgroup per row)
__global__ __launch_bounds__(1024) void k_active_prefix(const View v,
                                                        uint64_t nb) {
  const uint64_t row = blockIdx.x;
  const uint32_t *cnt = v.act_cnt + row * nb;
  uint32_t *off = v.act_off + row * nb;
  const uint64_t chunk = (nb + 1023) / 1024;
  const uint64_t lo = threadIdx.x * chunk;
  const uint64_t hi = lo + chunk < nb ? lo + chunk : nb;
  uint32_t sum = 0;
  for (uint64_t i = lo; i < hi; ++i) sum += cnt[i];
  __shared__ uint32_t part[1024];
  part[threadIdx.x] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive scan
    const uint32_t x = threadIdx.x >= o ? part[threadIdx.x - o] : 0u;
    __syncthreads();
    part[threadIdx.x] += x;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - sum;
  for (uint64_t i = lo; i < hi; ++i) {
    off[i] = run;
    run += cnt[i];
  }
  if (threadIdx.x == 1023) v.act_total[row] = part[1023];
  // (a lean round's escalation counts, per list row, start at zero)
  if (threadIdx.x < ESC_SPLIT && row < 2ull * v.R)
    v.esc_n[row * ESC_SPLIT + threadIdx.x] = 0;
}

__global__ __launch_bounds__(256) void k_active_scatter(const View v) {
  const uint32_t s = blockIdx.y;
  const uint64_t nb = gridDim.x;
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint32_t k = 0; k < 4; ++k) {
    const uint64_t lrow = (uint64_t)(k >> 1) * v.R + s;  // the list's row
    const uint64_t row = lrow * 2 + (k & 1);             // its count row
    const uint64_t *m = v.act_mask + (row * nb + blockIdx.x) * 4;
    const uint64_t mw = m[wave];
    if (!((mw >> lane) & 1ull)) continue;
    uint32_t before = 0;
    for (uint32_t w = 0; w < wave; ++w) before += (uint32_t)__popcll(m[w]);
    const uint64_t base = (k & 1) ? v.act_total[lrow * 2] : 0;  // light
    const uint64_t pos = base + v.act_off[row * nb + blockIdx.x] + before +
                         (uint32_t)__popcll(mw & ((1ull << lane) - 1ull));
    v.act_list[lrow * v.G + pos] = (uint32_t)g;
  }
}

// the largest round (workgroups of both launches) whose leader and
// follower launches run side by side (C2, 768 workgroups: 0.0882 against
// 0.0928 ms/round on one stream, profiles/r05_chunk)
constexpr uint64_t kSplitMaxBlocks = 2048;

// blk0 / nblk: a chunk of group blocks (drb_step_rounds; nblk 0: all), on
// stream st
template <int R>
static void launch_step(drb_engine *e, const RoundParams &p0,
                        hipStream_t st = nullptr, uint32_t blk0 = 0,
                        uint32_t nblk = 0) {
  const unsigned gx_all = (unsigned)((e->v.G + 255) / 256);
  const unsigned gx = nblk ? nblk : gx_all;
  if (!st) st = e->stream;
  if (p0.listed) {
    k_active_scan<R><<<gx, 256, 0, e->stream>>>(e->v, p0);
    k_active_prefix<<<4 * e->v.R, 1024, 0, e->stream>>>(e->v, gx);
    k_active_scatter<<<dim3(gx, e->v.R), 256, 0, e->stream>>>(e->v);
  }
  RoundParams pl = p0, pf = p0;
  pl.blk0 = pf.blk0 = blk0;
  pl.gx_all = pf.gx_all = nblk ? gx_all : 0u;
  uint32_t nl = 0, nf = 0;
  pl.slots = slot_list(e->role_slots[0], &nl);
  pf.slots = slot_list(e->role_slots[1], &nf);
  // the EXT instantiation only where its paths can run (drb_step.hpp)
  const bool ext =
      e->v.C16 > 4 || e->v.kv_ool || p0.encode_saves || e->v.quiesce ||
      e->v.kv_ovf_cap;
  pl.nrows = nl;
  pf.nrows = nf;
  // one-dimensional grids of the role's slot rows, row-major (block_pos);
  // both launches back to back on the engine stream (they touch disjoint
  // state; on two streams they measured 3 % slower at C3)
  const StepLaunchFn *launch = kStepLaunch[R - 1];
  // forwarded proposals and member kinds: the EXT kernels with the Propose
  // and nonVoting / witness paths
  const bool fwd = e->v.fwd_props || e->v.nv_mask || e->v.wt_mask;
  // without placement (no remote planes) the LOCAL instantiations, which
  // compile the remote-plane paths out (drb_launch.hpp)
  const bool local = !e->v.remote_mask;
  const int kl = fwd ? SK_LEAD_FWD
                 : ext ? (local ? SK_LEAD_EXT_LOCAL : SK_LEAD_EXT)
                       : (local ? SK_LEAD_LOCAL : SK_LEAD);
  const int kf = fwd ? SK_FOLLOW_FWD
                 : ext ? (local ? SK_FOLLOW_EXT_LOCAL : SK_FOLLOW_EXT)
                       : (local ? SK_FOLLOW_LOCAL : SK_FOLLOW);
  // a small round (C2: 64k groups, 768 workgroups, one wave per SIMD) runs
  // its two launches side by side on the engine's two streams: they touch
  // disjoint state, and neither fills the chip alone
  const bool split = nl && nf && !nblk && !e->v.elections &&
                     st == e->stream &&
                     (uint64_t)gx * (nl + nf) <= kSplitMaxBlocks;
  if (split) {
    (void)hipEventRecord(e->ev_fork, st);
    (void)hipStreamWaitEvent(e->stream2, e->ev_fork, 0);
  }
  // listed rounds of a plain EXT engine: the light lanes' heartbeat rounds
  // through the lean kernel first (drb_lean.hpp), the full kernel then
  // over the heavy lanes and the ones the lean kernel escalated
  const bool lean = p0.listed && ext && !fwd && !nblk &&
                    !e->v.elections && !e->v.remote_mask &&
                    !e->v.save_tan && !e->v.save_batched && !e->no_lean &&
                    st == e->stream;
  if (lean) {
    // the lean kernels, then the full ones over the heavy and the
    // escalated lanes, one stream.  Measured slower on two streams: the
    // heavy lanes' full launches beside the lean kernels (2.02 against 1.97
    // ms a C5 round), the two full launches side by side (1.92 against
    // 1.90), the two lean ones (1.93), both pairs (1.96;
    // profiles/r06_lean/c5_streams_ab.txt).
    if (split) {
      (void)hipEventRecord(e->ev_join, e->stream2);
      (void)hipStreamWaitEvent(st, e->ev_join, 0);
    }
    if (nl) launch[SK_LEAD_LEAN](e->v, pl, gx * nl, st);
    if (nf) launch[SK_FOLLOW_LEAN](e->v, pf, gx * nf, st);
    pl.lean = pf.lean = LEAN_ALL;
    if (nl) launch[kl](e->v, pl, gx * nl, st);
    if (nf) launch[kf](e->v, pf, gx * nf, st);
    return;
  }
  hipStream_t sf = split ? e->stream2 : st;
  if (nl) launch[kl](e->v, pl, gx * nl, st);
  if (nf) launch[kf](e->v, pf, gx * nf, sf);
  if (split) {
    (void)hipEventRecord(e->ev_join, e->stream2);
    (void)hipStreamWaitEvent(st, e->ev_join, 0);
  }
  if (e->v.elections) {  // the replicas the two launches routed (F_SLOW)
    RoundParams ps = p0;
    ps.slots = 0;
    ps.nrows = 1;
    launch[SK_SLOW](e->v, ps, (e->v.slow_cap + 255) / 256, e->stream);
  }
}

// role map: bit s of role_slots[0] when a hosted replica of slot s is a
// leader, of role_slots[1] when one is not (roles change on the host side
// only: init, import; a replica whose role would change falls back)
__global__ void k_role_scan(View v, uint32_t *out) {
  __shared__ uint32_t any[2];
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t s = blockIdx.y;
  if (threadIdx.x < 2) any[threadIdx.x] = 0;
  __syncthreads();
  if (g < v.G && (v.u32[u32_ix(v, W_FLAGS, s, g)] & DRB_F_HOSTED)) {
    const bool lead = v.u32[u32_ix(v, W_ROLE, s, g)] == DRB_LEADER;
    any[lead ? 0 : 1] = 1;  // benign race: every writer stores 1
  }
  __syncthreads();
  // one global atomic per block and role (not per lane: those serialise)
  if (threadIdx.x < 2 && any[threadIdx.x]) atomicOr(&out[threadIdx.x], 1u << s);
}

static int refresh_roles(drb_engine *e) {
  if (e->v.elections) {  // roles change on the device: both launches span
    e->role_slots[0] = e->role_slots[1] = (1u << e->v.R) - 1u;  // every slot
    return DRB_OK;
  }
  HIPCHK(hipMemsetAsync(e->role_dev, 0, 8, e->stream));
  dim3 grid((unsigned)((e->v.G + 255) / 256), e->v.R);
  k_role_scan<<<grid, 256, 0, e->stream>>>(e->v, e->role_dev);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->role_slots, e->role_dev, 8, hipMemcpyDeviceToHost,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

__global__ void k_role_census(View v, unsigned long long *out) {
  __shared__ unsigned long long part[8];
  if (threadIdx.x < 8) part[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t s = blockIdx.y;
  if (g < v.G) {
    const uint32_t fl = v.u32[u32_ix(v, W_FLAGS, s, g)];
    if ((fl & DRB_F_HOSTED) && !(fl & (DRB_F_FALLBACK | DRB_F_ERROR)))
      atomicAdd(&part[v.u32[u32_ix(v, W_ROLE, s, g)] & 7u], 1ull);
  }
  __syncthreads();
  if (threadIdx.x < 8 && part[threadIdx.x])
    atomicAdd(&out[s * 8 + threadIdx.x], part[threadIdx.x]);
}

extern "C" int drb_role_census(drb_engine *e, uint64_t *counts) {
  if (!e || !counts) return DRB_EINVAL;
  void *d;
  const size_t bytes = (size_t)e->v.R * 8 * sizeof(uint64_t);
  if (scratch(e, bytes, &d)) return DRB_EDEVICE;
  HIPCHK(hipMemsetAsync(d, 0, bytes, e->stream));
  dim3 grid((unsigned)((e->v.G + 255) / 256), e->v.R);
  k_role_census<<<grid, 256, 0, e->stream>>>(e->v,
                                             (unsigned long long *)d);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(counts, d, bytes, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

extern "C" int drb_role_slots(const drb_engine *e, uint32_t *leader_slots,
                              uint32_t *follower_slots) {
  if (!e) return DRB_EINVAL;
  if (leader_slots) *leader_slots = e->role_slots[0];
  if (follower_slots) *follower_slots = e->role_slots[1];
  return DRB_OK;
}

// a round's parameters from its drb_round_in (round t = e->round + 1 + ahead)
static int round_params(drb_engine *e, const drb_round_in *in, uint64_t ahead,
                        uint64_t ticks_before, RoundParams *out) {
  if (in->prop_slot != DRB_NONE && in->prop_slot >= e->cfg.prop_slots)
    return DRB_ERANGE;
  if (in->ri_slot != DRB_NONE && in->ri_slot >= e->cfg.ri_slots)
    return DRB_ERANGE;
  RoundParams p;
  memset(&p, 0, sizeof(p));
  p.slots = 0;
  p.nrows = 1;
  p.round = e->round + 1 + ahead;
  p.tick = in->tick ? 1 : 0;
  p.tick_no = ticks_before + p.tick;
  p.prop_slot = in->prop_slot;
  p.ri_slot = in->ri_slot;
  p.n_reads = in->reads_per_ctx;
  p.key_space = in->read_key_space;
  if (p.n_reads && !p.key_space) return DRB_EINVAL;
  if (p.n_reads && e->v.max_reads && p.n_reads > e->v.max_reads)
    return DRB_ERANGE;
  p.encode_saves = in->encode_saves ? 1 : 0;
  if (p.encode_saves && !e->v.save_cap16) return DRB_EINVAL;
  p.ri_replica = in->ri_replica;
  p.listed = in->listed ? 1 : 0;
  if (p.listed && e->v.remote_mask) return DRB_EINVAL;
  p.prop_replica = in->prop_replica;
  if (p.prop_replica > e->v.R || (p.prop_replica && !e->v.fwd_props))
    return DRB_EINVAL;
  if (p.ri_replica > e->v.R || (p.ri_replica && e->v.place_world > 1))
    return DRB_EINVAL;
  // a witness neither proposes nor reads: ErrInvalidOperation (node.go:
  // 425-429, nodehost.go:823, 909)
  if ((p.prop_replica && ((e->v.wt_mask >> (p.prop_replica - 1)) & 1u)) ||
      (p.ri_replica && ((e->v.wt_mask >> (p.ri_replica - 1)) & 1u)))
    return DRB_EINVAL;
  *out = p;
  return DRB_OK;
}

static int launch_any(drb_engine *e, const RoundParams &p,
                      hipStream_t st = nullptr, uint32_t blk0 = 0,
                      uint32_t nblk = 0) {
  switch (e->v.R) {
    case 1: launch_step<1>(e, p, st, blk0, nblk); break;
    case 2: launch_step<2>(e, p, st, blk0, nblk); break;
    case 3: launch_step<3>(e, p, st, blk0, nblk); break;
    case 4: launch_step<4>(e, p, st, blk0, nblk); break;
    case 5: launch_step<5>(e, p, st, blk0, nblk); break;
    case 6: launch_step<6>(e, p, st, blk0, nblk); break;
    case 7: launch_step<7>(e, p, st, blk0, nblk); break;
    case 8: launch_step<8>(e, p, st, blk0, nblk); break;
    default: return DRB_EINVAL;
  }
  HIPCHK(hipGetLastError());
  return DRB_OK;
}

// the host's bookkeeping after round p was enqueued
static void round_done(drb_engine *e, const RoundParams &p) {
  e->round++;
  e->ticks += p.tick;
  if (p.n_reads) {
    e->reads_round = e->round;
    e->reads_n = p.n_reads;
    e->reads_ks = p.key_space;
  }
}

extern "C" int drb_step_round_async(drb_engine *e, const drb_round_in *in) {
  if (!e || !in) return DRB_EINVAL;
  // transport threads stage the next round's inbox under this lock: a
  // round launches and advances e->round atomically with respect to them
  std::lock_guard<std::mutex> ingest_lock(e->ingest_mu);
  if (e->failed) return e->failed;
  // a durable LogDB: the last round's messages wait for its persistence
  if (e->cfg.durable_log && e->committed_round < e->round) return DRB_EINVAL;
  RoundParams p;
  if (int rc = round_params(e, in, 0, e->ticks, &p)) return rc;
  if (e->v.elections)  // this round's slow list
    HIPCHK(hipMemsetAsync(e->v.slow_n, 0, 8, e->stream));
  // plane summaries of this round only -- once a host reads them
  // (drb_plane_counts: the counted exchange); until then they only grow (a
  // max / or over rounds, an over-estimate a first counted read can take)
  if (e->v.remote_mask && e->xrows_used)
    HIPCHK(hipMemsetAsync(e->v.xrows, 0,
                          2ull * e->v.R * e->v.R * ((e->v.G + 255) / 256) * 4,
                          e->stream));
  if (e->v.xslow && e->xrows_used)
    HIPCHK(hipMemsetAsync(e->v.xslow, 0,
                          4ull * e->v.R * e->v.R * ((e->v.G + 255) / 256) * 4,
                          e->stream));
  if (int rc = launch_any(e, p)) return rc;
  if (p.encode_saves && e->v.save_tan) {
    int rc = launch_tan(e, (uint32_t)p.round);
    if (rc) return rc;
  }
  if (p.prop_slot != DRB_NONE)
    HIPCHK(hipEventRecord(e->ev_prop[p.prop_slot], e->stream));
  round_done(e, p);
  return DRB_OK;
}

// k rounds, chunk by chunk of the groups: each chunk of chunk_groups
// groups (a multiple of 256) runs all k rounds before the next chunk starts
// -- groups are independent (the reference steps each shard on its own,
// engine.go:1316-1328), so every group sees exactly the rounds of
// drb_step_round_async, and a chunk's rounds can find its mailbox, state
// and window rows still on-die.  Chunks alternate between two streams
// (joined back into the engine stream at the end).  Co-resident replicas,
// no elections, no listed rounds, no tan records, no durable LogDB.
extern "C" int drb_step_rounds(drb_engine *e, const drb_round_in *in,
                               uint32_t k, uint64_t chunk_groups) {
  if (!e || !in || !k) return DRB_EINVAL;
  std::lock_guard<std::mutex> ingest_lock(e->ingest_mu);
  if (e->failed) return e->failed;
  if (e->v.elections || e->v.remote_mask || e->v.save_tan ||
      e->cfg.durable_log)
    return DRB_EINVAL;
  const uint64_t gx = (e->v.G + 255) / 256;
  if (!chunk_groups || chunk_groups % 256) return DRB_EINVAL;
  const uint64_t cb = chunk_groups / 256;
  std::vector<RoundParams> ps(k);
  uint64_t ticks = e->ticks;
  for (uint32_t t = 0; t < k; ++t) {
    if (in[t].listed) return DRB_EINVAL;
    if (int rc = round_params(e, &in[t], t, ticks, &ps[t])) return rc;
    ticks += ps[t].tick;
  }
  // both streams start behind the engine stream's work
  HIPCHK(hipEventRecord(e->ev_fork, e->stream));
  HIPCHK(hipStreamWaitEvent(e->stream2, e->ev_fork, 0));
  int rc = DRB_OK;
  if (cb >= gx) {
    // one chunk of every group: the k rounds as plain rounds, each with its
    // two role launches side by side where they fit (launch_step), the
    // host's per-round cost one C call's (C2: a Python call per round left
    // the GPU idle a third of the time, profiles/r06_c2)
    for (uint32_t t = 0; t < k && !rc; ++t) rc = launch_any(e, ps[t]);
  } else {
    for (uint64_t c0 = 0, c = 0; c0 < gx && !rc; c0 += cb, ++c) {
      const uint32_t nb = (uint32_t)std::min<uint64_t>(cb, gx - c0);
      hipStream_t st = (c & 1) ? e->stream2 : e->stream;
      for (uint32_t t = 0; t < k && !rc; ++t)
        rc = launch_any(e, ps[t], st, (uint32_t)c0, nb);
    }
  }
  // the second stream joins the engine stream whatever happened
  const hipError_t j1 = hipEventRecord(e->ev_join, e->stream2);
  const hipError_t j2 = hipStreamWaitEvent(e->stream, e->ev_join, 0);
  if (rc || j1 != hipSuccess || j2 != hipSuccess) {
    // some chunks ran some of the rounds: the engine's round count no
    // longer matches the device, so it stops stepping
    e->failed = rc ? rc : DRB_EDEVICE;
    return e->failed;
  }
  for (uint32_t t = 0; t < k; ++t) {
    if (ps[t].prop_slot != DRB_NONE)
      HIPCHK(hipEventRecord(e->ev_prop[ps[t].prop_slot], e->stream));
    round_done(e, ps[t]);
  }
  return DRB_OK;
}

// sums the per-workgroup counter rows of the step kernels
__global__ void k_sum_counters(const unsigned long long *rows, uint64_t n,
                               unsigned long long *total) {
  __shared__ unsigned long long part[256];
  for (int c = 0; c < NUM_COUNTERS; ++c) {
    unsigned long long s = 0;
    for (uint64_t r = threadIdx.x; r < n; r += blockDim.x)
      s += rows[r * NUM_COUNTERS + c];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (threadIdx.x < (unsigned)o) part[threadIdx.x] += part[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) total[c] = part[0];
    __syncthreads();
  }
}

// per-phase cycle sums of the step kernels' lanes ([follower, leader] x
// {lanes, load + pre-pass, dispatch, tick + proposals, getUpdate, apply,
// store, reads}); zeros unless the engine was created with DRB_PHASE=1 and
// the step kernels built with DRB_PHASE_PROF=1 (a timing variant)
extern "C" int drb_debug_phase(drb_engine *e, uint64_t *out, int reset) {
  if (!e || !out) return DRB_EINVAL;
  memset(out, 0, 16 * sizeof(uint64_t));
  if (!e->v.phase) return DRB_OK;
  HIPCHK(hipMemcpyAsync(out, e->v.phase, 16 * sizeof(uint64_t),
                        hipMemcpyDeviceToHost, e->stream));
  if (reset)
    HIPCHK(hipMemsetAsync(e->v.phase, 0, 16 * sizeof(uint64_t), e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

extern "C" int drb_read_counters(drb_engine *e, drb_round_out *out,
                                 int reset) {
  if (!e || !out) return DRB_EINVAL;
  unsigned long long c[NUM_COUNTERS];
  k_sum_counters<<<1, 256, 0, e->stream>>>(e->v.counters, e->ctr_rows,
                                           e->ctr_total);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(c, e->ctr_total, sizeof(c), hipMemcpyDeviceToHost,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  out->round = e->round;
  out->committed_entries = c[C_COMMITTED];
  out->applied_entries = c[C_APPLIED];
  out->messages = c[C_MESSAGES];
  out->ready_to_reads = c[C_RTR];
  out->dropped_read_indexes = c[C_DROPPED_RI];
  out->fallbacks = c[C_FALLBACKS];
  out->errors = c[C_ERRORS];
  out->reads_served = c[C_READS];
  out->reads_deferred = c[C_READS_DEFERRED];
  out->saved_entries = c[C_SAVED_ENTRIES];
  out->saved_bytes = c[C_SAVED_BYTES];
  out->replicas_stepped = c[C_STEPPED];
  out->elections_stepped = c[C_ELECT];
  out->role_changes = c[C_ROLE];
  out->dropped_proposals = c[C_DPROP];
  out->lean_stepped = c[C_LEAN];
  out->log_records = 0;
  out->log_syncs = 0;
  out->log_new = 0;
  if (e->v.save_tan) {  // the tan records' bytes stand for the saves'
    unsigned long long t[4];
    int rc = read_tan_counters(e, t, reset);
    if (rc) return rc;
    out->saved_bytes = t[0];
    out->log_records = t[1];
    out->log_syncs = t[2];
    out->log_new = t[3];
  }
  if (reset) {
    HIPCHK(hipMemsetAsync(e->v.counters, 0,
                          e->ctr_rows * NUM_COUNTERS * sizeof(c[0]),
                          e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  return DRB_OK;
}

extern "C" int drb_commit_round(drb_engine *e, uint64_t round) {
  if (!e || round > e->round) return DRB_EINVAL;
  if (round > e->committed_round) e->committed_round = round;
  return DRB_OK;
}

extern "C" uint64_t drb_committed_round(const drb_engine *e) {
  return e ? e->committed_round : 0;
}

// the PIdx field i of replica (slot, g) from its packed record (device)
__device__ static uint64_t pk_field(const View &v, uint32_t slot, uint64_t g,
                                    int i) {
  const uint4 c0 = v.pk[pk_ix(v, 0, slot, g)];
  const uint4 c = v.pk[pk_ix(v, (4 + i / 2) / 4, slot, g)];
  const uint32_t w[4] = {c.x, c.y, c.z, c.w};
  const uint32_t code = (w[(4 + i / 2) % 4] >> (16 * (i & 1))) & 0xffffu;
  const uint64_t last = (uint64_t)c0.x | ((uint64_t)c0.y << 32);
  return code == PK_ESC16 ? v.u64[u64_ix(v, pi_field(i), slot, g)]
                          : pk_idx_value(code, last, i == PI_RING_GUARD);
}

// drb_apply_results: the entries (applied_index, sm_index] a replica applied
// in the round it last ran (updateAppliedIndex set applied_index to the
// state machine's index at that round's start); one output slot range per
// wave from a single atomic
__global__ __launch_bounds__(256) void k_apply_results(
    const View v, uint32_t slot, uint64_t first, uint64_t n,
    drb_apply_result *out, unsigned long long *count, uint64_t cap) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t g = first + i;
  uint64_t lo = 0, hi = 0;
  if (i < n) {
    const uint32_t fl = v.u32[u32_ix(v, W_FLAGS, slot, g)];
    const bool frozen = (fl & (DRB_F_FALLBACK | DRB_F_ERROR)) &&
                        !(fl & DRB_F_APPLY_STOPPED);
    if ((fl & DRB_F_HOSTED) && !frozen) {
      lo = pk_field(v, slot, g, PI_APPLIED_INDEX);
      hi = pk_field(v, slot, g, PI_SM_INDEX);
    }
  }
  const uint32_t cnt = hi > lo ? (uint32_t)(hi - lo) : 0u;
  const uint32_t lane = threadIdx.x & 63;
  uint32_t incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= (uint32_t)o) incl += t;
  }
  const uint32_t total = __shfl(incl, 63, 64);
  unsigned long long b = 0;
  if (lane == 0 && total) b = atomicAdd(count, (unsigned long long)total);
  b = __shfl(b, 0, 64);
  const uint64_t pos = b + incl - cnt;
  for (uint32_t k = 0; k < cnt; ++k) {
    if (pos + k >= cap) break;
    const uint64_t idx = lo + 1 + k;
    const uint4 m0 = v.ring[ring_ix(v, slot, idx, 0, g)];
    const uint4 m1 = v.ring[ring_ix(v, slot, idx, 1, g)];
    const uint4 m2 = v.ring[ring_ix(v, slot, idx, 2, g)];
    drb_apply_result r;
    r.group = g;
    r.index = idx;
    r.key = hi64(m0);
    r.client_id = lo64(m1);
    r.series_id = hi64(m1);
    const uint32_t type = m2.z, clen = m2.w;
    r.ignored = r.client_id == 0 ? 1u : 0u;  // an empty no-op entry
    // KVTest.Update's Result.Value: the payload length (kvtest.go:161)
    r.value = r.ignored ? 0
                        : (type == DRB_ENTRY_ENCODED && clen ? clen - 1 : clen);
    r.slot = slot;
    out[pos + k] = r;
  }
}

extern "C" int drb_apply_results(drb_engine *e, uint32_t slot,
                                 uint64_t first_group, uint64_t n_groups,
                                 drb_apply_result *out, size_t cap,
                                 size_t *n_out) {
  if (!e || slot >= e->v.R || (cap && !out)) return DRB_EINVAL;
  if (check_range(e, first_group, n_groups)) return DRB_ERANGE;
  if (!n_groups) {
    if (n_out) *n_out = 0;
    return DRB_OK;
  }
  void *s;
  const size_t bytes = 64 + cap * sizeof(drb_apply_result);
  if (scratch(e, bytes, &s)) return DRB_EDEVICE;
  unsigned long long *cnt = (unsigned long long *)s;
  drb_apply_result *dout = (drb_apply_result *)((char *)s + 64);
  HIPCHK(hipMemsetAsync(cnt, 0, 8, e->stream));
  k_apply_results<<<(unsigned)((n_groups + 255) / 256), 256, 0, e->stream>>>(
      e->v, slot, first_group, n_groups, dout, cnt, cap);
  HIPCHK(hipGetLastError());
  unsigned long long n = 0;
  HIPCHK(hipMemcpyAsync(&n, cnt, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  const size_t take = std::min<size_t>(n, cap);
  if (take) {
    HIPCHK(hipMemcpyAsync(out, dout, take * sizeof(drb_apply_result),
                          hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    std::sort(out, out + take,
              [](const drb_apply_result &a, const drb_apply_result &b) {
                return a.group != b.group ? a.group < b.group
                                          : a.index < b.index;
              });
  }
  if (n_out) *n_out = (size_t)n;
  return n > cap ? DRB_ERANGE : DRB_OK;
}

extern "C" int drb_take_flagged(drb_engine *e, drb_flagged *out, size_t cap,
                                size_t *n_out, uint64_t *lost, int reset) {
  if (!e || (cap && !out)) return DRB_EINVAL;
  const View &v = e->v;
  unsigned long long n = 0;
  HIPCHK(hipMemcpyAsync(&n, v.flog_n, sizeof(n), hipMemcpyDeviceToHost,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  const uint64_t have = std::min<uint64_t>(n, v.flog_cap);
  const uint64_t take = std::min<uint64_t>(have, cap);
  std::vector<uint4> recs(take);
  if (take) {
    HIPCHK(hipMemcpyAsync(recs.data(), v.flog, take * sizeof(uint4),
                          hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  for (uint64_t i = 0; i < take; ++i) {
    const uint4 q = recs[i];
    drb_flagged &o = out[i];
    memset(&o, 0, sizeof(o));
    o.group = (uint64_t)q.x | ((uint64_t)q.y << 32);
    o.slot = q.z & 0xffu;
    o.reason = (q.z >> 8) & 0xffu;
    o.flags = (q.z >> 16) & 0xffu;
    o.shard_id = v.first_shard_id + gid(v, o.slot, o.group);
    // the u32 round tag, widened against the engine's round counter
    o.round = (e->round & ~0xffffffffull) | q.w;
    if (o.round > e->round) o.round -= 1ull << 32;
  }
  if (n_out) *n_out = (size_t)take;
  if (lost) *lost = n > take ? n - take : 0;
  if (reset) {
    HIPCHK(hipMemsetAsync(v.flog_n, 0, sizeof(unsigned long long), e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  return DRB_OK;
}

extern "C" int drb_step_round(drb_engine *e, const drb_round_in *in,
                              drb_round_out *out) {
  if (!e || !in) return DRB_EINVAL;
  HIPCHK(hipMemsetAsync(e->v.counters, 0,
                        e->ctr_rows * NUM_COUNTERS * sizeof(unsigned long long),
                        e->stream));
  if (e->v.save_tan)
    HIPCHK(hipMemsetAsync(e->v.tan_ctr, 0,
                          e->tan_blocks * 4 * sizeof(unsigned long long),
                          e->stream));
  int rc = drb_step_round_async(e, in);
  if (rc) return rc;
  if (out) return drb_read_counters(e, out, 1);
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

// ---------------------------------------------------------------- outputs
// a remote plane's arrays as the step reads them (drb_step.hpp in_mbox &
// co.): the inbound copies, or a bound engine's sender outbox
struct InPlanes {
  uint4 *mbox, *meta, *embox;
  uint64_t *maxapp, *elo, *rterm;
};
static InPlanes in_planes(const drb_engine *e, uint32_t from, uint32_t to) {
  const View &v = e->v;
  if (v.peers && !e->peers_host.empty()) {
    const PeerPlanes &p = e->peers_host[plane_sender(v, from, to)];
    return {const_cast<uint4 *>(p.mbox), const_cast<uint4 *>(p.meta),
            const_cast<uint4 *>(p.embox), const_cast<uint64_t *>(p.maxapp),
            const_cast<uint64_t *>(p.elo), const_cast<uint64_t *>(p.rterm)};
  }
  return {v.mbox_in, v.meta_in, v.embox_in, v.maxapp_in, v.elo_in,
          v.rterm_in};
}

// entries [lo, hi] of a remote plane's entry rows (their first index elo),
// as drb_export_log writes them
static int export_entry_rows(drb_engine *e, uint32_t buf, uint64_t g,
                             uint32_t from, uint32_t to, uint64_t elo,
                             uint64_t lo, uint64_t hi, drb_entry *out,
                             uint8_t *pool, size_t pool_cap) {
  const View &v = e->v;
  if (hi < lo) return DRB_OK;
  if (lo < elo || hi - elo >= v.E) return DRB_ERANGE;
  std::vector<uint64_t> idx;
  for (uint64_t i = lo; i <= hi; ++i)
    for (uint32_t c = 0; c < ENT_META + v.C16; ++c)
      idx.push_back(embox_ix(v, buf, from, to, (uint32_t)(i - elo), c, g));
  std::vector<uint4> val;
  if (gather(e, in_planes(e, from, to).embox, idx, val)) return DRB_EDEVICE;
  size_t used = 0, k = 0;
  for (uint64_t i = lo; i <= hi; ++i, ++k) {
    const uint4 *c = &val[k * (ENT_META + v.C16)];
    drb_entry &o = out[k];
    o.term = lo64h(c[0]);
    o.key = hi64h(c[0]);
    o.client_id = lo64h(c[1]);
    o.series_id = hi64h(c[1]);
    o.responded_to = lo64h(c[2]);
    o.type = c[2].z;
    o.cmd_len = c[2].w;
    o.index = i;
    o.cmd_off = used;
    if (o.cmd_len > v.C16 * 16 || used + o.cmd_len > pool_cap)
      return DRB_ERANGE;
    memcpy(pool + used, &c[ENT_META], o.cmd_len);
    used += o.cmd_len;
  }
  return DRB_OK;
}

// the messages of one (sender, receiver) plane of mailbox buffer `buf`
// whose header carries round tag `tag`; remote: the inbound copies of a
// plane whose sender slot lives on another rank (C4 placement), entries in
// the plane's entry rows
static int export_pair(drb_engine *e, uint32_t buf, uint64_t g,
                       uint32_t from, uint32_t to, drb_message *out,
                       size_t cap, size_t *nm, drb_entry *ents, size_t ecap,
                       size_t *ne, uint8_t *pool, size_t pcap, size_t *np,
                       uint4 meta, uint64_t tag, bool remote = false) {
  const View &v = e->v;
  const bool cur = tag_is(meta.x, tag);
  const InPlanes ip = in_planes(e, from, to);
  uint4 *const mbox = remote ? ip.mbox : v.mbox;
  uint64_t *const rterm = remote ? ip.rterm : v.rterm;
  const uint32_t k = cur ? mi_count(meta.y) : 0;
  if (cur && (meta.x & MQ_QUIESCE)) {  // sendEnterQuiesceMessages
    if (*nm >= cap) return DRB_ERANGE;
    drb_message &m = out[(*nm)++];
    memset(&m, 0, sizeof(m));
    m.shard_id = v.first_shard_id + gid(v, remote ? to : from, g);
    m.from = from + 1;
    m.to = to + 1;
    m.type = DRB_MSG_QUIESCE;
    m.entries_off = *ne;
  }
  if (!k) return DRB_OK;
  // send order: the Replicates, then the others (drb_msg.hpp)
  std::vector<uint32_t> pos;
  for (uint32_t q = 0; q < mi_nrep(meta.y); ++q) pos.push_back(rec_pos(true, q, v.MB));
  for (uint32_t q = 0; q < mi_noth(meta.y); ++q)
    pos.push_back(rec_pos(false, q, v.MB));
  std::vector<uint64_t> idx;
  for (uint32_t q = 0; q < k; ++q)
    for (uint32_t c = 0; c < MSG_CHUNKS; ++c)
      idx.push_back(mbox_ix(v, buf, from, to, pos[q], c, g));
  std::vector<uint4> val;
  if (gather(e, mbox, idx, val)) return DRB_EDEVICE;
  uint64_t elo = 0;  // remote: the entry rows' first index
  if (remote && mi_nrep(meta.y)) {
    std::vector<uint64_t> li{mmeta_ix(v, buf, from, to, g)}, lv;
    if (gather(e, ip.elo, li, lv)) return DRB_EDEVICE;
    elo = lv[0];
  }
  uint64_t prev_lo = 0, prev_hi = 0;
  for (uint32_t q = 0; q < k; ++q) {
    if (*nm >= cap) return DRB_ERANGE;
    const uint4 *c = &val[q * MSG_CHUNKS];
    uint64_t rt = q_hi(meta);
    if ((c[0].x & MF_TERM_OTHER) && rterm) {  // its own term
      std::vector<uint64_t> ti{rterm_ix(v, buf, from, to, pos[q], g)}, tv;
      if (gather(e, rterm, ti, tv)) return DRB_EDEVICE;
      rt = tv[0];
    }
    Msg mm = msg_decode(c[0], c[1], rt, prev_lo, prev_hi);
    drb_message &m = out[(*nm)++];
    memset(&m, 0, sizeof(m));
    m.shard_id = v.first_shard_id + gid(v, remote ? to : from, g);
    m.from = from + 1;
    m.to = to + 1;
    m.type = mm.type;
    m.reject = mm.reject;
    m.term = mm.term;
    m.log_index = mm.log_index;
    m.log_term = mm.log_term;
    m.commit = mm.commit;
    m.hint = mm.hint;
    m.hint_high = mm.hint_high;
    uint64_t ne_ = mm.n;
    m.n_entries = ne_;
    m.entries_off = *ne;
    if (m.type == DRB_MSG_REPLICATE && ne_) {
      if (*ne + ne_ > ecap) return DRB_ERANGE;
      size_t used = 0;
      int rc = remote ? export_entry_rows(e, buf, g, from, to, elo,
                                          m.log_index + 1, m.log_index + ne_,
                                          ents + *ne, pool + *np, pcap - *np)
                      : drb_export_log(e, g, from, m.log_index + 1,
                                       m.log_index + ne_, ents + *ne,
                                       pool + *np, pcap - *np);
      if (rc) return rc;
      const bool wt = (v.wt_mask >> to) & 1u;
      for (uint64_t q2 = 0; q2 < ne_; ++q2) {
        drb_entry &en = ents[*ne + q2];
        used += en.cmd_len;  // the pool bytes drb_export_log wrote
        if (wt && en.type != DRB_ENTRY_CONFIG_CHANGE) {
          // a witness is sent metadata entries (makeMetadataEntries,
          // raft.go:771-785)
          const uint64_t t = en.term, x = en.index;
          memset(&en, 0, sizeof(en));
          en.type = DRB_ENTRY_METADATA;
          en.term = t;
          en.index = x;
        }
        en.cmd_off += *np;
      }
      *ne += ne_;
      *np += used;
    } else if (m.type == DRB_MSG_PROPOSE && ne_) {
      // the entries as proposed (no Term, no Index), from the sender's
      // forward rows of this round
      if (!v.fwd_props || ne_ > v.max_props) return DRB_EINVAL;
      if (*ne + ne_ > ecap) return DRB_ERANGE;
      const uint32_t chunks = PROP_META + v.C16, fw = fwd_ps(v, buf, from);
      std::vector<uint64_t> pi;
      for (uint64_t j = 0; j < ne_; ++j)
        for (uint32_t c = 0; c < chunks; ++c)
          pi.push_back(prop_ix(v, fw, (uint32_t)j, c, g));
      std::vector<uint4> pv;
      if (gather(e, v.props, pi, pv)) return DRB_EDEVICE;
      for (uint64_t j = 0; j < ne_; ++j) {
        const uint4 *q4 = &pv[j * chunks];
        drb_entry &en = ents[*ne + j];
        memset(&en, 0, sizeof(en));
        en.key = lo64h(q4[0]);
        en.client_id = hi64h(q4[0]);
        en.series_id = lo64h(q4[1]);
        en.responded_to = hi64h(q4[1]);
        en.type = q4[2].x;
        en.cmd_len = q4[2].y;
        if (en.cmd_len > v.C16 * 16) return DRB_EINVAL;
        if (*np + en.cmd_len > pcap) return DRB_ERANGE;
        en.cmd_off = *np;
        memcpy(pool + *np, &q4[PROP_META], en.cmd_len);
        *np += en.cmd_len;
      }
      *ne += ne_;
    }
  }
  return DRB_OK;
}

extern "C" int drb_export_outbox(drb_engine *e, uint64_t group,
                                 uint32_t from_slot, drb_message *out,
                                 size_t cap, drb_entry *ents, size_t ent_cap,
                                 uint8_t *pool, size_t pool_cap,
                                 size_t *n_msgs) {
  if (!e || group >= e->cfg.num_groups || from_slot >= e->cfg.num_replicas)
    return DRB_ERANGE;
  const View &v = e->v;
  const uint32_t buf = (uint32_t)(e->round & 1);
  std::vector<uint64_t> mi;
  for (uint32_t to = 0; to < v.R; ++to)
    mi.push_back(mmeta_ix(v, buf, from_slot, to, group));
  std::vector<uint4> meta;
  if (gather(e, v.mbox_meta, mi, meta)) return DRB_EDEVICE;
  size_t nm = 0, ne = 0, np = 0;
  if (e->round > 0) {
    // send order across destinations is not recorded per message; the
    // per-destination order is (messages are compared per destination)
    for (uint32_t to = 0; to < v.R; ++to) {
      if (to == from_slot) continue;
      int rc = export_pair(e, buf, group, from_slot, to, out, cap, &nm, ents,
                           ent_cap, &ne, pool, pool_cap, &np, meta[to],
                           e->round);
      if (rc) return rc;
    }
  }
  if (n_msgs) *n_msgs = nm;
  return DRB_OK;
}

extern "C" int drb_export_inbox(drb_engine *e, uint64_t group, uint32_t slot,
                                int last_round, drb_message *out, size_t cap,
                                drb_entry *ents, size_t ent_cap, uint8_t *pool,
                                size_t pool_cap, size_t *n_msgs) {
  if (!e || group >= e->cfg.num_groups || slot >= e->cfg.num_replicas)
    return DRB_ERANGE;
  const View &v = e->v;
  size_t nm = 0, ne = 0, np = 0;
  // the inbox round t + 1 takes is buffer t & 1 with tag t (what round t
  // sent and what was ingested since); the one round t took, t - 1
  const uint64_t tag = last_round ? e->round - 1 : e->round;
  if (!(last_round && e->round == 0)) {
    const uint32_t buf = (uint32_t)(tag & 1);
    for (uint32_t from = 0; from < v.R; ++from) {
      if (from == slot) continue;
      const bool rm = pair_remote(v, from, slot);
      std::vector<uint64_t> mi{mmeta_ix(v, buf, from, slot, group)};
      std::vector<uint4> meta;
      if (gather(e, rm ? in_planes(e, from, slot).meta : v.mbox_meta, mi, meta))
        return DRB_EDEVICE;
      int rc = export_pair(e, buf, group, from, slot, out, cap, &nm, ents,
                           ent_cap, &ne, pool, pool_cap, &np, meta[0], tag, rm);
      if (rc) return rc;
    }
  }
  if (n_msgs) *n_msgs = nm;
  return DRB_OK;
}

extern "C" int drb_export_ready_to_reads(drb_engine *e, uint64_t group,
                                         uint32_t slot, drb_ready_to_read *out,
                                         size_t cap, size_t *n_out) {
  if (!e || group >= e->cfg.num_groups || slot >= e->cfg.num_replicas)
    return DRB_ERANGE;
  const View &v = e->v;
  std::vector<uint64_t> ci = {ix(v, slot, group)};
  std::vector<uint32_t> cnt;
  if (gather(e, v.rtr_count, ci, cnt)) return DRB_EDEVICE;
  uint32_t n = std::min<uint32_t>(cnt[0], RTR_CAP);
  std::vector<uint64_t> idx;
  for (uint32_t k = 0; k < n; ++k)
    for (uint32_t c = 0; c < 2; ++c) idx.push_back(rtr_ix(v, slot, k, c, group));
  std::vector<uint4> val;
  if (gather(e, v.rtr, idx, val)) return DRB_EDEVICE;
  for (uint32_t k = 0; k < n && k < cap; ++k) {
    out[k].shard_id = v.first_shard_id + gid(v, slot, group);
    out[k].replica_id = slot + 1;
    out[k].index = lo64h(val[2 * k]);
    out[k].ctx_low = hi64h(val[2 * k]);
    out[k].ctx_high = lo64h(val[2 * k + 1]);
  }
  if (n_out) *n_out = n;
  return DRB_OK;
}

// ---------------------------------------------------------------- exchange
// the plane words (include/drb_engine.h DRB_PLANE_*) reduced over the
// per-block rows of both roles: max counts, OR of the flags
__global__ void k_plane_sum(const uint32_t *rows, const uint32_t *slow,
                            uint32_t RR, uint32_t blocks, uint32_t *out) {
  __shared__ uint32_t red[4][256];
  const uint32_t pair = blockIdx.x;
  uint32_t kr = 0, ko = 0, en = 0, f = 0;
  for (uint32_t role = 0; role < 2; ++role)
    for (uint32_t b = threadIdx.x; b < blocks; b += blockDim.x) {
      const uint32_t w = rows[((uint64_t)role * RR + pair) * blocks + b];
      kr = max(kr, DRB_PLANE_KREP(w));
      ko = max(ko, DRB_PLANE_KOTH(w));
      en = max(en, DRB_PLANE_E(w));
      f |= w & (DRB_PLANE_C1 | DRB_PLANE_HDR);
    }
  if (slow)  // the raft launch's lanes (elections)
    for (uint32_t b = threadIdx.x; b < blocks; b += blockDim.x) {
      const uint32_t *q = slow + ((uint64_t)pair * blocks + b) * 4;
      kr = max(kr, q[0]);
      ko = max(ko, q[1]);
      en = max(en, q[2]);
      f |= q[3] << 18;
    }
  red[0][threadIdx.x] = kr;
  red[1][threadIdx.x] = ko;
  red[2][threadIdx.x] = en;
  red[3][threadIdx.x] = f;
  __syncthreads();
  for (uint32_t o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      for (int q = 0; q < 3; ++q)
        red[q][threadIdx.x] = max(red[q][threadIdx.x], red[q][threadIdx.x + o]);
      red[3][threadIdx.x] |= red[3][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0)
    out[pair] = red[0][0] | (red[1][0] << 5) | (red[2][0] << 10) | red[3][0];
}

extern "C" int drb_plane_counts(drb_engine *e, uint32_t *words) {
  if (!e || !words) return DRB_EINVAL;
  const View &v = e->v;
  const uint32_t RR = v.R * v.R;
  if (!v.remote_mask || e->round == 0) {
    memset(words, 0, RR * sizeof(uint32_t));
    return DRB_OK;
  }
  e->xrows_used = true;  // the rounds clear the summaries from now on
  const uint32_t blocks = (uint32_t)((v.G + 255) / 256);
  k_plane_sum<<<RR, 256, 0, e->stream>>>(v.xrows, v.xslow, RR, blocks,
                                         e->xcount);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(words, e->xcount, RR * sizeof(uint32_t),
                        hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  for (uint32_t q = 0; q < RR; ++q)
    if (!((v.remote_mask >> q) & 1ull)) words[q] = 0;
  return DRB_OK;
}

extern "C" int drb_place_peer(uint32_t world, uint32_t rank, uint32_t from,
                              uint32_t to, int dir) {
  if (world <= 1 || rank >= world) return -1;
  const uint32_t N = world, d = (to % N + N - from % N) % N;
  if (d == 0) return -1;  // both replicas of the group on this rank
  return (int)(dir == 0 ? (rank + d) % N : (rank + N - d) % N);
}

extern "C" int drb_plane_peer(const drb_engine *e, uint32_t from, uint32_t to,
                              int dir) {
  if (!e || from >= e->v.R || to >= e->v.R || from == to) return -1;
  return drb_place_peer(e->v.place_world, e->v.place_rank, from, to, dir);
}

extern "C" int drb_plane_regions(drb_engine *e, uint32_t from, uint32_t to,
                                 uint32_t word, int dir, drb_region *out) {
  if (!e || !out || from >= e->v.R || to >= e->v.R) return DRB_EINVAL;
  if (dir && !e->bound.empty()) return DRB_EINVAL;  // (drb_ingest_ex)
  const View &v = e->v;
  if (!pair_remote(v, from, to) || e->round == 0) return 0;
  const uint32_t buf = (uint32_t)(e->round & 1);  // the last round's outbox
  const uint32_t Kr = DRB_PLANE_KREP(word), Ko = DRB_PLANE_KOTH(word),
                 En = DRB_PLANE_E(word);
  if (Kr + Ko > v.MB || En > v.E) return DRB_ERANGE;
  uint4 *mb = dir ? v.mbox_in : v.mbox;
  uint4 *meta = dir ? v.meta_in : v.mbox_meta;
  uint64_t *mx = dir ? v.maxapp_in : v.mbox_maxapp;
  uint64_t *elo = dir ? v.elo_in : v.elo;
  uint4 *eb = dir ? v.embox_in : v.embox;
  const uint64_t G = v.G;
  int n = 0;
  // Replicate records at positions [0, Kr), the others at [MB - Ko, MB)
  // (drb_msg.hpp), per chunk
  for (uint32_t c = 0; c < ((word & DRB_PLANE_C1) ? 2u : 1u); ++c) {
    if (Kr) out[n++] = {mb + mbox_ix(v, buf, from, to, 0, c, 0), Kr * G * 16};
    if (Ko)
      out[n++] = {mb + mbox_ix(v, buf, from, to, v.MB - Ko, c, 0),
                  Ko * G * 16};
  }
  if ((word & DRB_PLANE_TOTHER) && v.rterm_in) {
    // records with a term of their own (the raft launch): their rterm rows
    uint64_t *rt = dir ? v.rterm_in : v.rterm;
    if (Kr) out[n++] = {rt + rterm_ix(v, buf, from, to, 0, 0), Kr * G * 8};
    if (Ko)
      out[n++] = {rt + rterm_ix(v, buf, from, to, v.MB - Ko, 0), Ko * G * 8};
  }
  if (Kr || Ko || (word & DRB_PLANE_HDR))
    out[n++] = {meta + mmeta_ix(v, buf, from, to, 0), G * 16};
  if (Kr) out[n++] = {mx + mmeta_ix(v, buf, from, to, 0), G * 8};
  if (En) {
    out[n++] = {elo + mmeta_ix(v, buf, from, to, 0), G * 8};
    out[n++] = {eb + embox_ix(v, buf, from, to, 0, 0, 0),
                (uint64_t)En * (ENT_META + v.C16) * G * 16};
  }
  return n;
}

// every engine of one process at the same round, in placement order
static int exchange_check(drb_engine *const *engines, uint32_t n) {
  if (!engines || n == 0 || !engines[0]) return DRB_EINVAL;
  const uint32_t R = engines[0]->v.R;
  for (uint32_t r = 0; r < n; ++r) {
    const drb_engine *e = engines[r];
    // (the planes' shapes must match: the pull indexes a sender's planes
    // with the receiver's layout)
    const View &v0 = engines[0]->v;
    if (!e || e->v.R != R || e->v.place_world != n || e->v.place_rank != r ||
        e->round != engines[0]->round || e->v.G != v0.G ||
        e->v.MB != v0.MB || e->v.E != v0.E || e->v.C16 != v0.C16 ||
        (e->v.rterm_in == nullptr) != (v0.rterm_in == nullptr))
      return DRB_EINVAL;
  }
  return DRB_OK;
}

// the ingest locks of every engine, in rank order (drb_exchange_*: no
// transport thread writes an inbound plane while the exchange runs)
struct ExchangeLocks {
  std::vector<std::unique_lock<std::mutex>> l;
  ExchangeLocks(drb_engine *const *engines, uint32_t n) {
    for (uint32_t r = 0; r < n; ++r) l.emplace_back(engines[r]->ingest_mu);
  }
};

static int exchange_copy(drb_engine *const *engines, uint32_t n,
                         const std::vector<std::vector<uint32_t>> &words,
                         std::vector<uint32_t> *sent_to) {
  const uint32_t R = engines[0]->v.R;
  for (uint32_t r = 0; r < n; ++r)
    for (uint32_t a = 0; a < R; ++a)
      for (uint32_t b = 0; b < R; ++b) {
        const uint32_t w = words[r][a * R + b];
        const int peer = drb_plane_peer(engines[r], a, b, 0);
        if (peer < 0 || !w) continue;
        drb_engine *dst = engines[peer];
        if (sent_to) {  // the receiver waits for this sender's round once
          if (!(((*sent_to)[r] >> peer) & 1u))
            HIPCHK(hipStreamWaitEvent(dst->stream, engines[r]->ev_xsend, 0));
          (*sent_to)[r] |= 1u << peer;
        }
        drb_region src[DRB_PLANE_REGIONS], dreg[DRB_PLANE_REGIONS];
        const int ns = drb_plane_regions(engines[r], a, b, w, 0, src);
        const int nd = drb_plane_regions(dst, a, b, w, 1, dreg);
        if (ns < 0 || ns != nd) return DRB_EINVAL;
        for (int q = 0; q < ns; ++q) {
          HIPCHK(hipMemcpyAsync(dreg[q].ptr, src[q].ptr, src[q].bytes,
                                hipMemcpyDefault, dst->stream));
          dst->xcopy_bytes += src[q].bytes;
        }
      }
  return DRB_OK;
}

// the summary word of a plane at full capacity (drb_plane_regions): every
// record position, both chunks, the header; for a sender slot that may
// hold leaders the max-append word and every entry row too; with
// elections the rterm rows (dragonboat_amd/exchange.py full_word)
static uint32_t full_word(const View &v, bool leader_sender) {
  const uint32_t f = DRB_PLANE_C1 | DRB_PLANE_HDR;
  if (leader_sender || v.elections)
    return (v.MB & 0x1fu) | ((v.E & 0xffu) << 10) | f |
           (v.elections ? DRB_PLANE_TOTHER : 0u);
  return ((v.MB & 0x1fu) << 5) | f;
}

// ---- the one-device pull: every engine of the process on one GPU
// A receiver's kernel reads each sender's outbox plane header and copies,
// lane by lane, what the header counts: the header, the Replicate records
// [0, nrep) and the others [MB - noth, MB) (both chunks; with elections
// their rterm rows), the max-append word, and the entry rows [elo, maxapp]
// -- the bytes a counted exchange moves, with no host round trip.  A lane
// whose sender header is not of this round keeps its inbound plane as it is
// (its receiver reads only headers of the round, tag_is).
constexpr uint32_t PULL_MAX = 16;
constexpr uint32_t PULL_BATCH = 8;  // record / row chunks in flight per lane
struct PullSrc {
  const uint4 *mbox, *meta, *embox;
  const uint64_t *maxapp, *elo, *rterm;
};
struct PullArgs {
  PullSrc src[PULL_MAX];
  uint32_t N, d, buf;
  uint32_t tag;
};

__global__ void __launch_bounds__(256)
    k_plane_pull(View v, PullArgs a, unsigned long long *bytes) {
  const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint32_t from = blockIdx.y / v.R, to = blockIdx.y % v.R;
  uint64_t moved = 0;
  if (g < v.G && from != to && pair_remote(v, from, to)) {
    // the sender of plane (from, to) into rank d (drb_place_peer, dir 1)
    const uint32_t N = a.N, dd = (to % N + N - from % N) % N;
    const PullSrc &s = a.src[(a.d + N - dd) % N];
    const uint64_t hi = mmeta_ix(v, a.buf, from, to, g);
    const uint4 h = s.meta[hi];
    if (tag_is(h.x, a.tag)) {
      v.meta_in[hi] = h;
      moved += 16;
      const uint32_t nrep = mi_nrep(h.y), noth = mi_noth(h.y);
      const uint32_t n = nrep + noth;
      uint64_t mx = 0, lo = ~0ull;
      if (nrep) {
        mx = s.maxapp[hi];
        lo = s.elo[hi];
      }
      // the records, PULL_BATCH at a time: every load of a batch issued
      // before its stores (one memory round trip per batch)
      for (uint32_t j0 = 0; j0 < n; j0 += PULL_BATCH) {
        uint4 r0[PULL_BATCH], r1[PULL_BATCH];
#pragma unroll
        for (uint32_t t = 0; t < PULL_BATCH; ++t) {
          const uint32_t jj = j0 + t;
          const uint32_t k = rec_pos(jj < nrep, jj < nrep ? jj : jj - nrep, v.MB);
          if (jj < n) {
            r0[t] = s.mbox[mbox_ix(v, a.buf, from, to, k, 0, g)];
            r1[t] = s.mbox[mbox_ix(v, a.buf, from, to, k, 1, g)];
          }
        }
#pragma unroll
        for (uint32_t t = 0; t < PULL_BATCH; ++t) {
          const uint32_t jj = j0 + t;
          const uint32_t k = rec_pos(jj < nrep, jj < nrep ? jj : jj - nrep, v.MB);
          if (jj < n) {
            v.mbox_in[mbox_ix(v, a.buf, from, to, k, 0, g)] = r0[t];
            v.mbox_in[mbox_ix(v, a.buf, from, to, k, 1, g)] = r1[t];
            if (v.rterm_in) {
              const uint64_t ix = rterm_ix(v, a.buf, from, to, k, g);
              v.rterm_in[ix] = s.rterm[ix];
            }
          }
        }
      }
      moved += (uint64_t)n * (MSG_CHUNKS * 16 + (v.rterm_in ? 8 : 0));
      if (nrep) {
        v.maxapp_in[hi] = mx;
        v.elo_in[hi] = lo;
        moved += 16;
        if (v.E && lo != ~0ull && mx >= lo) {
          const uint64_t rows = mx - lo + 1 < v.E ? mx - lo + 1 : v.E;
          const uint32_t chunks = ENT_META + v.C16;
          const uint32_t total = (uint32_t)rows * chunks;
          for (uint32_t c0 = 0; c0 < total; c0 += PULL_BATCH) {
            uint4 q[PULL_BATCH];
#pragma unroll
            for (uint32_t t = 0; t < PULL_BATCH; ++t)
              if (c0 + t < total)
                q[t] = s.embox[embox_ix(v, a.buf, from, to, (c0 + t) / chunks,
                                        (c0 + t) % chunks, g)];
#pragma unroll
            for (uint32_t t = 0; t < PULL_BATCH; ++t)
              if (c0 + t < total)
                v.embox_in[embox_ix(v, a.buf, from, to, (c0 + t) / chunks,
                                    (c0 + t) % chunks, g)] = q[t];
          }
          moved += (uint64_t)total * 16;
        }
      }
    }
  }
  // the bytes moved, a wave sum and one atomic per wave
  for (int o = 32; o > 0; o >>= 1) moved += __shfl_down(moved, o, 64);
  if ((threadIdx.x & 63) == 0 && moved)
    atomicAdd(bytes, (unsigned long long)moved);
}

static bool pull_ok(drb_engine *const *engines, uint32_t n) {
  if (n > PULL_MAX) return false;
  for (uint32_t r = 1; r < n; ++r)
    if (engines[r]->cfg.device != engines[0]->cfg.device) return false;
  return true;
}

static int exchange_pull(drb_engine *const *engines, uint32_t n) {
  const View &v0 = engines[0]->v;
  PullArgs a;
  memset(&a, 0, sizeof(a));
  a.N = n;
  a.buf = (uint32_t)(engines[0]->round & 1);  // the last round's outbox
  a.tag = (uint32_t)engines[0]->round;
  for (uint32_t r = 0; r < n; ++r) {
    const View &v = engines[r]->v;
    a.src[r] = {v.mbox, v.mbox_meta, v.embox, v.mbox_maxapp, v.elo, v.rterm};
    HIPCHK(hipEventRecord(engines[r]->ev_xsend, engines[r]->stream));
  }
  const dim3 grid((unsigned)((v0.G + 255) / 256), v0.R * v0.R);
  for (uint32_t d = 0; d < n; ++d) {
    drb_engine *e = engines[d];
    if (!e->xpull_bytes && dalloc(e, &e->xpull_bytes, 1)) return DRB_ENOMEM;
    for (uint32_t r = 0; r < n; ++r)
      if (r != d) HIPCHK(hipStreamWaitEvent(e->stream, engines[r]->ev_xsend, 0));
    a.d = d;
    k_plane_pull<<<grid, 256, 0, e->stream>>>(e->v, a, e->xpull_bytes);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e->ev_xrecv, e->stream));
  }
  // a sender's next round overwrites the other outbox buffer, the one after
  // it this one: its stream waits for the pulls that read it
  for (uint32_t r = 0; r < n; ++r)
    for (uint32_t d = 0; d < n; ++d)
      if (r != d)
        HIPCHK(hipStreamWaitEvent(engines[r]->stream, engines[d]->ev_xrecv, 0));
  return DRB_OK;
}

// ---- the zero-copy exchange of one process's engines on one GPU
// Bound engines read each remote plane straight from the sender rank's
// outbox (View.peers, drb_step.hpp in_mbox & co.); drb_exchange_local then
// only orders the rounds: every engine's next round waits for every
// engine's last one, so a round reads its senders' finished outboxes and a
// sender overwrites an outbox buffer (two rounds later) only after its
// receivers read it.
static bool any_bound(drb_engine *const *engines, uint32_t n) {
  for (uint32_t r = 0; r < n; ++r)
    if (!engines[r]->bound.empty()) return true;
  return false;
}
static bool is_bound(drb_engine *const *engines, uint32_t n) {
  for (uint32_t r = 0; r < n; ++r)
    if (engines[r]->bound.size() != n || engines[r]->bound[r] != engines[r] ||
        engines[r]->bound != engines[0]->bound)
      return false;
  return n > 0;
}
static void exchange_barrier(drb_engine *const *engines, uint32_t n) {
  for (uint32_t r = 0; r < n; ++r)
    (void)hipEventRecord(engines[r]->ev_xsend, engines[r]->stream);
  for (uint32_t d = 0; d < n; ++d)
    for (uint32_t r = 0; r < n; ++r)
      if (r != d)
        (void)hipStreamWaitEvent(engines[d]->stream, engines[r]->ev_xsend, 0);
}

extern "C" int drb_exchange_local_bind(drb_engine *const *engines,
                                       uint32_t n) {
  if (int rc = exchange_check(engines, n)) return rc;
  if (n < 2 || !pull_ok(engines, n) || any_bound(engines, n))
    return DRB_EINVAL;
  for (uint32_t r = 0; r < n; ++r)
    if (engines[r]->v.place_world != n || engines[r]->v.place_rank != r)
      return DRB_EINVAL;  // (engines[r] is rank r of the placement)
  std::vector<PeerPlanes> src(n);
  for (uint32_t r = 0; r < n; ++r) {
    const View &v = engines[r]->v;
    src[r] = {v.mbox, v.mbox_meta, v.embox, v.mbox_maxapp, v.elo, v.rterm};
  }
  std::vector<drb_engine *> group(engines, engines + n);
  for (uint32_t r = 0; r < n; ++r) {
    drb_engine *e = engines[r];
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipStreamSynchronize(e->stream));
    PeerPlanes *d = nullptr;
    if (dalloc(e, &d, n)) return DRB_ENOMEM;
    HIPCHK(hipMemcpyAsync(d, src.data(), n * sizeof(PeerPlanes),
                          hipMemcpyHostToDevice, e->stream));
    e->v.peers = d;
    HIPCHK(hipMemcpyAsync(e->dview, &e->v, sizeof(View),
                          hipMemcpyHostToDevice, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  for (uint32_t r = 0; r < n; ++r) {
    engines[r]->bound = group;
    engines[r]->peers_host = src;
  }
  return DRB_OK;
}

extern "C" int drb_exchange_bytes(drb_engine *e, uint64_t *bytes, int reset) {
  if (!e || !bytes) return DRB_EINVAL;
  unsigned long long b = 0;
  if (e->xpull_bytes) {
    HIPCHK(hipMemcpyAsync(&b, e->xpull_bytes, 8, hipMemcpyDeviceToHost,
                          e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (reset) HIPCHK(hipMemsetAsync(e->xpull_bytes, 0, 8, e->stream));
  }
  *bytes = e->xcopy_bytes + b;
  if (reset) e->xcopy_bytes = 0;
  return DRB_OK;
}

extern "C" int drb_exchange_local(drb_engine *const *engines, uint32_t n) {
  if (int rc = exchange_check(engines, n)) return rc;
  const View &v = engines[0]->v;
  const uint32_t R = v.R;
  ExchangeLocks locks(engines, n);
  if (is_bound(engines, n)) {  // zero-copy: the rounds' order alone
    if (engines[0]->round == 0) return DRB_OK;
    exchange_barrier(engines, n);
    for (uint32_t r = 0; r < n; ++r)
      engines[r]->exchanged_round = engines[r]->round;
    return DRB_OK;
  }
  if (any_bound(engines, n)) return DRB_EINVAL;  // (not the bound group)
  if (pull_ok(engines, n)) {  // one GPU: counted, on the device
    if (engines[0]->round == 0) return DRB_OK;
    if (int rc = exchange_pull(engines, n)) return rc;
    for (uint32_t r = 0; r < n; ++r)
      engines[r]->exchanged_round = engines[r]->round;
    return DRB_OK;
  }
  // plane (a, b) can carry fast-path messages when a or b holds a leader on
  // some engine (followers send only to leaders); every plane when roles
  // change on the device
  uint32_t lead = 0;
  for (uint32_t r = 0; r < n; ++r) lead |= engines[r]->role_slots[0];
  std::vector<uint32_t> row(R * R, 0);
  for (uint32_t a = 0; a < R; ++a)
    for (uint32_t b = 0; b < R; ++b)
      if (a != b && (((lead >> a) | (lead >> b)) & 1u || v.elections))
        row[a * R + b] = full_word(v, (lead >> a) & 1u);
  std::vector<std::vector<uint32_t>> words(n, row);
  if (engines[0]->round == 0) return DRB_OK;
  for (uint32_t r = 0; r < n; ++r)
    HIPCHK(hipEventRecord(engines[r]->ev_xsend, engines[r]->stream));
  std::vector<uint32_t> sent_to(n, 0);
  if (int rc = exchange_copy(engines, n, words, &sent_to)) return rc;
  for (uint32_t d = 0; d < n; ++d)
    HIPCHK(hipEventRecord(engines[d]->ev_xrecv, engines[d]->stream));
  // a sender's next round overwrites the other outbox buffer, the one
  // after it this one: its stream waits for the copies that read it
  for (uint32_t r = 0; r < n; ++r)
    for (uint32_t d = 0; d < n; ++d)
      if ((sent_to[r] >> d) & 1u)
        HIPCHK(hipStreamWaitEvent(engines[r]->stream, engines[d]->ev_xrecv,
                                  0));
  for (uint32_t r = 0; r < n; ++r)
    engines[r]->exchanged_round = engines[r]->round;
  return DRB_OK;
}

extern "C" int drb_exchange_local_counted(drb_engine *const *engines,
                                          uint32_t n) {
  if (int rc = exchange_check(engines, n)) return rc;
  if (any_bound(engines, n)) return DRB_EINVAL;
  const uint32_t R = engines[0]->v.R;
  ExchangeLocks locks(engines, n);
  std::vector<std::vector<uint32_t>> words(n, std::vector<uint32_t>(R * R));
  for (uint32_t r = 0; r < n; ++r)
    if (int rc = drb_plane_counts(engines[r], words[r].data())) return rc;
  if (int rc = exchange_copy(engines, n, words, nullptr)) return rc;
  for (uint32_t r = 0; r < n; ++r) HIPCHK(hipStreamSynchronize(engines[r]->stream));
  for (uint32_t r = 0; r < n; ++r)
    engines[r]->exchanged_round = engines[r]->round;
  return DRB_OK;
}

extern "C" int drb_exchange_mark(drb_engine *e) {
  if (!e) return DRB_EINVAL;
  std::lock_guard<std::mutex> lock(e->ingest_mu);
  e->exchanged_round = e->round;
  return DRB_OK;
}

// ---------------------------------------------------------------- saves
extern "C" int drb_export_saved(drb_engine *e, uint64_t group, uint32_t slot,
                                uint8_t *buf, size_t cap, uint32_t *len,
                                uint32_t *crc) {
  if (!e || !len || (cap && !buf)) return DRB_EINVAL;
  const View &v = e->v;
  if (!v.save_cap16) return DRB_EINVAL;
  if (group >= v.G || slot >= v.R) return DRB_ERANGE;
  uint32_t l = 0, c = 0;
  HIPCHK(hipMemcpyAsync(&l, v.save_len + ix(v, slot, group), 4,
                        hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&c, v.save_crc + ix(v, slot, group), 4,
                        hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *len = l;
  if (crc) *crc = l ? c : 0;
  if (l > cap) return DRB_ERANGE;
  if (l) {
    HIPCHK(hipMemcpyAsync(buf, v.save_buf + ix(v, slot, group) * v.save_cap16,
                          l, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  return DRB_OK;
}

extern "C" int drb_export_save_records(drb_engine *e, uint64_t group,
                                       uint32_t slot, drb_save_record *out,
                                       size_t cap, size_t *n) {
  if (!e || !n || (cap && !out)) return DRB_EINVAL;
  const View &v = e->v;
  if (!v.save_batched) return DRB_EINVAL;
  if (group >= v.G || slot >= v.R) return DRB_ERANGE;
  uint32_t l = 0, k = 0;
  uint4 rec[DRB_SAVE_RECS];
  HIPCHK(hipMemcpyAsync(&l, v.save_len + ix(v, slot, group), 4,
                        hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(&k, v.save_nrec + ix(v, slot, group), 4,
                        hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemcpyAsync(rec, v.save_rec + ix(v, slot, group) * DRB_SAVE_RECS,
                        sizeof(rec), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *n = l ? k : 0;  // save_len 0: nothing saved this round
  if (*n > cap) return DRB_ERANGE;
  for (size_t i = 0; i < *n; ++i)
    out[i] = {rec[i].x, rec[i].y * 16, rec[i].z, rec[i].w, 0};
  return DRB_OK;
}

extern "C" int drb_saved_buffers(drb_engine *e, void **bytes, uint32_t **lens,
                                 uint32_t **crcs) {
  if (!e || !bytes || !lens || !crcs) return DRB_EINVAL;
  if (!e->v.save_cap16) return DRB_EINVAL;
  *bytes = e->v.save_buf;
  *lens = e->v.save_len;
  *crcs = e->v.save_crc;
  return DRB_OK;
}

static int read_kv_table(drb_engine *e, uint64_t group, uint32_t slot,
                         std::vector<uint4> &tbl) {
  const View &v = e->v;
  tbl.resize((uint64_t)v.KS * v.KVW);
  HIPCHK(hipMemcpyAsync(tbl.data(), v.kv + kv_ix(v, slot, group, 0),
                        tbl.size() * sizeof(uint4), hipMemcpyDeviceToHost,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

// the replica's overflow chain (drb_config.kv_overflow_buckets), its
// buckets' slots in chain order (4 x KVW chunks a bucket)
static int read_ovf_chain(drb_engine *e, uint64_t group, uint32_t slot,
                          std::vector<uint4> &out) {
  const View &v = e->v;
  out.clear();
  if (!v.kv_ovf_head) return DRB_OK;
  uint32_t b = 0;
  HIPCHK(hipMemcpyAsync(&b, v.kv_ovf_head + ix(v, slot, group), 4,
                        hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  std::vector<uint4> bk(4 * v.KVW);
  for (uint64_t guard = 0; b && guard <= v.kv_ovf_cap; ++guard) {
    if (b - 1 >= v.kv_ovf_cap) return DRB_EDEVICE;
    uint32_t next = 0;
    HIPCHK(hipMemcpyAsync(bk.data(), v.kv_ovf + (uint64_t)(b - 1) * 4 * v.KVW,
                          bk.size() * sizeof(uint4), hipMemcpyDeviceToHost,
                          e->stream));
    HIPCHK(hipMemcpyAsync(&next, v.kv_ovf_next + (b - 1), 4,
                          hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    out.insert(out.end(), bk.begin(), bk.end());
    b = next;
  }
  return DRB_OK;
}

static int slot_value(drb_engine *e, const uint4 *sl, uint8_t *val,
                      uint32_t vlen) {
  const View &v = e->v;
  if (v.kv_ool) {  // the key's value block
    if (sl[1].x >= v.kv_pool_blocks) return DRB_EDEVICE;
    HIPCHK(hipMemcpyAsync(val, v.kv_pool + (uint64_t)sl[1].x * v.VB, vlen,
                          hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return DRB_OK;
  }
  uint8_t tmp[16 * 9];
  memcpy(tmp, &sl[0].w, 4);
  for (uint32_t c = 1; c < v.KVW; ++c) memcpy(tmp + 4 + (c - 1) * 16, &sl[c], 16);
  memcpy(val, tmp, vlen);
  return DRB_OK;
}

extern "C" int drb_kv_lookup(drb_engine *e, uint64_t group, uint32_t slot,
                             const uint8_t *key, uint32_t key_len,
                             uint8_t *val, uint32_t val_cap,
                             uint32_t *val_len) {
  if (!e || group >= e->cfg.num_groups || slot >= e->cfg.num_replicas)
    return DRB_ERANGE;
  if (key_len > 8) return 1;
  const View &v = e->v;
  uint64_t k8 = 0;
  for (uint32_t i = 0; i < key_len; ++i) k8 |= (uint64_t)key[i] << (8 * i);
  std::vector<uint4> tbl;
  if (read_kv_table(e, group, slot, tbl)) return DRB_EDEVICE;
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < key_len; ++i)
    h = (h ^ ((k8 >> (8 * i)) & 0xff)) * 0x100000001b3ull;
  h ^= h >> 29;
  const uint32_t home = (uint32_t)h & (v.KS - 1);
  for (uint32_t p = 0; p < v.KS; ++p) {
    const uint4 *sl = &tbl[(uint64_t)kv_probe(v, home, p) * v.KVW];
    bool used = (sl[0].z >> 31) & 1u;
    if (!used) return 1;
    uint32_t klen = sl[0].z & 0xffu, vlen = (sl[0].z >> 8) & 0xfffu;
    if (klen == key_len && lo64h(sl[0]) == k8) {
      if (val_len) *val_len = vlen;
      if (vlen > val_cap) return DRB_ERANGE;
      return slot_value(e, sl, val, vlen);
    }
  }
  // a full table: the overflow chain
  std::vector<uint4> ch;
  if (read_ovf_chain(e, group, slot, ch)) return DRB_EDEVICE;
  for (size_t q = 0; q + v.KVW <= ch.size(); q += v.KVW) {
    const uint4 *sl = &ch[q];
    if (!((sl[0].z >> 31) & 1u)) continue;
    uint32_t klen = sl[0].z & 0xffu, vlen = (sl[0].z >> 8) & 0xfffu;
    if (klen == key_len && lo64h(sl[0]) == k8) {
      if (val_len) *val_len = vlen;
      if (vlen > val_cap) return DRB_ERANGE;
      return slot_value(e, sl, val, vlen);
    }
  }
  return 1;
}

extern "C" int drb_kv_import(drb_engine *e, uint64_t group, uint32_t slot,
                             const uint8_t *keys, const uint32_t *key_lens,
                             const uint8_t *vals, const uint32_t *val_lens,
                             size_t val_stride, size_t n) {
  if (!e || group >= e->cfg.num_groups || slot >= e->cfg.num_replicas)
    return DRB_ERANGE;
  if (n && (!keys || !key_lens || !vals || !val_lens)) return DRB_EINVAL;
  const View &v = e->v;
  if (n > v.KS && !v.kv_ovf_head) return DRB_ERANGE;
  std::vector<uint4> tbl((uint64_t)v.KS * v.KVW, make_uint4(0, 0, 0, 0));
  std::vector<size_t> spill;  // the pairs a full table sends to the chain
  const uint32_t mask = v.KS - 1;
  // one pair into its slot (the device's slot format, drb_step.hpp
  // apply_entry); an out-of-line value's block index is filled in below
  auto fill = [&](uint4 *sl, size_t i, uint64_t k8) {
    const uint32_t kl = key_lens[i], vl = val_lens[i];
    const uint8_t *val = vals + i * val_stride;
    uint32_t w0 = 0;
    for (uint32_t b = 0; b < 4 && b < vl; ++b) w0 |= (uint32_t)val[b] << (8 * b);
    sl[0] = make_uint4((uint32_t)k8, (uint32_t)(k8 >> 32),
                       (1u << 31) | (vl << 8) | kl, w0);
    if (!v.kv_ool) {
      uint8_t tmp[16 * 9] = {0};
      if (vl > 4) memcpy(tmp, val + 4, vl - 4);
      for (uint32_t c = 1; c < v.KVW; ++c) memcpy(&sl[c], tmp + 16 * (c - 1), 16);
    }
  };
  auto key8 = [&](size_t i) {
    uint64_t k8 = 0;
    for (uint32_t b = 0; b < key_lens[i]; ++b)
      k8 |= (uint64_t)keys[i * 8 + b] << (8 * b);
    return k8;
  };
  std::vector<std::pair<uint4 *, size_t>> ool;  // (slot, pair)
  for (size_t i = 0; i < n; ++i) {
    const uint32_t kl = key_lens[i], vl = val_lens[i];
    if (kl > 8 || vl > v.kv_val_cap) return DRB_ERANGE;
    const uint64_t k8 = key8(i);
    // the device's slot hash (drb_step.hpp kv_hash)
    uint64_t h = 0xcbf29ce484222325ull;
    for (uint32_t b = 0; b < kl; ++b)
      h = (h ^ ((k8 >> (8 * b)) & 0xff)) * 0x100000001b3ull;
    h ^= h >> 29;
    const uint32_t home = (uint32_t)h & mask;
    uint32_t ks = home, p = 0;
    while (p < v.KS && (tbl[(uint64_t)ks * v.KVW].z >> 31)) {
      ++p;
      ks = kv_probe(v, home, p);
    }
    if (p == v.KS) {
      spill.push_back(i);
      continue;
    }
    uint4 *sl = &tbl[(uint64_t)ks * v.KVW];
    fill(sl, i, k8);
    if (v.kv_ool) ool.push_back({sl, i});
  }
  // the chain: fresh buckets from the overflow pool (4 slots a bucket);
  // the replica's old chain, if any, is left behind like its old value
  // blocks (both pools are bump-allocated, drb_config.kv_overflow_buckets)
  const uint64_t nb = (spill.size() + 3) / 4;
  std::vector<uint4> ovf(nb * 4 * v.KVW, make_uint4(0, 0, 0, 0));
  unsigned long long obase = 0;
  if (v.kv_ovf_head) {
    HIPCHK(hipMemcpyAsync(&obase, v.kv_ovf_used, 8, hipMemcpyDeviceToHost,
                          e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (nb && obase + nb > v.kv_ovf_cap) return DRB_ERANGE;
  }
  for (size_t q = 0; q < spill.size(); ++q) {
    uint4 *sl = &ovf[q * v.KVW];
    fill(sl, spill[q], key8(spill[q]));
    if (v.kv_ool) ool.push_back({sl, spill[q]});
  }
  if (!ool.empty()) {  // fresh value blocks from the bump allocator
    unsigned long long next = 0;
    HIPCHK(hipMemcpyAsync(&next, v.kv_pool_next, 8, hipMemcpyDeviceToHost,
                          e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (next + ool.size() > v.kv_pool_blocks) return DRB_ERANGE;
    std::vector<uint4> blocks(ool.size() * v.VB, make_uint4(0, 0, 0, 0));
    for (size_t q = 0; q < ool.size(); ++q) {
      const size_t i = ool[q].second;
      ool[q].first[1] = make_uint4((uint32_t)(next + q), 0, 0, 0);
      memcpy(&blocks[q * v.VB], vals + i * val_stride, val_lens[i]);
    }
    HIPCHK(hipMemcpyAsync(v.kv_pool + next * v.VB, blocks.data(),
                          blocks.size() * sizeof(uint4), hipMemcpyHostToDevice,
                          e->stream));
    const unsigned long long nn = next + ool.size();
    HIPCHK(hipMemcpyAsync(v.kv_pool_next, &nn, 8, hipMemcpyHostToDevice,
                          e->stream));
  }
  if (v.kv_ovf_head) {
    std::vector<uint32_t> links(nb);
    for (uint64_t q = 0; q < nb; ++q)
      links[q] = q + 1 < nb ? (uint32_t)(obase + q + 2) : 0u;
    const uint32_t head = nb ? (uint32_t)(obase + 1) : 0u;
    if (nb) {
      HIPCHK(hipMemcpyAsync(v.kv_ovf + obase * 4 * v.KVW, ovf.data(),
                            ovf.size() * sizeof(uint4), hipMemcpyHostToDevice,
                            e->stream));
      HIPCHK(hipMemcpyAsync(v.kv_ovf_next + obase, links.data(), nb * 4,
                            hipMemcpyHostToDevice, e->stream));
      const unsigned long long nu = obase + nb;
      HIPCHK(hipMemcpyAsync(v.kv_ovf_used, &nu, 8, hipMemcpyHostToDevice,
                            e->stream));
    }
    HIPCHK(hipMemcpyAsync(v.kv_ovf_head + ix(v, slot, group), &head, 4,
                          hipMemcpyHostToDevice, e->stream));
  }
  HIPCHK(hipMemcpyAsync(v.kv + kv_ix(v, slot, group, 0), tbl.data(),
                        tbl.size() * sizeof(uint4), hipMemcpyHostToDevice,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

extern "C" int drb_kv_export(drb_engine *e, uint64_t group, uint32_t slot,
                             uint8_t *keys, uint32_t *key_lens, uint8_t *vals,
                             uint32_t *val_lens, size_t cap, size_t *n_out) {
  if (!e || group >= e->cfg.num_groups || slot >= e->cfg.num_replicas)
    return DRB_ERANGE;
  const View &v = e->v;
  std::vector<uint4> tbl;
  if (read_kv_table(e, group, slot, tbl)) return DRB_EDEVICE;
  std::vector<uint4> ch;  // the overflow chain's slots after the table's
  if (read_ovf_chain(e, group, slot, ch)) return DRB_EDEVICE;
  tbl.insert(tbl.end(), ch.begin(), ch.end());
  const uint64_t nslots = tbl.size() / v.KVW;
  size_t n = 0;
  for (uint64_t ks = 0; ks < nslots; ++ks) {
    const uint4 *sl = &tbl[(uint64_t)ks * v.KVW];
    if (!((sl[0].z >> 31) & 1u)) continue;
    if (n < cap) {
      uint32_t klen = sl[0].z & 0xffu, vlen = (sl[0].z >> 8) & 0xfffu;
      uint64_t k8 = lo64h(sl[0]);
      for (uint32_t i = 0; i < 8; ++i) keys[n * 8 + i] = (uint8_t)(k8 >> (8 * i));
      key_lens[n] = klen;
      if (int rc = slot_value(e, sl, vals + n * v.kv_val_cap, vlen)) return rc;
      val_lens[n] = vlen;
    }
    n++;
  }
  if (n_out) *n_out = n;
  return n > cap ? DRB_ERANGE : DRB_OK;
}

// ---------------------------------------------------------------- reads
// one lane per replica: the reads of the last round's ReadyToReads
// (the step kernels do the same in-round when drb_round_in.reads_per_ctx)
__global__ __launch_bounds__(256) void k_serve_reads(const View v,
                                                     uint32_t n_reads,
                                                     uint32_t key_space,
                                                     uint32_t slots) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t slot = (slots >> (4 * blockIdx.y)) & 0xfu;
  uint32_t served = 0, deferred = 0;
  if (g < v.G && (v.u32[u32_ix(v, W_FLAGS, slot, g)] & DRB_F_HOSTED)) {
    const uint32_t n = v.rtr_count[ix(v, slot, g)];
    if (n)
    {
      const uint4 c0 = v.pk[pk_ix(v, 0, slot, g)];
      const uint4 c1 = v.pk[pk_ix(v, 1, slot, g)];
      const uint64_t last = (uint64_t)c0.x | ((uint64_t)c0.y << 32);
      const uint32_t code = c1.z & 0xffffu;  // PI_SM_INDEX: word 6, low
      const uint64_t sm = code == PK_ESC16
                              ? v.u64[u64_ix(v, F_SM_INDEX, slot, g)]
                              : pk_idx_value(code, last, false);
      serve_reads_lane<true>(v, slot, g, n, sm, n_reads, key_space, served,
                             deferred);
    }
  }
  const uint32_t cnt[2] = {served, deferred};
  const BlockPos bp = {blockIdx.x, blockIdx.y, gridDim.x};
  block_counters<true, C_READS, 2>(v, slot, bp, cnt);
}

extern "C" int drb_serve_reads(drb_engine *e, uint32_t reads_per_ctx,
                               uint32_t key_space) {
  if (!e || key_space == 0) return DRB_EINVAL;
  if (e->v.max_reads && reads_per_ctx > e->v.max_reads) return DRB_ERANGE;
  dim3 grid((unsigned)((e->v.G + 255) / 256), e->v.R);
  uint32_t all = 0;
  for (uint32_t s = 0; s < e->v.R; ++s) all |= s << (4 * s);
  k_serve_reads<<<grid, 256, 0, e->stream>>>(e->v, reads_per_ctx, key_space,
                                             all);
  HIPCHK(hipGetLastError());
  e->reads_round = e->round;
  e->reads_n = reads_per_ctx;
  e->reads_ks = key_space;
  return DRB_OK;
}

extern "C" int drb_export_read_sums(drb_engine *e, uint64_t first_group,
                                    uint64_t n_groups, uint64_t *sums) {
  if (!e || !sums) return DRB_EINVAL;
  if (int rc = check_range(e, first_group, n_groups)) return rc;
  const View &v = e->v;
  const uint32_t R = v.R;
  std::vector<uint64_t> host(n_groups);
  for (uint32_t s = 0; s < R; ++s) {
    HIPCHK(hipMemcpyAsync(host.data(), v.read_sum + ix(v, s, first_group),
                          n_groups * sizeof(uint64_t), hipMemcpyDeviceToHost,
                          e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    for (uint64_t i = 0; i < n_groups; ++i) sums[i * R + s] = host[i];
  }
  return DRB_OK;
}

// ---------------------------------------------------------------- CRC32
// Slicing-by-8 CRC32-IEEE, one lane per buffer; the 8 x 256 table is
// staged in LDS once per workgroup.
__constant__ uint32_t c_crc_tab[8][256];

__global__ void k_crc32(const uint8_t *data, const uint64_t *off,
                        const uint32_t *len, uint32_t *crc, uint64_t n) {
  __shared__ uint32_t t[8][256];
  for (uint32_t i = threadIdx.x; i < 8 * 256; i += blockDim.x)
    t[i >> 8][i & 255] = c_crc_tab[i >> 8][i & 255];
  __syncthreads();
  uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n) return;
  const uint8_t *p = data + off[b];
  uint32_t l = len[b];
  uint32_t c = 0xffffffffu;
  while (l && ((uintptr_t)p & 7)) {
    c = t[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    l--;
  }
  while (l >= 8) {
    uint64_t w = *(const uint64_t *)p;
    uint32_t lo = (uint32_t)w ^ c, hi = (uint32_t)(w >> 32);
    c = t[7][lo & 0xff] ^ t[6][(lo >> 8) & 0xff] ^ t[5][(lo >> 16) & 0xff] ^
        t[4][lo >> 24] ^ t[3][hi & 0xff] ^ t[2][(hi >> 8) & 0xff] ^
        t[1][(hi >> 16) & 0xff] ^ t[0][hi >> 24];
    p += 8;
    l -= 8;
  }
  while (l--) c = t[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  crc[b] = c ^ 0xffffffffu;
}

extern "C" int drb_crc32_ieee_batch(drb_engine *e, const uint8_t *data,
                                    size_t data_len, const uint64_t *off,
                                    const uint32_t *len, size_t n,
                                    uint32_t *crc) {
  if (!e) return DRB_EINVAL;
  if (!n) return DRB_OK;
  for (size_t i = 0; i < n; ++i)
    if (off[i] + len[i] > data_len) return DRB_ERANGE;
  if (!e->crc_tab_ready) {
    uint32_t tab[8][256];
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      tab[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s)
        tab[s][i] = tab[0][tab[s - 1][i] & 0xff] ^ (tab[s - 1][i] >> 8);
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_tab), tab, sizeof(tab)));
    e->crc_tab_ready = true;
  }
  size_t bytes = ((data_len + 15) & ~15ull) + n * 8 + ((n * 4 + 15) & ~15ull) * 2;
  void *s;
  if (scratch(e, bytes + 64, &s)) return DRB_EDEVICE;
  uint8_t *dd = (uint8_t *)s;
  uint64_t *doff = (uint64_t *)(dd + ((data_len + 15) & ~15ull));
  uint32_t *dlen = (uint32_t *)(doff + n);
  uint32_t *dcrc = dlen + ((n + 3) & ~3ull);
  HIPCHK(hipMemcpyAsync(dd, data, data_len, hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipMemcpyAsync(doff, off, n * 8, hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipMemcpyAsync(dlen, len, n * 4, hipMemcpyHostToDevice, e->stream));
  k_crc32<<<(unsigned)((n + 255) / 256), 256, 0, e->stream>>>(dd, doff, dlen,
                                                               dcrc, n);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(crc, dcrc, n * 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

// ---------------------------------------------------------------- wire
#include "drb_wire.hpp"
#include "drb_ingest.hpp"
#include "drb_tan.hpp"

// ---------------------------------------------------------------- tan
static int launch_tan(drb_engine *e, uint32_t round) {
  const uint64_t max_log = e->cfg.tan_max_log ? e->cfg.tan_max_log
                                              : drb::TAN_MAX_LOG;
  HIPCHK(hipMemsetAsync(e->tan_n, 0, 64 * drb::TAN_LISTS * sizeof(uint32_t),
                        e->stream));
  tan_launch_select(e->v, round, max_log, e->tan_list, e->tan_per_list,
                    e->tan_n, (unsigned)e->tan_blocks, e->stream);
  HIPCHK(hipGetLastError());
  if (e->v.tan_mux) {
    tan_launch_chain(e->v, max_log, e->v.R * 16, e->stream);
    HIPCHK(hipGetLastError());
  }
  tan_launch_write(e->v, round, max_log, e->tan_list, e->tan_per_list,
                   e->tan_n, (unsigned)e->tan_wblocks, e->stream);
  HIPCHK(hipGetLastError());
  return DRB_OK;
}

__global__ void k_sum_tan(const unsigned long long *rows, uint64_t n,
                          unsigned long long *total) {
  __shared__ unsigned long long part[256];
  for (int c = 0; c < 4; ++c) {
    unsigned long long s = 0;
    for (uint64_t r = threadIdx.x; r < n; r += blockDim.x) s += rows[r * 4 + c];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (threadIdx.x < (unsigned)o) part[threadIdx.x] += part[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) total[c] = part[0];
    __syncthreads();
  }
}

static int read_tan_counters(drb_engine *e, unsigned long long *t4,
                             int reset) {
  k_sum_tan<<<1, 256, 0, e->stream>>>(e->v.tan_ctr, e->tan_blocks,
                                      e->tan_total);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(t4, e->tan_total, 4 * sizeof(t4[0]),
                        hipMemcpyDeviceToHost, e->stream));
  if (reset)
    HIPCHK(hipMemsetAsync(e->v.tan_ctr, 0, e->tan_blocks * 4 * sizeof(t4[0]),
                          e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

extern "C" int drb_export_tan(drb_engine *e, uint64_t group, uint32_t slot,
                              drb_tan_record *rec, uint8_t *buf, size_t cap) {
  if (!e || !rec || (cap && !buf)) return DRB_EINVAL;
  const View &v = e->v;
  if (!v.save_tan) return DRB_EINVAL;
  if (group >= v.G || slot >= v.R) return DRB_ERANGE;
  uint4 r, s[3];
  HIPCHK(hipMemcpyAsync(&r, v.tan_rec + ix(v, slot, group), sizeof(r),
                        hipMemcpyDeviceToHost, e->stream));
  for (uint32_t k = 0; k < 3; ++k)
    HIPCHK(hipMemcpyAsync(&s[k], v.tan_sum + tan_sum_ix(v, k, slot, group),
                          sizeof(uint4), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  memset(rec, 0, sizeof(*rec));
  rec->offset = (uint64_t)r.x | ((uint64_t)r.y << 32);
  rec->len = r.z;
  rec->flags = r.w & 0xffu;
  rec->log = r.w >> 8;
  if (rec->flags & DRB_TAN_WRITTEN) {
    const uint32_t n_save = s[2].x;
    const uint64_t save_lo = (uint64_t)s[1].z | ((uint64_t)s[1].w << 32);
    if (n_save) {
      rec->first_index = save_lo;
      rec->last_index = save_lo + n_save - 1;
    }
    if (s[2].y & TS_STATE)
      rec->commit = (uint64_t)s[1].x | ((uint64_t)s[1].y << 32);
  }
  if (rec->len > cap) return rec->len && buf ? DRB_ERANGE : DRB_OK;
  if (rec->len) {
    const uint8_t *src =
        reinterpret_cast<const uint8_t *>(v.save_buf + ix(v, slot, group) *
                                                           v.save_cap16);
    if (v.tan_mux) {  // its place in its log's staging
      uint4 p;
      HIPCHK(hipMemcpyAsync(&p, v.tanm_pos + tanm_ix(v, slot, group),
                            sizeof(p), hipMemcpyDeviceToHost, e->stream));
      HIPCHK(hipStreamSynchronize(e->stream));
      src = reinterpret_cast<const uint8_t *>(
                v.save_buf + ((uint64_t)slot * 16 + tanm_key(v, group)) *
                                 v.tanm_cap16) + p.z;
    }
    HIPCHK(hipMemcpyAsync(buf, src, rec->len, hipMemcpyDeviceToHost,
                          e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  return DRB_OK;
}

extern "C" int drb_export_tan_log(drb_engine *e, uint32_t slot, uint32_t key,
                                  drb_tan_log *out, uint8_t *buf, size_t cap) {
  if (!e || !out || (cap && !buf)) return DRB_EINVAL;
  const View &v = e->v;
  if (!v.tan_mux) return DRB_EINVAL;
  if (slot >= v.R || key >= 16) return DRB_ERANGE;
  uint4 lg[2];
  const uint64_t L = (uint64_t)slot * 16 + key;
  HIPCHK(hipMemcpyAsync(lg, v.tanm_log + 2 * L, sizeof(lg),
                        hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  memset(out, 0, sizeof(*out));
  out->start_offset = (uint64_t)lg[0].x | ((uint64_t)lg[0].y << 32);
  out->start_log = lg[0].z;
  out->flags = lg[0].w;
  out->bytes = lg[1].x;
  out->end_log = lg[1].y;
  out->end_offset = (uint64_t)lg[1].z | ((uint64_t)lg[1].w << 32);
  if (!buf) return DRB_OK;
  if (out->bytes > cap) return DRB_ERANGE;
  if (out->bytes) {
    HIPCHK(hipMemcpyAsync(buf, v.save_buf + L * v.tanm_cap16, out->bytes,
                          hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
  }
  return DRB_OK;
}

extern "C" int drb_tan_get(drb_engine *e, uint64_t group, uint32_t slot,
                           drb_tan_state *out) {
  if (!e || !out) return DRB_EINVAL;
  const View &v = e->v;
  if (!v.save_tan) return DRB_EINVAL;
  if (group >= v.G || slot >= v.R) return DRB_ERANGE;
  uint4 st, cur;
  HIPCHK(hipMemcpyAsync(&st, v.tan_st + ix(v, slot, group), sizeof(st),
                        hipMemcpyDeviceToHost, e->stream));
  if (v.tan_mux)  // the writer of the replica's multiplexed log
    HIPCHK(hipMemcpyAsync(&cur, v.tanm_cur + slot * 16 + tanm_key(v, group),
                          sizeof(cur), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (v.tan_mux) {
    st.x = cur.x;
    st.y = cur.y;
    st.z = cur.z;
  }
  out->offset = (uint64_t)st.x | ((uint64_t)st.y << 32);
  out->log = st.z;
  out->state_stored = st.w & TST_STATE;
  return DRB_OK;
}

extern "C" int drb_tan_set(drb_engine *e, uint64_t group, uint32_t slot,
                           const drb_tan_state *in) {
  if (!e || !in) return DRB_EINVAL;
  const View &v = e->v;
  if (!v.save_tan) return DRB_EINVAL;
  if (group >= v.G || slot >= v.R || in->log > 0xffffffu) return DRB_ERANGE;
  const uint4 st = make_uint4((uint32_t)in->offset,
                              (uint32_t)(in->offset >> 32), in->log,
                              in->state_stored ? TST_STATE : 0u);
  HIPCHK(hipMemcpyAsync(v.tan_st + ix(v, slot, group), &st, sizeof(st),
                        hipMemcpyHostToDevice, e->stream));
  if (v.tan_mux) {  // (the log's writer, shared by the slot's replicas)
    const uint4 cur = make_uint4(st.x, st.y, st.z, 0);
    HIPCHK(hipMemcpyAsync(v.tanm_cur + slot * 16 + tanm_key(v, group), &cur,
                          sizeof(cur), hipMemcpyHostToDevice, e->stream));
  }
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

extern "C" int drb_tan_buffers(drb_engine *e, void **bytes, void **recs) {
  if (!e || !bytes || !recs) return DRB_EINVAL;
  if (!e->v.save_tan) return DRB_EINVAL;
  *bytes = e->v.save_buf;
  *recs = e->v.tan_rec;
  return DRB_OK;
}

// ------------------------------------------------ batched round outputs
// The round's ReadyToReads and served-read results of one replica slot
// over a range of groups, compacted on the device: a per-lane record count,
// an exclusive scan (hipCUB), then each lane writes its records at its
// offset -- node.processReadyToRead (node.go:1081) and the clients'
// ReadLocalNode results (nodehost.go:849) for a whole step worker's groups
// without a device round trip per group.
namespace {
enum BatchKind : uint32_t { BK_RTR = 0, BK_READS = 1 };
}

// records of lane g of the range: ReadyToReads, or served reads (bit k of
// read_served for ctx k < rtr_count, n_reads each)
__global__ void k_batch_count(const View v, uint32_t slot, uint64_t g0,
                              uint64_t n, uint32_t kind, uint32_t n_reads,
                              uint32_t *cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  uint32_t c = 0;
  if (i < n) {
    const uint64_t g = g0 + i;
    const uint32_t nr = min(v.rtr_count[ix(v, slot, g)], (uint32_t)RTR_CAP);
    if (kind == BK_RTR) {
      c = nr;
    } else if (nr) {
      const uint32_t m = v.read_served[ix(v, slot, g)] & ((1u << nr) - 1u);
      c = (uint32_t)__popc(m) * n_reads;
    }
  }
  cnt[i] = c;  // cnt[n] = 0: the scan's last element is the total
}

__global__ void k_batch_rtr(const View v, uint32_t slot, uint64_t g0,
                            uint64_t n, const uint32_t *off,
                            drb_ready_to_read *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t g = g0 + i;
  const uint32_t nr = min(v.rtr_count[ix(v, slot, g)], (uint32_t)RTR_CAP);
  uint64_t o = off[i];
  for (uint32_t k = 0; k < nr; ++k, ++o) {
    const uint4 c0 = v.rtr[rtr_ix(v, slot, k, 0, g)];
    const uint4 c1 = v.rtr[rtr_ix(v, slot, k, 1, g)];
    drb_ready_to_read r;
    r.shard_id = v.first_shard_id + gid(v, slot, g);
    r.replica_id = slot + 1;
    r.index = (uint64_t)c0.x | ((uint64_t)c0.y << 32);
    r.ctx_low = (uint64_t)c0.z | ((uint64_t)c0.w << 32);
    r.ctx_high = (uint64_t)c1.x | ((uint64_t)c1.y << 32);
    out[o] = r;
  }
}

__global__ void k_batch_reads(const View v, uint32_t slot, uint64_t g0,
                              uint64_t n, uint32_t n_reads,
                              uint32_t key_space, const uint32_t *off,
                              drb_read_result *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t g = g0 + i;
  const uint32_t nr = min(v.rtr_count[ix(v, slot, g)], (uint32_t)RTR_CAP);
  if (!nr) return;
  const uint32_t m = v.read_served[ix(v, slot, g)] & ((1u << nr) - 1u);
  uint64_t o = off[i];
  for (uint32_t k = 0; k < nr; ++k) {
    if (!((m >> k) & 1u)) continue;
    const uint4 c0 = v.rtr[rtr_ix(v, slot, k, 0, g)];
    const uint4 c1 = v.rtr[rtr_ix(v, slot, k, 1, g)];
    const uint64_t low = (uint64_t)c0.z | ((uint64_t)c0.w << 32);
    for (uint32_t j = 0; j < n_reads; ++j, ++o) {
      const uint2 w = v.read_res[rres_ix(v, slot, k, j, g)];
      const uint64_t x =
          mix64(low ^ ((uint64_t)(j + 1) * 0x9E3779B97F4A7C15ull));
      drb_read_result r;
      r.shard_id = v.first_shard_id + gid(v, slot, g);
      r.index = (uint64_t)c0.x | ((uint64_t)c0.y << 32);
      r.ctx_low = low;
      r.ctx_high = (uint64_t)c1.x | ((uint64_t)c1.y << 32);
      r.key = x % key_space;  // serve_reads_lane's key (drb_step.hpp)
      r.replica_id = slot + 1;
      r.read = j;
      r.found = w.y >> 31;
      r.vlen = w.y & 0x7fffffffu;
      r.value = w.x;
      r.pad = 0;
      out[o] = r;
    }
  }
}

// ---- full ReadLocalNode values (drb_export_read_values)
// the slot of key8 in replica slot `slot`'s KV at lane g (table probes, then
// the overflow chain), or null
__device__ const uint4 *kv_find(const View &v, uint32_t slot, uint64_t g,
                                uint64_t key8) {
  const uint4 *tbl = v.kv + kv_ix(v, slot, g, 0);
  const uint32_t home = (uint32_t)kv_hash(key8, 8) & (v.KS - 1);
  for (uint32_t t = 0; t < v.KS; ++t) {
    const uint4 *sl = tbl + (uint64_t)kv_probe(v, home, t) * v.KVW;
    if (!kv_used(sl[0])) return nullptr;
    if (kv_match(sl[0], key8, 8)) return sl;
  }
  if (v.kv_ovf_head) {
    bool hit = false;
    const uint4 *sl = kv_ovf_walk(v, slot, g, key8, 8, false, hit);
    if (hit) return sl;
  }
  return nullptr;
}

// value bytes of the served reads of lane g, each padded to 16 B
__global__ void k_value_count(const View v, uint32_t slot, uint64_t g0,
                              uint64_t n, uint32_t n_reads, uint64_t *cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  uint64_t c = 0;
  if (i < n) {
    const uint64_t g = g0 + i;
    const uint32_t nr = min(v.rtr_count[ix(v, slot, g)], (uint32_t)RTR_CAP);
    const uint32_t m = nr ? v.read_served[ix(v, slot, g)] & ((1u << nr) - 1u)
                          : 0u;
    for (uint32_t k = 0; k < nr; ++k)
      if ((m >> k) & 1u)
        for (uint32_t j = 0; j < n_reads; ++j) {
          const uint2 w = v.read_res[rres_ix(v, slot, k, j, g)];
          if (w.y >> 31) c += ((w.y & 0x7fffffffu) + 15) & ~15u;
        }
  }
  cnt[i] = c;
}

// the values themselves: lookup again (the KV is as the round served it)
// and copy 16 B at a time into the pool at the read's offset
__global__ void k_batch_values(const View v, uint32_t slot, uint64_t g0,
                               uint64_t n, uint32_t n_reads,
                               uint32_t key_space, const uint32_t *off,
                               const uint64_t *voff, uint64_t *value_off,
                               uint4 *pool, unsigned long long *bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t g = g0 + i;
  const uint32_t nr = min(v.rtr_count[ix(v, slot, g)], (uint32_t)RTR_CAP);
  if (!nr) return;
  const uint32_t m = v.read_served[ix(v, slot, g)] & ((1u << nr) - 1u);
  uint64_t o = off[i], vo = voff[i];
  for (uint32_t k = 0; k < nr; ++k) {
    if (!((m >> k) & 1u)) continue;
    const uint4 c0 = v.rtr[rtr_ix(v, slot, k, 0, g)];
    const uint64_t low = (uint64_t)c0.z | ((uint64_t)c0.w << 32);
    for (uint32_t j = 0; j < n_reads; ++j, ++o) {
      const uint2 w = v.read_res[rres_ix(v, slot, k, j, g)];
      value_off[o] = vo;
      if (!(w.y >> 31)) continue;
      const uint32_t vlen = w.y & 0x7fffffffu;
      const uint64_t x =
          mix64(low ^ ((uint64_t)(j + 1) * 0x9E3779B97F4A7C15ull));
      const uint4 *sl = kv_find(v, slot, g, x % key_space);
      uint4 *dst = pool + vo / 16;
      vo += (vlen + 15) & ~15u;
      if (!sl || ((sl[0].z >> 8) & 0xfffu) != vlen) {
        atomicAdd(bad, 1ull);  // the KV changed since the round served it
        continue;
      }
      if (v.kv_ool) {  // the key's value block
        const uint4 *src = v.kv_pool + (uint64_t)sl[1].x * v.VB;
        for (uint32_t c = 0; c * 16 < vlen; ++c) dst[c] = src[c];
      } else {  // inline: 4 bytes in the header word, then the slot chunks
        uint4 prev = make_uint4(sl[0].w, 0, 0, 0);
        for (uint32_t c = 0; c * 16 < vlen; ++c) {
          const uint4 nx = c + 1 < v.KVW ? sl[c + 1] : make_uint4(0, 0, 0, 0);
          // bytes [16 c, 16 c + 16) of (w, sl[1], sl[2], ...)
          dst[c] = make_uint4(prev.x, nx.x, nx.y, nx.z);
          prev = make_uint4(nx.w, 0, 0, 0);
        }
      }
    }
  }
}

static int xout(drb_engine *e, size_t bytes, void **p) {
  if (bytes > e->xout_bytes) {
    if (e->xout) HIPCHK(hipFree(e->xout));
    e->xout = nullptr;
    e->xout_bytes = 0;
    HIPCHK(hipMalloc(&e->xout, bytes));
    e->xout_bytes = bytes;
  }
  *p = e->xout;
  return DRB_OK;
}

static int batch_export(drb_engine *e, uint32_t slot, uint64_t first,
                        uint64_t n, uint32_t kind, void *out, size_t rec,
                        size_t cap, size_t *n_out) {
  if (!e || !n_out || (cap && !out)) return DRB_EINVAL;
  if (slot >= e->v.R || check_range(e, first, n)) return DRB_ERANGE;
  *n_out = 0;
  const uint32_t n_reads = kind == BK_READS ? e->reads_n : 0;
  // reads: only the last round's, and only if that round served them
  if (kind == BK_READS && (!e->v.read_res || e->reads_round != e->round))
    return e->v.read_res ? DRB_OK : DRB_EINVAL;
  const View &v = e->v;
  // scratch: counts and offsets [n + 1] each, then the scan's temp storage
  size_t tb = 0;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (uint32_t *)nullptr,
                                          (uint32_t *)nullptr, (int)(n + 1),
                                          e->stream));
  const size_t a = ((n + 1) * 4 + 255) & ~(size_t)255;
  void *s;
  if (scratch(e, 2 * a + tb + 256, &s)) return DRB_EDEVICE;
  uint32_t *cnt = (uint32_t *)s;
  uint32_t *off = (uint32_t *)((char *)s + a);
  void *tmp = (char *)s + 2 * a;
  const unsigned blocks = (unsigned)((n + 1 + 255) / 256);
  k_batch_count<<<blocks, 256, 0, e->stream>>>(v, slot, first, n, kind,
                                               n_reads, cnt);
  HIPCHK(hipGetLastError());
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, off, (int)(n + 1),
                                          e->stream));
  uint32_t total = 0;
  HIPCHK(hipMemcpyAsync(&total, off + n, 4, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *n_out = total;
  if (total > cap) return DRB_ERANGE;
  if (!total) return DRB_OK;
  void *d;
  if (xout(e, (size_t)total * rec, &d)) return DRB_EDEVICE;
  const unsigned wb = (unsigned)((n + 255) / 256);
  if (kind == BK_RTR)
    k_batch_rtr<<<wb, 256, 0, e->stream>>>(v, slot, first, n, off,
                                           (drb_ready_to_read *)d);
  else
    k_batch_reads<<<wb, 256, 0, e->stream>>>(v, slot, first, n, n_reads,
                                             e->reads_ks, off,
                                             (drb_read_result *)d);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, d, (size_t)total * rec, hipMemcpyDeviceToHost,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}

extern "C" int drb_export_ready_to_reads_batch(drb_engine *e, uint32_t slot,
                                               uint64_t first_group,
                                               uint64_t n_groups,
                                               drb_ready_to_read *out,
                                               size_t cap, size_t *n_out) {
  return batch_export(e, slot, first_group, n_groups, BK_RTR, out,
                      sizeof(drb_ready_to_read), cap, n_out);
}

extern "C" int drb_export_read_results(drb_engine *e, uint32_t slot,
                                       uint64_t first_group, uint64_t n_groups,
                                       drb_read_result *out, size_t cap,
                                       size_t *n_out) {
  return batch_export(e, slot, first_group, n_groups, BK_READS, out,
                      sizeof(drb_read_result), cap, n_out);
}

extern "C" int drb_export_read_values(drb_engine *e, uint32_t slot,
                                      uint64_t first_group, uint64_t n_groups,
                                      drb_read_result *out,
                                      uint64_t *value_off, size_t cap,
                                      uint8_t *pool, size_t pool_cap,
                                      size_t *n_out, size_t *pool_bytes) {
  if (!e || !n_out || !pool_bytes || (cap && (!out || !value_off)))
    return DRB_EINVAL;
  *pool_bytes = 0;
  int rc = batch_export(e, slot, first_group, n_groups, BK_READS, out,
                        sizeof(drb_read_result), cap, n_out);
  if (rc || !*n_out) return rc;
  // the record offsets again (batch_export's scratch), and the value ones
  const View &v = e->v;
  const uint64_t n = n_groups;
  const uint32_t n_reads = e->reads_n;
  size_t tb = 0, tb2 = 0;
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (uint32_t *)nullptr,
                                          (uint32_t *)nullptr, (int)(n + 1),
                                          e->stream));
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, (uint64_t *)nullptr,
                                          (uint64_t *)nullptr, (int)(n + 1),
                                          e->stream));
  const size_t a = ((n + 1) * 4 + 255) & ~(size_t)255;
  const size_t a8 = ((n + 1) * 8 + 255) & ~(size_t)255;
  const size_t tmax = tb > tb2 ? tb : tb2;
  void *s;
  if (scratch(e, 2 * a + 2 * a8 + tmax + 256, &s)) return DRB_EDEVICE;
  uint32_t *cnt = (uint32_t *)s;
  uint32_t *off = (uint32_t *)((char *)s + a);
  uint64_t *vcnt = (uint64_t *)((char *)s + 2 * a);
  uint64_t *voff = (uint64_t *)((char *)s + 2 * a + a8);
  unsigned long long *bad = (unsigned long long *)((char *)s + 2 * a + 2 * a8);
  void *tmp = (char *)s + 2 * a + 2 * a8 + 256;
  const unsigned blocks = (unsigned)((n + 1 + 255) / 256);
  k_batch_count<<<blocks, 256, 0, e->stream>>>(v, slot, first_group, n,
                                               BK_READS, n_reads, cnt);
  HIPCHK(hipGetLastError());
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, off, (int)(n + 1),
                                          e->stream));
  k_value_count<<<blocks, 256, 0, e->stream>>>(v, slot, first_group, n,
                                               n_reads, vcnt);
  HIPCHK(hipGetLastError());
  HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, vcnt, voff, (int)(n + 1),
                                          e->stream));
  uint64_t total = 0;
  HIPCHK(hipMemcpyAsync(&total, voff + n, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipMemsetAsync(bad, 0, 8, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *pool_bytes = (size_t)total;
  if (total > pool_cap || (total && !pool)) return DRB_ERANGE;
  // device staging: the offsets, then the pool
  const size_t ob = ((size_t)*n_out * 8 + 255) & ~(size_t)255;
  void *d;
  if (xout(e, ob + (size_t)total + 16, &d)) return DRB_EDEVICE;
  uint64_t *doff = (uint64_t *)d;
  uint4 *dpool = (uint4 *)((char *)d + ob);
  const unsigned wb = (unsigned)((n + 255) / 256);
  k_batch_values<<<wb, 256, 0, e->stream>>>(v, slot, first_group, n, n_reads,
                                            e->reads_ks, off, voff, doff,
                                            dpool, bad);
  HIPCHK(hipGetLastError());
  unsigned long long nbad = 0;
  HIPCHK(hipMemcpyAsync(value_off, doff, (size_t)*n_out * 8,
                        hipMemcpyDeviceToHost, e->stream));
  if (total)
    HIPCHK(hipMemcpyAsync(pool, dpool, (size_t)total, hipMemcpyDeviceToHost,
                          e->stream));
  HIPCHK(hipMemcpyAsync(&nbad, bad, 8, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return nbad ? DRB_EDEVICE : DRB_OK;
}

// ---------------------------------------------------------------- worker
#include "drb_worker.hpp"

// ------------------------------------------------- RCCL exchange (C4, N > 1)
#include "drb_rccl.hpp"
