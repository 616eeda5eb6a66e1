// drb_step.hpp -- the fused step-round kernel.
//
// One lane = one replica (slot, group).  A round is one iteration of
// dragonboat's step loop (node_test.go:274-353, engine.go:1304-1364) for
// that replica: handleEvents (node.go:1161-1223) -> getUpdate
// (node.go:1025) -> apply (rsm StateMachine.Handle) -> Peer.Commit
// (peer.go:292).  Messages emitted in round t land in the mailbox buffer
// t&1 and are consumed in round t+1 -- exactly the delivery of the
// reference step loop, where all sends happen after every node has handled
// its events.  Inbox order = Replicate messages by sender slot, then all
// other messages by sender slot (node_test.go:311-339), then the LocalTick.
//
// The lane first runs a read-only pre-pass over its inbox and inputs; if
// the round would leave the fast path (term change, election, lost quorum,
// unsupported message/entry, capacity) it marks the replica
// DRB_F_FALLBACK and returns WITHOUT mutating anything.
#pragma once
#include "../../include/drb_engine.h"
#include "drb_codec.hpp"
#include "drb_layout.hpp"
#include "drb_msg.hpp"
#include "drb_ring.hpp"

namespace drb {

#define DRB_DEV __device__ __forceinline__

// minimum waves per SIMD the step kernels are compiled for, per role
// (caps the registers the compiler may allocate)
// (measured at C3 on MI355X, tools/exp_variants.sh: leader 3 / follower 4
// waves per SIMD ran 3-6 % faster than the unconstrained 2 / 3, the
// leader's few spilled values notwithstanding)
#ifndef DRB_LEAD_WAVES
#define DRB_LEAD_WAVES 3
#endif
// the EXT leader (C5 payloads, EntryBatch encoding) carries the most state.
// Two waves per SIMD spill nothing but measured slower at C5 128 B (3.83 vs
// 3.35 ms / round).  Note: the three-wave EXT leader built with
// DRB_PROBE_W=4 produced wrong EntriesToSave on the GPU (every W <= 2 build,
// and the two-wave build, were exact; tests/test_gpu_parity.py
// test_entries_to_save_entrybatch_crc catches it)
#ifndef DRB_EXT_LEAD_WAVES
#define DRB_EXT_LEAD_WAVES 3
#endif
// the raft launch steps only the replicas routed to it: its register
// budget matters more than its occupancy (at 3 waves it spilled ~400 VGPRs
// and ~330 SGPRs into VGPR lanes)
#ifndef DRB_SLOW_WAVES
#define DRB_SLOW_WAVES 1
#endif
#ifndef DRB_FOLLOW_WAVES
#define DRB_FOLLOW_WAVES 4
#endif
// KV slots loaded per probe step (apply upserts, lookups past the first two).
// Measured at C3 (same box): W=1 1.016, 2 1.033, 4 1.063, 8 1.240 ms/round,
// and kv_slots 1024 no faster than 512: the probe chains are not what the
// KV accesses wait on (the random line fetches are)
// (round 2, near-empty tables: W=1 1.016, 2 1.033, 4 1.063 ms/round.  At
// the steady state's load of 1/2 a lookup's first probe often misses, and
// the whole 64 B probe group -- one HBM fetch, see kv_probe -- is loaded at
// once: DRB_PROBE_W = 4 for the upserts, DRB_READ_W = 4 for the served
// reads' first group and DRB_PROBE_WR = 4 for their later groups.)
#ifndef DRB_PROBE_W
#define DRB_PROBE_W 4
#endif
#ifndef DRB_PROBE_WR
#define DRB_PROBE_WR DRB_PROBE_W
#endif
#ifndef DRB_READ_W
#define DRB_READ_W 4
#endif
// follower inbox prefetch: the first DRB_FPF records from the (one)
// sender with records, loaded to LDS at once by LDS-DMA (global_load_lds:
// no VGPRs) instead of one dependent load per record in the dispatch loop
#ifndef DRB_FPF
#define DRB_FPF 8
#endif
// (the leader's first records the same way measured neutral or slower,
// profiles/r03_lpf: the leader prefetches nothing)
#ifndef DRB_QS_DIRTY
#define DRB_QS_DIRTY 1
#endif
#ifndef DRB_REM_DIRTY
#define DRB_REM_DIRTY 1
#endif
// timing only: per-phase cycle sums of the leader / follower lanes
// (View.phase, drb_debug_phase); 0 in shipped builds
// the quiesce base stored and read every round, rtr_count cleared by every
// lean round (1: the behaviour before round 6's lazy forms; timing variant)
#ifndef DRB_QS_EAGER
#define DRB_QS_EAGER 0
#endif
// the zero-copy exchange's reads (in_mbox & co.; 0: timing variant only)
#ifndef DRB_PEERS
#define DRB_PEERS 1
#endif
#ifndef DRB_PHASE_PROF
#define DRB_PHASE_PROF 0
#endif

constexpr uint64_t MAX_ENTRY_SIZE = 64ull * 1024 * 1024;  // soft.go:186

// counters[] slots
enum : int {
  C_COMMITTED = 0,
  C_APPLIED,
  C_MESSAGES,
  C_RTR,
  C_DROPPED_RI,
  C_FALLBACKS,
  C_ERRORS,
  C_READS,        // drb_serve_reads
  C_READS_DEFERRED,
  C_SAVED_ENTRIES,  // encode_saves
  C_SAVED_BYTES,
  C_STEPPED,  // replicas that ran the round (not skipped as idle)
  C_ELECT,    // elections: replicas the raft launch stepped
  C_ROLE,     // elections: role changes
  C_DPROP,    // elections: proposals a transferring leader dropped
  C_LEAN,     // replicas the lean kernel of a listed round stepped
  NUM_COUNTERS
};

// A replica's state is one 64 B packed record (drb_layout.hpp, PIdx),
// loaded whole at the start of its round and stored whole at the end.  The
// fields most of the round uses are decoded into registers; the rest
// (vote, the randomized timeout, Peer's prevState, node's confirmed/pushed
// indexes, appliedTo*, sm_term) stay encoded in the record words and are
// read / written through ld_f / st_f.  tick_count and kv_count are plain
// u64 counters, read-modify-written where the round changes them.
template <int R>
struct Rep {
  uint32_t pw[16];  // the packed record (index offsets relative to base0)
  uint64_t base0;   // last at the start of the round
  uint64_t term, leader_id, election_tick, heartbeat_tick;
  uint64_t committed, processed, last, marker, saved_to;
  uint64_t applied_index, sm_index, ring_lo, ring_guard, term_start;
  uint64_t sm_term;      // valid when kv_added / applied_any
  uint32_t kv_added;     // KVTest.Count increments this round
  bool applied_any, lid_dirty;
  uint32_t role, flags, fb, ri_count;
  uint32_t votes;  // elections: answered | granted << 8, bit per slot
  // leader remotes live in LDS (RemLds), see rem_get/rem_put
  // leader: readIndex queue (the ctx of each entry in LDS, Lane.rq)
  uint64_t ri_ix[DRB_RI_DEPTH];
  uint32_t ri_fr[DRB_RI_DEPTH], ri_cf[DRB_RI_DEPTH];
  // round-local
  HintCtx hc;          // ctx dedup state of this sender (drb_msg.hpp)
  uint32_t nmsgs;
  uint32_t c1mask;     // destinations that got a record with a c1 chunk
  uint32_t nrtr;
  uint32_t ndropped_ri;
  uint32_t ndropped_props;  // reportDroppedProposal (entries)
  uint64_t guard_new;
  bool leader_update;
  bool oterm;  // raft launch: a record went out with a term not r.term
  bool err;
  // node.qs (Quiesce on, EXT instantiation): quiesce.go:23-33
  uint64_t qs_tick, qs_idle, qs_since, qs_exit;
  uint32_t qs_dirty;  // idle 1, since 2, exit 4: stored at the round's end
  bool qs_new;  // newQuiesceStateFlag: send Quiesce to the peers
};

// Per-lane remote progress table in LDS, [peer][lane]: dynamically
// indexed by the sender slot without spilling to scratch, and conflict-free
// (consecutive lanes hit consecutive banks).
template <int R>
struct RemLds {
  uint64_t m[R][256];
  uint64_t n[R][256];
  uint32_t st[R][256];
  uint32_t a[R][256];
  // fields changed this round, bit 4 * peer + {m, n, st, a}: the end of
  // the round stores only those (a heartbeat round, C5's common one,
  // changes none)
  uint32_t dirty[256];
};

struct Lane {
  void *rl;       // RemLds<R> of this workgroup
  uint32_t *oi;   // [R][256] outbox header info per destination (LDS)
  uint64_t *elo;  // [R][256] leader: lowest entry index sent to a remote
                  // follower this round (~0: none), LDS (placement C4)
  uint64_t *rq;   // [2][DRB_RI_DEPTH][256] leader: the readIndex queue's
                  // ctx {low, high} per entry, LDS
  uint32_t tid;   // lane within the workgroup
  const View *v;
  uint32_t slot;
  uint64_t g;
  uint32_t rbuf, wbuf;
  uint64_t round;
  bool slow;  // the raft launch (elections): records carry their own term
  // the remotes' fields are stored back only where they changed (the EXT
  // instantiation: C5's heartbeat rounds change none; the C3 path keeps
  // its registers for the unconditional stores)
  bool dirty;
  // member kinds (drb_config.nonvoting_slots / witness_slots) are stepped
  // by the FWD instantiations (and the raft launch) only; the C3 and C5
  // kernels compile them out
  bool members = false;
  // remote planes may be read in bound peers' outboxes (View.peers,
  // drb_exchange_local_bind): off in the LOCAL instantiations (engines
  // without placement), which compile that path out -- it costs the C3
  // kernels ~1-2 % in registers (profiles/r06_bind)
  bool peers = true;
};

// ------------------------------------------------------------ helpers
// the ctx of readIndex queue entry d (d a compile-time index)
DRB_DEV uint64_t &rq_lo(const Lane &L, int d) {
  return L.rq[(uint32_t)d * 256 + L.tid];
}
DRB_DEV uint64_t &rq_hi(const Lane &L, int d) {
  return L.rq[(uint32_t)(DRB_RI_DEPTH + d) * 256 + L.tid];
}
DRB_DEV uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
DRB_DEV uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
DRB_DEV uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }


template <int R>
DRB_DEV void set_error(Rep<R> &r, uint32_t reason) {
  if (!r.err) {
    r.err = true;
    r.fb = reason;
  }
}

// entry term at index (entryLog.term, logentry.go:142-155) from the
// resident window
template <int R>
DRB_DEV uint64_t log_term(const Lane &L, Rep<R> &r, uint64_t index) {
  if (index == 0 || index > r.last) return 0;  // first-1 == 0 on this path
  if (index >= r.term_start) return r.term;    // no HBM access on the tail
  if (index < r.ring_lo) {
    set_error(r, DRB_ERR_LOG_RANGE);
    return 0;
  }
  uint4 q = L.v->ring[ring_ix(*L.v, L.slot, index, 0, L.g)];
  return (uint64_t)q.x | ((uint64_t)q.y << 32);
}
DRB_DEV uint4 mk4(uint64_t a, uint64_t b) {
  return make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b,
                    (uint32_t)(b >> 32));
}

template <int R>
DRB_DEV uint64_t ring_term(const Lane &L, uint32_t slot, uint64_t index) {
  return lo64(L.v->ring[ring_ix(*L.v, slot, index, 0, L.g)]);
}

template <int R>
DRB_DEV void set_leader(Rep<R> &r, uint64_t id) {
  if (r.leader_id != id) {
    r.leader_id = id;
    r.lid_dirty = true;
  }
}

// ------------------------------------------------------------ quiesce
// quiesceState (quiesce.go:23-120) with electionTick = 2 x ElectionRTT
// (node.go:195-200); threshold = 10 x that.
template <int R>
DRB_DEV bool qs_quiesced(const Rep<R> &r) { return r.qs_since > 0; }
template <int R>
DRB_DEV void qs_enter(Rep<R> &r) {  // enterQuiesce (quiesce.go:104-109)
  r.qs_since = r.qs_tick;
  r.qs_idle = r.qs_tick;
  r.qs_dirty |= 3u;
  r.qs_new = true;
}
template <int R>
DRB_DEV void qs_exit(Rep<R> &r) {  // exitQuiesce (quiesce.go:111-114)
  r.qs_since = 0;
  r.qs_exit = r.qs_tick;
  r.qs_dirty |= 6u;
}
// record (quiesce.go:56-74); heartbeats carrying a ReadIndex ctx count as
// ReadIndex (node.recordMessage, node.go:1339-1345)
template <int R>
DRB_DEV void qs_record(const View &v, Rep<R> &r, uint32_t type) {
  if (type == DRB_MSG_HEARTBEAT || type == DRB_MSG_HEARTBEAT_RESP) {
    if (!qs_quiesced(r)) return;
    if (r.qs_tick - r.qs_since < 2ull * v.election_rtt) return;  // newToQuiesce
  }
  r.qs_idle = r.qs_tick;
  r.qs_dirty |= 1u;
  if (qs_quiesced(r)) qs_exit(r);
}
// tryEnterQuiesce (quiesce.go:91-102): a Quiesce message
template <int R>
DRB_DEV void qs_try_enter(const View &v, Rep<R> &r) {
  if (!qs_quiesced(r) && r.qs_tick - r.qs_exit < 20ull * v.election_rtt)
    return;  // justExitedQuiesce
  if (!qs_quiesced(r)) qs_enter(r);
}
// Whether this round's LocalTick is a quiesced tick, for a round whose
// inbox holds no record and no staged ReadIndex (only Quiesce messages):
// tryEnterQuiesce on a Quiesce, then tick (node.go:1385-1386, 1562-1570)
template <int R>
DRB_DEV bool qs_quiet_tick(const View &v, const Rep<R> &r, uint32_t qz_from) {
  const uint64_t thr = 20ull * v.election_rtt;
  bool q = qs_quiesced(r);
  if (!q && qz_from && !(r.qs_tick - r.qs_exit < thr)) q = true;
  return q || (r.qs_tick + 1 - r.qs_idle > thr);
}
// tick (quiesce.go:40-51)
template <int R>
DRB_DEV void qs_tick_once(const View &v, Rep<R> &r) {
  r.qs_tick++;
  if (!qs_quiesced(r) && r.qs_tick - r.qs_idle > 20ull * v.election_rtt)
    qs_enter(r);
}

// ------------------------------------------------------------ packed state
// the u64 array: overflow of escaped record fields, tick/kv counters
DRB_DEV uint64_t over_ld(const Lane &L, int f) {
  return L.v->u64[u64_ix(*L.v, f, L.slot, L.g)];
}
DRB_DEV void over_st(const Lane &L, int f, uint64_t x) {
  L.v->u64[u64_ix(*L.v, f, L.slot, L.g)] = x;
}
// index field i (a PIdx constant): offset from `base` in the record
template <int R>
DRB_DEV uint64_t pi_get(const Lane &L, const Rep<R> &r, int i) {
  const uint32_t c = pk_half(r.pw, 4 + i / 2, i & 1);
  return c == PK_ESC16 ? over_ld(L, pi_field(i))
                       : pk_idx_value(c, r.base0, i == PI_RING_GUARD);
}
template <int R>
DRB_DEV void pi_put(const Lane &L, Rep<R> &r, int i, uint64_t x,
                    uint64_t base) {
  const uint32_t c = pk_idx_code(x, base, i == PI_RING_GUARD);
  if (c == PK_ESC16) over_st(L, pi_field(i), x);
  pk_set_half(r.pw, 4 + i / 2, i & 1, c);
}
// term distances (word, half), ticks (word, half), replica ids (byte)
template <int R>
DRB_DEV uint64_t pt_get(const Lane &L, const Rep<R> &r, int w, int h, int f) {
  const uint32_t c = pk_half(r.pw, w, h);
  return c == PK_ESCU16 ? over_ld(L, f) : r.term - c;
}
template <int R>
DRB_DEV void pt_put(const Lane &L, Rep<R> &r, int w, int h, int f,
                    uint64_t x) {
  const uint32_t c = pk_term_code(x, r.term);
  if (c == PK_ESCU16) over_st(L, f, x);
  pk_set_half(r.pw, w, h, c);
}
template <int R>
DRB_DEV uint64_t pu_get(const Lane &L, const Rep<R> &r, int w, int h, int f) {
  const uint32_t c = pk_half(r.pw, w, h);
  return c == PK_ESCU16 ? over_ld(L, f) : c;
}
template <int R>
DRB_DEV void pu_put(const Lane &L, Rep<R> &r, int w, int h, int f,
                    uint64_t x) {
  const uint32_t c = pk_u16_code(x);
  if (c == PK_ESCU16) over_st(L, f, x);
  pk_set_half(r.pw, w, h, c);
}
template <int R>
DRB_DEV uint64_t pd_get(const Lane &L, const Rep<R> &r, int b, int f) {
  const uint32_t c = (r.pw[14] >> (8 * b)) & 0xffu;
  return c == PK_ESC8 ? over_ld(L, f) : c;
}
template <int R>
DRB_DEV void pd_put(const Lane &L, Rep<R> &r, int b, int f, uint64_t x) {
  const uint32_t c = pk_id_code(x);
  if (c == PK_ESC8) over_st(L, f, x);
  r.pw[14] = (r.pw[14] & ~(0xffu << (8 * b))) | (c << (8 * b));
}

// the record fields a round does not keep decoded (f: a U64Field constant)
template <int R>
DRB_DEV uint64_t ld_f(const Lane &L, const Rep<R> &r, int f) {
  switch (f) {
    case F_VOTE: return pd_get(L, r, 0, f);
    case F_PREV_VOTE: return pd_get(L, r, 2, f);
    case F_APPLIED_TO_TERM: return pt_get(L, r, 11, 0, f);
    case F_PREV_TERM: return pt_get(L, r, 11, 1, f);
    case F_SM_TERM: return pt_get(L, r, 12, 0, f);
    case F_RAND_TIMEOUT: return pu_get(L, r, 13, 1, f);
    case F_APPLIED: return pi_get(L, r, PI_APPLIED);
    case F_APPLIED_TO_INDEX: return pi_get(L, r, PI_APPLIED_TO_INDEX);
    case F_CONFIRMED_INDEX: return pi_get(L, r, PI_CONFIRMED);
    case F_PUSHED_INDEX: return pi_get(L, r, PI_PUSHED);
    case F_PREV_COMMIT: return pi_get(L, r, PI_PREV_COMMIT);
    default: return over_ld(L, f);  // tick_count, kv_count
  }
}
template <int R>
DRB_DEV void st_f(const Lane &L, Rep<R> &r, int f, uint64_t x) {
  switch (f) {
    case F_VOTE: pd_put(L, r, 0, f, x); break;
    case F_PREV_VOTE: pd_put(L, r, 2, f, x); break;
    case F_APPLIED_TO_TERM: pt_put(L, r, 11, 0, f, x); break;
    case F_PREV_TERM: pt_put(L, r, 11, 1, f, x); break;
    case F_SM_TERM: pt_put(L, r, 12, 0, f, x); break;
    case F_RAND_TIMEOUT: pu_put(L, r, 13, 1, f, x); break;
    case F_APPLIED: pi_put(L, r, PI_APPLIED, x, r.base0); break;
    case F_APPLIED_TO_INDEX: pi_put(L, r, PI_APPLIED_TO_INDEX, x, r.base0); break;
    case F_CONFIRMED_INDEX: pi_put(L, r, PI_CONFIRMED, x, r.base0); break;
    case F_PUSHED_INDEX: pi_put(L, r, PI_PUSHED, x, r.base0); break;
    case F_PREV_COMMIT: pi_put(L, r, PI_PREV_COMMIT, x, r.base0); break;
    default: over_st(L, f, x); break;  // tick_count, kv_count
  }
}

// ------------------------------------------------------------ messages
// send (raft.go:683-687): From = self; the Term of every non-request
// message is r.term and lives in the outbox meta word
// The header info of each destination accumulates in LDS ([dest][lane]:
// a runtime destination slot indexes it without scratch); the headers are
// written at the end of the round for the destinations that got records.
template <int R>
DRB_DEV void emit(const Lane &L, Rep<R> &r, uint32_t to_slot, const Msg &m) {
  const View &v = *L.v;
  uint32_t &w = L.oi[to_slot * 256 + L.tid];
  if (mi_count(w) >= v.MB) {  // bounded by the pre-pass; never expected
    set_error(r, DRB_FB_CAPACITY);
    return;
  }
  const bool rep = m.type == DRB_MSG_REPLICATE;
  const uint32_t k = rep ? mi_nrep(w) : rec_pos(false, mi_noth(w), v.MB);
  r.nmsgs++;
  Msg mm = m;
  mm.term = is_request_type(m.type) ? 0
            : is_prevote_type(m.type) ? m.term
                                      : r.term;
  if (mm.term != r.term && mm.term != 0) r.oterm = true;
  uint4 c0, c1;
  const bool has = msg_encode(mm, to_slot, &r.hc, c0, c1);
  const uint32_t inf = msg_info(mm.type, mm.term == 0, m.reject != 0, m.n);
  w = (w + (inf & MI_CNTS)) | (inf & ~MI_CNTS);
  v.mbox[mbox_ix(v, L.wbuf, L.slot, to_slot, k, 0, L.g)] = c0;
  // the raft launch may change its term after this record: keep the
  // record's own (the header gets the final term, drb_msg.hpp)
  if (L.slow) v.rterm[rterm_ix(v, L.wbuf, L.slot, to_slot, k, L.g)] = mm.term;
  if (has) {
    v.mbox[mbox_ix(v, L.wbuf, L.slot, to_slot, k, 1, L.g)] = c1;
    r.c1mask |= 1u << to_slot;
  }
  if (rep) {
    // entries to a replica on another rank travel by value: the rows
    // [lowest index sent, last] ship with the plane (end of the round)
    if (m.n && pair_remote(v, L.slot, to_slot)) {
      uint64_t &lo = L.elo[to_slot * 256 + L.tid];
      lo = umin64(lo, m.log_index + 1);
    }
    // LogIndex + n of successive Replicates never decreases in a round
    v.mbox_maxapp[mmeta_ix(v, L.wbuf, L.slot, to_slot, L.g)] =
        m.log_index + m.n;
  }
}

// ------------------------------------------------------------ members
// member kinds of the replica slots (drb_config.nonvoting_slots /
// witness_slots): slot s of every group
DRB_DEV uint32_t nv_mask_of(const Lane &L) {
  return L.members ? L.v->nv_mask : 0u;
}
DRB_DEV uint32_t wt_mask_of(const Lane &L) {
  return L.members ? L.v->wt_mask : 0u;
}
DRB_DEV bool is_nonvoting(const Lane &L, uint32_t s) {
  return (nv_mask_of(L) >> s) & 1u;
}
DRB_DEV bool is_witness(const Lane &L, uint32_t s) {
  return (wt_mask_of(L) >> s) & 1u;
}
// quorum (raft.go:385-389): voting members (remotes + witnesses) / 2 + 1
template <int R>
DRB_DEV uint32_t quorum_of(const Lane &L) {
  return L.members ? L.v->quorum : (uint32_t)(R / 2 + 1);
}
// a nonVoting or witness replica's state (raft.go:973-999)
DRB_DEV bool passive_role(uint32_t role) {
  return role == DRB_NONVOTING || role == DRB_WITNESS;
}
// the remote-dirty bit 3 of every nonVoting slot (RemLds.dirty nibbles)
DRB_DEV uint32_t nv_bits8(uint32_t nv_mask) {
  uint32_t b = 0;
#pragma unroll
  for (int s = 0; s < 8; ++s)
    if ((nv_mask >> s) & 1u) b |= 8u << (4 * s);
  return b;
}
// isSingleNodeQuorum (raft.go:391-393): quorum over the voting members
template <int R>
DRB_DEV bool single_quorum(const Lane &L) {
  return R == 1 || (nv_mask_of(L) && quorum_of<R>(L) == 1);
}

// ------------------------------------------------------------ remote FSM
// The remotes live in registers; a runtime slot index selects through a
// short chain of v_cndmask instead of indexing an array (which would put
// the whole array in scratch memory).
struct RemoteV {
  uint64_t m, n;
  uint32_t st, a;
};

template <int R>
DRB_DEV RemLds<R> &rl_of(const Lane &L) {
  return *(RemLds<R> *)L.rl;
}

template <int R>
DRB_DEV RemoteV rem_get(const Lane &L, int s) {
  RemLds<R> &t = rl_of<R>(L);
  return RemoteV{t.m[s][L.tid], t.n[s][L.tid], t.st[s][L.tid],
                 t.a[s][L.tid]};
}

template <int R>
DRB_DEV void rem_put(const Lane &L, int s, const RemoteV &x) {
  RemLds<R> &t = rl_of<R>(L);
  if (L.dirty) {  // EXT (C5): only changed fields go back to HBM
    const uint32_t d = (t.m[s][L.tid] != x.m ? 1u : 0u) |
                       (t.n[s][L.tid] != x.n ? 2u : 0u) |
                       (t.st[s][L.tid] != x.st ? 4u : 0u) |
                       (t.a[s][L.tid] != x.a ? 8u : 0u);
    if (d) t.dirty[L.tid] |= d << (4 * s);
  }
  t.m[s][L.tid] = x.m;
  t.n[s][L.tid] = x.n;
  t.st[s][L.tid] = x.st;
  t.a[s][L.tid] = x.a;
}

// remote.go:103-213 on a local copy
DRB_DEV void rv_wait_to_retry(RemoteV &x) {
  if (x.st == DRB_REMOTE_WAIT) x.st = DRB_REMOTE_RETRY;
}
DRB_DEV bool rv_is_paused(const RemoteV &x) {
  return x.st == DRB_REMOTE_WAIT || x.st == DRB_REMOTE_SNAPSHOT;
}
DRB_DEV bool rv_try_update(RemoteV &x, uint64_t index) {
  if (x.n < index + 1) x.n = index + 1;
  if (x.m < index) {
    rv_wait_to_retry(x);
    x.m = index;
    return true;
  }
  return false;
}

template <int R>
DRB_DEV bool rem_try_update(const Lane &L, int s, uint64_t index) {
  RemoteV x = rem_get<R>(L, s);
  bool u = rv_try_update(x, index);
  rem_put<R>(L, s, x);
  return u;
}

// A remote plane (pair_remote) as the step reads it: the inbound copy the
// exchange wrote, or -- engines bound for the zero-copy exchange
// (View.peers) -- the sender rank's outbox itself
DRB_DEV const PeerPlanes *in_peer(const Lane &L, uint32_t from, uint32_t to) {
  const View &v = *L.v;
  return DRB_PEERS && L.peers && v.peers ? &v.peers[plane_sender(v, from, to)]
                                         : nullptr;
}
DRB_DEV const uint4 *in_mbox(const Lane &L, uint32_t from, uint32_t to) {
  const PeerPlanes *q = in_peer(L, from, to);
  return q ? q->mbox : L.v->mbox_in;
}
DRB_DEV const uint4 *in_meta(const Lane &L, uint32_t from, uint32_t to) {
  const PeerPlanes *q = in_peer(L, from, to);
  return q ? q->meta : L.v->meta_in;
}
DRB_DEV const uint4 *in_embox(const Lane &L, uint32_t from, uint32_t to) {
  const PeerPlanes *q = in_peer(L, from, to);
  return q ? q->embox : L.v->embox_in;
}
DRB_DEV const uint64_t *in_maxapp(const Lane &L, uint32_t from, uint32_t to) {
  const PeerPlanes *q = in_peer(L, from, to);
  return q ? q->maxapp : L.v->maxapp_in;
}
DRB_DEV const uint64_t *in_elo(const Lane &L, uint32_t from, uint32_t to) {
  const PeerPlanes *q = in_peer(L, from, to);
  return q ? q->elo : L.v->elo_in;
}
DRB_DEV const uint64_t *in_rterm(const Lane &L, uint32_t from, uint32_t to) {
  const PeerPlanes *q = in_peer(L, from, to);
  return q ? q->rterm : L.v->rterm_in;
}

// ------------------------------------------------------------ log
// commitTo (logentry.go:336-349)
// The lowest next the round's ReplicateResps from remote s can leave it
// at (pre-pass): a reject goes back to match + 1 in Replicate state, else
// to max(1, min(LogIndex, Hint + 1)) (decreaseTo, remote.go:182-198); an
// accepted one to max(match, LogIndex) + 1 (tryUpdate + respondedTo,
// remote.go:143-176) -- a fresh leader's remotes (match 0) get their
// floors from the answers, not from 1.
template <int R>
DRB_DEV uint64_t resp_floor(const Lane &L, const RemoteV &x, int s,
                            uint32_t ns) {
  const View &v = *L.v;
  const bool rm = pair_remote(v, s, L.slot);
  const uint4 *mb = rm ? in_mbox(L, s, L.slot) : v.mbox;
  const uint32_t nrp = mi_nrep(
      (rm ? in_meta(L, s, L.slot) : v.mbox_meta)[mmeta_ix(v, L.rbuf, s, L.slot, L.g)].y);
  uint64_t f = x.n;
  for (uint32_t j = nrp; j < ns; ++j) {
    const uint32_t k = rec_pos(false, j - nrp, v.MB);
    const uint4 c0 = mb[mbox_ix(v, L.rbuf, s, L.slot, k, 0, L.g)];
    if ((c0.x & 0xffu) != DRB_MSG_REPLICATE_RESP) continue;
    const uint64_t idx = hi64(c0);
    uint64_t c;
    if (c0.x & MF_REJECT) {
      const uint64_t hint =
          (c0.x & MF_HAS_C1) ? lo64(mb[mbox_ix(v, L.rbuf, s, L.slot, k, 1, L.g)])
                             : 0;
      c = umin64(x.m + 1, umax64(1, umin64(idx, hint + 1)));
    } else {
      c = umax64(x.m, idx) + 1;
    }
    f = umin64(f, c);
  }
  return f;
}

template <int R>
DRB_DEV void commit_to(Rep<R> &r, uint64_t index) {
  if (index <= r.committed) return;
  if (index > r.last) {
    set_error(r, DRB_ERR_COMMIT);
    return;
  }
  r.committed = index;
}

// sendReplicateMessage (raft.go:787-819) + makeReplicateMessage (738-769)
template <int R>
DRB_DEV void send_replicate(const Lane &L, Rep<R> &r, int to) {
  RemoteV x = rem_get<R>(L, to);
  if (rv_is_paused(x)) return;
  const uint64_t next = x.n;
  Msg m = {};
  m.type = DRB_MSG_REPLICATE;
  m.log_index = next - 1;
  m.log_term = log_term(L, r, next - 1);
  m.commit = r.committed;
  // entries(next, maxEntrySize): [next, last]; limitSize never binds in the
  // resident window (W * (128 + cmd_cap) < 64 MiB, checked at create)
  uint64_t n = next <= r.last ? r.last - next + 1 : 0;
  if (n > 0) {
    if (next < r.ring_lo) {  // would come from LogDB (logentry.go:180-195)
      set_error(r, DRB_ERR_LOG_RANGE);
      return;
    }
    m.n = (uint32_t)n;
    r.guard_new = umin64(r.guard_new, next);
    // remote.progress (remote.go:159-168)
    if (x.st == DRB_REMOTE_REPLICATE)
      x.n = r.last + 1;
    else if (x.st == DRB_REMOTE_RETRY)
      x.st = DRB_REMOTE_WAIT;
    rem_put<R>(L, to, x);
  }
  emit(L, r, to, m);
}

// broadcastReplicateMessage (raft.go:821-833)
template <int R>
DRB_DEV void broadcast_replicate(const Lane &L, Rep<R> &r) {
#pragma unroll
  for (int s = 0; s < R; ++s)
    if ((uint32_t)s != L.slot) send_replicate(L, r, s);
}

// broadcastHeartbeatMessageWithHint (raft.go:859-871) + sendHeartbeat
template <int R>
DRB_DEV void broadcast_heartbeat_hint(const Lane &L, Rep<R> &r, uint64_t lo,
                                      uint64_t hi) {
#pragma unroll
  for (int s = 0; s < R; ++s) {
    if ((uint32_t)s == L.slot) continue;
    // the voting members (remotes, witnesses) with the ctx, the nonVotings
    // only without one (raft.go:859-871)
    if (is_nonvoting(L, (uint32_t)s) && (lo | hi) != 0) continue;
    Msg m = {};
    m.type = DRB_MSG_HEARTBEAT;
    m.commit = umin64(rem_get<R>(L, s).m, r.committed);
    m.hint = lo;
    m.hint_high = hi;
    emit(L, r, s, m);
  }
}

// broadcastHeartbeatMessage (raft.go:849-857)
template <int R>
DRB_DEV void broadcast_heartbeat(const Lane &L, Rep<R> &r) {
  uint64_t lo = 0, hi = 0;
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d)
    if ((uint32_t)d + 1 == r.ri_count) {  // peepCtx: last queued
      lo = rq_lo(L, d);
      hi = rq_hi(L, d);
    }
  broadcast_heartbeat_hint(L, r, lo, hi);
}

// sortMatchValues + tryCommit (raft.go:884-942): quorum-th largest match
template <int R>
DRB_DEV bool try_commit(const Lane &L, Rep<R> &r) {
  // the remotes' and witnesses' matches (raft.go:917-924); a nonVoting's
  // counts as 0, which sorts below them and leaves the quorum-th largest
  // voting match at m[R - quorum]
  uint64_t m[R];
#pragma unroll
  for (int s = 0; s < R; ++s)
    m[s] = is_nonvoting(L, (uint32_t)s) ? 0 : rl_of<R>(L).m[s][L.tid];
  // sorting network (odd-even transposition), ascending
#pragma unroll
  for (int p = 0; p < R; ++p)
#pragma unroll
    for (int i = (p & 1); i + 1 < R; i += 2) {
      uint64_t a = m[i], b = m[i + 1];
      m[i] = umin64(a, b);
      m[i + 1] = umax64(a, b);
    }
  uint64_t q = m[R - (R / 2 + 1)];  // the quorum without nonVotings
  if (nv_mask_of(L)) {
#pragma unroll
    for (int s = 0; s < R; ++s)
      if ((uint32_t)s == R - quorum_of<R>(L)) q = m[s];
  }
  // entryLog.tryCommit (logentry.go:395-410)
  if (q <= r.committed) return false;
  uint64_t lterm = log_term(L, r, q);
  if (lterm == r.term) {
    commit_to(r, q);
    return true;
  }
  return false;
}

// addReadyToRead (raft.go:1833-1839): written straight to the round output
template <int R>
DRB_DEV void add_ready(const Lane &L, Rep<R> &r, uint64_t index, uint64_t lo,
                       uint64_t hi) {
  const View &v = *L.v;
  if (r.nrtr >= RTR_CAP) {
    set_error(r, DRB_FB_CAPACITY);
    return;
  }
  v.rtr[rtr_ix(v, L.slot, r.nrtr, 0, L.g)] = mk4(index, lo);
  v.rtr[rtr_ix(v, L.slot, r.nrtr, 1, L.g)] = mk4(hi, 0);
  r.nrtr++;
}

// readIndex.addRequest (readindex.go:43-66)
template <int R>
DRB_DEV void ri_add_request(const Lane &L, Rep<R> &r, uint64_t index,
                            uint64_t lo, uint64_t hi, uint64_t from) {
  bool found = false;
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d)
    if ((uint32_t)d < r.ri_count && rq_lo(L, d) == lo && rq_hi(L, d) == hi)
      found = true;
  if (found) return;
  uint64_t tail_index = 0;
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d)
    if ((uint32_t)d + 1 == r.ri_count) tail_index = r.ri_ix[d];
  if (r.ri_count > 0 && index < tail_index) {
    set_error(r, DRB_ERR_READINDEX);
    return;
  }
  if (r.ri_count >= DRB_RI_DEPTH) {  // excluded by the pre-pass
    set_error(r, DRB_FB_CAPACITY);
    return;
  }
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d)
    if ((uint32_t)d == r.ri_count) {
      rq_lo(L, d) = lo;
      rq_hi(L, d) = hi;
      r.ri_ix[d] = index;
      r.ri_fr[d] = (uint32_t)from;
      r.ri_cf[d] = 0;
    }
  r.ri_count++;
}

// handleReadIndexLeaderConfirmation (raft.go:1955-1974) +
// readIndex.confirm (readindex.go:77-115)
template <int R>
DRB_DEV void ri_confirm(const Lane &L, Rep<R> &r, uint64_t lo, uint64_t hi,
                        uint32_t from_slot) {
  int pos = -1;
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d)
    if (pos < 0 && (uint32_t)d < r.ri_count && rq_lo(L, d) == lo &&
        rq_hi(L, d) == hi)
      pos = d;
  if (pos < 0) return;
  uint32_t cf = 0;
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d)
    if (d == pos) {
      r.ri_cf[d] |= 1u << from_slot;
      cf = r.ri_cf[d];
    }
  // the voting members' quorum (a nonVoting is sent no ctx to confirm)
  if ((int)__builtin_popcount(cf) + 1 < (int)quorum_of<R>(L)) return;
  uint64_t sidx = 0;
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d)
    if (d == pos) sidx = r.ri_ix[d];
  // release queue[0..pos], each with index rewritten to sidx
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d) {
    if (d > pos) continue;
    if (r.ri_ix[d] > sidx) set_error(r, DRB_ERR_READINDEX);
    uint64_t fr = r.ri_fr[d];
    if (fr == 0 || fr == (uint64_t)L.slot + 1) {
      add_ready(L, r, sidx, rq_lo(L, d), rq_hi(L, d));
    } else {
      Msg m = {};
      m.type = DRB_MSG_READ_INDEX_RESP;
      m.log_index = sidx;
      m.hint = lo;  // the confirming ctx (raft.go:1966-1970)
      m.hint_high = hi;
      emit(L, r, (uint32_t)(fr - 1), m);
    }
  }
  // shift the remaining queue down by pos+1
  uint32_t done = (uint32_t)pos + 1;
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d) {
    uint64_t nl = 0, nh = 0, ni = 0;
    uint32_t nf = 0, nc = 0;
#pragma unroll
    for (int e = 0; e < DRB_RI_DEPTH; ++e)
      if ((uint32_t)e == (uint32_t)d + done) {
        nl = rq_lo(L, e);
        nh = rq_hi(L, e);
        ni = r.ri_ix[e];
        nf = r.ri_fr[e];
        nc = r.ri_cf[e];
      }
    rq_lo(L, d) = nl;
    rq_hi(L, d) = nh;
    r.ri_ix[d] = ni;
    r.ri_fr[d] = nf;
    r.ri_cf[d] = nc;
  }
  r.ri_count -= done;
}

// ------------------------------------------------------------ handlers
// handleLeaderReplicateResp (raft.go:1878-1908), via lw (2309-2323)
// BC = false: a commit advance is returned in *bc for the caller's
// broadcast (the last thing the handler does), so one broadcast site
// serves it and handleLeaderPropose (dispatch)
template <int R, bool BC = true>
DRB_DEV bool leader_replicate_resp(const Lane &L, Rep<R> &r, int s,
                                   const Msg &m, bool *bc = nullptr) {
  RemoteV x = rem_get<R>(L, s);
  x.a = 1;  // setActive
  bool upd = false;
  if (!m.reject) {
    bool paused = rv_is_paused(x);
    upd = rv_try_update(x, m.log_index);
    if (upd && x.st == DRB_REMOTE_RETRY) {  // respondedTo (remote.go:170)
      x.n = x.m + 1;                        // becomeReplicate
      x.st = DRB_REMOTE_REPLICATE;
    }
    rem_put<R>(L, s, x);
    if (upd) {
      if (try_commit(L, r)) {
        if (BC)
          broadcast_replicate(L, r);
        else
          *bc = true;
      } else if (paused) {
        send_replicate(L, r, s);
      }
    }
  } else {
    // decreaseTo (remote.go:182-198)
    bool dec = false;
    if (x.st == DRB_REMOTE_REPLICATE) {
      if (m.log_index > x.m) {
        x.n = x.m + 1;
        dec = true;
      }
    } else if (x.n - 1 == m.log_index) {
      rv_wait_to_retry(x);
      x.n = umax64(1, umin64(m.log_index, m.hint + 1));
      dec = true;
    }
    if (dec && x.st == DRB_REMOTE_REPLICATE) {
      // enterRetryState (raft.go:2013-2017): becomeRetry
      x.n = x.m + 1;
      x.st = DRB_REMOTE_RETRY;
    }
    rem_put<R>(L, s, x);
    if (dec) send_replicate(L, r, s);
  }
  return upd;
}

// handleLeaderHeartbeatResp (raft.go:1910-1923)
template <int R>
DRB_DEV void leader_heartbeat_resp(const Lane &L, Rep<R> &r, int s,
                                   const Msg &m) {
  RemoteV x = rem_get<R>(L, s);
  x.a = 1;
  rv_wait_to_retry(x);
  rem_put<R>(L, s, x);
  if (x.m < r.last) send_replicate(L, r, s);
  if (m.hint != 0) ri_confirm(L, r, m.hint, m.hint_high, (uint32_t)s);
}

// hasCommittedEntryAtCurrentTerm (raft.go:1818-1827)
template <int R>
DRB_DEV bool committed_at_term(const Lane &L, Rep<R> &r) {
  return log_term(L, r, r.committed) == r.term;
}

// handleLeaderReadIndex (raft.go:1842-1876)
template <int R>
DRB_DEV void leader_read_index(const Lane &L, Rep<R> &r, uint64_t lo,
                               uint64_t hi, uint64_t from) {
  if (from && is_witness(L, (uint32_t)(from - 1))) {
    return;  // dropped: a witness node (raft.go:1848-1849)
  } else if (!single_quorum<R>(L)) {
    if (!committed_at_term(L, r)) {
      r.ndropped_ri++;  // reportDroppedReadIndex
      return;
    }
    ri_add_request(L, r, r.committed, lo, hi, from);
    broadcast_heartbeat_hint(L, r, lo, hi);
  } else {
    add_ready(L, r, r.committed, lo, hi);
    // a nonVoting requester is answered (raft.go:1863-1873)
    if (R > 1 && from && from != (uint64_t)L.slot + 1 &&
        is_nonvoting(L, (uint32_t)(from - 1))) {
      Msg m = {};
      m.type = DRB_MSG_READ_INDEX_RESP;
      m.log_index = r.committed;
      m.hint = lo;
      m.hint_high = hi;
      emit(L, r, (uint32_t)(from - 1), m);
    }
  }
}

// handleLeaderPropose (raft.go:1794-1815) -> appendEntries (:944-955): the
// n entries of proposal batch ps (staged, or a Propose's forward rows) at
// last + 1.., Term = r.term; the caller then broadcastReplicateMessage
template <int R>
DRB_DEV void append_props(const Lane &L, Rep<R> &r, uint32_t ps, uint32_t n) {
  const View &v = *L.v;
  const uint32_t chunks = PROP_META + v.C16;
  for (uint32_t j = 0; j < n; ++j) {
    const uint64_t idx = r.last + 1 + j;
    const uint4 p0 = v.props[prop_ix(v, ps, j, 0, L.g)];
    const uint4 p1 = v.props[prop_ix(v, ps, j, 1, L.g)];
    const uint4 p2 = v.props[prop_ix(v, ps, j, 2, L.g)];
    v.ring[ring_ix(v, L.slot, idx, 0, L.g)] = mk4(r.term, lo64(p0));
    v.ring[ring_ix(v, L.slot, idx, 1, L.g)] = mk4(hi64(p0), lo64(p1));
    v.ring[ring_ix(v, L.slot, idx, 2, L.g)] = make_uint4(p1.z, p1.w, p2.x, p2.y);
    for (uint32_t c = PROP_META; c < chunks; ++c)
      v.ring[ring_ix(v, L.slot, idx, c, L.g)] = v.props[prop_ix(v, ps, j, c, L.g)];
  }
  r.last += n;
  if (r.last + 1 > v.W) r.ring_lo = umax64(r.ring_lo, r.last + 1 - v.W);
  rem_try_update<R>(L, (int)L.slot, r.last);  // self remote
  if (single_quorum<R>(L)) try_commit(L, r);
}

// handleFollowerPropose (raft.go:2103-2116): the entry queue goes to the
// leader as a Propose (From = self, Term 0: a request type) carrying the
// entries by value in this replica's forward rows; dropped without a leader
template <int R>
DRB_DEV void forward_props(const Lane &L, Rep<R> &r, uint32_t ps, uint32_t n) {
  const View &v = *L.v;
  if (r.leader_id == 0 || r.leader_id > (uint64_t)R) {
    r.ndropped_props += n;  // reportDroppedProposal
    return;
  }
  const uint32_t chunks = PROP_META + v.C16;
  const uint32_t fw = fwd_ps(v, L.wbuf, L.slot);
  for (uint32_t j = 0; j < n; ++j)
    for (uint32_t c = 0; c < chunks; ++c)
      v.props[prop_ix(v, fw, j, c, L.g)] = v.props[prop_ix(v, ps, j, c, L.g)];
  Msg m = {};
  m.type = DRB_MSG_PROPOSE;
  m.n = n;
  emit(L, r, (uint32_t)(r.leader_id - 1), m);
}

// Where the entries of a Replicate from sender slot s are read: the
// sender's window when it is co-resident (the ring guard keeps them
// resident until the follower has read them), else the entry rows that
// came with the sender's plane (entry index lo at row 0).
struct EntSrc {
  bool remote;
  uint64_t lo;
};
DRB_DEV uint4 ent_chunk(const Lane &L, const EntSrc &src, uint32_t s,
                        uint64_t idx, uint32_t c) {
  const View &v = *L.v;
  if (src.remote)
    return in_embox(L, s, L.slot)[embox_ix(
        v, L.rbuf, s, L.slot, (uint32_t)(idx - src.lo), c, L.g)];
  return v.ring[ring_ix(v, s, idx, c, L.g)];
}

// handleFollowerReplicate (raft.go:2122) -> handleReplicateMessage
// (raft.go:1444-1484) -> tryAppend (logentry.go:296-310) -> merge
// (inmemory.go:199-230)
template <int R>
DRB_DEV void follower_replicate(const Lane &L, Rep<R> &r, int s,
                                const Msg &m, const EntSrc &src) {
  const View &v = *L.v;
  r.election_tick = 0;  // leaderIsAvailable
  set_leader(r, (uint64_t)s + 1);
  r.leader_update = true;
  Msg resp = {};
  resp.type = DRB_MSG_REPLICATE_RESP;
  if (m.log_index < r.committed) {
    resp.log_index = r.committed;
    emit(L, r, s, resp);
    return;
  }
  if (log_term(L, r, m.log_index) == m.log_term) {
    // getConflictIndex: first entry whose term differs
    uint64_t ci = 0;
    for (uint32_t i = 0; i < m.n; ++i) {
      uint64_t idx = m.log_index + 1 + i;
      uint64_t et = lo64(ent_chunk(L, src, (uint32_t)s, idx, 0));
      if (log_term(L, r, idx) != et) {
        ci = idx;
        break;
      }
    }
    if (ci != 0) {
      // tryAppend / append (logentry.go:296-321) panic when a committed
      // entry would change; unreachable here (LogIndex >= committed, see
      // above) but kept as the invariant it is
      if (ci <= r.committed) {
        set_error(r, DRB_ERR_APPEND);
        return;
      }
      uint64_t new_last = m.log_index + m.n;
      uint64_t first_term = lo64(ent_chunk(L, src, (uint32_t)s, ci, 0));
      bool inmem_nonempty = r.last >= r.marker;
      if (ci == r.marker + (inmem_nonempty ? r.last - r.marker + 1 : 0)) {
        // append at the end: checkEntriesToAppend(existing, ents)
        if (inmem_nonempty && log_term(L, r, r.last) > first_term)
          set_error(r, DRB_ERR_APPEND);
      } else if (ci <= r.marker) {
        r.marker = ci;
        r.saved_to = ci - 1;
      } else {
        // keep [marker, ci) then append
        if (ci - 1 > r.last) {
          set_error(r, DRB_ERR_APPEND);
          return;
        }
        if (log_term(L, r, ci - 1) > first_term)
          set_error(r, DRB_ERR_APPEND);
        r.saved_to = umin64(r.saved_to, ci - 1);
      }
      // copy entries [ci, new_last] from the leader's window; keep the
      // [term_start, last] == r.term invariant (terms never decrease
      // along a log and never exceed the leader's term)
      const uint32_t chunks = ENT_META + v.C16;
      // a witness keeps metadata entries: Index and Term, config changes as
      // they are (makeMetadataEntries, raft.go:771-785; the leader's send)
      const bool wt = is_witness(L, L.slot);
      uint64_t ts = new_last + 1;
      for (uint64_t idx = ci; idx <= new_last; ++idx) {
        uint4 m0 = ent_chunk(L, src, (uint32_t)s, idx, 0);
        if (ts > new_last && lo64(m0) == r.term) ts = idx;
        if (wt) {
          const uint4 m2 = ent_chunk(L, src, (uint32_t)s, idx, 2);
          if (m2.z != DRB_ENTRY_CONFIG_CHANGE) {
            m0.z = m0.w = 0;  // key
            v.ring[ring_ix(v, L.slot, idx, 0, L.g)] = m0;
            v.ring[ring_ix(v, L.slot, idx, 1, L.g)] = make_uint4(0, 0, 0, 0);
            v.ring[ring_ix(v, L.slot, idx, 2, L.g)] =
                make_uint4(0, 0, DRB_ENTRY_METADATA, 0);
            continue;
          }
        }
        v.ring[ring_ix(v, L.slot, idx, 0, L.g)] = m0;
        for (uint32_t c = 1; c < chunks; ++c)
          v.ring[ring_ix(v, L.slot, idx, c, L.g)] =
              ent_chunk(L, src, (uint32_t)s, idx, c);
      }
      if (ci <= r.term_start) r.term_start = ts;
      r.last = new_last;
      if (new_last + 1 > v.W) r.ring_lo = umax64(r.ring_lo, new_last + 1 - v.W);
    }
    uint64_t last_idx = m.log_index + m.n;
    commit_to(r, umin64(last_idx, m.commit));
    resp.log_index = last_idx;
  } else {
    resp.reject = 1;
    resp.log_index = m.log_index;
    resp.hint = r.last;
  }
  emit(L, r, s, resp);
}

// handleFollowerHeartbeat (raft.go:2128) -> handleHeartbeatMessage (1400)
template <int R>
DRB_DEV void follower_heartbeat(const Lane &L, Rep<R> &r, int s,
                                const Msg &m) {
  r.election_tick = 0;
  set_leader(r, (uint64_t)s + 1);
  r.leader_update = true;
  commit_to(r, m.commit);
  Msg resp = {};
  resp.type = DRB_MSG_HEARTBEAT_RESP;
  resp.hint = m.hint;
  resp.hint_high = m.hint_high;
  emit(L, r, s, resp);
}

// handleFollowerReadIndex (raft.go:2134-2144): forwarded to the leader
// (From = self, Term 0: a request type, raft.go:667-687)
template <int R>
DRB_DEV void follower_read_index(const Lane &L, Rep<R> &r, uint64_t lo,
                                 uint64_t hi) {
  if (r.leader_id == 0 || r.leader_id > (uint64_t)R) {
    r.ndropped_ri++;  // reportDroppedReadIndex
    return;
  }
  Msg m = {};
  m.type = DRB_MSG_READ_INDEX;
  m.hint = lo;
  m.hint_high = hi;
  emit(L, r, (uint32_t)(r.leader_id - 1), m);
}

// handleFollowerReadIndexResp (raft.go:2155-2164)
template <int R>
DRB_DEV void follower_read_index_resp(const Lane &L, Rep<R> &r, int s,
                                      const Msg &m) {
  r.election_tick = 0;
  set_leader(r, (uint64_t)s + 1);
  r.leader_update = true;
  add_ready(L, r, m.log_index, m.hint, m.hint_high);
}

// FWD: the instantiation carries forwarded proposals (EXT; an engine with
// drb_config.forward_proposals runs it, drb_engine.hip launch_step)
template <int R, bool FWD = true>
DRB_DEV void dispatch(const Lane &L, Rep<R> &r, int s, const Msg &m,
                      const EntSrc &src) {
  if (r.role == DRB_LEADER) {
    bool bc = false;
    if (m.type == DRB_MSG_REPLICATE_RESP) {
      leader_replicate_resp<R, false>(L, r, s, m, &bc);
    } else if (m.type == DRB_MSG_HEARTBEAT_RESP) {
      leader_heartbeat_resp(L, r, s, m);
    } else if (m.type == DRB_MSG_READ_INDEX) {
      leader_read_index(L, r, m.hint, m.hint_high, (uint64_t)s + 1);
    } else if (FWD && m.type == DRB_MSG_PROPOSE) {  // handleLeaderPropose
      append_props(L, r, fwd_ps(*L.v, L.rbuf, (uint32_t)s), m.n);
      bc = true;
    }
    if (bc) broadcast_replicate(L, r);
  } else {
    if (m.type == DRB_MSG_REPLICATE)
      follower_replicate(L, r, s, m, src);
    else if (m.type == DRB_MSG_HEARTBEAT)
      follower_heartbeat(L, r, s, m);
    else if (m.type == DRB_MSG_READ_INDEX_RESP)
      follower_read_index_resp(L, r, s, m);
  }
}

// ------------------------------------------------------------ elections
// The raft launch (drb_config.elections): the state changes
// the step round leaves to the CPU path -- term changes, votes, the
// candidate state, CheckQuorum step-down -- restated from raft.go for the
// replicas the step kernels routed to it (F_SLOW).

// raft.rand -> setRandomizedElectionTimeout (raft.go:658-661): one
// splitmix64 draw from the replica's generator state
template <int R>
DRB_DEV void el_rand_timeout(const Lane &L, Rep<R> &r) {
  const View &v = *L.v;
  uint64_t s = over_ld(L, F_RNG) + 0x9E3779B97F4A7C15ull;
  over_st(L, F_RNG, s);
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  st_f(L, r, F_RAND_TIMEOUT, v.election_rtt + z % v.election_rtt);
}

// a new term: the record's term-relative fields are re-coded against it,
// and no log entry carries it yet (term_start, log_term)
template <int R>
DRB_DEV void el_set_term(const Lane &L, Rep<R> &r, uint64_t t) {
  const uint64_t at = ld_f(L, r, F_APPLIED_TO_TERM);
  const uint64_t pt = ld_f(L, r, F_PREV_TERM);
  const uint64_t smt = r.applied_any ? r.sm_term : ld_f(L, r, F_SM_TERM);
  r.term = t;
  r.pw[2] = (uint32_t)t;
  r.pw[3] = (uint32_t)(t >> 32);
  st_f(L, r, F_APPLIED_TO_TERM, at);
  st_f(L, r, F_PREV_TERM, pt);
  if (!r.applied_any) st_f(L, r, F_SM_TERM, smt);
  r.term_start = r.last + 1;
}

// reset (raft.go:1052-1073) with resetRemotes (raft.go:1088-1097)
template <int R>
DRB_DEV void el_reset(const Lane &L, Rep<R> &r, uint64_t term,
                      bool reset_election) {
  if (r.term != term) {
    el_set_term(L, r, term);
    st_f(L, r, F_VOTE, 0);
  }
  if (reset_election) {
    r.election_tick = 0;
    el_rand_timeout(L, r);
  }
  r.votes = 0;
  r.heartbeat_tick = 0;
  r.ri_count = 0;
  r.flags &= ~F_XFER;  // abortLeaderTransfer (raft.go:1068)
#pragma unroll
  for (int s = 0; s < R; ++s)
    rem_put<R>(L, s,
               RemoteV{(uint32_t)s == L.slot ? r.last : 0, r.last + 1,
                       DRB_REMOTE_RETRY, 0});
}

// becomeFollower / becomeFollowerKE (raft.go:961-999)
template <int R>
DRB_DEV void el_become_follower(const Lane &L, Rep<R> &r, uint64_t term,
                                uint64_t leader, bool reset_election) {
  r.role = DRB_FOLLOWER;
  el_reset(L, r, term, reset_election);
  set_leader(r, leader);
  r.leader_update = true;
}

// becomeLeader (raft.go:1038-1050): the term-start no-op entry
// (appendEntries, raft.go:944-955); config-change entries never reach the
// GPU log, so preLeaderPromotionHandleConfigChange finds none
template <int R>
DRB_DEV void el_become_leader(const Lane &L, Rep<R> &r) {
  const View &v = *L.v;
  r.role = DRB_LEADER;
  el_reset(L, r, r.term, true);
  set_leader(r, (uint64_t)L.slot + 1);
  r.leader_update = true;
  const uint64_t idx = r.last + 1;
  v.ring[ring_ix(v, L.slot, idx, 0, L.g)] = mk4(r.term, 0);
  v.ring[ring_ix(v, L.slot, idx, 1, L.g)] = mk4(0, 0);
  v.ring[ring_ix(v, L.slot, idx, 2, L.g)] = make_uint4(0, 0, 0, 0);
  r.last = idx;
  if (r.last + 1 > v.W) r.ring_lo = umax64(r.ring_lo, r.last + 1 - v.W);
  if (r.term_start > idx) r.term_start = idx;
  rem_try_update<R>(L, (int)L.slot, r.last);  // self remote
  if (single_quorum<R>(L)) try_commit(L, r);
}

// handleVoteResp (raft.go:1125-1147): granted votes so far
template <int R>
DRB_DEV uint32_t el_vote_resp(Rep<R> &r, uint32_t from_slot, bool rejected) {
  if (!((r.votes >> from_slot) & 1u)) {
    r.votes |= 1u << from_slot;
    if (!rejected) r.votes |= 1u << (8 + from_slot);
  }
  return __builtin_popcount(r.votes >> 8);
}

// campaign (raft.go:1176-1217) after becomeCandidate (raft.go:1020-1036);
// xfer: isLeaderTransferTarget -- the RequestVotes name the candidate in
// Hint, which passes the voters' leader lease (raft.go:1192-1196, 1518)
template <int R>
DRB_DEV void el_campaign(const Lane &L, Rep<R> &r, bool xfer = false) {
  r.role = DRB_CANDIDATE;
  el_reset(L, r, r.term + 1, true);
  set_leader(r, 0);
  r.leader_update = true;
  st_f(L, r, F_VOTE, (uint64_t)L.slot + 1);
  el_vote_resp(r, L.slot, false);
  if (single_quorum<R>(L)) {  // a single-node quorum
    el_become_leader(L, r);
    return;
  }
  Msg m = {};
  m.type = DRB_MSG_REQUEST_VOTE;
  m.log_index = r.last;
  m.log_term = log_term(L, r, r.last);
  m.hint = xfer ? (uint64_t)L.slot + 1 : 0;
#pragma unroll
  for (int s = 0; s < R; ++s)  // votingMembers (raft.go:1202)
    if ((uint32_t)s != L.slot && !is_nonvoting(L, (uint32_t)s))
      emit(L, r, (uint32_t)s, m);
}

// preVoteCampaign (raft.go:1149-1174) after becomePreVoteCandidate
// (raft.go:1001-1018): RequestPreVote at term + 1, the term unchanged
template <int R>
DRB_DEV void el_pre_vote_campaign(const Lane &L, Rep<R> &r) {
  r.role = DRB_PREVOTE_CANDIDATE;
  el_reset(L, r, r.term, true);
  set_leader(r, 0);
  r.leader_update = true;
  el_vote_resp(r, L.slot, false);
  if (single_quorum<R>(L)) {  // a single-node quorum
    el_campaign(L, r);
    return;
  }
  Msg m = {};
  m.type = DRB_MSG_REQUEST_PREVOTE;
  m.term = r.term + 1;
  m.log_index = r.last;
  m.log_term = log_term(L, r, r.last);
#pragma unroll
  for (int s = 0; s < R; ++s)  // votingMembers (raft.go:1160)
    if ((uint32_t)s != L.slot && !is_nonvoting(L, (uint32_t)s))
      emit(L, r, (uint32_t)s, m);
}

// handleNodeElection (raft.go:1632-1668): not while a config change may be
// waiting to be applied (hasConfigChangeToApply, raft.go:1611-1622); with
// PreVote the pre-vote round first, unless this replica is a leader
// transfer's target (xfer, raft.go:1659)
template <int R>
DRB_DEV void el_election(const Lane &L, Rep<R> &r, bool xfer = false) {
  if (r.role == DRB_LEADER) return;
  if (r.committed > ld_f(L, r, F_APPLIED)) return;
  if (L.v->pre_vote && !xfer)
    el_pre_vote_campaign(L, r);
  else
    el_campaign(L, r, xfer);
}

// sendTimeoutNowMessage (raft.go:873-878)
template <int R>
DRB_DEV void el_send_timeout_now(const Lane &L, Rep<R> &r, uint32_t to_slot) {
  Msg m = {};
  m.type = DRB_MSG_TIMEOUT_NOW;
  emit(L, r, to_slot, m);
}

DRB_DEV uint32_t xfer_target(uint32_t flags) {
  return (flags & F_XFER) >> F_XFER_SHIFT;
}

// handleLeaderTransfer (raft.go:1925-1953): the target (a replica ID) is
// recorded and, when it already holds the whole log, told to campaign now
template <int R>
DRB_DEV void el_leader_transfer(const Lane &L, Rep<R> &r, uint64_t target) {
  if (target == 0) {  // plog.Panicf: target not set
    set_error(r, DRB_ERR_TRANSFER);
    return;
  }
  if (r.flags & F_XFER) return;                // a transfer is ongoing
  if (target == (uint64_t)L.slot + 1) return;  // pointing to itself
  if (target > (uint64_t)R) return;            // unknown target
  // r.remotes only: a nonVoting or witness is no target (raft.go:1942-1946)
  if (is_nonvoting(L, (uint32_t)target - 1) ||
      is_witness(L, (uint32_t)target - 1))
    return;
  r.flags = (r.flags & ~F_XFER) | ((uint32_t)target << F_XFER_SHIFT);
  r.election_tick = 0;
  if (rem_get<R>(L, (int)target - 1).m == r.last)
    el_send_timeout_now(L, r, (uint32_t)target - 1);
}

// upToDate (logentry.go:381-393)
template <int R>
DRB_DEV bool el_up_to_date(const Lane &L, Rep<R> &r, uint64_t index,
                           uint64_t term) {
  const uint64_t lt = log_term(L, r, r.last);
  return term > lt || (term == lt && index >= r.last);
}

// handleNodeRequestVote (raft.go:1697-1722)
template <int R>
DRB_DEV void el_request_vote(const Lane &L, Rep<R> &r, int s, const Msg &m) {
  const uint64_t vote = ld_f(L, r, F_VOTE);
  const bool can = vote == 0 || vote == (uint64_t)s + 1 || m.term > r.term;
  Msg resp = {};
  resp.type = DRB_MSG_REQUEST_VOTE_RESP;
  if (can && el_up_to_date(L, r, m.log_index, m.log_term)) {
    r.election_tick = 0;
    st_f(L, r, F_VOTE, (uint64_t)s + 1);
  } else {
    resp.reject = 1;
  }
  emit(L, r, (uint32_t)s, resp);
}

// handleNodeRequestPreVote (raft.go:1670-1695): granted at the asked term
// for an up-to-date log, else rejected at r.term
template <int R>
DRB_DEV void el_request_pre_vote(const Lane &L, Rep<R> &r, int s,
                                 const Msg &m) {
  Msg resp = {};
  resp.type = DRB_MSG_REQUEST_PREVOTE_RESP;
  if (m.term > r.term && el_up_to_date(L, r, m.log_index, m.log_term)) {
    resp.term = m.term;
  } else {
    resp.term = r.term;
    resp.reject = 1;
  }
  emit(L, r, (uint32_t)s, resp);
}

// handlePreVoteCandidateRequestPreVoteResp (raft.go:2259-2276)
template <int R>
DRB_DEV void el_pre_vote_resp(const Lane &L, Rep<R> &r, int s, const Msg &m) {
  const uint32_t quorum = quorum_of<R>(L);
  const uint32_t granted = el_vote_resp(r, (uint32_t)s, m.reject != 0);
  const uint32_t answered = __builtin_popcount(r.votes & 0xffu);
  if (granted == quorum)
    el_campaign(L, r);
  else if (answered - granted == quorum)
    el_become_follower(L, r, r.term, 0, true);
}

// handleCandidateRequestVoteResp (raft.go:2235-2253)
template <int R>
DRB_DEV void el_candidate_vote_resp(const Lane &L, Rep<R> &r, int s,
                                    const Msg &m) {
  const uint32_t quorum = quorum_of<R>(L);
  const uint32_t granted = el_vote_resp(r, (uint32_t)s, m.reject != 0);
  const uint32_t answered = __builtin_popcount(r.votes & 0xffu);
  if (granted == quorum) {
    el_become_leader(L, r);
    broadcast_replicate(L, r);
  } else if (answered - granted == quorum) {
    el_become_follower(L, r, r.term, 0, true);
  }
}

DRB_DEV bool el_leader_message(uint32_t t) {  // isLeaderMessage
  return t == DRB_MSG_REPLICATE || t == DRB_MSG_INSTALL_SNAPSHOT ||
         t == DRB_MSG_HEARTBEAT || t == DRB_MSG_TIMEOUT_NOW ||
         t == DRB_MSG_READ_INDEX_RESP;
}

// Handle's term gate (raft.go:1596-1609): onMessageTermNotMatched
// (raft.go:1540-1590) with dropRequestVoteFromHighTermNode (1507-1529);
// true: the message is dropped
template <int R>
DRB_DEV bool el_term_gate(const Lane &L, Rep<R> &r, int s, const Msg &m) {
  const View &v = *L.v;
  if (m.term == 0 || m.term == r.term) return false;
  if ((m.type == DRB_MSG_REQUEST_VOTE || m.type == DRB_MSG_REQUEST_PREVOTE) &&
      v.check_quorum && m.term > r.term && m.hint != (uint64_t)s + 1 &&
      r.leader_id != 0 && r.election_tick < v.election_rtt)
    return true;
  if (m.term > r.term) {
    // isPreVoteMessageWithExpectedHigherTerm (raft.go:1531-1534)
    if (m.type == DRB_MSG_REQUEST_PREVOTE ||
        (m.type == DRB_MSG_REQUEST_PREVOTE_RESP && !m.reject))
      return false;
    const uint64_t leader = el_leader_message(m.type) ? (uint64_t)s + 1 : 0;
    if (r.role == DRB_NONVOTING || r.role == DRB_WITNESS) {
      // becomeNonVoting / becomeWitness (raft.go:973-999)
      el_reset(L, r, m.term, true);
      set_leader(r, leader);
      r.leader_update = true;
      return false;
    }
    el_become_follower(L, r, m.term, leader,
                       m.type != DRB_MSG_REQUEST_VOTE);  // ...KE keeps ticks
    return false;
  }
  if (m.type == DRB_MSG_REQUEST_PREVOTE ||
      (el_leader_message(m.type) && (v.check_quorum || v.pre_vote))) {
    Msg resp = {};
    resp.type = DRB_MSG_NOOP;
    emit(L, r, (uint32_t)s, resp);
  }
  return true;
}

// the handler table (raft.go:2332-2417) for the three states of the path
template <int R>
DRB_DEV void el_dispatch(const Lane &L, Rep<R> &r, int s, const Msg &m,
                         const EntSrc &src) {
  if (el_term_gate(L, r, s, m)) return;
  const uint32_t t = m.type;
  if (t == DRB_MSG_REQUEST_PREVOTE) {  // any state (raft.go:2342-2413)
    el_request_pre_vote(L, r, s, m);
    return;
  }
  if (r.role == DRB_LEADER) {
    if (t == DRB_MSG_REQUEST_VOTE) {
      el_request_vote(L, r, s, m);
    } else if (t == DRB_MSG_LEADER_TRANSFER) {
      el_leader_transfer(L, r, m.hint);
    } else if (t == DRB_MSG_PROPOSE && (r.flags & F_XFER)) {
      r.ndropped_props += m.n;  // leaderTransfering (raft.go:1796-1800)
    } else if (t == DRB_MSG_REPLICATE_RESP) {
      // the transfer target caught up: TimeoutNow (raft.go:1890-1895)
      if (leader_replicate_resp(L, r, s, m) &&
          xfer_target(r.flags) == (uint32_t)s + 1 &&
          rem_get<R>(L, s).m == r.last)
        el_send_timeout_now(L, r, (uint32_t)s);
    } else if (t != DRB_MSG_REQUEST_PREVOTE_RESP) {
      dispatch(L, r, s, m, src);
    }
  } else if (r.role == DRB_NONVOTING || r.role == DRB_WITNESS) {
    // raft.go:2396-2416, re-routed to the follower's handlers
    if (t == DRB_MSG_REQUEST_VOTE)
      el_request_vote(L, r, s, m);
    else if (t == DRB_MSG_REPLICATE || t == DRB_MSG_HEARTBEAT)
      dispatch(L, r, s, m, src);
    else if (r.role == DRB_NONVOTING && t == DRB_MSG_READ_INDEX)
      follower_read_index(L, r, m.hint, m.hint_high);
    else if (r.role == DRB_NONVOTING && t == DRB_MSG_READ_INDEX_RESP)
      dispatch(L, r, s, m, src);
  } else if (r.role == DRB_FOLLOWER) {
    if (t == DRB_MSG_REQUEST_VOTE)
      el_request_vote(L, r, s, m);
    else if (t == DRB_MSG_READ_INDEX)  // handleFollowerReadIndex
      follower_read_index(L, r, m.hint, m.hint_high);
    else if (t == DRB_MSG_LEADER_TRANSFER)
      el_forward_transfer(L, r, m.hint);
    else if (t == DRB_MSG_TIMEOUT_NOW)
      el_timeout_now(L, r);
    else if (t != DRB_MSG_REQUEST_PREVOTE_RESP)
      dispatch(L, r, s, m, src);
  } else {  // candidate, preVoteCandidate
    if (t == DRB_MSG_REPLICATE || t == DRB_MSG_HEARTBEAT) {
      // handleCandidateReplicate / Heartbeat (raft.go:2205-2233)
      el_become_follower(L, r, r.term, (uint64_t)s + 1, true);
      dispatch(L, r, s, m, src);
    } else if (t == DRB_MSG_REQUEST_VOTE_RESP) {
      if (r.role == DRB_CANDIDATE) el_candidate_vote_resp(L, r, s, m);
    } else if (t == DRB_MSG_REQUEST_PREVOTE_RESP) {
      if (r.role == DRB_PREVOTE_CANDIDATE) el_pre_vote_resp(L, r, s, m);
    } else if (t == DRB_MSG_REQUEST_VOTE) {
      el_request_vote(L, r, s, m);
    } else if (t == DRB_MSG_READ_INDEX) {  // handleCandidateReadIndex
      r.ndropped_ri++;
    } else if (t == DRB_MSG_PROPOSE) {  // handleCandidatePropose (2197)
      r.ndropped_props += m.n;
    }
  }
}

// LocalTick (raft.go:571-648) for any role; CheckQuorum (raft.go:1785-1792)
// may step the leader down, and a transfer not done within an election
// timeout is abandoned (timeToAbortLeaderTransfer, raft.go:622-636)
template <int R>
DRB_DEV void el_tick(const Lane &L, Rep<R> &r, bool xfer = false) {
  const View &v = *L.v;
  over_st(L, F_TICK_COUNT, over_ld(L, F_TICK_COUNT) + 1);
  if (r.role == DRB_LEADER) {
    r.election_tick++;
    const bool abort_xfer =
        (r.flags & F_XFER) && r.election_tick >= v.election_rtt;
    if (r.election_tick >= v.election_rtt) {
      r.election_tick = 0;
      if (v.check_quorum) {  // leaderHasQuorum (raft.go:395-405)
        uint32_t c = 0;
#pragma unroll
        for (int s = 0; s < R; ++s) {  // over the voting members
          if (is_nonvoting(L, (uint32_t)s)) continue;
          RemoteV x = rem_get<R>(L, s);
          if ((uint32_t)s == L.slot || x.a) c++;
          x.a = 0;
          rem_put<R>(L, s, x);
        }
        if (c < quorum_of<R>(L)) el_become_follower(L, r, r.term, 0, true);
      }
    }
    if (abort_xfer) r.flags &= ~F_XFER;
    r.heartbeat_tick++;
    if (r.heartbeat_tick >= v.heartbeat_rtt) {
      r.heartbeat_tick = 0;
      if (r.role == DRB_LEADER) broadcast_heartbeat(L, r);
    }
    return;
  }
  r.election_tick++;
  // a nonVoting or witness takes no part in elections (raft.go:596-600)
  if (r.role == DRB_NONVOTING || r.role == DRB_WITNESS) return;
  if (r.election_tick >= ld_f(L, r, F_RAND_TIMEOUT)) {
    r.election_tick = 0;
    el_election(L, r, xfer);
  }
}

// handleFollowerTimeoutNow (raft.go:2172-2185): the clock moving forward
// quickly -- a tick at the election timeout, campaigning without PreVote
template <int R>
DRB_DEV void el_timeout_now(const Lane &L, Rep<R> &r) {
  r.election_tick = ld_f(L, r, F_RAND_TIMEOUT);
  el_tick(L, r, true);
}

// handleFollowerLeaderTransfer (raft.go:2145-2153): to the leader, if known
template <int R>
DRB_DEV void el_forward_transfer(const Lane &L, Rep<R> &r, uint64_t target) {
  if (r.leader_id == 0 || r.leader_id > (uint64_t)R) return;
  Msg m = {};
  m.type = DRB_MSG_LEADER_TRANSFER;
  m.hint = target;
  emit(L, r, (uint32_t)r.leader_id - 1, m);
}

// ------------------------------------------------------------ apply
// FNV-1a over the key bytes, for the open-addressing slot
DRB_DEV uint64_t kv_hash(uint64_t key8, uint32_t klen) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint32_t i = 0; i < klen; ++i)
    h = (h ^ ((key8 >> (8 * i)) & 0xff)) * 0x100000001b3ull;
  return h ^ (h >> 29);
}

// the Cmd staged in four registers-quads (no dynamically indexed arrays:
// those would be placed in scratch memory)
struct Cmd4 {
  uint4 c0, c1, c2, c3;
};

// 32-bit word w (0..15) of the Cmd through a select tree on values (by-
// value operands: a select between two lvalues becomes a select between
// addresses, and the Cmd then lives in scratch memory).
DRB_DEV uint32_t sel(bool c, uint32_t a, uint32_t b) { return c ? a : b; }
DRB_DEV uint32_t sel4(uint32_t w, uint4 q) {
  return sel(w & 2, sel(w & 1, q.w, q.z), sel(w & 1, q.y, q.x));
}
DRB_DEV uint32_t cmd_word(const Cmd4 &c, uint32_t w) {
  const uint32_t a = sel4(w, c.c0), b = sel4(w, c.c1), d = sel4(w, c.c2),
                 e = sel4(w, c.c3);
  const uint32_t x = sel(w & 8, sel(w & 4, e, d), sel(w & 4, b, a));
  return sel(w & 16, 0u, x);
}
DRB_DEV uint32_t cmd_byte(const Cmd4 &c, uint32_t i) {
  return (cmd_word(c, i >> 2) >> (8 * (i & 3))) & 0xffu;
}
// 4 bytes starting at byte offset o (little endian)
DRB_DEV uint32_t cmd_u32_at(const Cmd4 &c, uint32_t o) {
  const uint64_t x = (uint64_t)cmd_word(c, o >> 2) |
                     ((uint64_t)cmd_word(c, (o >> 2) + 1) << 32);
  return (uint32_t)(x >> (8 * (o & 3)));
}
DRB_DEV uint32_t byte_mask(uint32_t n) {  // low n (<= 4) bytes
  return n >= 4 ? 0xffffffffu : ((1u << (8 * n)) - 1u);
}

// 16 bytes at byte offset s (0..15) of the 32-byte window q0 || q1
DRB_DEV uint32_t sel8(uint32_t i, uint4 a, uint4 b) {
  return sel(i & 4, sel4(i, b), sel4(i, a));
}
DRB_DEV uint4 extract16(uint4 q0, uint4 q1, uint32_t s) {
  const uint32_t w = s >> 2, sh = 8 * (s & 3);
  uint32_t o[4];
#pragma unroll
  for (uint32_t t = 0; t < 4; ++t) {
    const uint32_t a = sel8(w + t, q0, q1);
    const uint32_t b = sel8(w + t + 1, q0, q1);  // w + t + 1 <= 7
    o[t] = sh ? (a >> sh) | (b << (32 - sh)) : a;
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}
// keep the low n (0..16) bytes of q
DRB_DEV uint4 mask16(uint4 q, uint32_t n) {
  return make_uint4(q.x & byte_mask(n), q.y & byte_mask(n > 4 ? n - 4 : 0),
                    q.z & byte_mask(n > 8 ? n - 8 : 0),
                    q.w & byte_mask(n > 12 ? n - 12 : 0));
}

// value bytes [16 c + base, 16 c + base + 16) of an entry's PBKV value at
// Cmd offset voff: two ring chunks and a byte shift
DRB_DEV uint4 value_chunk(const Lane &L, uint64_t index, uint32_t voff,
                          uint32_t vlen, uint32_t base, uint32_t c) {
  const View &v = *L.v;
  const uint32_t o = voff + base + 16 * c;  // Cmd byte offset
  const uint32_t q = o >> 4;
  const uint4 q0 = v.ring[ring_ix(v, L.slot, index, ENT_META + q, L.g)];
  const uint4 q1 = q + 1 < v.C16
                       ? v.ring[ring_ix(v, L.slot, index, ENT_META + q + 1, L.g)]
                       : make_uint4(0, 0, 0, 0);
  const uint32_t have = vlen > base + 16 * c ? vlen - base - 16 * c : 0;
  return mask16(extract16(q0, q1, o & 15), have > 16 ? 16 : have);
}

// Values of longer Cmds (C5's 128 B / 1 KB payloads), read 16 B at a time
// from the resident window: into the slot's following chunks (inline) or
// into the key's value block (out of line, allocated on insert).  Only the
// EXT instantiation of the step kernel carries this path.
DRB_DEV bool put_value_long(const View &v, uint32_t slot,
                                            uint64_t g, uint64_t index,
                                            uint4 *sl, bool hit,
                                            uint32_t voff, uint32_t vlen) {
  Lane L;
  L.v = &v;
  L.slot = slot;
  L.g = g;
  if (v.kv_ool) {
    uint32_t blk;
    if (hit) {
      blk = sl[1].x;
    } else {
      const uint64_t b = atomicAdd(v.kv_pool_next, 1ull);
      if (b >= v.kv_pool_blocks) return false;
      blk = (uint32_t)b;
      sl[1] = make_uint4(blk, 0, 0, 0);
    }
    uint4 *dst = v.kv_pool + (uint64_t)blk * v.VB;
    for (uint32_t c = 0; c * 16 < vlen; ++c)
      dst[c] = value_chunk(L, index, voff, vlen, 0, c);
  } else {
    for (uint32_t c = 1; c < v.KVW; ++c)
      sl[c] = value_chunk(L, index, voff, vlen, 4, c - 1);
  }
  return true;
}

// The KV's overflow chain (drb_config.kv_overflow_buckets): a replica
// whose table is full keeps further keys in buckets of 4 slots, newest
// first.  Returns the key's slot (hit) or, with `insert`, a free one -- the
// head bucket's next free slot, or slot 0 of a bucket taken from the pool
// and linked in front -- else null (absent, or the pool is used up).
DRB_DEV uint4 *kv_ovf_walk(const View &v, uint32_t slot, uint64_t g,
                           uint64_t key8, uint32_t klen, bool insert,
                           bool &hit) {
  hit = false;
  uint32_t *const headp = v.kv_ovf_head + ix(v, slot, g);
  uint4 *free_sl = nullptr;
  for (uint32_t b = *headp; b;) {
    uint4 *bk = v.kv_ovf + (uint64_t)(b - 1) * 4 * v.KVW;
    for (uint32_t t = 0; t < 4; ++t) {
      uint4 *sl = bk + (uint64_t)t * v.KVW;
      const uint4 h = sl[0];
      if (!((h.z >> 31) & 1u)) {
        if (!free_sl) free_sl = sl;
      } else if ((h.z & 0xffu) == klen && lo64(h) == key8) {
        hit = true;
        return sl;
      }
    }
    b = v.kv_ovf_next[b - 1];
  }
  if (!insert || free_sl) return free_sl;
  const unsigned long long nb = atomicAdd(v.kv_ovf_used, 1ull);
  if (nb >= v.kv_ovf_cap) return nullptr;
  v.kv_ovf_next[nb] = *headp;
  *headp = (uint32_t)nb + 1;
  return v.kv_ovf + (uint64_t)nb * 4 * v.KVW;
}

// handleEntry (statemachine.go:935-969) -> update (1057-1103) ->
// GetPayload (encoded.go:55-65) -> KVTest.Update (kvtest.go:145-162).
// Returns: 0 noop applied, 1 KV updated, -1 not on the fast path, -2 the
// KV table or the value pool is full.
// The PBKV header is parsed from the Cmd's first 64 bytes (registers); the
// value is copied 16 B at a time straight from the window into the slot
// (inline values) or the slot's value block (out-of-line, kv_val_cap >
// 124: 128 B / 1 KB payloads).
template <int R, bool EXT>
DRB_DEV int apply_entry(const Lane &L, Rep<R> &r, uint64_t index) {
  const View &v = *L.v;
  uint4 m0 = v.ring[ring_ix(v, L.slot, index, 0, L.g)];
  uint4 m1 = v.ring[ring_ix(v, L.slot, index, 1, L.g)];
  uint4 m2 = v.ring[ring_ix(v, L.slot, index, 2, L.g)];
  uint64_t term = lo64(m0);
  uint64_t client_id = lo64(m1), series_id = hi64(m1);
  uint32_t type = m2.z, clen = m2.w;
  if (type == DRB_ENTRY_CONFIG_CHANGE) return -1;
  if (client_id == 0) {  // not session managed
    if (clen != 0) return -1;  // reference panics
    r.sm_index = index;
    r.sm_term = term;
    r.applied_any = true;
    return 0;
  }
  if (series_id != 0) return -1;  // sessions stay on the CPU path
  // the Cmd's first 64 bytes in registers: the PBKV header lies there
  Cmd4 cmd;
  cmd.c0 = v.ring[ring_ix(v, L.slot, index, ENT_META, L.g)];
  cmd.c1 = cmd.c2 = cmd.c3 = make_uint4(0, 0, 0, 0);
  if (v.C16 > 1) cmd.c1 = v.ring[ring_ix(v, L.slot, index, ENT_META + 1, L.g)];
  if (v.C16 > 2) cmd.c2 = v.ring[ring_ix(v, L.slot, index, ENT_META + 2, L.g)];
  if (v.C16 > 3) cmd.c3 = v.ring[ring_ix(v, L.slot, index, ENT_META + 3, L.g)];
  uint32_t off = 0, plen = clen;
  if (type == DRB_ENTRY_ENCODED) {
    if (clen == 0) return -1;
    uint32_t h = cmd_byte(cmd, 0);
    if ((h & 0xf0) != 0 || (h & 0x0e) != 0 || (h & 1)) return -1;
    off = 1;
    plen = clen - 1;
  } else if (type != DRB_ENTRY_APPLICATION) {
    return -1;
  }
  // PBKV.Unmarshal (kvpb/kv.go:76-283): fields 1 (key) and 2 (value),
  // lengths as varints of up to two bytes, headers inside the first 64 B
  uint64_t key8 = 0;
  uint32_t klen = 0, voff = 0, vlen = 0;
  bool have_k = false, have_v = false;
  uint32_t i = 0;
  while (i < plen) {
    if (off + i + 3 > 64) return -1;
    uint32_t tag = cmd_byte(cmd, off + i);
    if (i + 1 >= plen) return -1;
    uint32_t l = cmd_byte(cmd, off + i + 1), hl = 2;
    if (l >= 0x80) {
      const uint32_t b2 = cmd_byte(cmd, off + i + 2);
      if (b2 >= 0x80 || i + 2 >= plen) return -1;
      l = (l & 0x7f) | (b2 << 7);
      hl = 3;
    }
    if (i + hl + l > plen) return -1;
    if (tag == 0x0a) {
      if (l > 8 || off + i + hl + l > 64) return -1;
      const uint32_t ko = off + i + hl;
      key8 = (uint64_t)(cmd_u32_at(cmd, ko) & byte_mask(l)) |
             ((uint64_t)(cmd_u32_at(cmd, ko + 4) &
                         byte_mask(l > 4 ? l - 4 : 0)) << 32);
      klen = l;
      have_k = true;
    } else if (tag == 0x12) {
      if (l > v.kv_val_cap) return -1;
      voff = off + i + hl;
      vlen = l;
      have_v = true;
    } else {
      return -1;
    }
    i += hl + l;
  }
  if (!have_k || !have_v) return -1;
  // the value's first 4 bytes (kept in the slot header word either way)
  const uint32_t w0 =
      (!EXT || voff + 4 <= 64 ? cmd_u32_at(cmd, voff)
                              : value_chunk(L, index, voff, vlen, 0, 0).x) &
      byte_mask(vlen);
  // open-addressing upsert into this replica's table: DRB_PROBE_W slots
  // are loaded per step (one memory round trip), then resolved in order
  const uint32_t home = (uint32_t)kv_hash(key8, klen) & (v.KS - 1);
  uint4 *tbl = v.kv + kv_ix(v, L.slot, L.g, 0);
  for (uint32_t p0 = 0; p0 < v.KS; p0 += DRB_PROBE_W) {
    uint4 hs[DRB_PROBE_W];
#pragma unroll
    for (uint32_t t = 0; t < DRB_PROBE_W; ++t)
      hs[t] = p0 + t < v.KS ? tbl[(uint64_t)kv_probe(v, home, p0 + t) * v.KVW]
                            : make_uint4(0, 0, 0, 1u << 31);
    uint32_t found = DRB_PROBE_W;
    bool hit = false;
#pragma unroll
    for (int t = DRB_PROBE_W - 1; t >= 0; --t) {
      const bool used = (hs[t].z >> 31) & 1u;
      const bool h = used && (hs[t].z & 0xffu) == klen && lo64(hs[t]) == key8;
      const bool pad = p0 + t >= v.KS;
      if (!pad && (!used || h)) {
        found = (uint32_t)t;
        hit = h;
      }
    }
    if (found < DRB_PROBE_W) {
      uint4 *sl = tbl + (uint64_t)kv_probe(v, home, p0 + found) * v.KVW;
      if (!EXT) {
        // inline value of a Cmd inside the 64 B register window: bytes 4..
        // in the slot's following chunks
        for (uint32_t c = 1; c < v.KVW; ++c) {
          uint32_t wv[4];
#pragma unroll
          for (uint32_t t = 0; t < 4; ++t) {
            const uint32_t src = 4 + (c - 1) * 16 + 4 * t;  // value byte
            wv[t] = src < vlen ? cmd_u32_at(cmd, voff + src) &
                                     byte_mask(vlen - src)
                               : 0u;
          }
          sl[c] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        }
      } else if (!put_value_long(v, L.slot, L.g, index, sl, hit, voff,
                                 vlen)) {
        return -2;  // value pool exhausted
      }
      sl[0] = make_uint4((uint32_t)key8, (uint32_t)(key8 >> 32),
                         (1u << 31) | (vlen << 8) | klen, w0);
      r.kv_added++;
      r.sm_index = index;
      r.sm_term = term;
      r.applied_any = true;
      return 1;
    }
  }
  if (EXT && v.kv_ovf_head) {  // the table is full: the overflow chain
    bool hit = false;
    uint4 *sl = kv_ovf_walk(v, L.slot, L.g, key8, klen, true, hit);
    if (sl && put_value_long(v, L.slot, L.g, index, sl, hit, voff, vlen)) {
      sl[0] = make_uint4((uint32_t)key8, (uint32_t)(key8 >> 32),
                         (1u << 31) | (vlen << 8) | klen, w0);
      r.kv_added++;
      r.sm_index = index;
      r.sm_term = term;
      r.applied_any = true;
      return 1;
    }
  }
  return -2;  // table full
}

// ------------------------------------------------------------ saves
// SaveRaftState's input for this replica (engine.go:1343): the round's
// pb.Update.EntriesToSave [lo, hi] (inMemory.entriesToSave,
// inmemory.go:116-122) encoded as one EntryBatch (entrybatch.go:25-58) of
// colfer Entries (raft_optimized.go:166-300) straight from the resident
// window, with its CRC32-IEEE.
// One EntryBatch.Entries element of window entry idx; `compact` writes it
// with Term and Index zero (compactBatchFields, logdb/batch.go:100-113).
DRB_DEV void encode_entry(ByteOut &o, const Lane &L, uint64_t idx,
                          bool compact) {
  const EntryHdr e = ring_entry_hdr(*L.v, L.slot, L.g, idx, compact);
  bo_byte(o, 0x0a);  // EntryBatch.Entries, wire type 2
  bo_varint(o, entry_size(e));
  emit_entry(o, *L.v, L.slot, L.g, idx, e);
}

template <int R>
DRB_DEV void encode_saves(const Lane &L, Rep<R> &r, uint64_t lo, uint64_t hi,
                          const uint32_t *crc_tab, uint32_t &n_ent,
                          uint32_t &n_bytes) {
  const View &v = *L.v;
  ByteOut o;
  bo_init(o, v.save_buf + ix(v, L.slot, L.g) * v.save_cap16, v.save_cap16,
          crc_tab);
  for (uint64_t idx = lo; idx <= hi; ++idx) {
    encode_entry(o, L, idx, false);
    n_ent++;
  }
  const uint32_t crc = bo_finish(o);
  if (o.overflow) {  // bounded by the pre-pass; never expected
    set_error(r, DRB_FB_CAPACITY);
    v.save_len[ix(v, L.slot, L.g)] = 0;
    return;
  }
  v.save_len[ix(v, L.slot, L.g)] = o.total;
  v.save_crc[ix(v, L.slot, L.g)] = crc;
  n_bytes += o.total;
}

// The batched LogDB's records of EntriesToSave [lo, hi]
// (batchedEntries.record / recordBatch, logdb/batch.go:288-346): one
// EntryBatch per batch id = index / 48 touched; the first is merged with
// the batch's entries this replica saved before (getMergedFirstBatch and
// getLastBatch, :115-141, :369-393 -- in a LogDB fed only by these saves
// that is the log from max(batch start, first saved index), resident in
// the window), then compactBatchFields when it holds more than one entry.
// Records start 16 B aligned in the replica's save buffer.
constexpr uint64_t LOGDB_BATCH = 48;  // LogDBEntryBatchSize (hard.go:125)
DRB_DEV uint64_t save_merge_start(uint64_t lo, uint64_t base) {
  const uint64_t b0 = lo / LOGDB_BATCH;
  return lo % LOGDB_BATCH ? umax64(b0 * LOGDB_BATCH, base) : lo;
}

template <int R>
DRB_DEV void encode_save_records(const Lane &L, Rep<R> &r, uint64_t lo,
                                 uint64_t hi, const uint32_t *crc_tab,
                                 uint32_t &n_ent, uint32_t &n_bytes) {
  const View &v = *L.v;
  uint64_t base = over_ld(L, F_SAVE_BASE);
  if (base == 0 || base > lo) {  // the record stream starts here
    base = lo;
    over_st(L, F_SAVE_BASE, base);
  }
  uint4 *buf = v.save_buf + ix(v, L.slot, L.g) * v.save_cap16;
  uint32_t off16 = 0, nrec = 0;
  for (uint64_t b = lo / LOGDB_BATCH; b <= hi / LOGDB_BATCH; ++b) {
    const uint64_t start =
        b == lo / LOGDB_BATCH ? save_merge_start(lo, base) : b * LOGDB_BATCH;
    const uint64_t end = umin64(hi, b * LOGDB_BATCH + LOGDB_BATCH - 1);
    // compactBatchFields: one term from the first entry to the last (the
    // indices are contiguous by construction)
    const bool compact =
        end > start && ring_term<R>(L, L.slot, start) ==
                           ring_term<R>(L, L.slot, end);
    ByteOut o;
    bo_init(o, buf + off16, off16 < v.save_cap16 ? v.save_cap16 - off16 : 0,
            crc_tab);
    for (uint64_t idx = start; idx <= end; ++idx)
      encode_entry(o, L, idx, compact && idx > start);
    const uint32_t crc = bo_finish(o);
    if (o.overflow || nrec >= DRB_SAVE_RECS) {  // bounded by the pre-pass
      set_error(r, DRB_FB_CAPACITY);
      v.save_len[ix(v, L.slot, L.g)] = 0;
      v.save_nrec[ix(v, L.slot, L.g)] = 0;
      return;
    }
    v.save_rec[ix(v, L.slot, L.g) * DRB_SAVE_RECS + nrec] =
        make_uint4((uint32_t)b, off16, o.total, crc);
    nrec++;
    off16 += (o.total + 15) / 16;
    n_bytes += o.total;
  }
  n_ent += (uint32_t)(hi - lo + 1);
  v.save_len[ix(v, L.slot, L.g)] = off16 * 16;
  v.save_crc[ix(v, L.slot, L.g)] = 0;
  v.save_nrec[ix(v, L.slot, L.g)] = nrec;
}

// ------------------------------------------------------------ served reads
// ReadLocalNode for the reads behind each ReadyToRead of the round
// (request.go:930-953 -> KVTest.Lookup kvtest.go:164-175): read j of a
// released ctx {low, high} looks up the 8-byte LE key
// mix64(low ^ (j+1)*GOLDEN) % key_space and folds the slot word
// (found: vlen << 32 | LE32(value), else ~0) into read_sum[slot][g].
// A lookup first reads its first two probes (one 128 B line: kv_probe
// wraps inside the home line), and the lookups of a batch are all issued
// before any is resolved: one memory round trip per batch.
DRB_DEV bool kv_used(uint4 h) { return (h.z >> 31) & 1u; }
DRB_DEV bool kv_match(uint4 h, uint64_t key8, uint32_t klen) {
  return kv_used(h) && (h.z & 0xffu) == klen && lo64(h) == key8;
}
DRB_DEV uint64_t kv_word(uint4 h) {
  const uint32_t vlen = (h.z >> 8) & 0xfffu;
  return ((uint64_t)vlen << 32) | (h.w & byte_mask(vlen));
}
// probes t0 .. KS-1 of home slot `home` (kv_probe), DRB_PROBE_WR slots
// per memory round trip
template <bool OVF>
DRB_DEV uint64_t kv_probe_word(const View &v, const uint4 *tbl, uint32_t home,
                               uint32_t t0, uint64_t key8, uint32_t klen,
                               uint32_t slot, uint64_t g) {
  for (uint32_t p0 = t0; p0 < v.KS; p0 += DRB_PROBE_WR) {
    uint4 hs[DRB_PROBE_WR];
#pragma unroll
    for (uint32_t t = 0; t < DRB_PROBE_WR; ++t)
      hs[t] = p0 + t < v.KS ? tbl[(uint64_t)kv_probe(v, home, p0 + t) * v.KVW]
                            : make_uint4(0, 0, 0, 0);
    // resolved in probe order without leaving the unrolled loop (an early
    // return from it put hs[] in scratch memory)
    uint32_t res = 0;  // 0: go on, 1: an empty slot, 2: found
    uint64_t w = ~0ull;
#pragma unroll
    for (uint32_t t = 0; t < DRB_PROBE_WR; ++t) {
      if (res) continue;
      if (!kv_used(hs[t])) {
        res = 1;  // also the padding past KS
      } else if (kv_match(hs[t], key8, klen)) {
        res = 2;
        w = kv_word(hs[t]);
      }
    }
    if (res) return w;
  }
  if (OVF && v.kv_ovf_head) {  // a full table: the overflow chain
    bool hit = false;
    const uint4 *sl = kv_ovf_walk(v, slot, g, key8, klen, false, hit);
    if (hit) return kv_word(sl[0]);
  }
  return ~0ull;
}

// lookups issued together (each loads its whole first probe group): at the
// steady state's 1/2 load, C3 ran 1.131 ms/round with 3, 1.139 with 5
// (profiles/r03_kvw); 9 spills
#ifndef DRB_READ_BATCH
#define DRB_READ_BATCH 3
#endif
constexpr uint32_t READ_BATCH = DRB_READ_BATCH;

template <bool OVF>
DRB_DEV void serve_reads_lane(const View &v, uint32_t slot, uint64_t g,
                              uint32_t nrtr, uint64_t sm_index,
                              uint32_t n_reads, uint32_t key_space,
                              uint32_t &served, uint32_t &deferred) {
  if (!nrtr) return;
  const uint32_t mask = v.KS - 1;
  const uint4 *tbl = v.kv + kv_ix(v, slot, g, 0);
  const bool ks_pow2 = (key_space & (key_space - 1)) == 0;
  uint64_t sum = 0;
  uint32_t served_mask = 0;
  for (uint32_t k = 0; k < nrtr; ++k) {
    const uint4 c0 = v.rtr[rtr_ix(v, slot, k, 0, g)];
    if (lo64(c0) > sm_index) {  // pendingReadIndex: index not applied yet
      deferred += n_reads;
      continue;
    }
    served_mask |= 1u << k;
    const uint64_t low = hi64(c0);
    for (uint32_t j0 = 0; j0 < n_reads; j0 += READ_BATCH) {
      uint64_t key[READ_BATCH];
      uint32_t ks[READ_BATCH];
      uint4 h[READ_BATCH][DRB_READ_W];
#pragma unroll
      for (uint32_t t = 0; t < READ_BATCH; ++t) {
        const uint64_t x =
            mix64(low ^ ((uint64_t)(j0 + t + 1) * 0x9E3779B97F4A7C15ull));
        key[t] = ks_pow2 ? (x & (key_space - 1)) : x % key_space;
        ks[t] = (uint32_t)kv_hash(key[t], 8) & mask;
        // the first DRB_READ_W probes (one 64 B group): independent loads
        // (plain: with the nontemporal hint the step kernel fetched 7 %
        // more bytes, profiles/r02_kvline)
#pragma unroll
        for (uint32_t q = 0; q < DRB_READ_W; ++q)
          h[t][q] = j0 + t < n_reads && q < v.KS
                        ? tbl[(uint64_t)kv_probe(v, ks[t], q) * v.KVW]
                        : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (uint32_t t = 0; t < READ_BATCH; ++t) {
        const uint32_t j = j0 + t;
        if (j >= n_reads) continue;
        uint64_t w = ~0ull;
        bool done = false;
#pragma unroll
        for (uint32_t q = 0; q < DRB_READ_W; ++q) {
          if (done) continue;
          if (!kv_used(h[t][q])) {
            done = true;  // an empty slot ends the probe sequence
          } else if (kv_match(h[t][q], key[t], 8)) {
            w = kv_word(h[t][q]);
            done = true;
          }
        }
        if (!done && (v.KS > DRB_READ_W || (OVF && v.kv_ovf_head)))
          w = kv_probe_word<OVF>(v, tbl, ks[t], DRB_READ_W, key[t], 8, slot,
                                 g);
        sum += mix64(w ^ key[t] ^ ((uint64_t)j << 56));
        served++;
        if (v.read_res)  // ReadLocalNode's result for the client
        {
          const uint64_t rv =
              w == ~0ull ? 0ull
                         : (w & 0xffffffffull) |
                               ((uint64_t)((uint32_t)(w >> 32) | 0x80000000u)
                                << 32);
          uint64_t *dst = (uint64_t *)&v.read_res[rres_ix(v, slot, k, j, g)];
          // (stored nontemporally they measured the same, profiles/r04_reads)
          *dst = rv;
        }
      }
    }
  }
  v.read_sum[ix(v, slot, g)] = sum;
  if (v.read_res) v.read_served[ix(v, slot, g)] = served_mask;
}

// ------------------------------------------------------------ load/store
template <int R, bool LEAD>
DRB_DEV void load_rep(const Lane &L, Rep<R> &r) {
  const View &v = *L.v;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint4 q = v.pk[pk_ix(v, c, L.slot, L.g)];
    r.pw[4 * c] = q.x;
    r.pw[4 * c + 1] = q.y;
    r.pw[4 * c + 2] = q.z;
    r.pw[4 * c + 3] = q.w;
  }
  r.last = (uint64_t)r.pw[0] | ((uint64_t)r.pw[1] << 32);
  r.term = (uint64_t)r.pw[2] | ((uint64_t)r.pw[3] << 32);
  r.base0 = r.last;
  r.leader_id = pd_get(L, r, 1, F_LEADER_ID);
  r.election_tick = pu_get(L, r, 12, 1, F_ELECTION_TICK);
  if (LEAD) r.heartbeat_tick = pu_get(L, r, 13, 0, F_HEARTBEAT_TICK);
  r.committed = pi_get(L, r, PI_COMMITTED);
  r.processed = pi_get(L, r, PI_PROCESSED);
  r.marker = pi_get(L, r, PI_MARKER);
  r.saved_to = pi_get(L, r, PI_SAVED_TO);
  r.applied_index = pi_get(L, r, PI_APPLIED_INDEX);
  r.sm_index = pi_get(L, r, PI_SM_INDEX);
  r.ring_lo = pi_get(L, r, PI_RING_LO);
  r.ring_guard = pi_get(L, r, PI_RING_GUARD);
  r.term_start = pi_get(L, r, PI_TERM_START);
  r.sm_term = 0;
  r.kv_added = 0;
  r.applied_any = false;
  r.lid_dirty = false;
  r.flags = v.u32[u32_ix(v, W_FLAGS, L.slot, L.g)];
  r.fb = v.u32[u32_ix(v, W_FB_REASON, L.slot, L.g)];
  r.ri_count = v.u32[u32_ix(v, W_RI_COUNT, L.slot, L.g)];
  if (LEAD) {
#pragma unroll
    for (int s = 0; s < R; ++s)
      rem_put<R>(L, s,
                 RemoteV{v.rem_match[rem_ix(v, L.slot, s, L.g)],
                         v.rem_next[rem_ix(v, L.slot, s, L.g)],
                         v.rem_state[rem_ix(v, L.slot, s, L.g)],
                         v.rem_active[rem_ix(v, L.slot, s, L.g)]});
    if (L.dirty) rl_of<R>(L).dirty[L.tid] = 0;
  }
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d) {
    if (LEAD && (uint32_t)d < r.ri_count) {
      uint4 c = v.ri_ctx[ri_ix(v, L.slot, d, L.g)];
      uint4 i = v.ri_idx[ri_ix(v, L.slot, d, L.g)];
      rq_lo(L, d) = lo64(c);
      rq_hi(L, d) = hi64(c);
      r.ri_ix[d] = lo64(i);
      r.ri_fr[d] = (uint32_t)hi64(i);
      r.ri_cf[d] = v.ri_conf[ri_ix(v, L.slot, d, L.g)];
    } else {
      if (LEAD) rq_lo(L, d) = rq_hi(L, d) = 0;
      r.ri_ix[d] = 0;
      r.ri_fr[d] = 0;
      r.ri_cf[d] = 0;
    }
  }
}

template <int R, bool LEAD>
DRB_DEV void store_rep(const Lane &L, Rep<R> &r, uint32_t flags0,
                       uint32_t fb0) {
  const View &v = *L.v;
  // re-base the record on the final last: the cold index fields first
  // (still relative to base0), then the decoded ones
  const uint64_t base = r.last;
#pragma unroll
  for (int i = PI_APPLIED; i < NUM_PI; ++i) {
    const uint32_t c = pk_half(r.pw, 4 + i / 2, i & 1);
    if (c != PK_ESC16)
      pi_put(L, r, i, pk_idx_value(c, r.base0, false), base);
  }
  pi_put(L, r, PI_COMMITTED, r.committed, base);
  pi_put(L, r, PI_PROCESSED, r.processed, base);
  pi_put(L, r, PI_MARKER, r.marker, base);
  pi_put(L, r, PI_SAVED_TO, r.saved_to, base);
  pi_put(L, r, PI_SM_INDEX, r.sm_index, base);
  pi_put(L, r, PI_APPLIED_INDEX, r.applied_index, base);
  pi_put(L, r, PI_RING_LO, r.ring_lo, base);
  pi_put(L, r, PI_RING_GUARD, r.ring_guard, base);
  pi_put(L, r, PI_TERM_START, r.term_start, base);
  // term, vote, prevVote, randomizedElectionTimeout never change on the
  // fast path (a round that would change them falls back first)
  if (r.lid_dirty) pd_put(L, r, 1, F_LEADER_ID, r.leader_id);
  pu_put(L, r, 12, 1, F_ELECTION_TICK, r.election_tick);
  if (LEAD) pu_put(L, r, 13, 0, F_HEARTBEAT_TICK, r.heartbeat_tick);
  if (r.applied_any) pt_put(L, r, 12, 0, F_SM_TERM, r.sm_term);
  if (r.kv_added)
    over_st(L, F_KV_COUNT, over_ld(L, F_KV_COUNT) + r.kv_added);
  r.pw[0] = (uint32_t)r.last;
  r.pw[1] = (uint32_t)(r.last >> 32);
#pragma unroll
  for (int c = 0; c < 4; ++c)
    v.pk[pk_ix(v, c, L.slot, L.g)] =
        make_uint4(r.pw[4 * c], r.pw[4 * c + 1], r.pw[4 * c + 2],
                   r.pw[4 * c + 3]);
  if (r.flags != flags0) v.u32[u32_ix(v, W_FLAGS, L.slot, L.g)] = r.flags;
  if (r.fb != fb0) v.u32[u32_ix(v, W_FB_REASON, L.slot, L.g)] = r.fb;
  if (!LEAD) return;  // followers keep no remotes and no readIndex queue
  v.u32[u32_ix(v, W_RI_COUNT, L.slot, L.g)] = r.ri_count;
  {
    const uint32_t dm = L.dirty ? rl_of<R>(L).dirty[L.tid] : 0xffffffffu;
#pragma unroll
    for (int s = 0; s < R; ++s) {
      const uint32_t d = dm >> (4 * s);
      if (!(d & 15u)) continue;
      RemoteV x = rem_get<R>(L, s);
      if (d & 1u) v.rem_match[rem_ix(v, L.slot, s, L.g)] = x.m;
      if (d & 2u) v.rem_next[rem_ix(v, L.slot, s, L.g)] = x.n;
      if (d & 4u) v.rem_state[rem_ix(v, L.slot, s, L.g)] = x.st;
      if (d & 8u) v.rem_active[rem_ix(v, L.slot, s, L.g)] = x.a;
    }
  }
#pragma unroll
  for (int d = 0; d < DRB_RI_DEPTH; ++d) {
    if ((uint32_t)d >= r.ri_count) continue;
    v.ri_ctx[ri_ix(v, L.slot, d, L.g)] = mk4(rq_lo(L, d), rq_hi(L, d));
    v.ri_idx[ri_ix(v, L.slot, d, L.g)] = mk4(r.ri_ix[d], r.ri_fr[d]);
    v.ri_conf[ri_ix(v, L.slot, d, L.g)] = r.ri_cf[d];
  }
}

// ------------------------------------------------------------ flagged list
// One record per replica newly marked FALLBACK / ERROR (drb_take_flagged);
// rare, so one global atomic per marked lane
DRB_DEV void flag_log(const View &v, uint64_t g, uint32_t slot,
                      uint32_t reason, uint32_t flags, uint64_t round) {
  const unsigned long long i = atomicAdd(v.flog_n, 1ull);
  if (i < v.flog_cap)
    v.flog[i] = make_uint4((uint32_t)g, (uint32_t)(g >> 32),
                           slot | ((reason & 0xffu) << 8) |
                               ((flags & 0xffu) << 16),
                           (uint32_t)round);
}

// ------------------------------------------------------------ the kernel
struct RoundParams {
  uint64_t round;      // t (>= 1)
  uint32_t tick;
  uint32_t prop_slot;  // DRB_NONE: none
  uint32_t ri_slot;    // DRB_NONE: none
  uint32_t n_reads;    // reads served per released ctx (0: none)
  uint32_t key_space;  // served-read key space
  uint32_t encode_saves;
  uint32_t slots;  // slot of block row y = (slots >> 4 * y) & 15
  uint32_t nrows;  // block rows (slots) of this launch; see block_pos
  uint64_t tick_no;  // engine ticks so far, this round's included
  uint32_t ri_replica;  // staged ReadIndex at: 0 the leader, else ID
  uint32_t listed;      // 1: step the active list (k_active_*), see below
  uint32_t prop_replica;  // staged proposals at: 0 the leader, else ID
  // a launch over a chunk of the groups (drb_step_rounds): its first group
  // block, and the engine's group blocks (0: the launch covers them all)
  uint32_t blk0;
  uint32_t gx_all;
  // listed rounds with the lean kernel (drb_lean.hpp): the full EXT kernel
  // steps the heavy part of its row's list (LEAN_HEAVY, concurrently with
  // the lean kernel) or the lanes the lean kernel escalated (LEAN_ESC,
  // after it)
  uint32_t lean;
};

// RoundParams.lean: the full kernel of a lean round steps the heavy part
// of its row's list and the lanes the lean kernel escalated (LEAN_ALL), or
// one of the two (LEAN_HEAVY, LEAN_ESC)
constexpr uint32_t LEAN_HEAVY = 1, LEAN_ESC = 2, LEAN_ALL = 3;

// Whether this replica takes the lane's staged proposals / ReadIndex
// (co-resident: the leader, or replica ri_replica for reads; replicas
// spread over ranks: the stage slot's).
DRB_DEV bool stage_here(const View &v, uint32_t slot, bool lead) {
  return lead && (v.place_world <= 1 || slot == v.stage_slot);
}
DRB_DEV bool ri_here(const View &v, const RoundParams &p, uint32_t slot,
                     bool lead) {
  if (p.ri_slot == DRB_NONE) return false;
  return p.ri_replica == 0 ? stage_here(v, slot, lead)
                           : slot + 1 == p.ri_replica;
}
// the staged proposals: the leader's, or replica prop_replica's (whose
// NodeHost's entry queue they are; a follower forwards them)
DRB_DEV bool prop_here(const View &v, const RoundParams &p, uint32_t slot,
                       bool lead) {
  if (p.prop_slot == DRB_NONE) return false;
  return p.prop_replica == 0 ? stage_here(v, slot, lead)
                             : slot + 1 == p.prop_replica;
}

// Idle rounds: a replica at rest -- its last round left
// nothing pending, see the end of the round -- whose round brings no
// input changes nothing (node.stepNode finds no event, node.go:1139-1159):
// no tick, no staged proposal or ReadIndex, and no record from a
// co-resident sender, which the senders' one-byte round tags tell
// without reading the mailbox headers.  Its round outputs are already
// empty (a round that produced any does not leave the replica at rest).
// With Quiesce on, a quiesced replica at rest also skips tick rounds
// without input: a quiesced tick only advances its tick counters
// (node.tick node.go:1562-1579, raft.quiescedTick raft.go:650-656),
// which the next round it runs applies at once (F_QS_BASE).
// idle_round_of is the same rule over preloaded inputs -- the flags, the
// slot's inbox tag word, the group's staged proposal count and ReadIndex
// row (looked at only where prop_here / ri_here) -- which k_active_scan
// loads all at once; idle_round loads them as the rule needs them.
template <int R>
DRB_DEV bool idle_round_of(const View &v, const RoundParams &p, uint32_t slot,
                           bool lead, uint32_t flags, uint64_t tags,
                           uint32_t pcount, uint4 ri) {
  if (!(flags & F_AT_REST) || v.remote_mask) return false;
  if (p.tick && !(v.quiesce && (flags & F_QUIESCED))) return false;
#pragma unroll
  for (int s = 0; s < R; ++s)
    if ((uint32_t)s != slot &&
        tag_current((uint32_t)(tags >> (8 * s)) & 0xffu, p.round - 1))
      return false;
  if (prop_here(v, p, slot, lead) && pcount != 0) return false;
  if (ri_here(v, p, slot, lead) && (ri.x | ri.y)) return false;
  return true;
}
template <int R>
DRB_DEV bool idle_round(const View &v, const RoundParams &p, uint32_t slot,
                        uint64_t g, bool lead, uint32_t flags) {
  if (!(flags & F_AT_REST) || v.remote_mask) return false;
  if (p.tick && !(v.quiesce && (flags & F_QUIESCED))) return false;
  const uint32_t rbuf = (uint32_t)((p.round - 1) & 1);
  const uint64_t tags = v.inbox_tag[((uint64_t)rbuf * v.R + slot) * v.G + g];
#pragma unroll
  for (int s = 0; s < R; ++s)
    if ((uint32_t)s != slot &&
        tag_current((uint32_t)(tags >> (8 * s)) & 0xffu, p.round - 1))
      return false;
  if (prop_here(v, p, slot, lead) &&
      v.prop_count[(uint64_t)p.prop_slot * v.G + g] != 0)
    return false;
  if (ri_here(v, p, slot, lead) &&
      (v.ri_in[(uint64_t)p.ri_slot * v.G + g].x |
       v.ri_in[(uint64_t)p.ri_slot * v.G + g].y))
    return false;
  return true;
}

// The logical (x = group block, y = slot row) of this workgroup: the launch
// is one-dimensional, gx * nrows workgroups, row-major.  (Rows interleaved
// in runs of 8, so that a group block's follower replicas share an XCD's
// L2, measured neutral at C3 and 7 % slower at C4 N = 1:
// profiles/r01_pair_xcd, r01_c4_pair.)
struct BlockPos {
  uint32_t x, y, gx;
};
DRB_DEV BlockPos block_pos(const RoundParams &p) {
  const uint32_t n = p.nrows ? p.nrows : 1u;
  const uint32_t b = blockIdx.x, gx = gridDim.x / n;
  BlockPos bp;
  // (a chunk's launch: its blocks are group blocks blk0.. of the engine's
  // gx_all, so lanes and counter rows are the full launch's)
  bp.gx = p.gx_all ? p.gx_all : gx;
  bp.y = b / gx;
  bp.x = p.blk0 + b % gx;
  return bp;
}

// Round counters: each workgroup owns one row of NUM_COUNTERS u64 in
// v.counters ([2 roles][R slots][gridDim.x][NUM_COUNTERS]) and adds its
// totals to it with plain loads and stores; drb_read_counters sums the rows.
// (Global atomics from every wave onto 8 shared addresses serialise at the
// memory side -- ~14 ns each -- and were the round's critical path.)
DRB_DEV uint32_t wave_sum(uint32_t x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// counters [FIRST, FIRST + N) of this workgroup's row (256 threads)
template <bool LEAD, int FIRST, int N>
DRB_DEV void block_counters(const View &v, uint32_t slot, BlockPos bp,
                            const uint32_t (&c)[N]) {
  __shared__ uint32_t red[4][N];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint32_t s = wave_sum(c[i]);
    if (lane == 0) red[wave][i] = s;
  }
  __syncthreads();
  if (threadIdx.x < N) {
    const uint32_t i = threadIdx.x;
    const uint64_t s = (uint64_t)red[0][i] + red[1][i] + red[2][i] + red[3][i];
    if (s) {
      const uint64_t row =
          ((uint64_t)(LEAD ? 0 : 1) * v.R + slot) * bp.gx + bp.x;
      // (an atomic: a lean round's kernels run concurrently, and two of
      // them may own the same row; rows are per block, so no contention)
      atomicAdd(&v.counters[row * NUM_COUNTERS + FIRST + i],
                (unsigned long long)s);
    }
  }
}

// one row per workgroup of xrows[role][from][to][block]:
// K | E << 8 | flags << 16 (max, max, or over the block's lanes)
template <bool LEAD>
DRB_DEV void block_plane_summary(const View &v, BlockPos bp, uint32_t from,
                                 uint32_t to, uint32_t Kr, uint32_t Ko,
                                 uint32_t E, uint32_t fl) {
  __shared__ uint32_t red[4][4];
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Kr = max(Kr, (uint32_t)__shfl_xor(Kr, o, 64));
    Ko = max(Ko, (uint32_t)__shfl_xor(Ko, o, 64));
    E = max(E, (uint32_t)__shfl_xor(E, o, 64));
    fl |= (uint32_t)__shfl_xor(fl, o, 64);
  }
  __syncthreads();  // red[] is reused across destinations
  if (lane == 0) {
    red[wave][0] = Kr;
    red[wave][1] = Ko;
    red[wave][2] = E;
    red[wave][3] = fl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t kr = 0, ko = 0, e = 0, f = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      kr = max(kr, red[w][0]);
      ko = max(ko, red[w][1]);
      e = max(e, red[w][2]);
      f |= red[w][3];
    }
    const uint64_t row = (((uint64_t)(LEAD ? 0 : 1) * v.R + from) * v.R + to) *
                             bp.gx + bp.x;
    // the DRB_PLANE_* word of include/drb_engine.h
    v.xrows[row] = kr | (ko << 5) | (e << 10) | (f << 18);
  }
}

// LEAD selects the role this launch steps: the leader kernel takes the
// replicas whose role is LEADER, the follower kernel every other replica
// (non-FOLLOWER roles fall back).  Both read round t-1's mailbox and write
// round t's, so the two launches of a round are independent; compiling the
// roles apart keeps each one's register footprint (and so its occupancy)
// to what its own handlers need.
// EXT: the instantiation for Cmds longer than 64 B, out-of-line values or
// encode_saves (C5); the other one keeps the common path lean
// SLOW: the raft launch of an elections engine (LEAD = EXT = true): it
// steps the replicas on the slow list (F_SLOW) with the election state
// machine (el_*, above) as well, whatever their role.
// FWD: forwarded proposals (drb_config.forward_proposals; an EXT
// instantiation of its own, so C5's EXT kernels keep their registers)
template <int R, bool LEAD, bool EXT, bool SLOW = false, bool FWD = false,
          bool LOCAL = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SLOW ? DRB_SLOW_WAVES : LEAD ? (EXT ? DRB_EXT_LEAD_WAVES : DRB_LEAD_WAVES) : DRB_FOLLOW_WAVES))) void step_kernel(const View v,
                                                   RoundParams p) {
  // the View is a by-value kernel argument: its fields are wave-uniform
  // kernarg loads, and the pointers loaded from it are known to address
  // global memory (global_load/store, not flat: no LDS-counter waits)
  const View *vp = &v;
  const BlockPos bp = block_pos(p);
  // the slots this launch steps (4 bits each): a role's launch covers only
  // the slots where that role occurs (drb_engine.hip role map); the raft
  // launch takes (group, slot) from the slow list
  uint4 slow_e = make_uint4(0, 0, 0, 0);
  if (SLOW) {
    const uint64_t slow_n = umin64(*v.slow_n, v.slow_cap);
    if ((uint64_t)blockIdx.x * blockDim.x >= slow_n) return;  // uniform
    const uint64_t si = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    slow_e = si < slow_n ? v.slow_list[si]
                         : make_uint4(0xffffffffu, 0xffffffffu, 0, 0);
  }
  const uint32_t slot = SLOW ? slow_e.z : (p.slots >> (4 * bp.y)) & 0xfu;
  // Listed rounds step only the replicas k_active_scan found with work,
  // packed in group order into dense waves (drb_engine.hip); the blocks
  // past the list's end have nothing to do.
  const uint64_t lrow = ((uint64_t)(LEAD ? 0 : 1) * v.R + slot);
  const uint64_t li = (uint64_t)bp.x * blockDim.x + threadIdx.x;
  uint64_t nlisted = 0, nheavy = 0, nesc = 0;
  const uint32_t lean = EXT && !SLOW ? p.lean : 0u;
  // (the raft launch takes its lanes from the slow list, listed or not)
  if (!SLOW && p.listed) {  // the heavy part of the row's list, then light
    // (a lean round: the heavy part alone, or the light lanes the lean
    // kernel escalated, from the ESC_SPLIT segments of the row's list)
    nheavy = lean == LEAN_ESC ? 0 : v.act_total[2 * lrow];
    if (lean & LEAN_ESC)
      for (uint32_t k = 0; k < ESC_SPLIT; ++k)
        nesc += v.esc_n[lrow * ESC_SPLIT + k];
    nlisted = nheavy + (lean & LEAN_ESC ? nesc
                        : lean == LEAN_HEAVY ? 0
                                             : v.act_total[2 * lrow + 1]);
    if ((uint64_t)bp.x * blockDim.x >= nlisted) return;  // uniform
  }
  uint64_t g = SLOW ? lo64(slow_e) : li;
  if (!SLOW && p.listed) {
    if (li >= nlisted) {
      g = v.G;
    } else if ((lean & LEAN_ESC) && li >= nheavy) {  // li's segment
      uint64_t x = li - nheavy, k = 0;
      for (; k + 1 < ESC_SPLIT; ++k) {
        const uint32_t c = v.esc_n[lrow * ESC_SPLIT + k];
        if (x < c) break;
        x -= c;
      }
      g = v.esc_list[(lrow * ESC_SPLIT + k) * esc_seg(v.G) + x];
    } else {
      g = v.act_list[lrow * v.G + li];
    }
  }
  __shared__ RemLds<R> rl;
  __shared__ uint32_t oinfo[R * 256];
  __shared__ uint32_t crc_tab[EXT ? 256 : 1];
  __shared__ uint64_t rq_lds[LEAD ? 2 * DRB_RI_DEPTH : 1][256];
  // inbox prefetch (LDS-DMA): PFS senders x PFN records.  One sender row:
  // the LDS destination of global_load_lds goes through M0 and must be
  // wave-uniform, and the row a lane's first sender with records lands in
  // is uniform only while there is one row (the first such sender differs
  // between lanes)
  constexpr int PFN = SLOW || LEAD ? 0 : DRB_FPF;
  constexpr bool FPF = PFN > 0;
  constexpr int PFS = 1;
  // the LDS row of a prefetch goes through M0 (wave-uniform): one sender
  // row only, whose index does not depend on the lane
  static_assert(PFS == 1 || !FPF, "per-lane prefetch rows need PFS == 1");
  __shared__ uint4 pf_lds[FPF ? PFS : 1][FPF ? PFN : 1][FPF ? 256 : 1];
  constexpr int NPH = (DRB_PHASE_PROF && !SLOW) ? 8 : 1;
  __shared__ uint32_t ph_lds[NPH][NPH > 1 ? 256 : 1];
  uint32_t ph_t = 0;
  if (NPH > 1)
#pragma unroll
    for (int i = 0; i < NPH; ++i) ph_lds[i][threadIdx.x] = 0;
#define DRB_PH(i)                                                   \
  do {                                                              \
    if (NPH > 1) {                                                  \
      const uint32_t now = (uint32_t)__builtin_readcyclecounter();  \
      ph_lds[(i) < NPH ? (i) : 0][NPH > 1 ? threadIdx.x : 0] = now - ph_t; \
      ph_t = now;                                                   \
    }                                                               \
  } while (0)
  // placement C4 only: [R][256] (the launch sizes it, drb_step_inst.hip)
  extern __shared__ uint64_t elo_dyn[];
  uint64_t(*elo_lds)[256] = reinterpret_cast<uint64_t(*)[256]>(elo_dyn);
  if (EXT && p.encode_saves) {  // uniform: every thread reaches the barrier
    crc32_table_init(crc_tab, threadIdx.x);
    __syncthreads();
  }
  Lane L;
  L.rl = &rl;
  L.oi = oinfo;
  L.elo = elo_dyn;
  L.rq = &rq_lds[0][0];
  L.tid = threadIdx.x;
  L.v = vp;
  L.slot = slot;
  L.g = g;
  L.round = p.round;
  L.rbuf = (uint32_t)((p.round - 1) & 1);
  L.wbuf = (uint32_t)(p.round & 1);
  L.slow = SLOW;
  L.dirty = EXT && DRB_REM_DIRTY;
  L.members = FWD;
  L.peers = !LOCAL;
  uint32_t c_commit = 0, c_applied = 0, c_fb = 0, c_err = 0, c_msgs = 0;
  uint32_t c_rtr = 0, c_drop = 0;
  uint32_t c_served = 0, c_deferred = 0, c_saved = 0, c_saved_bytes = 0;
  uint32_t c_stepped = 0, c_elect = 0, c_role = 0, c_dprop = 0;
  uint32_t sent_c1 = 0;     // remote planes: destinations given a c1 chunk
  uint32_t qz_out = 0;      // destinations sent a Quiesce message
  uint64_t last_final = 0;  // leader: last index at the end of the round
  bool active = g < v.G;
  uint32_t flags = active ? v.u32[u32_ix(v, W_FLAGS, slot, g)] : 0;
  uint32_t role = active ? v.u32[u32_ix(v, W_ROLE, slot, g)] : 0;
  if (SLOW) {
    if (!(flags & DRB_F_HOSTED) || !(flags & F_SLOW)) active = false;
  } else if (!(flags & DRB_F_HOSTED) || ((role == DRB_LEADER) != LEAD)) {
    // an unhosted replica (stopped, or on another NodeHost) has no round
    // output; the launch of its role clears what an earlier round left
    if (active && !(flags & DRB_F_HOSTED) && (role == DRB_LEADER) == LEAD) {
      v.rtr_count[ix(v, slot, g)] = 0;
      if (p.encode_saves) v.save_len[ix(v, slot, g)] = 0;
    }
    active = false;
  }
  if (active && (flags & (DRB_F_FALLBACK | DRB_F_ERROR))) {
    // left the fast path in an earlier round: no round output
    v.rtr_count[ix(v, slot, g)] = 0;
    if (p.encode_saves) v.save_len[ix(v, slot, g)] = 0;
    active = false;
  }
  if (!SLOW && active && !p.listed &&
      idle_round<R>(v, p, slot, g, LEAD, flags))
    active = false;
  if (active) {
    c_stepped = 1;
    if (NPH > 1) ph_t = (uint32_t)__builtin_readcyclecounter();
    Rep<R> r;
    load_rep<R, LEAD>(L, r);
    r.role = SLOW ? role : LEAD ? DRB_LEADER : DRB_FOLLOWER;
    r.votes = SLOW ? v.u32[u32_ix(v, W_VOTES, slot, g)] : 0u;
    if (SLOW) {  // off the slow list
      r.flags &= ~F_SLOW;
      v.u32[u32_ix(v, W_FLAGS, slot, g)] = r.flags;
      c_elect = 1;
    }
    const uint64_t term0 = r.term;
    const uint32_t role0 = r.role, votes0 = r.votes;
#pragma unroll
    for (int s = 0; s < R; ++s) {
      oinfo[s * 256 + threadIdx.x] = 0;
      if (LEAD && v.remote_mask) elo_lds[s][threadIdx.x] = ~0ull;
    }
    r.c1mask = 0;
    r.hc.lo = r.hc.hi = 0;
    r.hc.dests = 0;
    r.nmsgs = 0;
    r.nrtr = 0;
    r.ndropped_ri = 0;
    r.ndropped_props = 0;
    r.guard_new = ~0ull;
    r.leader_update = false;
    r.oterm = false;
    r.err = false;
    r.qs_new = false;
    const uint32_t flags0 = r.flags, fb0 = r.fb;
    const uint32_t tag_prev = (uint32_t)(p.round - 1);
    const bool qon = EXT && v.quiesce;
    uint64_t qs_owed = 0;
    if (qon) {
      r.qs_tick = over_ld(L, F_QS_TICK);
      r.qs_idle = over_ld(L, F_QS_IDLE);
      r.qs_since = over_ld(L, F_QS_SINCE);
      r.qs_exit = over_ld(L, F_QS_EXIT);
      r.qs_dirty = 0;
      // the quiesced ticks this replica skipped: only a replica that ended
      // its last round quiesced and at rest skips rounds (idle_round), and
      // only such a round stores the base (below)
      if (DRB_QS_EAGER ||
          (flags0 & (F_QUIESCED | F_AT_REST)) == (F_QUIESCED | F_AT_REST))
        qs_owed = p.tick_no - p.tick - over_ld(L, F_QS_BASE);
      r.election_tick += qs_owed;
      r.qs_tick += qs_owed;
    }

    // ---------------------------------------------- pre-pass (read only)
    uint32_t fb = DRB_FB_NONE;
    const bool is_leader = SLOW ? r.role == DRB_LEADER : LEAD;
    if (SLOW) {
      if (role != DRB_LEADER && role != DRB_FOLLOWER && role != DRB_CANDIDATE &&
          role != DRB_PREVOTE_CANDIDATE && !passive_role(role))
        fb = DRB_FB_ROLE;
    } else if (!LEAD && ((role != DRB_FOLLOWER && !passive_role(role)) ||
                         r.ri_count != 0)) {
      fb = DRB_FB_ROLE;
    } else if (flags & (F_XFER | F_XFER_REQ)) {
      fb = DRB_FB_ROLE;  // a leader transfer: the raft launch's
    }
    bool higher_in = false;  // raft launch: a message may raise the term
    bool higher_lead = false;  // ... and one of them is a leader message
    uint32_t n_lt = 0;       // raft launch: LeaderTransfer records
    // the inbox, from the per-sender headers alone (drb_msg.hpp)
    uint64_t nin_packed = 0;  // 5-bit inbox record count per sender
    uint32_t total_in = 0, n_ri_msgs = 0, n_rr = 0, resp_from = 0;
    uint32_t rej_from = 0;  // senders with a rejecting ReplicateResp
    uint32_t qz_from = 0;   // senders whose Quiesce message arrived
    // leader: 5-bit count per sender s of the sends back to s that its own
    // records and queued requests can cause (the mailbox bound below)
    uint64_t own_packed = 0;
    uint64_t max_app = 0;
    uint32_t prop_from = 0;     // senders with a Propose (MI_PROP)
    uint64_t nprop_packed = 0;  // 4-bit forwarded entry count per sender
    uint32_t n_fwd = 0;         // ... and their sum
    int pf_s[2] = {-1, -1};    // the senders whose records are in pf_lds
    uint32_t pf_nrp[2] = {0, 0};  // ... and their Replicate counts
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if ((uint32_t)s == slot) continue;
      const bool rm = pair_remote(v, s, slot);
      const uint4 meta = (rm ? in_meta(L, s, slot) : v.mbox_meta)[mmeta_ix(v, L.rbuf, s,
                                                                 slot, g)];
      const bool cur = tag_is(meta.x, tag_prev);
      const uint32_t info = cur ? meta.y : 0u;
      const uint32_t ns = mi_count(info);
      nin_packed |= (uint64_t)ns << (5 * s);
      if (cur && (meta.x & MQ_QUIESCE)) qz_from |= 1u << s;
      if (SLOW) {
        // the types the raft launch handles (el_dispatch); anything else
        // (snapshots, leader transfer, ...) is the CPU path's
        if (info & (MI_OFF_LEADER | MI_OFF_FOLLOWER)) {
          const uint4 *mb = rm ? in_mbox(L, s, slot) : v.mbox;
          const uint32_t nrp = mi_nrep(info);
          for (uint32_t j = 0; j < ns; ++j) {
            const uint32_t k = rec_pos(j < nrp, j < nrp ? j : j - nrp, v.MB);
            const uint32_t t =
                mb[mbox_ix(v, L.rbuf, s, slot, k, 0, g)].x & 0xffu;
            const bool ok =
                t == DRB_MSG_REPLICATE || t == DRB_MSG_REPLICATE_RESP ||
                t == DRB_MSG_HEARTBEAT || t == DRB_MSG_HEARTBEAT_RESP ||
                t == DRB_MSG_READ_INDEX || t == DRB_MSG_READ_INDEX_RESP ||
                t == DRB_MSG_REQUEST_VOTE || t == DRB_MSG_REQUEST_VOTE_RESP ||
                t == DRB_MSG_NOOP || t == DRB_MSG_LEADER_TRANSFER ||
                t == DRB_MSG_TIMEOUT_NOW ||
                (v.pre_vote && is_prevote_type(t)) ||
                (v.fwd_props && t == DRB_MSG_PROPOSE);
            if (!ok && fb == DRB_FB_NONE) fb = DRB_FB_MESSAGE_TYPE;
            n_lt += t == DRB_MSG_LEADER_TRANSFER;
          }
        }
        const bool hterm = (info & MI_TERM) && hi64(meta) > r.term;
        if (hterm) higher_in = true;
        if (hterm || (info & MI_TERM_OTHER)) {
          // the records above this replica's term: records with a term of
          // their own (rterm), and the leader messages among them -- a
          // leader that steps down for one learns the new leader, and would
          // forward its queued proposals to it (handleFollowerPropose,
          // raft.go:2103-2116); without one it drops them
          const uint4 *mb = rm ? in_mbox(L, s, slot) : v.mbox;
          const uint32_t nrp = mi_nrep(info);
          for (uint32_t j = 0; j < ns; ++j) {
            const uint32_t k = rec_pos(j < nrp, j < nrp ? j : j - nrp, v.MB);
            const uint32_t x = mb[mbox_ix(v, L.rbuf, s, slot, k, 0, g)].x;
            // (a RequestPreVote or a granted pre-vote raises no term,
            // isPreVoteMessageWithExpectedHigherTerm, raft.go:1531-1534)
            const bool pv = (x & 0xffu) == DRB_MSG_REQUEST_PREVOTE ||
                            ((x & 0xffu) == DRB_MSG_REQUEST_PREVOTE_RESP &&
                             !(x & MF_REJECT));
            const uint64_t rt =
                (x & MF_TERM_OTHER)
                    ? (rm ? in_rterm(L, s, slot) : v.rterm)[rterm_ix(v, L.rbuf, s, slot,
                                                           k, g)]
                    : (x & MF_TERM_ZERO) ? 0 : hi64(meta);
            if ((x & MF_TERM_OTHER) && !pv && rt > r.term) higher_in = true;
            if (rt > r.term && el_leader_message(x & 0xffu))
              higher_lead = true;
          }
        }
      } else {
        if ((info & (LEAD ? MI_OFF_LEADER : MI_OFF_FOLLOWER)) &&
            fb == DRB_FB_NONE)
          fb = DRB_FB_MESSAGE_TYPE;
        if (((info & MI_TERM_OTHER) ||
             ((info & MI_TERM) && hi64(meta) != r.term)) &&
            fb == DRB_FB_NONE)
          fb = DRB_FB_TERM_MISMATCH;
      }
      const uint32_t nri_s = (info >> MI_NRI) & 0x1fu;
      const uint32_t nrr_s = (info >> MI_NRR) & 0x1fu;
      n_ri_msgs += nri_s;
      n_rr += nrr_s;
      if (LEAD && is_leader) {
        // the sends to s that s's records cause (raft.go:1878-1923,
        // 1955-1974): a ReadIndexResp per request of s released (queued or
        // new), one answer per HeartbeatResp (and, in the raft launch, per
        // record of another type), and per ReplicateResp a resend only
        // while s is paused -- an accepted answer from Wait resends once and
        // leaves s in Replicate, where only a commit broadcast (counted for
        // every follower below) sends to it; s is paused again only after a
        // reject or a HeartbeatResp (remote.go:103-213)
        const uint32_t hb_s = ns - nri_s - nrr_s - ((info & MI_PROP) ? 1u : 0u);
        const uint32_t w0 =
            rem_get<R>(L, s).st != DRB_REMOTE_REPLICATE ? 1u : 0u;
        const uint32_t rr = (info & MI_REJECT) ? nrr_s : umin32(nrr_s, w0 + hb_s);
        uint32_t riq = 0;
#pragma unroll
        for (int d = 0; d < DRB_RI_DEPTH; ++d)
          riq += ((uint32_t)d < r.ri_count && r.ri_fr[d] == (uint32_t)s + 1u)
                     ? 1u : 0u;
        own_packed |= (uint64_t)umin32(riq + nri_s + hb_s + rr, 31u) << (5 * s);
      }
      if (info & MI_RESP) resp_from |= 1u << s;
      if (info & MI_PROP) {
        prop_from |= 1u << s;
        if (FWD) {
          nprop_packed |= (uint64_t)mi_nprop(info) << (4 * s);
          n_fwd += mi_nprop(info);
        }
      }
      if (info & MI_REJECT) rej_from |= 1u << s;
      if (!is_leader && mi_nrep(info))
        max_app = umax64(max_app, (rm ? in_maxapp(L, s, slot) : v.mbox_maxapp)[mmeta_ix(
                                      v, L.rbuf, s, slot, g)]);
      if (FPF && ns && (pf_s[0] < 0 || (PFS > 1 && pf_s[1] < 0))) {
        // the records go to LDS in one batch; the dispatch loop reads them
        // there (after the wait below)
        const int q = pf_s[0] < 0 ? 0 : 1;
        pf_s[q] = s;
        pf_nrp[q] = mi_nrep(info);
        const uint4 *mb = rm ? in_mbox(L, s, slot) : v.mbox;
#pragma unroll
        for (int j = 0; j < (FPF ? PFN : 1); ++j)
          if ((uint32_t)j < ns) {
            const uint32_t jj = (uint32_t)j, nr = pf_nrp[q];
            const uint32_t k = rec_pos(jj < nr, jj < nr ? jj : jj - nr, v.MB);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(
                    mb + mbox_ix(v, L.rbuf, s, slot, k, 0, g)),
                (__attribute__((address_space(3))) void *)&pf_lds[FPF ? q : 0][
                    FPF ? j : 0][FPF ? threadIdx.x & ~63u : 0],
                16, 0, 0);
          }
      }
      total_in += ns;
    }
    uint32_t nprops = 0;   // staged proposals this replica takes
    uint32_t nappend = 0;  // leader: entries the round may append
    uint64_t in_lo = 0, in_hi = 0;
    // lowest index the round may still read: apply cursor, commit term,
    // applied-to term
    const uint64_t keep_common =
        umin64(umin64(r.processed + 1, r.committed), r.sm_index);
    // staged inputs are per lane: with replicas spread over ranks a lane
    // holds R different groups, and they go to the stage slot's leader
    if (ri_here(v, p, slot, is_leader)) {
      uint4 c = v.ri_in[(uint64_t)p.ri_slot * v.G + g];
      in_lo = lo64(c);
      in_hi = hi64(c);
    }
    if ((FWD || is_leader) && prop_here(v, p, slot, is_leader))
      nprops = v.prop_count[(uint64_t)p.prop_slot * v.G + g];
    if (is_leader) {
      // with elections a group can hold two leaders (a stale one and the
      // new one): its entry queue goes to the hosted leader in the highest
      // slot (the NodeHost the client reaches; tests/gpu_harness.py)
      if (v.elections && nprops && v.place_world <= 1 && !p.prop_replica) {
#pragma unroll
        for (int s = 0; s < R; ++s)
          if ((uint32_t)s > slot &&
              (v.u32[u32_ix(v, W_FLAGS, s, g)] & DRB_F_HOSTED) &&
              v.u32[u32_ix(v, W_ROLE, s, g)] == DRB_LEADER)
            nprops = 0;
      }
      if (r.ri_count + (in_lo != 0) + n_ri_msgs > DRB_RI_DEPTH &&
          fb == DRB_FB_NONE)
        fb = DRB_FB_CAPACITY;
      for (uint32_t j = 0; j < nprops; ++j) {
        // p2 = {type, cmd_len, fast}: the staging side's prop_fast check
        // (drb_layout.hpp) -- config change, session and compressed
        // entries go to the CPU path before anything is appended
        uint4 p2 = v.props[prop_ix(v, p.prop_slot, j, 2, g)];
        if (!p2.z && fb == DRB_FB_NONE) fb = DRB_FB_ENTRY_TYPE;
        if (p2.y > v.C16 * 16 && fb == DRB_FB_NONE) fb = DRB_FB_CAPACITY;
      }
      // the Proposes of the inbox (handleLeaderPropose): their entries in
      // the senders' forward rows, checked as staged ones are
      if (prop_from) {
        if ((!FWD || !v.fwd_props) && fb == DRB_FB_NONE)
          fb = DRB_FB_MESSAGE_TYPE;
#pragma unroll
        for (int s = 0; s < R; ++s) {
          const uint32_t ns = (uint32_t)(nprop_packed >> (4 * s)) & 0xfu;
          for (uint32_t j = 0; FWD && v.fwd_props && j < ns; ++j) {
            const uint4 p2 = v.props[prop_ix(v, fwd_ps(v, L.rbuf, (uint32_t)s),
                                             j, 2, g)];
            if (!p2.z && fb == DRB_FB_NONE) fb = DRB_FB_ENTRY_TYPE;
            if (p2.y > v.C16 * 16 && fb == DRB_FB_NONE) fb = DRB_FB_CAPACITY;
          }
        }
      }
      nappend = nprops + n_fwd;
      // The window: the lowest index a Replicate of this round may read
      // for remote s is next - 1 (its LogTerm), or match - 1 after a
      // rejection lowers next (decreaseTo / enterRetryState, remote.go:
      // 182-198, raft.go:2013-2017).  Below the resident window the
      // reference reads LogDB (logentry.go:180-195): the CPU path's job,
      // so the leader falls back before it sends.  Appended entries must
      // not evict anything still needed either.  A remote being sent a
      // snapshot (remote.go:128-141) is the CPU path's as well.
      uint64_t keep = umin64(r.ring_guard, keep_common);
#pragma unroll
      for (int s = 0; s < R; ++s) {
        if ((uint32_t)s == slot) continue;
        const RemoteV x = rem_get<R>(L, s);
        if (x.st == DRB_REMOTE_SNAPSHOT && fb == DRB_FB_NONE)
          fb = DRB_FB_SNAPSHOT;
        // a paused remote (Wait) that sent nothing this round is sent no
        // Replicate (isPaused, remote.go:200-213; only its own responses
        // unpause it): it holds no rows of the window this round -- a
        // stopped follower does not hold the leader back.  When it answers
        // again below the window, that round falls back.
        if (x.st == DRB_REMOTE_WAIT && !((nin_packed >> (5 * s)) & 31u))
          continue;
        uint64_t lowest = ((rej_from >> s) & 1) ? umin64(x.m, x.n) : x.n;
        // an accepting answer outside Replicate state may lower next to
        // the answer's match + 1 (respondedTo: a fresh leader's remotes)
        if (!((rej_from >> s) & 1) && ((resp_from >> s) & 1) &&
            x.st != DRB_REMOTE_REPLICATE)
          lowest = umin64(lowest, resp_floor<R>(L, x, s,
                                                (uint32_t)((nin_packed >>
                                                            (5 * s)) & 31u)));
        const uint64_t need = lowest > 0 ? lowest - 1 : 0;  // LogTerm index
        keep = umin64(keep, need);
        const bool ents_below = need < r.last && need + 1 < r.ring_lo;
        const bool term_below =
            need != 0 && need < r.ring_lo && need < r.term_start;
        if ((ents_below || term_below) && fb == DRB_FB_NONE)
          fb = DRB_FB_CAPACITY;
      }
      if (nappend && r.last + nappend >= keep + v.W && fb == DRB_FB_NONE)
        fb = DRB_FB_CAPACITY;
      // entry rows of a remote follower's plane: the round sends it
      // entries [floor, new last], floor = its next, or above its match
      // where a reject or respondedTo (remote.go:170-198) may lower next
      if (v.remote_mask) {
#pragma unroll
        for (int s = 0; s < R; ++s)
          if ((uint32_t)s != slot && pair_remote(v, slot, s)) {
            const RemoteV x = rem_get<R>(L, s);
            if (x.st == DRB_REMOTE_WAIT && !((nin_packed >> (5 * s)) & 31u))
              continue;  // paused and silent: nothing is sent to it
            const bool lowers = ((rej_from >> s) & 1) ||
                                (((resp_from >> s) & 1) &&
                                 x.st != DRB_REMOTE_REPLICATE);
            const uint64_t floor =
                lowers ? resp_floor<R>(L, x, s,
                                       (uint32_t)((nin_packed >> (5 * s)) & 31u))
                       : x.n;
            if (r.last + nappend + 1 > floor + v.E && fb == DRB_FB_NONE)
              fb = DRB_FB_CAPACITY;
          }
      }
      // mailbox: messages the round can send to each follower s: the
      // broadcasts every follower gets -- the tick's heartbeat, one
      // heartbeat per ReadIndex (staged or from any follower), one
      // Replicate per proposal batch and per Propose, and one per commit
      // advance (raft.go:1885: at most min(#ReplicateResp, last -
      // committed), an answer only acknowledges entries the round began
      // with) -- plus what s's own records cause (own_packed, above).
      // tools/mailbox_bound.py checks it against the oracle's sends.
      {
        uint64_t adv = r.last > r.committed ? r.last - r.committed : 0;
        uint32_t nb = (uint32_t)umin64((uint64_t)n_rr, adv);
        uint32_t base = (in_lo != 0) + (p.tick ? 1 : 0) + (nprops ? 1 : 0) +
                        __builtin_popcount(prop_from) + n_ri_msgs + nb +
                        (SLOW ? 1 : 0);
#pragma unroll
        for (int s = 0; s < R; ++s) {
          if ((uint32_t)s == slot) continue;
          uint32_t bound = base + (uint32_t)((own_packed >> (5 * s)) & 31u);
          // a transfer: one TimeoutNow from the ReplicateResps (it needs
          // match == lastIndex after a successful tryUpdate, and match only
          // grows while lastIndex stands: raft.go:1883-1895), plus a
          // TimeoutNow or Replicate per LeaderTransfer handled
          // (handleLeaderTransfer, raft.go:1925-1953)
          if (SLOW && (n_lt || (flags & (F_XFER | F_XFER_REQ))))
            bound += 1 + n_lt + ((flags & F_XFER_REQ) ? 1u : 0u);
          if (bound > v.MB && fb == DRB_FB_NONE) fb = DRB_FB_CAPACITY;
        }
      }
      // tick: CheckQuorum (raft.go:623-633) -- not on a quiesced tick
      const bool qtick = qon && p.tick && total_in == 0 && in_lo == 0 &&
                         qs_quiet_tick(v, r, qz_from);
      if (p.tick && !qtick && v.check_quorum &&
          r.election_tick + 1 >= v.election_rtt) {
        uint32_t c = 1;
#pragma unroll
        for (int s = 0; s < R; ++s)  // the voting members (raft.go:395-405)
          if ((uint32_t)s != slot && !is_nonvoting(L, (uint32_t)s) &&
              (rem_get<R>(L, s).a || ((resp_from >> s) & 1)))
            c++;
        // (the raft launch steps the leader down at the tick, el_tick)
        if (c < quorum_of<R>(L) && !SLOW && fb == DRB_FB_NONE)
          fb = DRB_FB_CHECK_QUORUM;
      }
      // a leader that may step down before handleProposals and learn the
      // new leader in the same round would forward its proposals to it
      // (handleFollowerPropose, raft.go:2103-2116): the CPU path's.  One
      // that steps down for a vote, a NoOP or CheckQuorum knows no leader
      // and drops them (below).
      // (with forward rows it forwards them, as the reference does)
      if (SLOW && nprops && higher_lead && !v.fwd_props && fb == DRB_FB_NONE)
        fb = DRB_FB_TERM_MISMATCH;
      // a Propose the leader may not handle as leader (it steps down first)
      if (SLOW && prop_from && higher_in && fb == DRB_FB_NONE)
        fb = DRB_FB_MESSAGE_TYPE;
    } else {
      if (max_app && max_app >= keep_common + v.W &&
          fb == DRB_FB_NONE)
        fb = DRB_FB_CAPACITY;
      // a Propose at a follower (or a candidate) is the CPU path's
      // (handleFollowerPropose would forward it again)
      if (prop_from && fb == DRB_FB_NONE) fb = DRB_FB_MESSAGE_TYPE;
      // the entry queue this follower forwards: Cmds that fit the rows
      for (uint32_t j = 0; j < nprops; ++j) {
        const uint4 p2 = v.props[prop_ix(v, p.prop_slot, j, 2, g)];
        if (p2.y > v.C16 * 16 && fb == DRB_FB_NONE) fb = DRB_FB_CAPACITY;
      }
      // mailbox: one response per message of a sender, plus the
      // forwarded ReadIndex (handleFollowerReadIndex) and Propose
#pragma unroll
      for (int s = 0; s < R; ++s)
        if ((uint32_t)s != slot &&
            ((nin_packed >> (5 * s)) & 31u) + (in_lo != 0) + (nprops != 0) +
                    (SLOW ? 1 : 0) +
                    (SLOW ? n_lt + ((flags & F_XFER_REQ) ? 1u : 0u) : 0u) >
                v.MB &&
            fb == DRB_FB_NONE)
          fb = DRB_FB_CAPACITY;
      // (a staged ReadIndex ends the quiesce before the tick: node.
      // handleReadIndex -> qs.record, node.go:1296-1298)
      const bool qtick = qon && p.tick && total_in == 0 && in_lo == 0 &&
                         qs_quiet_tick(v, r, qz_from);
      if (!SLOW && p.tick && !qtick) {
        uint64_t et = (total_in ? 0 : r.election_tick) + 1;
        // (a nonVoting or witness member never campaigns, nonLeaderTick)
        if (et >= ld_f(L, r, F_RAND_TIMEOUT) && fb == DRB_FB_NONE &&
            !passive_role(role))
          fb = DRB_FB_ELECTION;
      }
    }
    if (p.encode_saves && fb == DRB_FB_NONE) {
      // EntriesToSave lie in [min(committed, saved_to) + 1, new last]
      const uint64_t top = umax64(r.last + nappend, max_app);
      const uint64_t base = umin64(r.committed, r.saved_to);
      uint64_t n_save = top > base ? top - base : 0;
      uint64_t slack = 0;
      if (v.save_batched && n_save) {
        // the records also hold the first batch's earlier entries, which
        // must still be resident, and start 16 B aligned
        uint64_t sb = over_ld(L, F_SAVE_BASE);
        if (sb == 0 || sb > base + 1) sb = base + 1;
        const uint64_t start = save_merge_start(base + 1, sb);
        if (start < r.ring_lo ||
            top / LOGDB_BATCH - (base + 1) / LOGDB_BATCH + 1 > DRB_SAVE_RECS)
          fb = DRB_FB_CAPACITY;
        n_save = top - start + 1;
        slack = 16 * DRB_SAVE_RECS;
      }
      if (v.save_tan) slack = v.save_slack;
      if (n_save * entrybatch_elem_bound(v.C16 * 16) + slack >
          (uint64_t)v.save_cap16 * 16)
        fb = DRB_FB_CAPACITY;
    }
    DRB_PH(1);  // load + pre-pass
    // elections: what the raft launch handles goes there, untouched
    bool to_slow = false;
    if (!SLOW && v.elections &&
        (fb == DRB_FB_TERM_MISMATCH || fb == DRB_FB_MESSAGE_TYPE ||
         fb == DRB_FB_ELECTION || fb == DRB_FB_CHECK_QUORUM ||
         fb == DRB_FB_ROLE)) {
      const unsigned long long i = atomicAdd(v.slow_n, 1ull);
      if (i < v.slow_cap) {
        v.slow_list[i] = make_uint4((uint32_t)g, (uint32_t)(g >> 32), slot, 0);
        v.u32[u32_ix(v, W_FLAGS, slot, g)] = r.flags | F_SLOW;
        to_slow = true;
        c_stepped = 0;
      }
    }
    if (to_slow) {
      // the raft launch runs this replica's round after this launch
    } else if (fb != DRB_FB_NONE) {
      r.flags |= DRB_F_FALLBACK;
      r.fb = fb;
      v.u32[u32_ix(v, W_FLAGS, slot, g)] = r.flags;
      v.u32[u32_ix(v, W_FB_REASON, slot, g)] = r.fb;
      c_fb = 1;
      if (qs_owed) {  // the pre-round state includes the skipped ticks
        pu_put(L, r, 12, 1, F_ELECTION_TICK, r.election_tick);
        v.pk[pk_ix(v, 3, slot, g)] =
            make_uint4(r.pw[12], r.pw[13], r.pw[14], r.pw[15]);
        over_st(L, F_QS_TICK, r.qs_tick);
        over_st(L, F_QS_BASE, p.tick_no - p.tick);
      }
    } else {
      // ---------------------------------------- handleEvents (node.go)
      // updateAppliedIndex (node.go:1133-1137)
      r.applied_index = r.sm_index;
      st_f(L, r, F_APPLIED, r.applied_index);  // applied_index: hot
      // handleReadIndex (node.go:1296) -> Peer.ReadIndex (peer.go:309)
      if (in_lo != 0) {
        if (qon) qs_record(v, r, DRB_MSG_READ_INDEX);
        if (is_leader)
          leader_read_index(L, r, in_lo, in_hi, 0);
        else
          follower_read_index(L, r, in_lo, in_hi);
      }
      // handleReceivedMessages: Replicates by sender, then the rest
      if (FPF && pf_s[0] >= 0)
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): pf_lds landed
#pragma unroll 1
      for (int pass = 0; pass < 2; ++pass) {
#pragma unroll 1
        for (int s = 0; s < R; ++s) {
          if ((uint32_t)s == slot) continue;
          // a Quiesce from s precedes its other non-Replicate messages
          // (node.handleMessage -> tryEnterQuiesce, node.go:1385-1386)
          if (qon && pass == 1 && ((qz_from >> s) & 1)) qs_try_enter(v, r);
          if (!((nin_packed >> (5 * s)) & 31u)) continue;
          const bool rm = pair_remote(v, s, slot);
          const uint4 *mb = rm ? in_mbox(L, s, slot) : v.mbox;
          const uint4 meta = (rm ? in_meta(L, s, slot) : v.mbox_meta)[mmeta_ix(
              v, L.rbuf, s, slot, g)];
          const uint64_t sterm = hi64(meta);
          // records of this pass: the Replicates, then the others
          const uint32_t cnt = pass == 0 ? mi_nrep(meta.y) : mi_noth(meta.y);
          EntSrc src;
          src.remote = rm;
          src.lo = 0;
          if (rm && pass == 0 && cnt)
            src.lo = in_elo(L, s, slot)[mmeta_ix(v, L.rbuf, s, slot, g)];
          uint64_t prev_lo = 0, prev_hi = 0;
          // (a window of prefetched records measured slower: the leader
          // spills more, profiles/r02_kvline/README.md)
          for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t k = rec_pos(pass == 0, j, v.MB);
            const int q = s == pf_s[0] ? 0 : (PFS > 1 && s == pf_s[1]) ? 1 : -1;
            const uint32_t ord = pass == 0 ? j : pf_nrp[q > 0 ? 1 : 0] + j;
            const uint4 c0 = (FPF && q >= 0 && ord < (uint32_t)PFN)
                                 ? pf_lds[FPF ? q : 0][FPF ? ord : 0]
                                         [FPF ? threadIdx.x : 0]
                                 : mb[mbox_ix(v, L.rbuf, s, slot, k, 0, g)];
            uint4 c1 = make_uint4(0, 0, 0, 0);
            if (c0.x & MF_HAS_C1) c1 = mb[mbox_ix(v, L.rbuf, s, slot, k, 1, g)];
            // the raft launch: a record whose sender changed terms
            // within its round carries its own term (rterm)
            const uint64_t rt =
                (SLOW && (c0.x & MF_TERM_OTHER))
                    ? (rm ? in_rterm(L, s, slot) : v.rterm)[rterm_ix(v, L.rbuf, s, slot,
                                                           k, g)]
                    : sterm;
            const Msg m = msg_decode(c0, c1, rt, prev_lo, prev_hi);
            if (qon)  // node.recordMessage (node.go:1339-1345)
              qs_record(v, r,
                        (m.type == DRB_MSG_HEARTBEAT ||
                         m.type == DRB_MSG_HEARTBEAT_RESP) && m.hint > 0
                            ? (uint32_t)DRB_MSG_READ_INDEX
                            : m.type);
            if (SLOW)
              el_dispatch(L, r, s, m, src);
            else
              dispatch<R, FWD>(L, r, s, m, src);
          }
        }
      }
      DRB_PH(2);  // handleEvents: the inbox dispatch
      // LocalTick (node.tick node.go:1562 -> raft.tick raft.go:571-648)
      bool quiet = false;
      if (p.tick && qon) {
        qs_tick_once(v, r);
        quiet = qs_quiesced(r);
      }
      if (p.tick && quiet) {
        r.election_tick++;  // raft.quiescedTick (raft.go:650-656)
      } else if (SLOW && p.tick) {
        el_tick(L, r);  // any role; may campaign or step down
      } else if (p.tick) {
        over_st(L, F_TICK_COUNT, over_ld(L, F_TICK_COUNT) + 1);
        if (is_leader) {
          r.election_tick++;
          if (r.election_tick >= v.election_rtt) {
            r.election_tick = 0;
            if (v.check_quorum) {
              // leaderHasQuorum (raft.go:395-405): quorum held (pre-pass);
              // the voting members' active flags are cleared
#pragma unroll
              for (int s = 0; s < R; ++s)
                if (!is_nonvoting(L, (uint32_t)s)) rl_of<R>(L).a[s][L.tid] = 0;
              if (L.dirty)
                rl_of<R>(L).dirty[L.tid] |=
                    0x88888888u & ~nv_bits8(nv_mask_of(L));
            }
          }
          r.heartbeat_tick++;
          if (r.heartbeat_tick >= v.heartbeat_rtt) {
            r.heartbeat_tick = 0;
            broadcast_heartbeat(L, r);
          }
        } else {
          r.election_tick++;
        }
      }
      // handleProposals (node.go:1275) -> handleLeaderPropose
      // (raft.go:1794-1815) -> appendEntries (raft.go:944-955); a leader
      // transferring its leadership drops them (raft.go:1796-1800)
      if (nprops && (SLOW ? r.role == DRB_LEADER : LEAD)) {
        if (SLOW && (r.flags & F_XFER))
          r.ndropped_props += nprops;  // leaderTransfering
        else {
          append_props(L, r, p.prop_slot, nprops);
          broadcast_replicate(L, r);
        }
      } else if (FWD && nprops &&
                 (r.role == DRB_FOLLOWER || r.role == DRB_NONVOTING) &&
                 v.fwd_props) {
        // handleFollowerPropose, handleNonVotingPropose (raft.go:2103-2116,
        // 2071-2073)
        forward_props(L, r, p.prop_slot, nprops);
      } else if (nprops) {
        // stepped down this round: handleCandidatePropose, or
        // handleFollowerPropose with no leader known (raft.go:2197-2201,
        // 2103-2108) -- reportDroppedProposal; one that knows the new
        // leader forwards (above), or without forward rows was routed to
        // the CPU path by the pre-pass
        if ((r.role == DRB_FOLLOWER || r.role == DRB_NONVOTING) &&
            r.leader_id != 0)
          set_error(r, DRB_ERR_PROPOSE);
        else
          r.ndropped_props += nprops;
      }
      // handleLeaderTransfer (node.go:1249-1257) -> Peer.RequestLeader-
      // Transfer (peer.go:106-113): a LeaderTransfer to itself, term 0
      if (SLOW && (r.flags & F_XFER_REQ)) {
        r.flags &= ~F_XFER_REQ;
        const uint64_t target = v.xfer_in[ix(v, slot, g)];
        if (r.role == DRB_LEADER)
          el_leader_transfer(L, r, target);
        else if (r.role == DRB_FOLLOWER)
          el_forward_transfer(L, r, target);
      }
      // stepNode: newQuiesceState -> sendEnterQuiesceMessages to every
      // other member (node.go:993-1005, 1148-1150), sent ahead of the
      // Update's messages (a header bit per destination, drb_msg.hpp)
      if (qon && r.qs_new) {
        qz_out = ((1u << R) - 1u) & ~(1u << slot);
        r.nmsgs += R - 1;
      }

      DRB_PH(3);  // tick + proposals
      // ---------------------------------------- getUpdate (node.go:1025)
      bool inmem_nonempty = r.last >= r.marker;
      uint64_t save_lo = r.saved_to + 1;
      bool has_save = inmem_nonempty && save_lo >= r.marker && save_lo <= r.last;
      bool has_apply = r.committed > r.processed;
      // Peer.prevState (peer.go:59) and node's cursors, in place
      const uint64_t vote = ld_f(L, r, F_VOTE);
      const uint64_t prev_term = ld_f(L, r, F_PREV_TERM);
      const uint64_t prev_vote = ld_f(L, r, F_PREV_VOTE);
      const uint64_t prev_commit = ld_f(L, r, F_PREV_COMMIT);
      const uint64_t confirmed_index = ld_f(L, r, F_CONFIRMED_INDEX);
      bool state_changed = !(r.term == prev_term && vote == prev_vote &&
                             r.committed == prev_commit);
      bool state_empty = r.term == 0 && vote == 0 && r.committed == 0;
      bool has_update = has_save || r.leader_update || r.nmsgs > 0 ||
                        has_apply || (!state_empty && state_changed) ||
                        r.nrtr > 0 || r.ndropped_ri > 0 ||
                        r.ndropped_props > 0;
      uint64_t apply_lo = 0, apply_hi = 0;
      if (has_update || confirmed_index != r.applied_index) {
        // validateUpdate / pushEntries (node.go:1100) / Peer.Commit
        if (has_apply) {
          // pb.EntriesToApply(CommittedEntries, pushedIndex, strict)
          // (raftpb/entry.go:27-47) then node.pushEntries (node.go:625)
          const uint64_t pushed = ld_f(L, r, F_PUSHED_INDEX);
          apply_lo = r.processed + 1;
          apply_hi = r.committed;
          if (apply_hi <= pushed || apply_lo > pushed + 1) {
            set_error(r, DRB_ERR_APPLY);
            apply_lo = 0;
          } else {
            apply_lo = pushed + 1;
            st_f(L, r, F_PUSHED_INDEX, apply_hi);
          }
        }
        if (state_changed && !state_empty) {
          if (prev_term != r.term) st_f(L, r, F_PREV_TERM, r.term);
          if (prev_vote != vote) st_f(L, r, F_PREV_VOTE, vote);
          st_f(L, r, F_PREV_COMMIT, r.committed);
        }
        if (confirmed_index != r.applied_index)
          st_f(L, r, F_CONFIRMED_INDEX, r.applied_index);
        // SaveRaftState (engine.go:1343) of EntriesToSave
        if (EXT && p.encode_saves && v.save_tan) {
          // the Update a tan LogDB writes, for k_tan_encode (drb_tan.hpp)
          const uint32_t n_save =
              has_save ? (uint32_t)(r.last - save_lo + 1) : 0u;
          const uint32_t tf =
              1u /*TS_HAVE*/ | (state_changed && !state_empty ? 2u : 0u) |
              (prev_term != r.term || prev_vote != vote ? 4u : 0u);
          const uint64_t RG = (uint64_t)v.R * v.G, ti = ix(v, L.slot, L.g);
          v.tan_sum[ti] = make_uint4((uint32_t)r.term,
                                     (uint32_t)(r.term >> 32), (uint32_t)vote,
                                     (uint32_t)(vote >> 32));
          v.tan_sum[RG + ti] = make_uint4(
              (uint32_t)r.committed, (uint32_t)(r.committed >> 32),
              (uint32_t)save_lo, (uint32_t)(save_lo >> 32));
          v.tan_sum[2 * RG + ti] = make_uint4(n_save, tf, (uint32_t)p.round, 0);
          c_saved += n_save;
        } else if (EXT && has_save && p.encode_saves) {
          if (v.save_batched)
            encode_save_records(L, r, save_lo, r.last, crc_tab, c_saved,
                                c_saved_bytes);
          else
            encode_saves(L, r, save_lo, r.last, crc_tab, c_saved,
                         c_saved_bytes);
        }
        // Peer.Commit -> entryLog.commitUpdate (logentry.go:351-371)
        if (has_save) r.saved_to = r.last;  // savedLogTo(last, term(last))
        if (has_apply) r.processed = apply_hi;
        uint64_t la = r.applied_index;
        if (la > 0) {
          if (la > r.committed || la > r.processed)
            set_error(r, DRB_ERR_COMMIT);
          // inMemory.appliedLogTo (inmemory.go:138-164)
          if (la >= r.marker && r.last >= r.marker && la <= r.last) {
            st_f(L, r, F_APPLIED_TO_INDEX, la);
            st_f(L, r, F_APPLIED_TO_TERM, log_term(L, r, la));
            r.marker = la + 1;
          }
        }
        // clearReadyToRead: records stay in the round output buffer
      }
      DRB_PH(4);  // getUpdate
      // ---------------------------------------- StateMachine.Handle
      if (apply_hi >= apply_lo && apply_lo != 0) {
        uint64_t from = umax64(apply_lo, r.sm_index + 1);
        for (uint64_t idx = from; idx <= apply_hi; ++idx) {
          const int rc = apply_entry<R, EXT>(L, r, idx);
          if (rc < 0) {
            // the rsm apply of this replica leaves the fast path at idx;
            // the raft round itself completed: (sm_index, pushed_index]
            // stay pushed but unapplied (include/drb_engine.h)
            r.flags |= DRB_F_FALLBACK | DRB_F_APPLY_STOPPED;
            r.fb = rc == -2 ? DRB_FB_CAPACITY : DRB_FB_ENTRY_TYPE;
            c_fb = 1;
            break;
          }
          c_applied++;
          if (rc == 1 && (SLOW ? r.role == DRB_LEADER : is_leader))
            c_commit++;
        }
      }
      DRB_PH(5);  // apply
      // the entry rows of remote followers' planes: [lowest sent, last]
      if (LEAD && v.remote_mask) {
        const uint32_t chunks = ENT_META + v.C16;
#pragma unroll
        for (int s = 0; s < R; ++s) {
          if ((uint32_t)s == slot || !pair_remote(v, slot, s)) continue;
          const uint64_t lo = elo_lds[LEAD ? s : 0][threadIdx.x];
          if (lo == ~0ull) continue;
          if (r.last + 1 - lo > v.E || lo < r.ring_lo) {  // pre-pass bound
            set_error(r, DRB_FB_CAPACITY);
            elo_lds[LEAD ? s : 0][threadIdx.x] = ~0ull;
            continue;
          }
          for (uint64_t idx = lo; idx <= r.last; ++idx)
            for (uint32_t c = 0; c < chunks; ++c)
              v.embox[embox_ix(v, L.wbuf, slot, s, (uint32_t)(idx - lo), c,
                               g)] = v.ring[ring_ix(v, slot, idx, c, g)];
          v.elo[mmeta_ix(v, L.wbuf, slot, s, g)] = lo;
        }
        last_final = r.last;
      }
      // the leader's served reads issued before the state store and the
      // outbox headers, their loads overlapping those stores (0.3-0.8 %
      // faster at C3 than after them, profiles/r04_reads)
      if (LEAD && p.n_reads)
        serve_reads_lane<EXT>(v, slot, g, r.nrtr, r.sm_index, p.n_reads,
                              p.key_space, c_served, c_deferred);
      sent_c1 = r.c1mask;
      // ring guard for the next round's appends
      r.ring_guard = r.guard_new;
      if (r.err) {
        r.flags |= DRB_F_ERROR;
        c_err = 1;
      }
      // at rest: with no input the next round would change nothing --
      // updateAppliedIndex finds applied == sm index, nothing to apply, no
      // Replicate in flight to guard, and no round output to clear
      const bool rest = r.sm_index == r.applied_index &&
                        r.committed == r.processed && r.guard_new == ~0ull &&
                        r.nrtr == 0 && !has_save &&
                        !(r.flags & (DRB_F_FALLBACK | DRB_F_ERROR));
      r.flags = rest ? (r.flags | F_AT_REST) : (r.flags & ~F_AT_REST);
      if (EXT && p.encode_saves)  // (save_len: 0 below iff nothing saved)
        r.flags = c_saved == 0 ? (r.flags | F_SAVE_ZERO)
                               : (r.flags & ~F_SAVE_ZERO);
      if (qon) {
        r.flags = qs_quiesced(r) ? (r.flags | F_QUIESCED)
                                 : (r.flags & ~F_QUIESCED);
        // (a heartbeat round moves only the tick and the base)
        over_st(L, F_QS_TICK, r.qs_tick);
        const uint32_t qd = DRB_QS_DIRTY ? r.qs_dirty : 7u;
        if (qd & 1u) over_st(L, F_QS_IDLE, r.qs_idle);
        if (qd & 2u) over_st(L, F_QS_SINCE, r.qs_since);
        if (qd & 4u) over_st(L, F_QS_EXIT, r.qs_exit);
        if (DRB_QS_EAGER ||
            (r.flags & (F_QUIESCED | F_AT_REST)) == (F_QUIESCED | F_AT_REST))
          over_st(L, F_QS_BASE, p.tick_no);  // (it may skip rounds now)
      }
      store_rep<R, LEAD>(L, r, flags0, fb0);
      if (SLOW) {  // what only the raft launch changes
        if (r.role != role0) {
          v.u32[u32_ix(v, W_ROLE, slot, g)] = r.role;
          c_role = 1;
        }
        if (r.votes != votes0) v.u32[u32_ix(v, W_VOTES, slot, g)] = r.votes;
      }
      c_msgs = r.nmsgs;
      c_rtr = r.nrtr;
      c_drop = r.ndropped_ri;
      c_dprop = r.ndropped_props;
    }
    if (c_fb | c_err) flag_log(v, g, slot, r.fb, r.flags, p.round);
    // outbox headers for this round (tag = round), for the destinations
    // that got records: a receiver reads a stale tag as an empty inbox
#pragma unroll
    for (int s = 0; s < R; ++s) {
      uint32_t w = oinfo[s * 256 + threadIdx.x];
      const bool qz = (qz_out >> s) & 1u;
      if (SLOW && (r.term != term0 || r.oterm) && mi_count(w)) {
        // the records sent before the term changed keep theirs (rterm)
        const uint32_t nrp = mi_nrep(w), nt = mi_count(w);
        for (uint32_t j = 0; j < nt; ++j) {
          const uint32_t k = rec_pos(j < nrp, j < nrp ? j : j - nrp, v.MB);
          const uint64_t ci = mbox_ix(v, L.wbuf, slot, (uint32_t)s, k, 0, g);
          uint4 c0 = v.mbox[ci];
          if (!(c0.x & MF_TERM_ZERO) &&
              v.rterm[rterm_ix(v, L.wbuf, slot, (uint32_t)s, k, g)] !=
                  r.term) {
            c0.x |= MF_TERM_OTHER;
            v.mbox[ci] = c0;
            w |= MI_TERM_OTHER;
          }
        }
        oinfo[s * 256 + threadIdx.x] = w;  // (the plane summary's flag)
      }
      if (mi_count(w) || qz) {
        uint4 meta = mk4(0, r.term);
        meta.x = ((uint32_t)p.round & MQ_TAG) | (qz ? MQ_QUIESCE : 0u);
        meta.y = w;
        v.mbox_meta[mmeta_ix(v, L.wbuf, slot, (uint32_t)s, g)] = meta;
        // the receiver's round tag byte for this sender (a byte store: the
        // other senders own the other bytes of the word)
        ((uint8_t *)&v.inbox_tag[((uint64_t)L.wbuf * v.R + s) * v.G + g])
            [slot] = tag_byte(p.round, w);
      }
    }
    v.rtr_count[ix(v, slot, g)] = r.nrtr;
    if (p.encode_saves && c_saved == 0) v.save_len[ix(v, slot, g)] = 0;
    DRB_PH(6);  // state store + outbox headers
    // ReadLocalNode of the released reads, against the state just applied
    if (!LEAD && p.n_reads)
      serve_reads_lane<EXT>(v, slot, g, r.nrtr, r.sm_index, p.n_reads,
                       p.key_space, c_served, c_deferred);
    DRB_PH(7);  // served reads
  }
  if (NPH > 1 && v.phase) {  // uniform: the lanes' phase sums, one atomic
    // per wave and phase (lane 0: stepped lanes)
#pragma unroll
    for (int i = 0; i < NPH; ++i) {
      uint64_t x =
          i ? (c_stepped ? ph_lds[i][NPH > 1 ? threadIdx.x : 0] : 0u) : c_stepped;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
        x += (uint64_t)__shfl_xor((long long)x, o, 64);
      if ((threadIdx.x & 63) == 0 && x)
        atomicAdd(&v.phase[(LEAD ? 8 : 0) + i], (unsigned long long)x);
    }
  }
#undef DRB_PH
  // per-block summary of this rank's remote planes (drb_exchange_*): max
  // records, max entry rows, c1 / Replicate flags; the raft launch adds its
  // lanes' to the slow rows, lane by lane (its lanes are no slot's block)
  if (SLOW && v.remote_mask && active) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if ((uint32_t)s == slot || !pair_remote(v, slot, s)) continue;
      const uint32_t w = oinfo[s * 256 + threadIdx.x];
      uint32_t E = 0;
      const uint64_t lo = elo_lds[s][threadIdx.x];
      if (lo != ~0ull) E = (uint32_t)(last_final + 1 - lo);
      const uint32_t fl = ((sent_c1 >> s) & 1u) | (((qz_out >> s) & 1u) << 1) |
                          ((w & MI_TERM_OTHER) ? 4u : 0u);
      if (!(mi_count(w) | E | fl)) continue;
      uint32_t *q = v.xslow + (((uint64_t)slot * v.R + s) * ((v.G + 255) / 256) +
                               g / 256) * 4;
      atomicMax(&q[0], mi_nrep(w));
      atomicMax(&q[1], mi_noth(w));
      atomicMax(&q[2], E);
      atomicOr(&q[3], fl);
    }
  }
  if (!SLOW && v.remote_mask) {  // uniform
#pragma unroll
    for (int s = 0; s < R; ++s) {
      if ((uint32_t)s == slot || !pair_remote(v, slot, s)) continue;
      uint32_t Kr = 0, Ko = 0, E = 0, fl = 0;
      if (active) {
        const uint32_t w = oinfo[s * 256 + threadIdx.x];
        Kr = mi_nrep(w);
        Ko = mi_noth(w);
        fl = ((sent_c1 >> s) & 1u) | (((qz_out >> s) & 1u) << 1);
        if (LEAD) {
          const uint64_t lo = elo_lds[LEAD ? s : 0][threadIdx.x];
          if (lo != ~0ull) E = (uint32_t)(last_final + 1 - lo);
        }
      }
      block_plane_summary<LEAD>(v, bp, slot, (uint32_t)s, Kr, Ko, E, fl);
    }
  }
  const uint32_t cnt[NUM_COUNTERS] = {
      (uint32_t)c_commit, (uint32_t)c_applied, (uint32_t)c_msgs,
      (uint32_t)c_rtr,    (uint32_t)c_drop,    (uint32_t)c_fb,
      (uint32_t)c_err,    c_served,            c_deferred,
      c_saved,            c_saved_bytes,       c_stepped,
      c_elect,            c_role,              c_dprop};
  block_counters<LEAD, 0, NUM_COUNTERS>(v, SLOW ? 0u : slot, bp, cnt);
}

}  // namespace drb

#include "drb_lean.hpp"
