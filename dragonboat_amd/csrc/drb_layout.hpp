// drb_layout.hpp -- HBM layout of the engine (structure-of-arrays).
//
// Every per-replica array is indexed [slot][group]: lanes of a wavefront
// step 64 consecutive groups of the SAME replica slot, so each field load
// is one coalesced 512 B (u64) or 1 KiB (uint4) access and every wave is
// role-homogeneous (all leaders or all followers) -- no divergence on the
// steady-state path.
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace drb {

// the tan select pass's replica lists (drb_tan.hpp)
constexpr uint32_t TAN_LISTS = 64;

__host__ __device__ inline uint64_t lo64(uint4 q) {
  return (uint64_t)q.x | ((uint64_t)q.y << 32);
}
__host__ __device__ inline uint64_t hi64(uint4 q) {
  return (uint64_t)q.z | ((uint64_t)q.w << 32);
}

// splitmix64 finaliser: seeded synthetic inputs and the served-read keys
__host__ __device__ inline uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// per-replica u64 fields (drb_replica_state order), array [F][slot][g]
enum U64Field : int {
  F_TERM = 0,
  F_VOTE,
  F_LEADER_ID,
  F_APPLIED,
  F_ELECTION_TICK,
  F_HEARTBEAT_TICK,
  F_RAND_TIMEOUT,
  F_TICK_COUNT,
  F_COMMITTED,
  F_PROCESSED,
  F_LAST_INDEX,
  F_MARKER_INDEX,
  F_SAVED_TO,
  F_APPLIED_TO_INDEX,
  F_APPLIED_TO_TERM,
  F_APPLIED_INDEX,
  F_CONFIRMED_INDEX,
  F_PUSHED_INDEX,
  F_PREV_TERM,
  F_PREV_VOTE,
  F_PREV_COMMIT,
  F_SM_INDEX,
  F_SM_TERM,
  F_KV_COUNT,
  F_QS_TICK,     // quiesceState.currentTick (quiesce.go:23-33)
  F_QS_IDLE,     // .idleSince
  F_QS_SINCE,    // .quiescedSince (0: not quiesced)
  F_QS_EXIT,     // .exitQuiesceTick
  F_RNG,         // raft.rand state (splitmix64): randomized timeouts
  // internal (not part of drb_replica_state)
  F_RING_LO,     // lowest index still resident in the window
  F_RING_GUARD,  // lowest index referenced by last round's Replicates
  F_TERM_START,  // every entry in [term_start, last] has term == r.term
  F_QS_BASE,     // engine tick count the replica's ticks are applied up to
                 // (a quiesced replica's ticks are applied lazily)
  F_SAVE_BASE,   // save_batched: first index of the replica's record
                 // stream (0: nothing saved yet)
  NUM_U64
};
constexpr int NUM_U64_EXPORTED = F_RING_LO;

// ---- packed per-replica state ------------------------------------------
// One 64 B record per replica (v.pk, [4 chunks][R][G] uint4 = words w0..15):
//   w0-1 last, w2-3 term,
//   w4..w10  the PIdx fields as signed 16-bit offsets from last (2 a word),
//   w11 term - appliedToTerm | (term - prevTerm) << 16,
//   w12 term - smTerm | electionTick << 16,
//   w13 heartbeatTick | randomizedElectionTimeout << 16,
//   w14 vote | leaderID << 8 | prevVote << 16, w15 0.
// A value that does not fit stores the field's escape code and lives in
// the u64 field array, which also keeps tick_count and kv_count.  A round
// reads and writes 64 B of state per replica instead of ~340 B of u64
// fields.
enum PIdx : int {
  PI_COMMITTED = 0,
  PI_PROCESSED,
  PI_MARKER,
  PI_SAVED_TO,
  PI_SM_INDEX,
  PI_APPLIED_INDEX,
  PI_RING_LO,
  PI_RING_GUARD,  // ~0 (no Replicate in flight) is PK_INF16
  PI_TERM_START,
  PI_APPLIED,
  PI_APPLIED_TO_INDEX,
  PI_CONFIRMED,
  PI_PUSHED,
  PI_PREV_COMMIT,
  NUM_PI
};
constexpr uint32_t PK_ESC16 = 0x8000u;  // index offset escape
constexpr uint32_t PK_INF16 = 0x7fffu;  // ring guard +inf
constexpr uint32_t PK_ESCU16 = 0xffffu;  // term distance / tick escape
constexpr uint32_t PK_ESC8 = 0xffu;      // replica id escape

// the u64 field that holds a PIdx field's overflow
__host__ __device__ constexpr int pi_field(int i) {
  return i == PI_COMMITTED          ? F_COMMITTED
         : i == PI_PROCESSED        ? F_PROCESSED
         : i == PI_MARKER           ? F_MARKER_INDEX
         : i == PI_SAVED_TO         ? F_SAVED_TO
         : i == PI_SM_INDEX         ? F_SM_INDEX
         : i == PI_APPLIED_INDEX    ? F_APPLIED_INDEX
         : i == PI_RING_LO          ? F_RING_LO
         : i == PI_RING_GUARD       ? F_RING_GUARD
         : i == PI_TERM_START       ? F_TERM_START
         : i == PI_APPLIED          ? F_APPLIED
         : i == PI_APPLIED_TO_INDEX ? F_APPLIED_TO_INDEX
         : i == PI_CONFIRMED        ? F_CONFIRMED_INDEX
         : i == PI_PUSHED           ? F_PUSHED_INDEX
                                    : F_PREV_COMMIT;
}
__host__ __device__ inline uint32_t pk_half(const uint32_t *w, int word,
                                            int hi) {
  return (w[word] >> (16 * hi)) & 0xffffu;
}
__host__ __device__ inline void pk_set_half(uint32_t *w, int word, int hi,
                                            uint32_t x) {
  w[word] = (w[word] & ~(0xffffu << (16 * hi))) | ((x & 0xffffu) << (16 * hi));
}
// index field codes relative to base (the record's last)
__host__ __device__ inline uint32_t pk_idx_code(uint64_t x, uint64_t base,
                                                bool guard) {
  if (guard && x == ~0ull) return PK_INF16;
  const int64_t d = (int64_t)(x - base);
  if (d < -32767 || d > (guard ? 32766 : 32767)) return PK_ESC16;
  return (uint32_t)(uint16_t)(int16_t)d;
}
__host__ __device__ inline uint64_t pk_idx_value(uint32_t code,
                                                 uint64_t base, bool guard) {
  if (guard && code == PK_INF16) return ~0ull;
  return base + (uint64_t)(int64_t)(int16_t)code;
}
__host__ __device__ inline uint32_t pk_term_code(uint64_t x, uint64_t term) {
  return (x <= term && term - x < PK_ESCU16) ? (uint32_t)(term - x) : PK_ESCU16;
}
__host__ __device__ inline uint32_t pk_u16_code(uint64_t x) {
  return x < PK_ESCU16 ? (uint32_t)x : PK_ESCU16;
}
__host__ __device__ inline uint32_t pk_id_code(uint64_t x) {
  return x < PK_ESC8 ? (uint32_t)x : PK_ESC8;
}

// the whole record from / to field values indexed by U64Field (vals),
// escapes through the overflow array `over` (same index); tick_count and
// kv_count are not in the record
__host__ __device__ inline void pk_encode(uint32_t *w, const uint64_t *vals,
                                          uint64_t *over) {
  const uint64_t last = vals[F_LAST_INDEX], term = vals[F_TERM];
  for (int q = 0; q < 16; ++q) w[q] = 0;
  w[0] = (uint32_t)last;
  w[1] = (uint32_t)(last >> 32);
  w[2] = (uint32_t)term;
  w[3] = (uint32_t)(term >> 32);
  for (int i = 0; i < NUM_PI; ++i) {
    const uint64_t x = vals[pi_field(i)];
    const uint32_t c = pk_idx_code(x, last, i == PI_RING_GUARD);
    if (c == PK_ESC16) over[pi_field(i)] = x;
    pk_set_half(w, 4 + i / 2, i & 1, c);
  }
  const int tf[3] = {F_APPLIED_TO_TERM, F_PREV_TERM, F_SM_TERM};
  const int tw[3] = {11, 11, 12}, th[3] = {0, 1, 0};
  for (int k = 0; k < 3; ++k) {
    const uint32_t c = pk_term_code(vals[tf[k]], term);
    if (c == PK_ESCU16) over[tf[k]] = vals[tf[k]];
    pk_set_half(w, tw[k], th[k], c);
  }
  const int uf[3] = {F_ELECTION_TICK, F_HEARTBEAT_TICK, F_RAND_TIMEOUT};
  const int uw[3] = {12, 13, 13}, uh[3] = {1, 0, 1};
  for (int k = 0; k < 3; ++k) {
    const uint32_t c = pk_u16_code(vals[uf[k]]);
    if (c == PK_ESCU16) over[uf[k]] = vals[uf[k]];
    pk_set_half(w, uw[k], uh[k], c);
  }
  const int df[3] = {F_VOTE, F_LEADER_ID, F_PREV_VOTE};
  for (int k = 0; k < 3; ++k) {
    const uint32_t c = pk_id_code(vals[df[k]]);
    if (c == PK_ESC8) over[df[k]] = vals[df[k]];
    w[14] |= c << (8 * k);
  }
}
__host__ __device__ inline void pk_decode(const uint32_t *w,
                                          const uint64_t *over,
                                          uint64_t *vals) {
  const uint64_t last = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  const uint64_t term = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  vals[F_LAST_INDEX] = last;
  vals[F_TERM] = term;
  for (int i = 0; i < NUM_PI; ++i) {
    const uint32_t c = pk_half(w, 4 + i / 2, i & 1);
    vals[pi_field(i)] = c == PK_ESC16
                            ? over[pi_field(i)]
                            : pk_idx_value(c, last, i == PI_RING_GUARD);
  }
  const int tf[3] = {F_APPLIED_TO_TERM, F_PREV_TERM, F_SM_TERM};
  const int tw[3] = {11, 11, 12}, th[3] = {0, 1, 0};
  for (int k = 0; k < 3; ++k) {
    const uint32_t c = pk_half(w, tw[k], th[k]);
    vals[tf[k]] = c == PK_ESCU16 ? over[tf[k]] : term - c;
  }
  const int uf[3] = {F_ELECTION_TICK, F_HEARTBEAT_TICK, F_RAND_TIMEOUT};
  const int uw[3] = {12, 13, 13}, uh[3] = {1, 0, 1};
  for (int k = 0; k < 3; ++k) {
    const uint32_t c = pk_half(w, uw[k], uh[k]);
    vals[uf[k]] = c == PK_ESCU16 ? over[uf[k]] : c;
  }
  const int df[3] = {F_VOTE, F_LEADER_ID, F_PREV_VOTE};
  for (int k = 0; k < 3; ++k) {
    const uint32_t c = (w[14] >> (8 * k)) & 0xffu;
    vals[df[k]] = c == PK_ESC8 ? over[df[k]] : c;
  }
  vals[F_TICK_COUNT] = over[F_TICK_COUNT];
  vals[F_KV_COUNT] = over[F_KV_COUNT];
  for (int f = F_QS_TICK; f <= F_QS_EXIT; ++f) vals[f] = over[f];
  vals[F_RNG] = over[F_RNG];
  vals[F_QS_BASE] = over[F_QS_BASE];
}

// per-replica u32 fields, array [F][slot][g]
enum U32Field : int {
  W_ROLE = 0,
  W_FLAGS,
  W_FB_REASON,
  W_RI_COUNT,
  W_VOTES,  // candidate votes: answered | granted << 8, bit per slot
  NUM_U32
};

// internal W_FLAGS bits (masked out of drb_replica_state.flags)
constexpr uint32_t F_AT_REST = 1u << 16;  // a round without input is a no-op
constexpr uint32_t F_QUIESCED = 1u << 17;  // node.qs.quiesced() (Quiesce on)
// elections: the replica's round goes to the raft launch (slow list)
constexpr uint32_t F_SLOW = 1u << 18;
// elections: a staged NodeHost.RequestLeaderTransfer (target in v.xfer_in)
// that this replica's next round takes (node.handleLeaderTransfer,
// node.go:1249-1257); the round goes to the raft launch
constexpr uint32_t F_XFER_REQ = 1u << 19;
// a leader's raft.leaderTransferTarget (raft.go:375-381), a replica ID;
// a leader with one steps in the raft launch until it is cleared
constexpr int F_XFER_SHIFT = 20;
constexpr uint32_t F_XFER = 0xfu << F_XFER_SHIFT;
// save_len is 0: the replica's last encode_saves round saved nothing (set
// and cleared by the EXT rounds, the lean kernel's clear then skipped; any
// other writer of save_len writes 0 or leaves the bit clear, and an import
// clears it)
constexpr uint32_t F_SAVE_ZERO = 1u << 24;
constexpr uint32_t F_PUBLIC = 0xffffu;

// message record: 1-2 x uint4 (drb_msg.hpp)
constexpr int MSG_CHUNKS = 2;
// entry meta in the ring: 3 x uint4 = 48 B (+ cmd_cap bytes of Cmd)
//   m0 = {term, key}  m1 = {client_id, series_id}
//   m2 = {responded_to, type u32 | cmd_len u32 << 32}
constexpr int ENT_META = 3;
// staged proposal: 3 x uint4 + cmd chunks
//   p0 = {key, client_id} p1 = {series_id, responded_to}
//   p2 = {type, cmd_len, fast, 0}: fast = 1 when the rsm fast path can
//   apply the entry (prop_fast; checked by the leader's pre-pass)
constexpr int PROP_META = 3;

// Whether the rsm fast path applies this proposal (statemachine.go:935-
// 969, encoded.go:55-65, kvtest.go:145-162): an application or encoded
// entry of the NoOP session (SeriesID 0; ClientID 0 only when empty), an
// encoded Cmd carrying the v0 header byte 0x00 (no compression, no
// session).  Computed when the proposal is staged; anything else (config
// change, session management, regular sessions, Snappy) makes the leader
// fall back before it appends (DRB_FB_ENTRY_TYPE).
__host__ __device__ inline uint32_t prop_fast(uint32_t type, uint64_t client_id,
                                              uint64_t series_id,
                                              uint32_t cmd_len,
                                              uint32_t first_byte) {
  if (type != 0 /*APPLICATION*/ && type != 2 /*ENCODED*/) return 0;
  if (series_id != 0) return 0;
  if (client_id == 0) return cmd_len == 0;
  if (type == 2 && (cmd_len == 0 || first_byte != 0)) return 0;
  return 1;
}
constexpr int RTR_CAP = 8;  // ReadyToRead records per replica per round

// one engine's outbox planes (drb_exchange_local_bind; the device pull)
struct PeerPlanes {
  const uint4 *mbox, *meta, *embox;
  const uint64_t *maxapp, *elo, *rterm;
};

struct View {
  uint64_t G;      // groups
  uint32_t R;      // replicas
  uint32_t W;      // window entries (pow2)
  uint32_t C16;    // cmd chunks of 16 B
  uint32_t MB;     // mailbox messages per (sender, receiver)
  uint32_t KS;     // kv slots per replica (pow2)
  uint32_t KVW;    // kv slot stride in uint4 units
  uint32_t kv_val_cap;
  uint32_t max_props;
  uint32_t election_rtt, heartbeat_rtt, check_quorum;
  uint32_t quiesce;  // Config.Quiesce; qs.electionTick = 2 x election_rtt
  // member kinds per replica slot (drb_config.nonvoting_slots /
  // witness_slots) and the quorum of the voting members (remotes +
  // witnesses, raft.go:383-389)
  uint32_t nv_mask, wt_mask, quorum;
  uint64_t first_shard_id;

  uint64_t *u64;          // [NUM_U64][R][G] (overflow, tick/kv counts)
  uint4 *pk;              // [4][R][G] packed state records (see PIdx)
  uint32_t *u32;          // [NUM_U32][R][G]
  uint64_t *rem_match;    // [R(self)][R(peer)][G]
  uint64_t *rem_next;     // [R][R][G]
  uint32_t *rem_state;    // [R][R][G]
  uint32_t *rem_active;   // [R][R][G]
  uint4 *ri_ctx;          // [R][D][G] {low, high}
  uint4 *ri_idx;          // [R][D][G] {index, from}
  uint32_t *ri_conf;      // [R][D][G]
  uint4 *ring;            // [R][W][ENT_META + C16][G]
  uint4 *mbox;            // [2][R*R][MB][MSG_CHUNKS][G]
  uint4 *mbox_meta;       // [2][R(from)][R(to)][G] {tag, info, term}
  uint64_t *inbox_tag;    // [2][R(to)][G]: byte `from` = round & 0xff of
                          // the sender's last records to this replica
  uint64_t *mbox_maxapp;  // [2][R][R][G] max LogIndex+n of the Replicates
  uint4 *kv;              // [R][G][KS][KVW]
  // out-of-line values (kv_val_cap > 124): slot = {key8, meta, val0} +
  // {block}, the value in block chunks [VB] of kv_pool
  uint4 *kv_pool;
  unsigned long long *kv_pool_next;  // bump allocator
  uint64_t kv_pool_blocks;
  uint32_t kv_ool, VB;
  // KV overflow (drb_config.kv_overflow_buckets): buckets of 4 slots
  // [bucket][4][KVW], per bucket the next one (+1, 0: end), per replica its
  // chain's head (+1), the bump counter and the pool's size
  uint4 *kv_ovf;
  uint32_t *kv_ovf_next;
  uint32_t *kv_ovf_head;  // [R][G]
  unsigned long long *kv_ovf_used;
  uint64_t kv_ovf_cap;
  // DRB_PHASE_PROF step builds: [2 roles][8] cycle sums per round phase
  // (drb_debug_phase; allocated when DRB_PHASE=1 at drb_engine_create)
  unsigned long long *phase;
  uint4 *props;           // [P (+ 2R)][max_props][PROP_META + C16][G]
  uint32_t *prop_count;   // [P][G]
  // drb_config.forward_proposals: a Propose's entries travel by value in
  // proposal batch fwd_ps(buf, sender) = P + buf * R + sender, after the P
  // staged ones
  uint32_t fwd_props;
  uint32_t P;
  uint4 *ri_in;           // [RS][G] {low, high}
  uint4 *rtr;             // [R][RTR_CAP][G] x 2 chunks {index, low},{high,0}
  uint32_t *rtr_count;    // [R][G]
  uint64_t *read_sum;     // [R][G] served-read checksum (drb_serve_reads)
  // served-read results (drb_config.max_reads_per_ctx > 0): [R][RTR_CAP]
  // [max_reads][G] {LE32 value, vlen | found << 31}, and per replica the
  // ReadyToReads whose reads were served (bit k)
  uint2 *read_res;
  uint32_t *read_served;  // [R][G]
  uint32_t max_reads;
  uint4 *save_buf;        // [R][G][save_cap16] EntryBatch of EntriesToSave
  uint32_t *save_len;     // [R][G] bytes (0: nothing saved)
  uint32_t *save_crc;     // [R][G] CRC32-IEEE of those bytes
  uint32_t save_cap16;    // save_buf chunks per replica (0: no encoding)
  uint32_t save_batched;  // drb_config.save_batched
  uint4 *save_rec;        // [R][G][DRB_SAVE_RECS] {batch, off16, len, crc}
  uint32_t *save_nrec;    // [R][G] records of the round
  // save_tan (drb_tan.hpp): the round's pb.Update per replica as the
  // step kernel leaves it, the tan writer position, the round's record
  uint32_t save_tan;
  uint32_t save_slack;    // pre-pass bound: Update framing + chunk headers
  uint4 *tan_sum;         // [3][R][G] {term, vote} {commit, save_lo}
                          // {n_save, flags, round, 0}
  uint4 *tan_st;          // [R][G] {offset lo, hi, log, TST_* flags}
  uint4 *tan_rec;         // [R][G] {offset lo, hi, len, DRB_TAN_* | log << 8}
  unsigned long long *tan_ctr;  // [blocks][4] bytes, records, syncs, logs
  // multiplexed tan (CreateLogMultiplexedTan): 16 logs per replica slot,
  // key = ShardID % 16 (db_keeper.go:84-123), records in group order
  uint32_t pre_vote;      // Config.PreVote (elections)
  uint32_t tan_mux;
  uint32_t tanm_J;        // records per log row: >= ceil(G / 16), 256 | J
  uint32_t *tanm_len;     // [R][16][J] payload bytes | sync << 31, 0: none
  uint4 *tanm_pos;        // [R][16][J] {offset lo, hi, staging byte,
                          //  log << 1 | new log}
  uint4 *tanm_cur;        // [R][16] the log writer {offset lo, hi, log, 0}
  uint4 *tanm_log;        // [R][16][2] the round: {start offset lo, hi,
                          //  start log, flags} {bytes, end log, end lo, hi}
  uint64_t tanm_cap16;    // staging chunks per log (in save_buf)
  // elections (drb_config.elections): the replicas the raft launch steps
  // this round {g lo, g hi, slot, 0}, their count, and the term of every
  // record it wrote whose term differs from its header's (MF_TERM_OTHER)
  uint32_t elections;
  uint32_t slow_cap;
  uint4 *slow_list;
  unsigned long long *slow_n;
  uint64_t *rterm;        // [2][R][R][MB][G]
  uint8_t *xfer_in;       // [R][G] a staged leader transfer's target (the
                          // replica's F_XFER_REQ; drb_request_leader_transfer)
  // placement (drb_config) and the cross-rank planes (world >= 2)
  uint32_t place_world, place_rank;
  uint64_t total_groups;
  uint64_t remote_mask;   // bit from*R+to: that plane is on another rank
  uint32_t E;             // entry rows per remote plane
  uint32_t stage_slot;    // world >= 2: the slot staged inputs go to
  uint4 *mbox_in;         // inbound remote planes, shaped as mbox
  uint4 *meta_in;         // shaped as mbox_meta
  uint64_t *maxapp_in;    // shaped as mbox_maxapp
  uint64_t *elo;          // [2][R][R][G] first entry index in embox rows
  uint64_t *elo_in;
  uint4 *embox;           // [2][R][R][E][ENT_META + C16][G] entries
  uint4 *embox_in;
  uint32_t *xrows;        // [2 roles][R][R][blocks] per-block plane summary
  // elections with placement: the raft launch's lanes are not a block of
  // one slot, so it adds its planes' summaries per lane to [R][R][blocks][4]
  // {max K rep, max K other, max E, flags} (atomics), and the records with
  // a term of their own bring their rterm rows along (rterm_in, shaped as
  // rterm)
  uint32_t *xslow;
  uint64_t *rterm_in;
  // engines of one process on one device bound for the zero-copy exchange
  // (drb_exchange_local_bind): per rank its outbox planes, from which the
  // step kernels read their remote planes in place of the *_in copies
  const struct PeerPlanes *peers;
  unsigned long long *counters;  // [8] (drb_round_out order from index 1)
  // flagged-replica list (drb_take_flagged): {g lo, g hi, slot | reason
  // << 8 | flags << 16, round}, appended with one atomic per marked lane
  uint4 *flog;
  unsigned long long *flog_n;
  uint64_t flog_cap;
  // listed rounds (drb_round_in.listed): per (role, slot) row the lanes
  // with work this round in group order, and their count
  uint32_t *act_list;               // [2][R][G]
  unsigned long long *act_total;    // [2][R][2 (heavy, light)]
  uint32_t *act_cnt, *act_off;      // [2][R][2][blocks]
  uint64_t *act_mask;               // [2][R][2][blocks][4] (a word a wave)
  // lean listed rounds (drb_lean.hpp): per row the light lanes the lean
  // kernel left to the full one, in ESC_SPLIT segments (a workgroup's by
  // its block index mod ESC_SPLIT), and their counts
  uint32_t *esc_list;               // [2][R][ESC_SPLIT][esc_seg(G)]
  uint32_t *esc_n;                  // [2][R][ESC_SPLIT]
};

// The escalation list of a row is split so that no one counter takes every
// wave's atomic: a lean round escalates a few lanes of nearly every wave,
// and atomics on one address serialise at ~14 ns each (profiles/r06_lean).
constexpr uint32_t ESC_SPLIT = 64;
__host__ __device__ inline uint64_t esc_seg(uint64_t G) {
  return ((((G + 255) / 256) + ESC_SPLIT - 1) / ESC_SPLIT) * 256;
}

__host__ __device__ inline uint64_t ix(const View &v, uint32_t slot,
                                       uint64_t g) {
  return (uint64_t)slot * v.G + g;
}
__host__ __device__ inline uint64_t u64_ix(const View &v, int f,
                                           uint32_t slot, uint64_t g) {
  return ((uint64_t)f * v.R + slot) * v.G + g;
}
__host__ __device__ inline uint64_t pk_ix(const View &v, int chunk,
                                          uint32_t slot, uint64_t g) {
  return ((uint64_t)chunk * v.R + slot) * v.G + g;
}
__host__ __device__ inline uint64_t u32_ix(const View &v, int f,
                                           uint32_t slot, uint64_t g) {
  return ((uint64_t)f * v.R + slot) * v.G + g;
}
__host__ __device__ inline uint64_t rem_ix(const View &v, uint32_t self,
                                           uint32_t peer, uint64_t g) {
  return ((uint64_t)self * v.R + peer) * v.G + g;
}
__host__ __device__ inline uint64_t ri_ix(const View &v, uint32_t slot,
                                          uint32_t d, uint64_t g) {
  return ((uint64_t)slot * 4 /*DRB_RI_DEPTH*/ + d) * v.G + g;
}
__host__ __device__ inline uint64_t ring_ix(const View &v, uint32_t slot,
                                            uint64_t index, uint32_t chunk,
                                            uint64_t g) {
  uint64_t rs = index & (v.W - 1);
  return (((uint64_t)slot * v.W + rs) * (ENT_META + v.C16) + chunk) * v.G + g;
}
// [buf][pair][chunk][k][g]: the first K records of a (sender, receiver)
// plane are one contiguous region per chunk (what a cross-rank exchange
// ships)
__host__ __device__ inline uint64_t mbox_ix(const View &v, uint32_t buf,
                                            uint32_t from, uint32_t to,
                                            uint32_t k, uint32_t chunk,
                                            uint64_t g) {
  uint64_t pair = (uint64_t)from * v.R + to;
  return ((((uint64_t)buf * v.R * v.R + pair) * MSG_CHUNKS + chunk) * v.MB +
          k) * v.G + g;
}
// entry rows of a remote (leader, follower) plane: [buf][pair][e][chunk][g]
__host__ __device__ inline uint64_t embox_ix(const View &v, uint32_t buf,
                                             uint32_t from, uint32_t to,
                                             uint32_t e, uint32_t chunk,
                                             uint64_t g) {
  uint64_t pair = (uint64_t)from * v.R + to;
  return ((((uint64_t)buf * v.R * v.R + pair) * v.E + e) *
              (ENT_META + v.C16) + chunk) * v.G + g;
}
// placement: is the (from, to) plane on another rank?
__host__ __device__ inline bool pair_remote(const View &v, uint32_t from,
                                            uint32_t to) {
  return (v.remote_mask >> (from * v.R + to)) & 1ull;
}
// the rank whose outbox holds this rank's inbound plane (from, to): slot s
// of group g lives on rank (g + s) mod N at lane g / N, so every lane of
// the plane comes from one rank, at the same lane (drb_place_peer, dir 1)
__host__ __device__ inline uint32_t plane_sender(const View &v,
                                                 uint32_t from, uint32_t to) {
  const uint32_t N = v.place_world, d = (to % N + N - from % N) % N;
  return (v.place_rank + N - d) % N;
}
// the global group of replica slot s at lane g (include/drb_engine.h)
__host__ __device__ inline uint64_t rterm_ix(const View &v, uint32_t buf,
                                             uint32_t from, uint32_t to,
                                             uint32_t k, uint64_t g) {
  return ((((uint64_t)buf * v.R + from) * v.R + to) * v.MB + k) * v.G + g;
}
__host__ __device__ inline uint64_t gid(const View &v, uint32_t s,
                                        uint64_t g) {
  if (v.place_world <= 1) return g;
  const uint32_t N = v.place_world;
  return (uint64_t)N * g + (v.place_rank + N - (s % N)) % N;
}
// The lane of a message's receiver on this engine (drb_ingest's shape
// checks): co-resident, the group; with replicas spread over ranks
// (drb_config.place_world), replica slot s of global group g lives on rank
// (g + s) mod N at lane g / N -- a message for another rank's replica is
// not this NodeHost's (ErrShardNotFound, nodehost.go:2072-2122).
__host__ __device__ inline bool ing_target(const View &v, uint64_t shard,
                                           uint64_t from, uint64_t to,
                                           uint64_t *lane) {
  const uint64_t gid = shard - v.first_shard_id;
  if (!(to >= 1 && to <= v.R && from >= 1 && from <= v.R && from != to))
    return false;
  uint64_t g = gid;
  if (v.place_world > 1) {
    if (gid >= v.total_groups ||
        (gid + (to - 1)) % v.place_world != v.place_rank)
      return false;
    g = gid / v.place_world;
  }
  *lane = g;
  return g < v.G;
}

__host__ __device__ inline uint64_t mmeta_ix(const View &v, uint32_t buf,
                                             uint32_t from, uint32_t to,
                                             uint64_t g) {
  return (((uint64_t)buf * v.R + from) * v.R + to) * v.G + g;
}
__host__ __device__ inline uint64_t kv_ix(const View &v, uint32_t slot,
                                          uint64_t g, uint32_t ks) {
  return (((uint64_t)slot * v.G + g) * v.KS + ks) * v.KVW;
}
// KV probe sequence: the slot of probe t (0 <= t < KS) for home slot h.
// The probes walk the home slot's 64 B group first, wrapping inside it,
// then the following groups: one 64 B fetch -- HBM's access granule for a
// random read (MI355X_MICROARCH.md; profiles/r02_kvline/calib.log) --
// holds a lookup's first spl probes, and a lookup loads the whole group at
// once (serve_reads_lane, apply_entry), so at the steady state's load of
// about 1/2 it nearly always resolves in one memory round trip.  Tables
// are 64 B aligned (KS * KVW * 16 B per replica).
__host__ __device__ inline uint32_t kv_spl(const View &v) {
  // slots per 64 B group: 4 / KVW when KVW is a power of two <= 4, else 1
  return (v.KVW <= 4 && (v.KVW & (v.KVW - 1)) == 0 && v.KS >= 4 / v.KVW)
             ? 4u / v.KVW
             : 1u;
}
__host__ __device__ inline uint32_t kv_probe(const View &v, uint32_t h,
                                             uint32_t t) {
  const uint32_t spl = kv_spl(v);
  const uint32_t grp = ((h / spl) + (t / spl)) & (v.KS / spl - 1);
  return grp * spl + ((h + t) & (spl - 1));
}
__host__ __device__ inline uint64_t prop_ix(const View &v, uint32_t ps,
                                            uint32_t j, uint32_t chunk,
                                            uint64_t g) {
  return (((uint64_t)ps * v.max_props + j) * (PROP_META + v.C16) + chunk) *
             v.G + g;
}
__host__ __device__ inline uint32_t fwd_ps(const View &v, uint32_t buf,
                                           uint32_t sender) {
  return v.P + buf * v.R + sender;
}
__host__ __device__ inline uint64_t rres_ix(const View &v, uint32_t slot,
                                            uint32_t k, uint32_t j,
                                            uint64_t g) {
  return (((uint64_t)slot * RTR_CAP + k) * v.max_reads + j) * v.G + g;
}
__host__ __device__ inline uint64_t rtr_ix(const View &v, uint32_t slot,
                                           uint32_t k, uint32_t chunk,
                                           uint64_t g) {
  return (((uint64_t)slot * RTR_CAP + k) * 2 + chunk) * v.G + g;
}

}  // namespace drb
