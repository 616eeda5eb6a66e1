// drb_msg.hpp -- compact in-HBM encoding of pb.Message (raftpb/message.go)
// for the messages of the fast path.
//
// A record is one 16 B chunk, plus a second 16 B chunk only when the fields
// do not fit the first.  Per (sender, receiver, round) the mailbox holds a
// header {round tag, info, sender term}: every fast-path message carries the
// sender's current term (raft.go:667-681) -- request types (ReadIndex)
// carry 0 and set TERM_ZERO -- so the term is stored once per header, and
// the info word summarises the records so a receiver decides whether the
// round stays on the fast path from the header alone.
//
//   c0 = {meta u32, x u32, a u64}       c1 = {b u64, c u64}
//   meta: type[0:8] reject[8] has_c1[9] term_zero[10] term_other[11]
//         lt_self[12] c_delta[13] hint_prev[14] hh32[15] n_entries[16:32]
//   Replicate      a=LogIndex; LogTerm = sender term (lt_self) else c1.b;
//                  Commit = LogIndex + (int32)x (c_delta) else c1.c
//   ReplicateResp  a=LogIndex  c1={Hint, 0}           (only when Reject/Hint)
//   Heartbeat      a=Commit    c1={Hint, HintHigh}    (when Hint set)
//   HeartbeatResp  a=Hint x=HintHigh (hh32)  else c1={Hint, HintHigh}
//   ReadIndex      a=Commit    c1={Hint, HintHigh}
//   ReadIndexResp  a=LogIndex  c1={Hint, HintHigh}
//   RequestVote    a=LogIndex  c1={LogTerm, Hint}      (elections)
//   RequestVoteResp, NoOP      Reject in meta, nothing else
//   other          a=LogIndex  c1={Hint, HintHigh}
// term_other: the record's term is not its header's; it is in the rterm
// side array (elections: a sender whose term changed within the round)
// hint_prev: the ReadIndex ctx {Hint, HintHigh} equals the last ctx written
// explicitly in this (sender, receiver) record sequence (a leader sends the
// same ctx twice per round: with the ReadIndex broadcast and, as peepCtx,
// with the tick heartbeat, raft.go:849-871; followers echo both).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "../../include/drb_engine.h"

namespace drb {

constexpr uint32_t MF_REJECT = 1u << 8;
constexpr uint32_t MF_HAS_C1 = 1u << 9;
constexpr uint32_t MF_TERM_ZERO = 1u << 10;
constexpr uint32_t MF_TERM_OTHER = 1u << 11;  // ingest: term != header term
constexpr uint32_t MF_LT_SELF = 1u << 12;
constexpr uint32_t MF_C_DELTA = 1u << 13;
constexpr uint32_t MF_HINT_PREV = 1u << 14;
constexpr uint32_t MF_HH32 = 1u << 15;

// Records of a (sender, receiver, round) sit in send order: the
// Replicates ascending from position 0 (node.sendReplicateMessages sends
// them ahead of the rest, engine.go:1334-1336, node.go:1016-1023), the
// other messages descending from position MB - 1 (processRaftUpdate ->
// sendMessages, node.go:1104-1108).
// header info word, per (sender, receiver, round)
constexpr uint32_t MI_NREP = 0x1fu;       // [0:5] Replicate records
constexpr int MI_NOTH = 5;                // [5:10] other records
constexpr int MI_NRI = 10;                // [10:15] ReadIndex records
constexpr int MI_NRR = 15;                // [15:20] ReplicateResp records
constexpr uint32_t MI_CNTS = MI_NREP | (0x1fu << MI_NOTH) |
                             (0x1fu << MI_NRI) | (0x1fu << MI_NRR);
constexpr uint32_t MI_RESP = 1u << 20;    // a ReplicateResp / HeartbeatResp
constexpr uint32_t MI_OFF_LEADER = 1u << 21;    // a type a leader leaves
constexpr uint32_t MI_OFF_FOLLOWER = 1u << 22;  // the fast path for / a
                                                // follower does
constexpr uint32_t MI_TERM = 1u << 23;        // a record carries the term
constexpr uint32_t MI_TERM_OTHER = 1u << 24;  // a record's term != header's
constexpr uint32_t MI_REJECT = 1u << 25;  // a rejecting ReplicateResp
// a Propose record (drb_config.forward_proposals: at most one per plane and
// round), and its entry count [27:31]: the entries travel by value in the
// sender's forward batch (View.fwd_props, prop_ix)
constexpr uint32_t MI_PROP = 1u << 26;
constexpr int MI_NPROP = 27;
__host__ __device__ inline uint32_t mi_nprop(uint32_t w) {
  return (w >> MI_NPROP) & 0xfu;
}
constexpr uint32_t MAX_FWD_PROPS = 15;
constexpr uint32_t MB_MAX = 24;  // records per (sender, receiver, round)
__host__ __device__ inline uint32_t mi_nrep(uint32_t w) { return w & MI_NREP; }
__host__ __device__ inline uint32_t mi_noth(uint32_t w) {
  return (w >> MI_NOTH) & 0x1fu;
}
__host__ __device__ inline uint32_t mi_count(uint32_t w) {
  return mi_nrep(w) + mi_noth(w);
}
// position of the j-th record of its kind
__host__ __device__ inline uint32_t rec_pos(bool rep, uint32_t j,
                                            uint32_t MB) {
  return rep ? j : MB - 1 - j;
}
// header tag word: bits [0:31] the round tag, bit 31 a Quiesce message
// (node.sendEnterQuiesceMessages, node.go:993-1005) from the sender this
// round; it precedes the sender's other non-Replicate messages (it is sent
// straight from stepNode, before the Update's messages)
constexpr uint32_t MQ_QUIESCE = 1u << 31;
constexpr uint32_t MQ_TAG = 0x7fffffffu;
__host__ __device__ inline bool tag_is(uint32_t word, uint64_t round) {
  return (word & MQ_TAG) == ((uint32_t)round & MQ_TAG);
}

// inbox round-tag byte, one per sender in the receiver's word: bits 0-6
// the round (mod 128) of the sender's last records to this replica, bit 7
// set when they include a Replicate or a ReplicateResp -- the receiver's
// round then appends, commits or applies, and a listed round steps it in
// the dense "heavy" part of its list (drb_engine.hip, k_active_scan)
constexpr uint32_t TAG_HEAVY = 0x80u;
__host__ __device__ inline uint8_t tag_byte(uint64_t round, uint32_t info) {
  const bool heavy = mi_nrep(info) != 0 || ((info >> MI_NRR) & 0x1fu) != 0 ||
                     (info & MI_PROP);
  return (uint8_t)((round & 0x7fu) | (heavy ? TAG_HEAVY : 0u));
}
__host__ __device__ inline bool tag_current(uint32_t byte, uint64_t round) {
  return (byte & 0x7fu) == (uint32_t)(round & 0x7fu);
}

struct Msg {
  uint32_t type, reject, n;
  uint64_t term, log_index, log_term, commit, hint, hint_high;
};

// ctx last written explicitly, per sender, with the receivers it went to
struct HintCtx {
  uint64_t lo, hi;
  uint32_t dests;  // bit d: receiver d's last explicit ctx is {lo, hi}
};

__host__ __device__ inline uint4 pack2(uint64_t a, uint64_t b) {
  uint4 q;
  q.x = (uint32_t)a;
  q.y = (uint32_t)(a >> 32);
  q.z = (uint32_t)b;
  q.w = (uint32_t)(b >> 32);
  return q;
}
__host__ __device__ inline uint64_t q_lo(uint4 q) {
  return (uint64_t)q.x | ((uint64_t)q.y << 32);
}
__host__ __device__ inline uint64_t q_hi(uint4 q) {
  return (uint64_t)q.z | ((uint64_t)q.w << 32);
}

// PreVote messages carry a term of their own (r.term + 1, or the one a
// pre-vote is granted at), not the sender's
__host__ __device__ inline bool is_prevote_type(uint32_t t) {
  return t == DRB_MSG_REQUEST_PREVOTE || t == DRB_MSG_REQUEST_PREVOTE_RESP;
}
__host__ __device__ inline bool is_request_type(uint32_t t) {
  return t == DRB_MSG_PROPOSE || t == DRB_MSG_READ_INDEX ||
         t == DRB_MSG_LEADER_TRANSFER;
}
// types whose {Hint, HintHigh} is a ReadIndex ctx (dedup candidates)
__host__ __device__ inline bool is_ctx_type(uint32_t t) {
  return t == DRB_MSG_HEARTBEAT || t == DRB_MSG_HEARTBEAT_RESP ||
         t == DRB_MSG_READ_INDEX || t == DRB_MSG_READ_INDEX_RESP;
}

// header info contribution of one record (n: a Propose's entries)
__host__ __device__ inline uint32_t msg_info(uint32_t type, bool term_zero,
                                             bool reject = false,
                                             uint32_t n = 0) {
  uint32_t i = type == DRB_MSG_REPLICATE ? 1u : 1u << MI_NOTH;  // counts
  if (reject && type == DRB_MSG_REPLICATE_RESP) i |= MI_REJECT;
  if (type == DRB_MSG_PROPOSE)
    i |= MI_PROP | ((n < MAX_FWD_PROPS ? n : MAX_FWD_PROPS) << MI_NPROP);
  if (type == DRB_MSG_READ_INDEX) i += 1u << MI_NRI;
  if (type == DRB_MSG_REPLICATE_RESP) i += 1u << MI_NRR;
  if (type == DRB_MSG_REPLICATE_RESP || type == DRB_MSG_HEARTBEAT_RESP)
    i |= MI_RESP;
  if (!(type == DRB_MSG_REPLICATE_RESP || type == DRB_MSG_HEARTBEAT_RESP ||
        type == DRB_MSG_READ_INDEX || type == DRB_MSG_PROPOSE))
    i |= MI_OFF_LEADER;  // (a Propose without forward rows: the pre-pass)
  if (!(type == DRB_MSG_REPLICATE || type == DRB_MSG_HEARTBEAT ||
        type == DRB_MSG_READ_INDEX_RESP))
    i |= MI_OFF_FOLLOWER;
  if (!term_zero) i |= MI_TERM;
  return i;
}

// Encodes m (m.term must be the header term or 0 for request types) to
// receiver `dest`.  hc may be null (no ctx dedup).  Returns has_c1.
__host__ __device__ inline bool msg_encode(const Msg &m, uint32_t dest,
                                           HintCtx *hc, uint4 &c0, uint4 &c1) {
  uint64_t a = 0, b = 0, c = 0;
  uint32_t x = 0, fl = 0;
  bool has = false;
  const bool ctx = is_ctx_type(m.type) && (m.hint | m.hint_high) != 0;
  bool dedup = false;
  if (ctx && hc) {
    dedup = hc->lo == m.hint && hc->hi == m.hint_high &&
            ((hc->dests >> dest) & 1u);
    if (!dedup) {
      if (hc->lo == m.hint && hc->hi == m.hint_high) {
        hc->dests |= 1u << dest;
      } else {
        hc->lo = m.hint;
        hc->hi = m.hint_high;
        hc->dests = 1u << dest;
      }
    }
  }
  switch (m.type) {
    case DRB_MSG_REPLICATE: {
      a = m.log_index;
      const int64_t d = (int64_t)(m.commit - m.log_index);
      if (m.log_term == m.term && m.term != 0 && d >= INT32_MIN &&
          d <= INT32_MAX) {
        fl |= MF_LT_SELF | MF_C_DELTA;
        x = (uint32_t)(int32_t)d;
      } else {
        b = m.log_term;
        c = m.commit;
        has = true;
      }
      break;
    }
    case DRB_MSG_REPLICATE_RESP:
      a = m.log_index;
      b = m.hint;
      has = m.reject || m.hint;
      break;
    case DRB_MSG_HEARTBEAT:
      a = m.commit;
      b = m.hint;
      c = m.hint_high;
      has = ctx && !dedup;
      break;
    case DRB_MSG_HEARTBEAT_RESP:
      if (ctx && !dedup) {
        if (m.hint_high <= 0xffffffffull) {
          fl |= MF_HH32;
          a = m.hint;
          x = (uint32_t)m.hint_high;
        } else {
          b = m.hint;
          c = m.hint_high;
          has = true;
        }
      }
      break;
    case DRB_MSG_READ_INDEX:
      a = m.commit;
      b = m.hint;
      c = m.hint_high;
      has = !dedup;
      break;
    case DRB_MSG_READ_INDEX_RESP:
      a = m.log_index;
      b = m.hint;
      c = m.hint_high;
      has = !dedup;
      break;
    case DRB_MSG_REQUEST_VOTE:
    case DRB_MSG_REQUEST_PREVOTE:
      a = m.log_index;
      b = m.log_term;
      c = m.hint;
      has = true;
      break;
    case DRB_MSG_REQUEST_VOTE_RESP:
    case DRB_MSG_REQUEST_PREVOTE_RESP:
    case DRB_MSG_NOOP:
      break;
    case DRB_MSG_PROPOSE:  // {Type, From, Entries} (peer.go:118-124)
      a = m.log_index;
      b = m.hint;
      c = m.hint_high;
      has = (b | c) != 0;
      break;
    default:
      a = m.log_index;
      b = m.hint;
      c = m.hint_high;
      has = true;
      break;
  }
  if (dedup) fl |= MF_HINT_PREV;
  fl |= (m.type & 0xffu) | (m.reject ? MF_REJECT : 0) | (has ? MF_HAS_C1 : 0) |
        (m.n << 16);
  if (is_request_type(m.type) && m.term == 0) fl |= MF_TERM_ZERO;
  c0 = pack2(0, a);
  c0.x = fl;
  c0.y = x;
  c1 = pack2(b, c);
  return has;
}

// c1 is only read when MF_HAS_C1 is set.  prev_lo/prev_hi: the receiver's
// last explicit ctx of this (sender, receiver) sequence, updated here.
__host__ __device__ inline Msg msg_decode(uint4 c0, uint4 c1,
                                          uint64_t sender_term,
                                          uint64_t &prev_lo,
                                          uint64_t &prev_hi) {
  Msg m;
  const uint32_t meta = c0.x;
  const bool has = (meta & MF_HAS_C1) != 0;
  m.type = meta & 0xffu;
  m.reject = (meta & MF_REJECT) ? 1 : 0;
  m.n = meta >> 16;
  m.term = (meta & MF_TERM_ZERO) ? 0 : sender_term;
  const uint64_t a = q_hi(c0);
  const uint64_t b = has ? q_lo(c1) : 0, c = has ? q_hi(c1) : 0;
  m.log_index = m.log_term = m.commit = m.hint = m.hint_high = 0;
  switch (m.type) {
    case DRB_MSG_REPLICATE:
      m.log_index = a;
      if (meta & MF_LT_SELF) {
        m.log_term = sender_term;
        m.commit = a + (uint64_t)(int64_t)(int32_t)c0.y;
      } else {
        m.log_term = b;
        m.commit = c;
      }
      break;
    case DRB_MSG_REPLICATE_RESP:
      m.log_index = a;
      m.hint = b;
      break;
    case DRB_MSG_HEARTBEAT:
      m.commit = a;
      m.hint = b;
      m.hint_high = c;
      break;
    case DRB_MSG_HEARTBEAT_RESP:
      if (meta & MF_HH32) {
        m.hint = a;
        m.hint_high = c0.y;
      } else {
        m.hint = b;
        m.hint_high = c;
      }
      break;
    case DRB_MSG_READ_INDEX:
      m.commit = a;
      m.hint = b;
      m.hint_high = c;
      break;
    case DRB_MSG_REQUEST_VOTE:
    case DRB_MSG_REQUEST_PREVOTE:
      m.log_index = a;
      m.log_term = b;
      m.hint = c;
      break;
    case DRB_MSG_REQUEST_VOTE_RESP:
    case DRB_MSG_REQUEST_PREVOTE_RESP:
    case DRB_MSG_NOOP:
      break;
    default:
      m.log_index = a;
      m.hint = b;
      m.hint_high = c;
      break;
  }
  if (is_ctx_type(m.type)) {
    if (meta & MF_HINT_PREV) {
      m.hint = prev_lo;
      m.hint_high = prev_hi;
    } else if ((m.hint | m.hint_high) != 0) {
      prev_lo = m.hint;
      prev_hi = m.hint_high;
    }
  }
  return m;
}

}  // namespace drb
