// drb_msg.hpp -- compact in-HBM encoding of pb.Message (raftpb/message.go)
// for the messages of the fast path.
//
// A record is one 16 B chunk, plus a second 16 B chunk only when the type
// carries more than one 64-bit field.  The sender's term is stored once per
// (sender, round) in the mailbox meta word instead of in every message:
// within a fast-path round every message a replica sends carries its
// current term (raft.go:667-681), except request types (ReadIndex), which
// carry 0 and set TERM_ZERO.
//
//   c0 = {meta u32, 0, a u64}       c1 = {b u64, c u64}
//   meta: type[0:8] reject[8] has_c1[9] term_zero[10] term_other[11]
//         n_entries[16:32]
//   Replicate      a=LogIndex  c1={LogTerm, Commit}
//   ReplicateResp  a=LogIndex  c1={Hint, 0}            (only when Reject)
//   Heartbeat      a=Commit    c1={Hint, HintHigh}     (only when Hint set)
//   HeartbeatResp  a=0         c1={Hint, HintHigh}     (only when Hint set)
//   ReadIndexResp  a=LogIndex  c1={Hint, HintHigh}
//   ReadIndex      a=Commit    c1={Hint, HintHigh}
//   other          a=LogIndex  c1={Hint, HintHigh}
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "../../include/drb_engine.h"

namespace drb {

constexpr uint32_t MF_REJECT = 1u << 8;
constexpr uint32_t MF_HAS_C1 = 1u << 9;
constexpr uint32_t MF_TERM_ZERO = 1u << 10;
constexpr uint32_t MF_TERM_OTHER = 1u << 11;  // ingest: term != meta term

struct Msg {
  uint32_t type, reject, n;
  uint64_t term, log_index, log_term, commit, hint, hint_high;
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

__host__ __device__ inline bool is_request_type(uint32_t t) {
  return t == DRB_MSG_PROPOSE || t == DRB_MSG_READ_INDEX ||
         t == DRB_MSG_LEADER_TRANSFER;
}

// returns true when c1 is needed
__host__ __device__ inline bool msg_encode(const Msg &m, uint4 &c0, uint4 &c1) {
  uint64_t a = 0, b = 0, c = 0;
  bool has = false;
  switch (m.type) {
    case DRB_MSG_REPLICATE:
      a = m.log_index;
      b = m.log_term;
      c = m.commit;
      has = true;
      break;
    case DRB_MSG_REPLICATE_RESP:
      a = m.log_index;
      b = m.hint;
      has = m.reject || m.hint;
      break;
    case DRB_MSG_HEARTBEAT:
      a = m.commit;
      b = m.hint;
      c = m.hint_high;
      has = m.hint || m.hint_high;
      break;
    case DRB_MSG_HEARTBEAT_RESP:
      b = m.hint;
      c = m.hint_high;
      has = m.hint || m.hint_high;
      break;
    case DRB_MSG_READ_INDEX:
      a = m.commit;
      b = m.hint;
      c = m.hint_high;
      has = true;
      break;
    default:
      a = m.log_index;
      b = m.hint;
      c = m.hint_high;
      has = true;
      break;
  }
  uint32_t meta = (m.type & 0xffu) | (m.reject ? MF_REJECT : 0) |
                  (has ? MF_HAS_C1 : 0) | (m.n << 16);
  if (is_request_type(m.type) && m.term == 0) meta |= MF_TERM_ZERO;
  c0 = pack2(0, a);
  c0.x = meta;
  c0.y = 0;
  c1 = pack2(b, c);
  return has;
}

// c1 is only read by the caller when MF_HAS_C1 is set
__host__ __device__ inline Msg msg_decode(uint4 c0, uint4 c1, bool has_c1,
                                          uint64_t sender_term) {
  Msg m;
  uint32_t meta = c0.x;
  m.type = meta & 0xffu;
  m.reject = (meta & MF_REJECT) ? 1 : 0;
  m.n = meta >> 16;
  m.term = (meta & MF_TERM_ZERO) ? 0 : sender_term;
  uint64_t a = q_hi(c0);
  uint64_t b = has_c1 ? q_lo(c1) : 0, c = has_c1 ? q_hi(c1) : 0;
  m.log_index = m.log_term = m.commit = m.hint = m.hint_high = 0;
  switch (m.type) {
    case DRB_MSG_REPLICATE:
      m.log_index = a;
      m.log_term = b;
      m.commit = c;
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
      m.hint = b;
      m.hint_high = c;
      break;
    case DRB_MSG_READ_INDEX:
      m.commit = a;
      m.hint = b;
      m.hint_high = c;
      break;
    default:
      m.log_index = a;
      m.hint = b;
      m.hint_high = c;
      break;
  }
  return m;
}

}  // namespace drb
