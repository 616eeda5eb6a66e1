// drb_ring.hpp -- the resident window's entries as the byte encoders see
// them (the step kernel's EntriesToSave, the tan record writer).
#pragma once
#include "drb_codec.hpp"
#include "drb_layout.hpp"

namespace drb {

// The fields of window entry idx of replica (slot, g) as the encoder sees
// them; `compact` zeroes Term and Index (compactBatchFields).
__device__ __forceinline__ EntryHdr ring_entry_hdr(const View &v, uint32_t slot, uint64_t g,
                                uint64_t idx, bool compact) {
  const uint4 m0 = v.ring[ring_ix(v, slot, idx, 0, g)];
  const uint4 m1 = v.ring[ring_ix(v, slot, idx, 1, g)];
  const uint4 m2 = v.ring[ring_ix(v, slot, idx, 2, g)];
  EntryHdr e;
  e.term = compact ? 0 : lo64(m0);
  e.index = compact ? 0 : idx;
  e.key = hi64(m0);
  e.client_id = lo64(m1);
  e.series_id = hi64(m1);
  e.responded_to = lo64(m2);
  e.type = m2.z;
  e.cmd_len = m2.w;
  return e;
}

// Entry.marshalTo (raft_optimized.go:166-300) of e, its Cmd read from the
// window chunk by chunk, into any byte sink O
template <class O>
__device__ __forceinline__ void emit_entry(O &o, const View &v, uint32_t slot, uint64_t g,
                        uint64_t idx, const EntryHdr &e) {
  colfer_u64(o, 0, e.term);
  colfer_u64(o, 1, e.index);
  if (e.type != 0) {
    bo_byte(o, 2);
    bo_varint(o, e.type);
  }
  colfer_u64(o, 3, e.key);
  colfer_u64(o, 4, e.client_id);
  colfer_u64(o, 5, e.series_id);
  colfer_u64(o, 6, e.responded_to);
  if (e.cmd_len != 0) {
    bo_byte(o, 7);
    bo_varint(o, e.cmd_len);
    for (uint32_t c = 0; c * 16 < e.cmd_len; ++c) {
      const uint4 q = v.ring[ring_ix(v, slot, idx, ENT_META + c, g)];
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (uint32_t b = 0; b < 16; ++b)
        if (c * 16 + b < e.cmd_len) bo_byte(o, w[b >> 2] >> (8 * (b & 3)));
    }
  }
  bo_byte(o, 0x7f);
}

}  // namespace drb
