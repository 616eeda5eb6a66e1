// drb_tan.hpp -- the tan LogDB's log records on the GPU.
//
// The regular tan (internal/tan/logdb.go:103-109, the plugin/tan Factory)
// keeps one log per raft node.  SaveRaftState (logdb.go:306-340) hands
// every pb.Update of a step round to db.write (internal/tan/db.go:97-130):
// the Update is marshalled (raftpb/update.go:128-169), written as one
// record by the record writer (internal/tan/record.go:548-591) -- 7-byte
// chunk headers inside 32 KiB blocks, each chunk's checksum the low 32 bits
// of XXH64 over its type byte and payload (internal/tan/crc.go:21-23,
// github.com/cespare/xxhash/v2) -- and the node's state is remembered for
// the next Update's skip / sync decision.
//
// Here one lane is one replica: every replica's log is independent, so the
// round's records are built in parallel straight from the step round's
// Update summary (tan_sum, written by step_kernel) and the resident
// window.  Each lane writes the bytes its log file grows by -- zero padding
// included -- into its save buffer, with {file offset, length, sync,
// new-log} for the host's pwrite / fsync.  Chunk checksums are folded as
// the bytes are produced (streaming XXH64 over 32-byte stripes in
// registers) and patched into the chunk headers, so nothing is read back.
#pragma once
#include "drb_codec.hpp"
#include "drb_layout.hpp"
#include "drb_step.hpp"  // ring_entry_hdr, emit_entry

namespace drb {

constexpr uint32_t TAN_BLOCK = 32768;  // blockSize (record.go:128)
constexpr uint32_t TAN_HDR = 7;        // legacyHeaderSize (record.go:130)
constexpr uint64_t TAN_MAX_LOG = 64ull << 20;  // MaxLogFileSize (options.go:29)

// tan_sum[2] flags (step_kernel, getUpdate block)
constexpr uint32_t TS_HAVE = 1;   // the replica produced a pb.Update
constexpr uint32_t TS_STATE = 2;  // its State is not empty
constexpr uint32_t TS_TV = 4;     // Term or Vote differ from Peer.prevState
// tan_st.w: nodeStates state of the replica is not empty
constexpr uint32_t TST_STATE = 1;

// ------------------------------------------------------------ XXH64
constexpr uint64_t XP1 = 0x9E3779B185EBCA87ull;
constexpr uint64_t XP2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t XP3 = 0x165667B19E3779F9ull;
constexpr uint64_t XP4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t XP5 = 0x27D4EB2F165667C5ull;

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
  return (x << r) | (x >> (64 - r));
}
__device__ __forceinline__ uint64_t xx_round(uint64_t acc, uint64_t in) {
  return rotl64(acc + in * XP2, 31) * XP1;
}
__device__ __forceinline__ uint64_t xx_merge(uint64_t acc, uint64_t v) {
  return (acc ^ xx_round(0, v)) * XP1 + XP4;
}

// streaming XXH64 with seed 0: the current 32-byte stripe in four words
struct Xxh {
  uint64_t v0, v1, v2, v3;
  uint64_t b0, b1, b2, b3;
  uint32_t n;      // bytes in the stripe
  uint32_t total;  // bytes hashed
};

__device__ __forceinline__ void xx_init(Xxh &h) {
  h.v0 = XP1 + XP2;
  h.v1 = XP2;
  h.v2 = 0;
  h.v3 = 0 - XP1;
  h.b0 = h.b1 = h.b2 = h.b3 = 0;
  h.n = h.total = 0;
}

__device__ __forceinline__ void xx_byte(Xxh &h, uint32_t b) {
  const uint64_t x = (uint64_t)(b & 0xffu) << (8 * (h.n & 7));
  const uint32_t w = h.n >> 3;
  h.b0 |= w == 0 ? x : 0;
  h.b1 |= w == 1 ? x : 0;
  h.b2 |= w == 2 ? x : 0;
  h.b3 |= w == 3 ? x : 0;
  h.total++;
  if (++h.n == 32) {
    h.v0 = xx_round(h.v0, h.b0);
    h.v1 = xx_round(h.v1, h.b1);
    h.v2 = xx_round(h.v2, h.b2);
    h.v3 = xx_round(h.v3, h.b3);
    h.b0 = h.b1 = h.b2 = h.b3 = 0;
    h.n = 0;
  }
}

// Sum64's tail and avalanche over the bytes left in the stripe
__device__ __forceinline__ uint64_t xx_final(const Xxh &h) {
  uint64_t acc;
  if (h.total >= 32) {
    acc = rotl64(h.v0, 1) + rotl64(h.v1, 7) + rotl64(h.v2, 12) +
          rotl64(h.v3, 18);
    acc = xx_merge(acc, h.v0);
    acc = xx_merge(acc, h.v1);
    acc = xx_merge(acc, h.v2);
    acc = xx_merge(acc, h.v3);
  } else {
    acc = XP5;
  }
  acc += h.total;
  const uint32_t words = h.n >> 3;
  if (words > 0) acc = rotl64(acc ^ xx_round(0, h.b0), 27) * XP1 + XP4;
  if (words > 1) acc = rotl64(acc ^ xx_round(0, h.b1), 27) * XP1 + XP4;
  if (words > 2) acc = rotl64(acc ^ xx_round(0, h.b2), 27) * XP1 + XP4;
  uint64_t t = words == 0 ? h.b0 : words == 1 ? h.b1 : words == 2 ? h.b2 : h.b3;
  uint32_t r = h.n & 7;
  if (r >= 4) {
    acc = rotl64(acc ^ (t & 0xffffffffull) * XP1, 23) * XP2 + XP3;
    t >>= 32;
    r -= 4;
  }
  for (uint32_t k = 0; k < r; ++k) {
    acc = rotl64(acc ^ (t & 0xffull) * XP5, 11) * XP1;
    t >>= 8;
  }
  acc ^= acc >> 33;
  acc *= XP2;
  acc ^= acc >> 29;
  acc *= XP3;
  acc ^= acc >> 32;
  return acc;
}

// ------------------------------------------------------------ record out
// The bytes one record adds to its log file: zero padding when the chunk
// header does not fit in the block (getNext, record.go:548-573), then the
// chunks (singleWriter.Write, :628-653), headers filled by fillHeader
// (:468-487).  Bytes leave as 16-byte stores from a register accumulator;
// a finished chunk's checksum is patched into its header.
struct TanOut {
  uint4 *dst;
  uint32_t cap16;
  uint64_t lo, hi;  // pending bytes
  uint32_t n;       // pending byte count
  uint32_t pos;     // 16 B chunks stored
  uint32_t total;   // bytes produced
  uint32_t bpos;    // position in the block of the next byte
  uint32_t hdr;     // output position of the current chunk's header
  uint32_t cleft;   // payload bytes left in the current chunk
  uint32_t rleft;   // payload bytes of the record not yet in a chunk
  bool first;       // the current chunk is the record's first
  bool overflow;
  Xxh h;
};

__device__ __forceinline__ void to_flush16(TanOut &o) {
  if (o.pos < o.cap16)
    o.dst[o.pos] = make_uint4((uint32_t)o.lo, (uint32_t)(o.lo >> 32),
                              (uint32_t)o.hi, (uint32_t)(o.hi >> 32));
  else
    o.overflow = true;
  o.pos++;
  o.lo = o.hi = 0;
  o.n = 0;
}

__device__ __forceinline__ void to_raw(TanOut &o, uint32_t b) {
  b &= 0xffu;
  if (o.n < 8)
    o.lo |= (uint64_t)b << (8 * o.n);
  else
    o.hi |= (uint64_t)b << (8 * (o.n - 8));
  o.total++;
  if (++o.bpos == TAN_BLOCK) o.bpos = 0;
  if (++o.n == 16) to_flush16(o);
}

// byte p of the output, already produced as 0: set it
__device__ __forceinline__ void to_patch(TanOut &o, uint32_t p, uint32_t b) {
  b &= 0xffu;
  const uint32_t flushed = o.pos * 16;
  if (p < flushed) {
    if (p / 16 < o.cap16) reinterpret_cast<uint8_t *>(o.dst)[p] = (uint8_t)b;
  } else {
    const uint32_t k = p - flushed;
    if (k < 8)
      o.lo |= (uint64_t)b << (8 * k);
    else
      o.hi |= (uint64_t)b << (8 * (k - 8));
  }
}

// a chunk header at the current position: checksum placeholder, length,
// type; its checksum covers the type byte and the payload
__device__ __forceinline__ void to_chunk(TanOut &o, bool first) {
  const uint32_t room = TAN_BLOCK - o.bpos - TAN_HDR;
  const uint32_t len = o.rleft < room ? o.rleft : room;
  o.rleft -= len;
  const bool last = o.rleft == 0;
  // fullChunkType 1, firstChunkType 2, middleChunkType 3, lastChunkType 4
  const uint32_t type = last ? (first ? 1u : 4u) : (first ? 2u : 3u);
  o.hdr = o.total;
  for (int k = 0; k < 4; ++k) to_raw(o, 0);
  to_raw(o, len);
  to_raw(o, len >> 8);
  to_raw(o, type);
  xx_init(o.h);
  xx_byte(o.h, type);
  o.cleft = len;
}

__device__ __forceinline__ void to_end_chunk(TanOut &o) {
  const uint32_t c = (uint32_t)xx_final(o.h);
  for (int k = 0; k < 4; ++k) to_patch(o, o.hdr + k, c >> (8 * k));
}

// begins a record of `len` payload bytes at block position bpos
__device__ __forceinline__ void to_begin(TanOut &o, uint4 *dst, uint32_t cap16,
                                         uint32_t bpos, uint32_t len) {
  o.dst = dst;
  o.cap16 = cap16;
  o.lo = o.hi = 0;
  o.n = o.pos = o.total = 0;
  o.bpos = bpos;
  o.overflow = false;
  if (bpos + TAN_HDR > TAN_BLOCK)  // the rest of the block stays zero
    while (o.bpos != 0) to_raw(o, 0);
  o.rleft = len;
  to_chunk(o, true);
}

// one payload byte (the colfer / Update encoders' sink)
__device__ __forceinline__ void bo_byte(TanOut &o, uint32_t b) {
  if (o.cleft == 0) {  // the block is full: the next chunk (record.go:639)
    to_end_chunk(o);
    to_chunk(o, false);
  }
  to_raw(o, b);
  xx_byte(o.h, b);
  o.cleft--;
}

__device__ __forceinline__ void to_le32(TanOut &o, uint32_t x) {
  for (int k = 0; k < 4; ++k) bo_byte(o, x >> (8 * k));
}

__device__ __forceinline__ void to_finish(TanOut &o) {
  to_end_chunk(o);
  if (o.n) to_flush16(o);
}

// bytes a record of `len` payload bytes adds at block position bpos
__device__ __forceinline__ uint32_t tan_appended(uint32_t bpos, uint32_t len) {
  uint32_t pad = 0;
  if (bpos + TAN_HDR > TAN_BLOCK) {
    pad = TAN_BLOCK - bpos;
    bpos = 0;
  }
  uint32_t total = pad, left = len;
  for (;;) {
    const uint32_t room = TAN_BLOCK - bpos - TAN_HDR;
    const uint32_t k = left < room ? left : room;
    total += TAN_HDR + k;
    left -= k;
    if (left == 0) return total;
    bpos = 0;
  }
}

// ------------------------------------------------------------ the kernel
__host__ __device__ inline uint64_t tan_sum_ix(const View &v, uint32_t k,
                                               uint32_t slot, uint64_t g) {
  return ((uint64_t)k * v.R + slot) * v.G + g;
}

// State.Size (raftpb/state.go:44-54)
__device__ __forceinline__ uint32_t state_size(uint64_t t, uint64_t vo,
                                               uint64_t c) {
  return 3 + varint_size(t) + varint_size(vo) + varint_size(c);
}

// per block: {bytes, records, syncs, new logs} added to tan_ctr rows
__global__ __launch_bounds__(256) void k_tan_encode(View v, uint32_t round,
                                                    uint64_t max_log) {
  __shared__ unsigned long long part[4];
  if (threadIdx.x < 4) part[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t slot = (uint32_t)(t / v.G);
  const uint64_t g = t - (uint64_t)slot * v.G;
  uint32_t c_bytes = 0, c_rec = 0, c_sync = 0, c_new = 0;
  if (slot < v.R) {
    const uint64_t i = ix(v, slot, g);
    const uint4 s2 = v.tan_sum[tan_sum_ix(v, 2, slot, g)];
    const uint32_t fl = v.u32[u32_ix(v, W_FLAGS, slot, g)];
    uint4 rec = make_uint4(0, 0, 0, 0);
    // an Update of this round from a replica that stayed on the fast path
    if (s2.z == round && (s2.y & TS_HAVE) && (fl & DRB_F_HOSTED) &&
        !(fl & (DRB_F_FALLBACK | DRB_F_ERROR))) {
      const uint4 s0 = v.tan_sum[tan_sum_ix(v, 0, slot, g)];
      const uint4 s1 = v.tan_sum[tan_sum_ix(v, 1, slot, g)];
      uint4 st = v.tan_st[i];
      uint64_t off = (uint64_t)st.x | ((uint64_t)st.y << 32);
      const uint32_t n_save = s2.x;
      const bool u_state = (s2.y & TS_STATE) != 0;
      const bool st_state = (st.w & TST_STATE) != 0;
      rec.x = st.x;
      rec.y = st.y;
      rec.w = st.z << 8;
      // db.write (db.go:97-116): IsStateEqual(u.State, st) with no entries
      // (the stored state is the empty one or Peer.prevState, see DESIGN)
      if (u_state || st_state || n_save > 0) {
        const uint64_t term = lo64(s0), vote = hi64(s0), commit = lo64(s1);
        const uint64_t save_lo = hi64(s1);
        // stateSyncChange (db.go:88-90)
        const bool sync =
            n_save > 0 ||
            (u_state ? (!st_state || (s2.y & TS_TV)) : st_state);
        // makeRoomForWrite (db.go:175-180) -> createNewLog (open.go:171)
        const bool new_log = off >= max_log;
        if (new_log) {
          off = 0;
          st.z++;
        }
        // the marshalled Update's size (update.go:128-169)
        const uint64_t shard = v.first_shard_id + gid(v, slot, g);
        uint32_t len = varint_size(shard) + varint_size(slot + 1) + 1 + 4 + 1;
        if (u_state) len += 4 + state_size(term, vote, commit);
        for (uint32_t k = 0; k < n_save; ++k)
          len += 4 + entry_size(ring_entry_hdr(v, slot, g, save_lo + k, false));
        const uint32_t bpos = (uint32_t)(off % TAN_BLOCK);
        const uint32_t add = tan_appended(bpos, len);
        if (add > v.save_cap16 * 16) {  // bounded by the pre-pass
          rec.w = (st.z << 8) | DRB_TAN_OVERFLOW;
        } else {
          TanOut o;
          to_begin(o, v.save_buf + i * v.save_cap16, v.save_cap16, bpos, len);
          bo_varint(o, shard);
          bo_varint(o, slot + 1);
          if (u_state) {
            bo_byte(o, 1);
            to_le32(o, state_size(term, vote, commit));
            bo_byte(o, 0x08);
            bo_varint(o, term);
            bo_byte(o, 0x10);
            bo_varint(o, vote);
            bo_byte(o, 0x18);
            bo_varint(o, commit);
          } else {
            bo_byte(o, 0);
          }
          to_le32(o, n_save);
          for (uint32_t k = 0; k < n_save; ++k) {
            const EntryHdr e = ring_entry_hdr(v, slot, g, save_lo + k, false);
            to_le32(o, entry_size(e));
            emit_entry(o, v, slot, g, save_lo + k, e);
          }
          bo_byte(o, 0);  // IsEmptySnapshot
          to_finish(o);
          // writeRecord's offset (record.go:589) = the file's new size
          rec.x = (uint32_t)off;
          rec.y = (uint32_t)(off >> 32);
          rec.z = o.total;
          rec.w = (st.z << 8) | DRB_TAN_WRITTEN | (sync ? DRB_TAN_SYNC : 0) |
                  (new_log ? DRB_TAN_NEW_LOG : 0);
          off += o.total;
          st.x = (uint32_t)off;
          st.y = (uint32_t)(off >> 32);
          st.w = u_state ? TST_STATE : 0;  // nodeStates.setState(u.State)
          v.tan_st[i] = st;
          c_bytes = o.total;
          c_rec = 1;
          c_sync = sync;
          c_new = new_log;
        }
      }
    }
    v.tan_rec[i] = rec;
    v.save_len[i] = rec.z;
  }
  if (c_rec) {
    atomicAdd(&part[0], (unsigned long long)c_bytes);
    atomicAdd(&part[1], 1ull);
    if (c_sync) atomicAdd(&part[2], 1ull);
    if (c_new) atomicAdd(&part[3], 1ull);
  }
  __syncthreads();
  if (threadIdx.x < 4)
    v.tan_ctr[(uint64_t)blockIdx.x * 4 + threadIdx.x] += part[threadIdx.x];
}

}  // namespace drb
