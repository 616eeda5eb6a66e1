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
// Here one lane is one record: every replica's log is independent, so the
// round's records are built in parallel straight from the step round's
// Update summary (tan_sum, written by step_kernel) and the resident
// window.  Each lane writes the bytes its log file grows by -- zero padding
// included -- into its save buffer, with {file offset, length, sync,
// new-log} for the host's pwrite / fsync, in one pass: 16-byte stores, the
// chunk checksums hashed on the way out.
#pragma once
#include "drb_codec.hpp"
#include "drb_layout.hpp"
#include "../../include/drb_engine.h"
#include "drb_ring.hpp"  // ring_entry_hdr, emit_entry

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

// ------------------------------------------------------------ record out
// The bytes one record adds to its log file go out as 16-byte stores from a
// register accumulator: zero padding when the header does not fit in the
// block (getNext, record.go:548-573), a 7-byte header, the payload, and a
// new header wherever the payload reaches a block's end with bytes left
// (singleWriter.Write, :628-653).  Each chunk's checksum -- the low 32 bits
// of XXH64 (seed 0) over its type byte and payload (fillHeader, :468-487)
// -- is computed as the bytes go out, by a streaming XXH64 kept in
// registers, and patched into the chunk's header when the chunk ends
// (into the accumulator if that header has not been stored yet).
struct TanOut {
  uint4 *dst;
  uint32_t cap16;
  uint32_t start;   // byte position of the record in dst
  uint32_t skip;    // bytes of the first 16 B word that precede the record
  bool shared;      // dst is a log's staging: the last word is shared too
  uint64_t lo, hi;  // pending bytes
  uint32_t n;       // pending byte count
  uint32_t pos;     // 16 B chunks stored
  uint32_t total;   // bytes produced
  uint32_t bpos;    // position in the block of the next byte
  uint32_t left;    // payload bytes still to come
  uint32_t hdr;     // byte position of the open chunk's header
  bool first;       // no chunk opened yet
  // XXH64 of the open chunk: stripe accumulators, the partial stripe
  uint64_t v0, v1, v2, v3, h0, h1, h2, h3;
  uint32_t hn;    // bytes in the partial stripe
  uint32_t hlen;  // bytes hashed
};

// bytes [from, to) of the pending word, one byte store each (a word the
// record shares with its neighbour in a log's staging)
__device__ __forceinline__ void to_store_bytes(TanOut &o, uint32_t from,
                                               uint32_t to) {
  if (o.pos >= o.cap16) return;
  uint8_t *b = reinterpret_cast<uint8_t *>(o.dst + o.pos);
  for (uint32_t k = from; k < to; ++k)
    b[k] = (uint8_t)(k < 8 ? o.lo >> (8 * k) : o.hi >> (8 * (k - 8)));
}

__device__ __forceinline__ void to_flush16(TanOut &o) {
  if (o.skip) {
    to_store_bytes(o, o.skip, 16);
    o.skip = 0;
  } else if (o.pos < o.cap16) {
    o.dst[o.pos] = make_uint4((uint32_t)o.lo, (uint32_t)(o.lo >> 32),
                              (uint32_t)o.hi, (uint32_t)(o.hi >> 32));
  }
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
  o.bpos++;
  if (++o.n == 16) to_flush16(o);
}

__device__ __forceinline__ void to_zeros(TanOut &o, uint32_t k) {
  for (uint32_t i = 0; i < k; ++i) to_raw(o, 0);
}

// byte p of the output (a zero placeholder) becomes b: in the accumulator
// when p has not been stored yet, else a byte store behind the lane's own
// 16-byte store of that word (same address, program order)
__device__ __forceinline__ void to_patch(TanOut &o, uint32_t p, uint32_t b) {
  const uint32_t base = o.pos * 16;
  b &= 0xffu;
  if (p >= base) {
    const uint32_t q = p - base;
    if (q < 8)
      o.lo |= (uint64_t)b << (8 * q);
    else
      o.hi |= (uint64_t)b << (8 * (q - 8));
  } else if (p < o.cap16 * 16) {
    reinterpret_cast<uint8_t *>(o.dst)[p] = (uint8_t)b;
  }
}

__device__ __forceinline__ void xs_byte(TanOut &o, uint32_t b) {
  const uint64_t x = (uint64_t)(b & 0xffu) << ((o.hn & 7) * 8);
  const uint32_t w = o.hn >> 3;
  o.h0 |= w == 0 ? x : 0;
  o.h1 |= w == 1 ? x : 0;
  o.h2 |= w == 2 ? x : 0;
  o.h3 |= w == 3 ? x : 0;
  o.hlen++;
  if (++o.hn == 32) {
    o.v0 = xx_round(o.v0, o.h0);
    o.v1 = xx_round(o.v1, o.h1);
    o.v2 = xx_round(o.v2, o.h2);
    o.v3 = xx_round(o.v3, o.h3);
    o.h0 = o.h1 = o.h2 = o.h3 = 0;
    o.hn = 0;
  }
}

// XXH64_digest of the open chunk (xxhash.go Sum64 / Digest.Sum64)
__device__ __forceinline__ uint64_t xs_final(const TanOut &o) {
  uint64_t acc;
  if (o.hlen >= 32) {
    acc = rotl64(o.v0, 1) + rotl64(o.v1, 7) + rotl64(o.v2, 12) +
          rotl64(o.v3, 18);
    acc = xx_merge(acc, o.v0);
    acc = xx_merge(acc, o.v1);
    acc = xx_merge(acc, o.v2);
    acc = xx_merge(acc, o.v3);
  } else {
    acc = XP5;
  }
  acc += o.hlen;
  const uint64_t hw[4] = {o.h0, o.h1, o.h2, o.h3};
  uint32_t left = o.hn;
#pragma unroll
  for (uint32_t k = 0; k < 3; ++k)
    if (left >= 8 * (k + 1))
      acc = rotl64(acc ^ xx_round(0, hw[k]), 27) * XP1 + XP4;
  const uint32_t w = left >> 3;
  uint64_t t = w == 0 ? o.h0 : w == 1 ? o.h1 : w == 2 ? o.h2 : o.h3;
  left &= 7;
  if (left >= 4) {
    acc = rotl64(acc ^ (t & 0xffffffffull) * XP1, 23) * XP2 + XP3;
    t >>= 32;
    left -= 4;
  }
  for (; left; --left) {
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

// the open chunk is complete: its checksum into its header
__device__ __forceinline__ void to_close(TanOut &o) {
  const uint32_t c = (uint32_t)xs_final(o);
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) to_patch(o, o.hdr + k, c >> (8 * k));
}

// a chunk header at the current block position: checksum placeholder,
// length, type (fullChunkType 1, first 2, middle 3, last 4); the hash
// starts over with the type byte
__device__ __forceinline__ void to_open(TanOut &o) {
  const uint32_t room = TAN_BLOCK - o.bpos - TAN_HDR;
  const uint32_t k = o.left < room ? o.left : room;
  const bool last = k == o.left;
  const uint32_t type = last ? (o.first ? 1u : 4u) : (o.first ? 2u : 3u);
  o.first = false;
  o.hdr = o.start + o.total;
  to_zeros(o, 4);
  to_raw(o, k);
  to_raw(o, k >> 8);
  to_raw(o, type);
  o.v0 = XP1 + XP2;
  o.v1 = XP2;
  o.v2 = 0;
  o.v3 = 0 - XP1;
  o.h0 = o.h1 = o.h2 = o.h3 = 0;
  o.hn = o.hlen = 0;
  xs_byte(o, type);
}

// begins a record of `len` payload bytes at block position bpos, byte
// `start` of dst: padding and the first header
__device__ __forceinline__ void to_begin(TanOut &o, uint4 *dst, uint32_t cap16,
                                         uint32_t bpos, uint32_t len,
                                         uint32_t start = 0,
                                         bool shared = false) {
  o.dst = dst;
  o.cap16 = cap16;
  o.start = start;
  o.shared = shared;
  o.lo = o.hi = 0;
  o.pos = start / 16;
  o.n = o.skip = start % 16;
  o.total = 0;
  o.bpos = bpos;
  o.left = len;
  o.first = true;
  if (bpos + TAN_HDR > TAN_BLOCK) {  // the rest of the block stays zero
    to_zeros(o, TAN_BLOCK - bpos);
    o.bpos = 0;
  }
  to_open(o);
}

// one payload byte (the colfer / Update encoders' sink)
__device__ __forceinline__ void bo_byte(TanOut &o, uint32_t b) {
  if (o.bpos == TAN_BLOCK) {  // the block is full: the next chunk
    to_close(o);
    o.bpos = 0;
    to_open(o);
  }
  to_raw(o, b);
  xs_byte(o, b);
  o.left--;
}

__device__ __forceinline__ void to_le32(TanOut &o, uint32_t x) {
  for (int k = 0; k < 4; ++k) bo_byte(o, x >> (8 * k));
}

__device__ __forceinline__ void to_finish(TanOut &o) {
  to_close(o);
  if (o.n > o.skip) {
    if (o.shared || o.skip) {
      to_store_bytes(o, o.skip, o.n);
      o.pos++;
    } else {
      to_flush16(o);
    }
  }
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

// The records of a round can be sparse (C5: 3 % of the replicas) and long
// (a 1 KB entry is 64 window chunks): a lane-per-replica pass would run
// waves with one or two busy lanes.  So the select pass writes the records
// of dense workgroups in place (C3: every replica has one) and lists the
// replicas of sparse ones -- wave-aggregated appends spread over TAN_LISTS
// counters (TAN_LISTS, drb_layout.hpp) -- for the write pass: one listed record per lane, full waves.
constexpr uint32_t TAN_DENSE = 64;  // of a 256-lane workgroup

// the Update of this round that db.write does not skip (db.go:97-116)
__device__ __forceinline__ bool tan_pending(const View &v, uint32_t round,
                                            uint32_t slot, uint64_t g,
                                            uint4 &s2, uint4 &st, bool &have) {
  const uint64_t i = ix(v, slot, g);
  s2 = v.tan_sum[tan_sum_ix(v, 2, slot, g)];
  const uint32_t fl = v.u32[u32_ix(v, W_FLAGS, slot, g)];
  // an Update of this round from a replica that stayed on the fast path
  have = s2.z == round && (s2.y & TS_HAVE) && (fl & DRB_F_HOSTED) &&
         !(fl & (DRB_F_FALLBACK | DRB_F_ERROR));
  st = have ? v.tan_st[i] : make_uint4(0, 0, 0, 0);
  if (!have) return false;
  // IsStateEqual(u.State, st) with no entries (the stored state is the
  // empty one or Peer.prevState, see DESIGN)
  return (s2.y & TS_STATE) || (st.w & TST_STATE) || s2.x > 0;
}

struct TanCount {
  uint32_t bytes = 0, rec = 0, sync = 0, fresh = 0;
};

// the multiplexed logs: log (slot, key) holds the groups g with
// (first_shard_id + g) % 16 == key, record j of the round being the j-th
// such group (place_world 1: ShardID = first_shard_id + g)
__host__ __device__ inline uint32_t tanm_key(const View &v, uint64_t g) {
  return (uint32_t)((v.first_shard_id + g) % 16);
}
__host__ __device__ inline uint64_t tanm_ix(const View &v, uint32_t slot,
                                            uint64_t g) {
  return ((uint64_t)slot * 16 + tanm_key(v, g)) * v.tanm_J + g / 16;
}

// the marshalled Update's size (update.go:128-169) and stateSyncChange
// (db.go:88-90) of replica (slot, g)'s pending Update
__device__ __forceinline__ uint32_t tan_len(const View &v, uint32_t slot,
                                            uint64_t g, uint4 s2, uint4 st,
                                            bool &sync) {
  const uint4 s0 = v.tan_sum[tan_sum_ix(v, 0, slot, g)];
  const uint4 s1 = v.tan_sum[tan_sum_ix(v, 1, slot, g)];
  const uint32_t n_save = s2.x;
  const bool u_state = (s2.y & TS_STATE) != 0;
  const bool st_state = (st.w & TST_STATE) != 0;
  sync = n_save > 0 || (u_state ? (!st_state || (s2.y & TS_TV)) : st_state);
  const uint64_t shard = v.first_shard_id + gid(v, slot, g);
  uint32_t len = varint_size(shard) + varint_size(slot + 1) + 1 + 4 + 1;
  if (u_state) len += 4 + state_size(lo64(s0), hi64(s0), lo64(s1));
  for (uint32_t k = 0; k < n_save; ++k)
    len += 4 + entry_size(ring_entry_hdr(v, slot, g, hi64(s1) + k, false));
  return len;
}

// db.write of replica (slot, g)'s pending Update: its record into the
// replica's save buffer (multiplexed: at its place in its log's staging,
// laid out by k_tanm_chain), {offset, length, flags} into tan_rec
__device__ __forceinline__ void tan_write_one(const View &v, uint32_t slot,
                                              uint64_t g, uint4 s2, uint4 st,
                                              uint64_t max_log, TanCount &c) {
  const uint64_t i = ix(v, slot, g);
  const uint4 s0 = v.tan_sum[tan_sum_ix(v, 0, slot, g)];
  const uint4 s1 = v.tan_sum[tan_sum_ix(v, 1, slot, g)];
  const uint32_t n_save = s2.x;
  const bool u_state = (s2.y & TS_STATE) != 0;
  const uint64_t term = lo64(s0), vote = hi64(s0), commit = lo64(s1);
  const uint64_t save_lo = hi64(s1);
  bool sync;
  const uint32_t len = tan_len(v, slot, g, s2, st, sync);
  uint64_t off;
  uint32_t logn, start = 0;
  bool new_log;
  uint4 *dst;
  uint32_t cap16;
  if (v.tan_mux) {
    const uint4 p = v.tanm_pos[tanm_ix(v, slot, g)];
    off = (uint64_t)p.x | ((uint64_t)p.y << 32);
    start = p.z;
    logn = p.w >> 1;
    new_log = p.w & 1;
    dst = v.save_buf + ((uint64_t)slot * 16 + tanm_key(v, g)) * v.tanm_cap16;
    cap16 = (uint32_t)v.tanm_cap16;
  } else {
    off = (uint64_t)st.x | ((uint64_t)st.y << 32);
    logn = st.z;
    // makeRoomForWrite (db.go:175-180) -> createNewLog (open.go:171)
    new_log = off >= max_log;
    if (new_log) {
      off = 0;
      logn++;
    }
    dst = v.save_buf + i * v.save_cap16;
    cap16 = v.save_cap16;
  }
  uint4 rec = make_uint4(st.x, st.y, 0, st.z << 8);
  const uint32_t bpos = (uint32_t)(off % TAN_BLOCK);
  const uint32_t add = tan_appended(bpos, len);
  if (add > v.save_cap16 * 16) {  // bounded by the pre-pass
    rec.w = (st.z << 8) | DRB_TAN_OVERFLOW;
  } else {
    const uint64_t shard = v.first_shard_id + gid(v, slot, g);
    TanOut o;
    to_begin(o, dst, cap16, bpos, len, start, v.tan_mux != 0);
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
    rec.w = (logn << 8) | DRB_TAN_WRITTEN | (sync ? DRB_TAN_SYNC : 0) |
            (new_log ? DRB_TAN_NEW_LOG : 0);
    if (!v.tan_mux) {  // (a multiplexed log's writer: k_tanm_chain)
      off += o.total;
      st.x = (uint32_t)off;
      st.y = (uint32_t)(off >> 32);
      st.z = logn;
    }
    st.w = u_state ? TST_STATE : 0;  // nodeStates.setState(u.State)
    v.tan_st[i] = st;
    c.bytes += o.total;
    c.rec++;
    c.sync += sync;
    c.fresh += new_log;
  }
  v.tan_rec[i] = rec;
  v.save_len[i] = rec.z;
}

// a workgroup's {bytes, records, syncs, new logs} added to its tan_ctr row
__device__ __forceinline__ void tan_count_row(const View &v, const TanCount &c,
                                              unsigned long long *part) {
  if (c.rec) {
    atomicAdd(&part[0], (unsigned long long)c.bytes);
    atomicAdd(&part[1], (unsigned long long)c.rec);
    if (c.sync) atomicAdd(&part[2], (unsigned long long)c.sync);
    if (c.fresh) atomicAdd(&part[3], (unsigned long long)c.fresh);
  }
  __syncthreads();
  if (threadIdx.x < 4)
    v.tan_ctr[(uint64_t)blockIdx.x * 4 + threadIdx.x] += part[threadIdx.x];
}

// The kernels are compiled in their own translation units
// (drb_tan_inst.hip: DRB_TAN_KERNELS 1 = select + chain, 2 = write; the
// engine launches them through drb_launch.hpp), so the engine's other code
// does not wait on their long register allocation.
#if DRB_TAN_KERNELS == 1
// list r of the select pass holds the replicas of workgroups b = r mod
// TAN_LISTS, at most per_list of them; its count is n[r * 64]
__global__ __launch_bounds__(256) void k_tan_select(View v, uint32_t round,
                                                    uint64_t max_log,
                                                    uint32_t *list,
                                                    uint32_t per_list,
                                                    uint32_t *n) {
  __shared__ unsigned long long part[4];
  if (threadIdx.x < 4) part[threadIdx.x] = 0;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t slot = (uint32_t)(t / v.G);
  const uint64_t g = t - (uint64_t)slot * v.G;
  bool pend = false;
  uint4 s2 = make_uint4(0, 0, 0, 0), st = s2;
  if (slot < v.R) {
    bool have = false;
    pend = tan_pending(v, round, slot, g, s2, st, have);
    if (!pend) {
      const uint64_t i = ix(v, slot, g);
      v.tan_rec[i] = v.tan_mux ? make_uint4(0, 0, 0, 0)
                               : make_uint4(st.x, st.y, 0, have ? st.z << 8 : 0);
      v.save_len[i] = 0;
    }
    if (v.tan_mux) {  // the record sizes k_tanm_chain lays out
      bool sync = false;
      const uint32_t len = pend ? tan_len(v, slot, g, s2, st, sync) : 0;
      v.tanm_len[tanm_ix(v, slot, g)] = len | (sync ? 1u << 31 : 0u);
    }
  }
  TanCount c;
  // (multiplexed: every record waits for the chain, so all are listed)
  if (!v.tan_mux && __syncthreads_count(pend) >= (int)TAN_DENSE) {
    if (pend) tan_write_one(v, slot, g, s2, st, max_log, c);
  } else {
    const uint64_t m = __ballot(pend);
    if (m) {
      const uint32_t r = blockIdx.x % TAN_LISTS;
      const uint32_t lane = __lane_id();
      const uint32_t first = (uint32_t)__ffsll((unsigned long long)m) - 1;
      uint32_t base = 0;
      if (lane == first) base = atomicAdd(&n[r * 64], (uint32_t)__popcll(m));
      base = __shfl(base, first);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi(
          (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (pend) list[(uint64_t)r * per_list + base + below] = (uint32_t)t;
    }
  }
  tan_count_row(v, c, part);
}

// wave-wide exclusive prefix sum with DPP lane moves (no LDS round trips):
// row_shr 1, 2, 4, 8 scan each row of 16 lanes, row_bcast 15 / 31 carry
// the row totals into the rows above
__device__ __forceinline__ uint32_t wave_excl(uint32_t x, uint32_t) {
  int v = (int)x;
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false); // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false); // row_bcast:31
  return (uint32_t)v - x;
}

// One wave per multiplexed log (slot, key): the offsets of the round's
// records in group order (concurrentSaveState, logdb.go:265-304; each
// db.write's makeRoomForWrite and writeRecord, db.go:97-130), 256 records
// per step, 4 per lane.  A record of len bytes takes len + 7 unless it
// starts too close to a block's end for its header (padding), runs past
// the block (more chunks), or finds the log full (a new log at offset 0):
// the first such record of a step is placed exactly (tan_appended) and
// the step continues after it.  Each record gets {offset, staging byte,
// log, new log}; the log's staging is the round's bytes back to back.
__global__ __launch_bounds__(64) void k_tanm_chain(View v, uint64_t max_log) {
  const uint32_t L = blockIdx.x;  // slot * 16 + key
  const uint32_t lane = threadIdx.x;
  const uint4 cur = v.tanm_cur[L];
  uint64_t off = (uint64_t)cur.x | ((uint64_t)cur.y << 32);
  uint32_t logn = cur.z;
  const uint64_t off0 = off;
  const uint32_t log0 = logn;
  uint32_t spos = 0;
  bool any_sync = false, switched = false;
  const uint32_t J = v.tanm_J;
  const uint4 *lens4 = reinterpret_cast<const uint4 *>(v.tanm_len + (uint64_t)L * J);
  uint4 *pos = v.tanm_pos + (uint64_t)L * J;
  uint4 nxt = lens4[lane];
  for (uint32_t base = 0; base < J; base += 256) {
    const uint4 cl = nxt;
    if (base + 256 < J) nxt = lens4[(base + 256) / 4 + lane];
    const uint32_t raw[4] = {cl.x, cl.y, cl.z, cl.w};
    uint32_t len[4];
    uint32_t todo = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      len[k] = raw[k] & 0x7fffffffu;
      any_sync |= (raw[k] >> 31) != 0;
      todo |= (raw[k] ? 1u : 0u) << k;
    }
    any_sync = __ballot(any_sync) != 0;
    if (__ballot(todo != 0) == 0) continue;
    uint4 out[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) out[k] = make_uint4(0, 0, 0, 0);
    for (;;) {
      uint32_t sz[4], lp[4], sum = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sz[k] = (todo >> k & 1u) ? len[k] + TAN_HDR : 0;
        lp[k] = sum;
        sum += sz[k];
      }
      const uint32_t ex = wave_excl(sum, lane);
      // the first record of this lane whose naive size is not exact
      uint32_t kk = 4;
#pragma unroll
      for (int k = 3; k >= 0; --k) {
        const uint64_t st = off + ex + lp[k];
        const uint32_t b = (uint32_t)(st % TAN_BLOCK);
        if ((todo >> k & 1u) && (st >= max_log || b + TAN_HDR + len[k] > TAN_BLOCK))
          kk = k;
      }
      const uint64_t m = __ballot(kk < 4);
      const uint32_t fl = m ? (uint32_t)__ffsll((unsigned long long)m) - 1 : 64;
      const uint32_t fk = __shfl(kk, fl < 64 ? fl : 0);
      // the records before it are placed at their naive offsets
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if ((todo >> k & 1u) && (lane < fl || (lane == fl && (uint32_t)k < fk))) {
          const uint64_t st = off + ex + lp[k];
          out[k] = make_uint4((uint32_t)st, (uint32_t)(st >> 32),
                              spos + ex + lp[k], logn << 1);
          todo &= ~(1u << k);
        }
      }
      if (fl == 64) {
        const uint32_t tot = __shfl(ex + sum, 63);
        off += tot;
        spos += tot;
        break;
      }
      // the record that is not: placed exactly
      uint32_t rel = 0, flen = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if ((uint32_t)k == kk) {
          rel = ex + lp[k];
          flen = len[k];
        }
      rel = __shfl(rel, fl);
      flen = __shfl(flen, fl);
      off += rel;
      spos += rel;
      bool fresh = false;
      if (off >= max_log) {  // makeRoomForWrite (db.go:175-180)
        off = 0;
        logn++;
        fresh = switched = true;
      }
      if (lane == fl) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((uint32_t)k == fk) {
            out[k] = make_uint4((uint32_t)off, (uint32_t)(off >> 32), spos,
                                (logn << 1) | (fresh ? 1u : 0u));
            todo &= ~(1u << k);
          }
      }
      const uint32_t add = tan_appended((uint32_t)(off % TAN_BLOCK), flen);
      off += add;
      spos += add;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (raw[k]) pos[base + lane * 4 + k] = out[k];
  }
  if (lane == 0) {
    v.tanm_cur[L] = make_uint4((uint32_t)off, (uint32_t)(off >> 32), logn, 0);
    v.tanm_log[2 * (uint64_t)L] =
        make_uint4((uint32_t)off0, (uint32_t)(off0 >> 32), log0,
                   (any_sync ? DRB_TAN_SYNC : 0u) |
                       (switched ? DRB_TAN_NEW_LOG : 0u));
    v.tanm_log[2 * (uint64_t)L + 1] =
        make_uint4(spos, logn, (uint32_t)off, (uint32_t)(off >> 32));
  }
}

#endif  // DRB_TAN_KERNELS == 1

#if DRB_TAN_KERNELS == 2
// the listed records, one per lane (grid-stride over the lists' total);
// its workgroups add into tan_ctr rows 0.. as well (the launches run in
// stream order)
__global__ __launch_bounds__(256) void k_tan_write(View v, uint32_t round,
                                                   uint64_t max_log,
                                                   const uint32_t *list,
                                                   uint32_t per_list,
                                                   const uint32_t *n) {
  __shared__ unsigned long long part[4];
  __shared__ uint32_t pre[TAN_LISTS + 1];
  if (threadIdx.x < 4) part[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    uint32_t a = 0;
    for (uint32_t r = 0; r < TAN_LISTS; ++r) {
      pre[r] = a;
      a += n[r * 64];
    }
    pre[TAN_LISTS] = a;
  }
  __syncthreads();
  const uint32_t cnt = pre[TAN_LISTS];
  TanCount c;
  for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < cnt;
       j += gridDim.x * blockDim.x) {
    uint32_t lo = 0, hi = TAN_LISTS;  // the list r with pre[r] <= j < pre[r+1]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) / 2;
      if (pre[mid] <= j) lo = mid; else hi = mid;
    }
    const uint64_t t = list[(uint64_t)lo * per_list + (j - pre[lo])];
    const uint32_t slot = (uint32_t)(t / v.G);
    const uint64_t g = t - (uint64_t)slot * v.G;
    uint4 s2, st;
    bool have;
    if (slot < v.R && tan_pending(v, round, slot, g, s2, st, have))
      tan_write_one(v, slot, g, s2, st, max_log, c);
  }
  tan_count_row(v, c, part);
}
#endif  // DRB_TAN_KERNELS == 2

}  // namespace drb
