// drb_codec.hpp -- device encoders of the raftpb wire formats on the path:
// the colfer Entry (raftpb/raft_optimized.go:84-300), EntryBatch
// (raftpb/entrybatch.go:25-58) and CRC32-IEEE (Go hash/crc32
// ChecksumIEEE, as used at internal/transport/tcp.go:146).
//
// One lane encodes one replica's byte stream.  Bytes collect in a 16-byte
// register accumulator and leave as 16 B stores; the CRC is folded in as
// the bytes are produced (byte-wise table in LDS), so the encoded record
// is never read back.
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>

namespace drb {

constexpr uint32_t CRC32_IEEE_POLY = 0xEDB88320u;  // reflected 0x04C11DB7

// fills the 256-entry byte table (one entry per thread of a 256-thread
// block; the caller synchronises the block afterwards)
__device__ __forceinline__ void crc32_table_init(uint32_t *tab, uint32_t i) {
  uint32_t c = i;
#pragma unroll
  for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ CRC32_IEEE_POLY : c >> 1;
  tab[i] = c;
}

struct ByteOut {
  uint4 *dst;           // 16 B aligned output of this lane
  const uint32_t *tab;  // CRC table (LDS)
  uint64_t lo, hi;      // pending bytes, little endian
  uint32_t n;           // pending byte count (0..15)
  uint32_t pos;         // 16 B chunks stored
  uint32_t cap16;       // capacity in chunks
  uint32_t crc;         // running CRC (inverted form)
  uint32_t total;       // bytes produced
  bool overflow;
};

__device__ __forceinline__ void bo_init(ByteOut &o, uint4 *dst, uint32_t cap16,
                                        const uint32_t *tab) {
  o.dst = dst;
  o.tab = tab;
  o.lo = o.hi = 0;
  o.n = 0;
  o.pos = 0;
  o.cap16 = cap16;
  o.crc = 0xffffffffu;
  o.total = 0;
  o.overflow = false;
}

__device__ __forceinline__ void bo_flush16(ByteOut &o) {
  if (o.pos < o.cap16)
    o.dst[o.pos] = make_uint4((uint32_t)o.lo, (uint32_t)(o.lo >> 32),
                              (uint32_t)o.hi, (uint32_t)(o.hi >> 32));
  else
    o.overflow = true;
  o.pos++;
  o.lo = o.hi = 0;
  o.n = 0;
}

__device__ __forceinline__ void bo_byte(ByteOut &o, uint32_t b) {
  b &= 0xffu;
  o.crc = o.tab[(o.crc ^ b) & 0xffu] ^ (o.crc >> 8);
  if (o.n < 8)
    o.lo |= (uint64_t)b << (8 * o.n);
  else
    o.hi |= (uint64_t)b << (8 * (o.n - 8));
  o.total++;
  if (++o.n == 16) bo_flush16(o);
}

// the tail chunk (zero padded); returns the final CRC
__device__ __forceinline__ uint32_t bo_finish(ByteOut &o) {
  if (o.n) bo_flush16(o);
  return o.crc ^ 0xffffffffu;
}

// protobuf / colfer varint (raftpb/common.go:11-19); O is any byte sink
// with a bo_byte(O &, uint32_t) overload (ByteOut, TanOut)
template <class O>
__device__ __forceinline__ void bo_varint(O &o, uint64_t x) {
  while (x >= 0x80) {
    bo_byte(o, (uint32_t)(x | 0x80));
    x >>= 7;
  }
  bo_byte(o, (uint32_t)x);
}
__device__ __forceinline__ uint32_t varint_size(uint64_t x) {
  uint32_t n = 1;
  while (x >= 0x80) {
    x >>= 7;
    n++;
  }
  return n;
}

// colfer u64 field (raft_optimized.go:172-187 and siblings): absent when
// 0, 0x80|tag + 8 bytes big endian from 2^49 on, else tag + varint
__device__ __forceinline__ uint32_t colfer_u64_size(uint64_t x) {
  if (x >= (1ull << 49)) return 9;
  if (x == 0) return 0;
  return 1 + varint_size(x);
}
template <class O>
__device__ __forceinline__ void colfer_u64(O &o, uint32_t tag, uint64_t x) {
  if (x >= (1ull << 49)) {
    bo_byte(o, tag | 0x80);
#pragma unroll
    for (int k = 0; k < 8; ++k) bo_byte(o, (uint32_t)(x >> (56 - 8 * k)));
  } else if (x != 0) {
    bo_byte(o, tag);
    bo_varint(o, x);
  }
}

// the fields of one pb.Entry (raftpb/entry.go:6-16) as the encoder sees
// them; the Cmd stays in the resident window and is read chunk by chunk
struct EntryHdr {
  uint64_t term, index, key, client_id, series_id, responded_to;
  uint32_t type, cmd_len;
};

// Entry.Size (raft_optimized.go:84-158)
__device__ __forceinline__ uint32_t entry_size(const EntryHdr &e) {
  uint32_t l = 1;  // terminator 0x7f
  l += colfer_u64_size(e.term) + colfer_u64_size(e.index);
  if (e.type != 0) l += 1 + varint_size(e.type);
  l += colfer_u64_size(e.key) + colfer_u64_size(e.client_id) +
       colfer_u64_size(e.series_id) + colfer_u64_size(e.responded_to);
  if (e.cmd_len != 0) l += 1 + varint_size(e.cmd_len) + e.cmd_len;
  return l;
}

// upper bound of one EntryBatch element: 0x0a + size varint + Entry with
// every u64 field in its 9-byte form (Entry.SizeUpperLimit,
// raft_optimized.go:77-81, plus the repeated-field framing)
__host__ __device__ inline uint32_t entrybatch_elem_bound(uint32_t cmd_len) {
  return 1 + 5 + (1 + 6 * 9 + 6 + (1 + 5 + cmd_len));
}

}  // namespace drb
