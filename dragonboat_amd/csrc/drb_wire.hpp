// drb_wire.hpp -- the outbound wire path for replicas that are not on
// this GPU: the messages one replica
// slot sent to another in the last round, for every group, encoded as the
// byte stream dragonboat's TCP transport puts on the connection to the
// NodeHost hosting the receivers:
//
//   Transport.processMessages (internal/transport/transport.go:443-508)
//     batches the send queue into pb.MessageBatch{Requests, DeploymentId,
//     SourceAddress, BinVer} (messagebatch.go:23-51), cutting a batch when
//     the sum of Message.SizeUpperLimit (raft_optimized.go:1210-1221)
//     reaches MaxMessageBatchSize (settings/hard.go:95): the messages
//     before the one that crossed the limit form one batch, that one
//     message a second (the `twoBatch` case);
//   sendMessageBatch -> writeMessage (tcp.go:142-178) frames each batch as
//     magic {0xAE,0x7D} | requestHeader{method 100, size, header CRC,
//     payload CRC32-IEEE} (tcp.go:64-90) | payload.
//
// The queue is taken as fully drained (every message of the round queued
// before the sender goroutine runs), group-major in shard order and in
// send order within a group, so the cut points are a function of the
// round's messages.
//
// Parallel structure (all kernels on the engine stream):
//   k_wire_measure   lane = group: decodes its mailbox records of the
//                    (from, to) plane and the Replicate entries from the
//                    sender's window; writes the count, wire bytes and
//                    SizeUpperLimit sum of its messages
//   k_scan3_*        exclusive prefix sums of the three (message ordinals,
//                    byte offsets, upper-limit offsets)
//   k_wire_plan      one wave: the batch cut points by 64-way searches on
//                    the upper-limit prefix; frame offsets
//   k_wire_encode    lane = group: writes its messages at their absolute
//                    byte offsets (full 16 B chunks as vector stores, the
//                    shared head/tail chunk bytes as byte stores) and
//                    folds each run's CRC32 into its frame's payload CRC:
//                    CRC(A|B) = CRC(A)*x^(8|B|) ^ CRC(B) mod P, so a run's
//                    contribution is its CRC shifted by the bytes that
//                    follow it in the payload (zlib crc32_combine algebra)
//   k_wire_finish    thread = frame: MessageBatch trailer, payload CRC,
//                    request header.
#pragma once

namespace drb {

constexpr uint32_t WIRE_MAX_FRAMES = 4096;
constexpr uint32_t WIRE_MAX_SRC = 256;
constexpr uint32_t WIRE_EMPTY_SNAPSHOT_FIELD = 26;  // 0x62 0x18 + 24 B

// x^(2^k) mod P, k = 0..31, reflected (zlib x2n_table)
__constant__ uint32_t c_x2n[32];
// slicing-by-4 tables (c_crc_s4[0..255]: the byte table), staged into LDS
// per block
__constant__ uint32_t c_crc_s4[4 * 256];

DRB_DEV void crc_s4_stage(uint32_t *t) {
  for (uint32_t i = threadIdx.x; i < 4 * 256; i += blockDim.x)
    t[i] = c_crc_s4[i];
  __syncthreads();
}

__host__ __device__ inline uint32_t gf2_multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ CRC32_IEEE_POLY : b >> 1;
  }
  return p;
}

// crc * x^(8n) mod P: the CRC of A followed by n more bytes' worth of
// shift (crc32_combine(crc, 0, n) without the second operand)
__device__ inline uint32_t crc_shift(uint32_t crc, uint64_t n) {
  if (!crc || !n) return crc;
  uint32_t p = 1u << 31;  // x^0
  uint32_t k = 3;         // 8n = n * 2^3
  while (n) {
    if (n & 1) p = gf2_multmodp(c_x2n[k & 31], p);
    n >>= 1;
    k++;
  }
  return gf2_multmodp(p, crc);
}

struct WireFrame {
  uint64_t first, last;    // message ordinals [first, last]
  uint64_t msg_off;        // byte offset of `first` in the message stream
  uint64_t msg_bytes;      // bytes of its Requests fields
  uint64_t off;            // frame offset in the output stream
  uint32_t crc;            // payload CRC accumulator (XOR of contributions)
  uint32_t pad;
};

struct WirePlan {
  uint64_t n_msgs, n_frames, total_bytes, overflow;
};

struct WireArgs {
  uint32_t from, to, buf, round_tag;
  uint64_t deployment_id, max_batch;
  uint32_t bin_ver, src_len;
  uint32_t trailer;        // bytes of DeploymentId + SourceAddress + BinVer
  uint32_t pad;
};

__host__ __device__ inline uint32_t sov64(uint64_t x) {
  uint32_t n = 1;
  while (x >= 0x80) {
    x >>= 7;
    n++;
  }
  return n;
}

// one decoded outbound message of a (from, to) plane
struct WireMsg {
  Msg m;
  uint64_t shard_id;
};

// walks the records of lane g's (from, to) plane in send order
// (a Quiesce message -- a header bit, drb_msg.hpp -- comes first)
struct WireCursor {
  uint4 meta;
  uint32_t k, q;
  uint32_t qz;  // a Quiesce message still to produce
  uint64_t prev_lo, prev_hi;
};

DRB_DEV void wc_init(WireCursor &c, const View &v, const WireArgs &a,
                     uint64_t g) {
  c.meta = v.mbox_meta[mmeta_ix(v, a.buf, a.from, a.to, g)];
  const bool cur = tag_is(c.meta.x, a.round_tag);
  c.qz = cur && (c.meta.x & MQ_QUIESCE) ? 1u : 0u;
  c.k = (cur ? mi_count(c.meta.y) : 0) + c.qz;
  c.q = 0;
  c.prev_lo = c.prev_hi = 0;
}

DRB_DEV WireMsg wc_next(WireCursor &c, const View &v, const WireArgs &a,
                        uint64_t g) {
  if (c.qz) {  // node.sendEnterQuiesceMessages (node.go:993-1005)
    c.qz = 0;
    WireMsg w;
    w.m = Msg{};
    w.m.type = DRB_MSG_QUIESCE;
    w.shard_id = v.first_shard_id + gid(v, a.from, g);
    return w;
  }
  // send order: the Replicates, then the others (drb_msg.hpp)
  const uint32_t nr = mi_nrep(c.meta.y);
  const uint32_t k = c.q < nr ? rec_pos(true, c.q, v.MB)
                              : rec_pos(false, c.q - nr, v.MB);
  const uint4 c0 = v.mbox[mbox_ix(v, a.buf, a.from, a.to, k, 0, g)];
  uint4 c1 = make_uint4(0, 0, 0, 0);
  if (c0.x & MF_HAS_C1) c1 = v.mbox[mbox_ix(v, a.buf, a.from, a.to, k, 1, g)];
  WireMsg w;
  w.m = msg_decode(c0, c1, q_hi(c.meta), c.prev_lo, c.prev_hi);
  w.shard_id = v.first_shard_id + gid(v, a.from, g);
  c.q++;
  return w;
}

DRB_DEV EntryHdr wire_entry(const View &v, uint32_t slot, uint64_t idx,
                            uint64_t g) {
  const uint4 m0 = v.ring[ring_ix(v, slot, idx, 0, g)];
  const uint4 m1 = v.ring[ring_ix(v, slot, idx, 1, g)];
  const uint4 m2 = v.ring[ring_ix(v, slot, idx, 2, g)];
  EntryHdr e;
  e.term = q_lo(m0);
  e.index = idx;
  e.key = q_hi(m0);
  e.client_id = q_lo(m1);
  e.series_id = q_hi(m1);
  e.responded_to = q_lo(m2);
  e.type = m2.z;
  e.cmd_len = m2.w;
  return e;
}

// entries of a Replicate (raft.go:738-769): [LogIndex+1, LogIndex+n] of
// the sender's log; of a forwarded Propose (raft.go:2103-2116): the sender's
// forward rows, as proposed (no Term, no Index)
DRB_DEV uint32_t wire_n_entries(const WireMsg &w) {
  return w.m.type == DRB_MSG_REPLICATE || w.m.type == DRB_MSG_PROPOSE ? w.m.n
                                                                      : 0;
}
// entry q of message w and its Cmd's first chunk (the next ones G apart)
DRB_DEV EntryHdr wire_msg_entry(const View &v, const WireArgs &a, uint64_t g,
                                const WireMsg &w, uint32_t q,
                                const uint4 **cmd0) {
  if (w.m.type == DRB_MSG_PROPOSE) {
    const uint32_t fw = fwd_ps(v, a.buf, a.from);
    const uint4 p0 = v.props[prop_ix(v, fw, q, 0, g)];
    const uint4 p1 = v.props[prop_ix(v, fw, q, 1, g)];
    const uint4 p2 = v.props[prop_ix(v, fw, q, 2, g)];
    EntryHdr e;
    e.term = e.index = 0;
    e.key = q_lo(p0);
    e.client_id = q_hi(p0);
    e.series_id = q_lo(p1);
    e.responded_to = q_hi(p1);
    e.type = p2.x;
    e.cmd_len = p2.y;
    *cmd0 = v.props + prop_ix(v, fw, q, PROP_META, g);
    return e;
  }
  const uint64_t idx = w.m.log_index + 1 + q;
  *cmd0 = v.ring + ring_ix(v, a.from, idx, ENT_META, g);
  EntryHdr e = wire_entry(v, a.from, idx, g);
  // a witness is sent metadata entries: Index and Term, config changes as
  // they are (makeMetadataEntries, raft.go:771-785)
  if (((v.wt_mask >> a.to) & 1u) && e.type != DRB_ENTRY_CONFIG_CHANGE) {
    e.key = e.client_id = e.series_id = e.responded_to = 0;
    e.type = DRB_ENTRY_METADATA;
    e.cmd_len = 0;
  }
  return e;
}

// Message.Size (message.go:92-124) and Message.SizeUpperLimit
// (raft_optimized.go:1210-1221); *bytes is the MessageBatch.Requests
// field: 0x0a + varint(size) + size
DRB_DEV void wire_sizes(const View &v, const WireArgs &a, uint64_t g,
                        const WireMsg &w, uint64_t &msize, uint64_t &bytes,
                        uint64_t &upper) {
  const Msg &m = w.m;
  uint64_t n = 1 + sov64(m.type) + 1 + sov64(a.to + 1) + 1 +
               sov64(a.from + 1) + 1 + sov64(w.shard_id) + 1 + sov64(m.term) +
               1 + sov64(m.log_term) + 1 + sov64(m.log_index) + 1 +
               sov64(m.commit) + 2 + 1 + sov64(m.hint);
  uint64_t up = 16 * 12 + 24;
  const uint32_t ne = wire_n_entries(w);
  for (uint32_t q = 0; q < ne; ++q) {
    const uint4 *cmd0;
    const EntryHdr e = wire_msg_entry(v, a, g, w, q, &cmd0);
    const uint32_t l = entry_size(e);
    n += 1 + l + sov64(l);
    up += 16 + 16 * 8 + e.cmd_len;  // EntryNonCmdFieldsSize (soft.go:20)
  }
  n += WIRE_EMPTY_SNAPSHOT_FIELD + 1 + sov64(m.hint_high);
  msize = n;
  bytes = 1 + sov64(n) + n;
  upper = up;
}

// ------------------------------------------------------------ stream out
// Bytes at absolute stream offsets.  A lane owns [start, pos); chunks it
// owns entirely leave as 16 B stores, the chunks it shares with its
// neighbours (its first and last) as byte stores of its own bytes.
// The CRC advances a 32-bit word at a time through slicing-by-4 tables in
// LDS (one dependent table step per 4 bytes).
struct StreamOut {
  uint8_t *base;
  const uint32_t *tab;  // LDS: 4 x 256 slicing tables
  uint64_t start, pos;
  uint64_t lo, hi;
  uint32_t crc, cw, cn;
};

DRB_DEV void so_init(StreamOut &o, uint8_t *base, uint64_t at,
                     const uint32_t *tab) {
  o.base = base;
  o.tab = tab;
  o.start = o.pos = at;
  o.lo = o.hi = 0;
  o.crc = 0xffffffffu;
  o.cw = o.cn = 0;
}

DRB_DEV void so_store(StreamOut &o, uint64_t cbase, uint32_t end) {
  const uint32_t first = o.start > cbase ? (uint32_t)(o.start - cbase) : 0;
  if (first == 0 && end == 16) {
    *(uint4 *)(o.base + cbase) =
        make_uint4((uint32_t)o.lo, (uint32_t)(o.lo >> 32), (uint32_t)o.hi,
                   (uint32_t)(o.hi >> 32));
  } else {
    for (uint32_t b = first; b < end; ++b)
      o.base[cbase + b] =
          (uint8_t)((b < 8 ? o.lo >> (8 * b) : o.hi >> (8 * (b - 8))) & 0xff);
  }
  o.lo = o.hi = 0;
}

DRB_DEV void so_byte(StreamOut &o, uint32_t b) {
  b &= 0xffu;
  o.cw |= b << (8 * o.cn);
  if (++o.cn == 4) {
    const uint32_t x = o.crc ^ o.cw;
    o.crc = o.tab[3 * 256 + (x & 0xffu)] ^ o.tab[2 * 256 + ((x >> 8) & 0xffu)] ^
            o.tab[256 + ((x >> 16) & 0xffu)] ^ o.tab[x >> 24];
    o.cw = o.cn = 0;
  }
  const uint32_t s = (uint32_t)(o.pos & 15);
  if (s < 8)
    o.lo |= (uint64_t)b << (8 * s);
  else
    o.hi |= (uint64_t)b << (8 * (s - 8));
  o.pos++;
  if ((o.pos & 15) == 0) so_store(o, o.pos - 16, 16);
}

// flushes the partial tail chunk; returns the run's CRC32-IEEE
DRB_DEV uint32_t so_finish(StreamOut &o) {
  if (o.pos & 15) so_store(o, o.pos & ~15ull, (uint32_t)(o.pos & 15));
  for (uint32_t i = 0; i < o.cn; ++i)
    o.crc = o.tab[(o.crc ^ (o.cw >> (8 * i))) & 0xffu] ^ (o.crc >> 8);
  o.cw = o.cn = 0;
  return o.crc ^ 0xffffffffu;
}

DRB_DEV void so_varint(StreamOut &o, uint64_t x) {
  while (x >= 0x80) {
    so_byte(o, (uint32_t)(x | 0x80));
    x >>= 7;
  }
  so_byte(o, (uint32_t)x);
}

DRB_DEV void so_colfer_u64(StreamOut &o, uint32_t tag, uint64_t x) {
  if (x >= (1ull << 49)) {
    so_byte(o, tag | 0x80);
#pragma unroll
    for (int k = 0; k < 8; ++k) so_byte(o, (uint32_t)(x >> (56 - 8 * k)));
  } else if (x != 0) {
    so_byte(o, tag);
    so_varint(o, x);
  }
}

// Entry.MarshalTo (raft_optimized.go:166-300), the Cmd from the window (or
// a Propose's forward rows): chunk c at cmd0[c * G]
DRB_DEV void so_entry(StreamOut &o, const View &v, const EntryHdr &e,
                      const uint4 *cmd0) {
  so_colfer_u64(o, 0, e.term);
  so_colfer_u64(o, 1, e.index);
  if (e.type != 0) {
    so_byte(o, 2);
    so_varint(o, e.type);
  }
  so_colfer_u64(o, 3, e.key);
  so_colfer_u64(o, 4, e.client_id);
  so_colfer_u64(o, 5, e.series_id);
  so_colfer_u64(o, 6, e.responded_to);
  if (e.cmd_len != 0) {
    so_byte(o, 7);
    so_varint(o, e.cmd_len);
    for (uint32_t c = 0; c * 16 < e.cmd_len; ++c) {
      const uint4 q = cmd0[(uint64_t)c * v.G];
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (uint32_t b = 0; b < 16; ++b)
        if (c * 16 + b < e.cmd_len) so_byte(o, w[b >> 2] >> (8 * (b & 3)));
    }
  }
  so_byte(o, 0x7f);
}

// MessageBatch.Requests element: 0x0a varint(size) Message.MarshalTo
// (message.go:32-90) with the empty Snapshot (snapshot.go:72-150)
DRB_DEV void so_message(StreamOut &o, const View &v, const WireArgs &a,
                        uint64_t g, const WireMsg &w, uint64_t msize) {
  const Msg &m = w.m;
  so_byte(o, 0x0a);
  so_varint(o, msize);
  so_byte(o, 0x08);
  so_varint(o, m.type);
  so_byte(o, 0x10);
  so_varint(o, a.to + 1);
  so_byte(o, 0x18);
  so_varint(o, a.from + 1);
  so_byte(o, 0x20);
  so_varint(o, w.shard_id);
  so_byte(o, 0x28);
  so_varint(o, m.term);
  so_byte(o, 0x30);
  so_varint(o, m.log_term);
  so_byte(o, 0x38);
  so_varint(o, m.log_index);
  so_byte(o, 0x40);
  so_varint(o, m.commit);
  so_byte(o, 0x48);
  so_byte(o, m.reject ? 1 : 0);
  so_byte(o, 0x50);
  so_varint(o, m.hint);
  const uint32_t ne = wire_n_entries(w);
  for (uint32_t q = 0; q < ne; ++q) {
    const uint4 *cmd0;
    const EntryHdr e = wire_msg_entry(v, a, g, w, q, &cmd0);
    so_byte(o, 0x5a);
    so_varint(o, entry_size(e));
    so_entry(o, v, e, cmd0);
  }
  // Snapshot (field 12): the 24-byte empty pb.Snapshot
  so_byte(o, 0x62);
  so_byte(o, 24);
  const uint8_t snap[24] = {0x12, 0, 0x18, 0, 0x20, 0, 0x28, 0,
                            0x32, 2, 0x08, 0, 0x48, 0, 0x50, 0,
                            0x58, 0, 0x60, 0, 0x68, 0, 0x70, 0};
#pragma unroll
  for (int k = 0; k < 24; ++k) so_byte(o, snap[k]);
  so_byte(o, 0x68);
  so_varint(o, m.hint_high);
}

// ------------------------------------------------------------ kernels
__global__ __launch_bounds__(256) void k_wire_measure(const View v,
                                                      const WireArgs a,
                                                      uint64_t *cnt,
                                                      uint64_t *bytes,
                                                      uint64_t *upper) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= v.G) return;
  WireCursor c;
  wc_init(c, v, a, g);
  uint64_t b = 0, u = 0;
  for (uint32_t q = 0; q < c.k; ++q) {
    const WireMsg w = wc_next(c, v, a, g);
    uint64_t ms, mb, mu;
    wire_sizes(v, a, g, w, ms, mb, mu);
    b += mb;
    u += mu;
  }
  cnt[g] = c.k;
  bytes[g] = b;
  upper[g] = u;
}

// exclusive scan of three u64 arrays of n elements, in place; tot[3]
constexpr uint32_t SCAN_ITEMS = 4;
constexpr uint32_t SCAN_TILE = 256 * SCAN_ITEMS;

__device__ inline void block_excl_scan3(uint64_t (&x)[3], uint64_t (&sum)[3]) {
  __shared__ uint64_t s[3][256];
  const uint32_t t = threadIdx.x;
  for (int j = 0; j < 3; ++j) s[j][t] = x[j];
  __syncthreads();
  for (uint32_t o = 1; o < 256; o <<= 1) {
    uint64_t y[3];
    for (int j = 0; j < 3; ++j) y[j] = t >= o ? s[j][t - o] : 0;
    __syncthreads();
    for (int j = 0; j < 3; ++j) s[j][t] += y[j];
    __syncthreads();
  }
  for (int j = 0; j < 3; ++j) {
    sum[j] = s[j][255];
    x[j] = s[j][t] - x[j];
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_scan3_up(uint64_t *a0, uint64_t *a1,
                                                  uint64_t *a2, uint64_t n,
                                                  uint64_t *bsum) {
  uint64_t *arr[3] = {a0, a1, a2};
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  uint64_t x[3] = {0, 0, 0};
  for (uint32_t i = 0; i < SCAN_ITEMS; ++i) {
    const uint64_t k = base + (uint64_t)threadIdx.x * SCAN_ITEMS + i;
    if (k < n)
      for (int j = 0; j < 3; ++j) x[j] += arr[j][k];
  }
  uint64_t sum[3];
  block_excl_scan3(x, sum);
  if (threadIdx.x == 0)
    for (int j = 0; j < 3; ++j) bsum[(uint64_t)blockIdx.x * 3 + j] = sum[j];
}

// one block: exclusive scan of the block sums, totals into tot[3]
__global__ __launch_bounds__(256) void k_scan3_top(uint64_t *bsum,
                                                   uint64_t nb,
                                                   uint64_t *tot) {
  uint64_t carry[3] = {0, 0, 0};
  for (uint64_t b0 = 0; b0 < nb; b0 += 256) {
    const uint64_t b = b0 + threadIdx.x;
    uint64_t x[3];
    for (int j = 0; j < 3; ++j) x[j] = b < nb ? bsum[b * 3 + j] : 0;
    uint64_t sum[3];
    block_excl_scan3(x, sum);
    if (b < nb)
      for (int j = 0; j < 3; ++j) bsum[b * 3 + j] = x[j] + carry[j];
    for (int j = 0; j < 3; ++j) carry[j] += sum[j];
  }
  if (threadIdx.x == 0)
    for (int j = 0; j < 3; ++j) tot[j] = carry[j];
}

__global__ __launch_bounds__(256) void k_scan3_down(uint64_t *a0, uint64_t *a1,
                                                    uint64_t *a2, uint64_t n,
                                                    const uint64_t *bsum) {
  uint64_t *arr[3] = {a0, a1, a2};
  const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
  uint64_t v[3][SCAN_ITEMS];
  uint64_t x[3] = {0, 0, 0};
  for (uint32_t i = 0; i < SCAN_ITEMS; ++i) {
    const uint64_t k = base + (uint64_t)threadIdx.x * SCAN_ITEMS + i;
    for (int j = 0; j < 3; ++j) {
      v[j][i] = k < n ? arr[j][k] : 0;
      x[j] += v[j][i];
    }
  }
  uint64_t sum[3];
  block_excl_scan3(x, sum);
  for (int j = 0; j < 3; ++j) x[j] += bsum[(uint64_t)blockIdx.x * 3 + j];
  for (uint32_t i = 0; i < SCAN_ITEMS; ++i) {
    const uint64_t k = base + (uint64_t)threadIdx.x * SCAN_ITEMS + i;
    for (int j = 0; j < 3; ++j) {
      if (k < n) arr[j][k] = x[j];
      x[j] += v[j][i];
    }
  }
}

// Wave-cooperative search: the smallest x in [lo, hi] with pred(x) true,
// pred monotone (false ... true) and pred(hi) true without being asked.
// Each of the 64 lanes probes one of 64 evenly spaced points and a ballot
// keeps the gap holding the first true one: log64 instead of log2
// dependent loads (3-4 for a million groups, not 20).  Every lane returns
// the same value.
template <class P>
DRB_DEV uint64_t wave_first_true(uint64_t lo, uint64_t hi, P pred) {
  const uint32_t lane = threadIdx.x & 63u;
  while (lo < hi) {
    const uint64_t step = (hi - lo + 63) / 64;
    const uint64_t pi = min(lo + (uint64_t)lane * step, hi);
    const bool t = pi == hi || pred(pi);
    const uint64_t b = __ballot(t);
    if (!b) {
      lo = min(lo + 63 * step, hi) + 1;
      continue;
    }
    const uint32_t k = (uint32_t)__ffsll((long long)b) - 1;
    const uint64_t pk = min(lo + (uint64_t)k * step, hi);
    if (k == 0) return pk;
    lo = min(lo + (uint64_t)(k - 1) * step, hi) + 1;
    hi = pk;
  }
  return lo;
}

// Transport.processMessages' cut points (transport.go:459-500) with the
// queue drained in one go.  One thread; per frame one binary search over
// the group-level upper-limit prefix and one walk of the group where the
// limit is reached.
__global__ void k_wire_plan(const View v, const WireArgs a,
                            const uint64_t *pcnt, const uint64_t *pbytes,
                            const uint64_t *pupper, const uint64_t *tot,
                            WireFrame *fr, WirePlan *plan) {
  if (blockIdx.x) return;
  const bool lane0 = threadIdx.x == 0;
  const uint64_t M = tot[0], B = tot[1], U = tot[2];
  uint64_t nf = 0, off = 0, ovf = 0;
  auto emit = [&](uint64_t first, uint64_t last, uint64_t b0, uint64_t b1) {
    if (nf >= WIRE_MAX_FRAMES) {
      ovf = 1;
      return;
    }
    WireFrame f;
    f.first = first;
    f.last = last;
    f.msg_off = b0;
    f.msg_bytes = b1 - b0;
    f.off = off;
    f.crc = 0;
    f.pad = 0;
    if (lane0) fr[nf] = f;
    ++nf;
    off += 20 + f.msg_bytes + a.trailer;
  };
  // s: first message of the next batch; bs: its byte offset; base: the
  // upper-limit prefix before it
  uint64_t s = 0, bs = 0, base = 0;
  while (s < M && !ovf) {
    const uint64_t T = base + a.max_batch;
    if (U < T) {  // the queue drains before the limit: one batch
      emit(s, M - 1, bs, B);
      break;
    }
    // the group holding message s: the last g with pcnt[g] <= s
    const uint64_t gs =
        wave_first_true(1, v.G, [&](uint64_t x) { return pcnt[x] > s; }) - 1;
    // the group whose messages reach T: smallest g with prefix(g+1) >= T
    const uint64_t lo = wave_first_true(gs, v.G - 1, [&](uint64_t x) {
      return pupper[x + 1] >= T;
    });
    WireCursor c;
    wc_init(c, v, a, lo);
    uint64_t u = pupper[lo], bj = pbytes[lo], mbj = 0;
    uint32_t q = 0;
    for (; q < c.k; ++q) {
      const WireMsg w = wc_next(c, v, a, lo);
      uint64_t ms, mb, mu;
      wire_sizes(v, a, lo, w, ms, mb, mu);
      u += mu;
      mbj = mb;
      if (u >= T) break;
      bj += mb;
    }
    const uint64_t j = pcnt[lo] + q;  // the message that reaches the limit
    if (j == s) {
      emit(s, s, bs, bj + mbj);
    } else {
      emit(s, j - 1, bs, bj);
      emit(j, j, bj, bj + mbj);
    }
    s = j + 1;
    bs = bj + mbj;
    base = u;
  }
  if (!lane0) return;
  plan->n_msgs = M;
  plan->n_frames = nf;
  plan->total_bytes = off;
  plan->overflow = ovf;
}

DRB_DEV uint32_t wire_frame_of(const WireFrame *fr, uint32_t nf,
                               uint64_t ord) {
  uint32_t lo = 0, hi = nf;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (fr[mid].first <= ord)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_wire_encode(
    const View v, const WireArgs a, const uint64_t *pcnt,
    const uint64_t *pbytes, WireFrame *fr, const WirePlan *plan,
    uint8_t *out) {
  __shared__ uint32_t blk_crc;
  __shared__ uint32_t blk_frame;
  __shared__ uint32_t tab[4 * 256];
  crc_s4_stage(tab);
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nf = (uint32_t)plan->n_frames;
  const uint64_t g0 = (uint64_t)blockIdx.x * blockDim.x;
  if (threadIdx.x == 0) {
    blk_crc = 0;
    blk_frame = nf ? wire_frame_of(fr, nf, g0 < v.G ? pcnt[g0] : 0) : 0;
  }
  __syncthreads();
  uint32_t acc = 0;
  if (g < v.G && nf) {
    WireCursor c;
    wc_init(c, v, a, g);
    uint64_t ord = pcnt[g], boff = pbytes[g];
    uint32_t f = c.k ? wire_frame_of(fr, nf, ord) : 0;
    StreamOut o;
    bool open = false;
    uint64_t run_end = 0;
    auto close_run = [&]() {
      if (!open) return;
      const uint32_t crc = so_finish(o);
      const WireFrame &F = fr[f];
      const uint64_t pend = F.off + 20 + F.msg_bytes + a.trailer;
      const uint32_t contrib = crc_shift(crc, pend - run_end);
      if (f == blk_frame)
        acc ^= contrib;
      else
        atomicXor(&fr[f].crc, contrib);
      open = false;
    };
    for (uint32_t q = 0; q < c.k; ++q, ++ord) {
      const WireMsg w = wc_next(c, v, a, g);
      uint64_t ms, mb, mu;
      wire_sizes(v, a, g, w, ms, mb, mu);
      const uint32_t fq = wire_frame_of(fr, nf, ord);
      if (fq != f) {
        close_run();
        f = fq;
      }
      const WireFrame &F = fr[f];
      const uint64_t at = F.off + 20 + (boff - F.msg_off);
      if (!open) {
        so_init(o, out, at, tab);
        open = true;
      }
      so_message(o, v, a, g, w, ms);
      run_end = at + mb;
      boff += mb;
    }
    close_run();
  }
  if (acc) atomicXor(&blk_crc, acc);
  __syncthreads();
  if (threadIdx.x == 0 && blk_crc && nf) atomicXor(&fr[blk_frame].crc, blk_crc);
}

DRB_DEV void put_be(uint8_t *p, uint64_t x, int n) {
  for (int k = 0; k < n; ++k) p[k] = (uint8_t)(x >> (8 * (n - 1 - k)));
}

__global__ void k_wire_finish(const WireArgs a, const uint8_t *src,
                              WireFrame *fr, const WirePlan *plan,
                              uint8_t *out) {
  __shared__ uint32_t tab[4 * 256];
  crc_s4_stage(tab);
  const uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= plan->n_frames) return;
  const WireFrame F = fr[f];
  // MessageBatch trailer (messagebatch.go:41-50)
  StreamOut o;
  so_init(o, out, F.off + 20 + F.msg_bytes, tab);
  so_byte(o, 0x10);
  so_varint(o, a.deployment_id);
  so_byte(o, 0x1a);
  so_varint(o, a.src_len);
  for (uint32_t k = 0; k < a.src_len; ++k) so_byte(o, src[k]);
  so_byte(o, 0x20);
  so_varint(o, a.bin_ver);
  const uint32_t pcrc = F.crc ^ so_finish(o);
  // writeMessage (tcp.go:142-160): magic, requestHeader.encode (tcp.go:79-90)
  uint8_t h[20];
  h[0] = 0xAE;
  h[1] = 0x7D;
  put_be(h + 2, 100, 2);  // raftType
  put_be(h + 4, F.msg_bytes + a.trailer, 8);
  put_be(h + 12, 0, 4);
  put_be(h + 16, pcrc, 4);
  uint32_t c = 0xffffffffu;
  for (int k = 2; k < 20; ++k) c = tab[(c ^ h[k]) & 0xffu] ^ (c >> 8);
  put_be(h + 12, c ^ 0xffffffffu, 4);
  for (int k = 0; k < 20; ++k) out[F.off + k] = h[k];
  fr[f].crc = pcrc;
}

}  // namespace drb

// ------------------------------------------------------------ host side
struct WireState {
  uint64_t G = 0;
  uint64_t *cnt = nullptr, *bytes = nullptr, *upper = nullptr;
  uint64_t *bsum = nullptr, *tot = nullptr;
  drb::WireFrame *frames = nullptr;
  drb::WirePlan *plan = nullptr;
  uint8_t *src = nullptr;
  uint8_t *out = nullptr;
  uint64_t out_cap = 0, out_len = 0, n_frames = 0;
};

static void wire_free(drb_engine *e) {
  WireState *w = e->wire;
  if (!w) return;
  void *ps[] = {w->cnt, w->bytes, w->upper, w->bsum, w->tot,
                w->frames, w->plan, w->src, w->out};
  for (void *p : ps)
    if (p) (void)hipFree(p);
  delete w;
  e->wire = nullptr;
}

static int wire_tables_ready = 0;

static int wire_init(drb_engine *e) {
  if (!wire_tables_ready) {
    uint32_t x2n[32], tab[256], s4[4 * 256];
    uint32_t p = 1u << 30;  // x^1
    x2n[0] = p;
    for (int n = 1; n < 32; ++n) x2n[n] = p = drb::gf2_multmodp(p, p);
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k)
        c = (c & 1) ? drb::CRC32_IEEE_POLY ^ (c >> 1) : c >> 1;
      tab[i] = c;
    }
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(drb::c_x2n), x2n, sizeof(x2n)));
    for (uint32_t i = 0; i < 256; ++i) {
      s4[i] = tab[i];
      for (int k = 1; k < 4; ++k)
        s4[k * 256 + i] =
            tab[s4[(k - 1) * 256 + i] & 0xff] ^ (s4[(k - 1) * 256 + i] >> 8);
    }
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(drb::c_crc_s4), s4, sizeof(s4)));
    wire_tables_ready = 1;
  }
  if (e->wire) return DRB_OK;
  WireState *w = new WireState();
  e->wire = w;
  const uint64_t G = e->cfg.num_groups;
  const uint64_t nb = (G + drb::SCAN_TILE - 1) / drb::SCAN_TILE;
  w->G = G;
  HIPCHK(hipMalloc(&w->cnt, G * 8));
  HIPCHK(hipMalloc(&w->bytes, G * 8));
  HIPCHK(hipMalloc(&w->upper, G * 8));
  HIPCHK(hipMalloc(&w->bsum, (nb + 1) * 3 * 8));
  HIPCHK(hipMalloc(&w->tot, 4 * 8));
  HIPCHK(hipMalloc(&w->frames, drb::WIRE_MAX_FRAMES * sizeof(drb::WireFrame)));
  HIPCHK(hipMalloc(&w->plan, sizeof(drb::WirePlan)));
  HIPCHK(hipMalloc(&w->src, drb::WIRE_MAX_SRC));
  return DRB_OK;
}

extern "C" int drb_encode_wire(drb_engine *e, uint32_t from_slot,
                               uint32_t to_slot, const drb_wire_cfg *cfg,
                               drb_wire_out *res) {
  // a durable LogDB: the round's responses leave only once it is saved
  if (e && e->cfg.durable_log && e->committed_round < e->round)
    return DRB_EINVAL;
  if (!e || !cfg || from_slot >= e->cfg.num_replicas ||
      to_slot >= e->cfg.num_replicas || from_slot == to_slot ||
      cfg->source_len > drb::WIRE_MAX_SRC ||
      (cfg->source_len && !cfg->source_address))
    return DRB_EINVAL;
  int rc = wire_init(e);
  if (rc) return rc;
  WireState *w = e->wire;
  w->out_len = w->n_frames = 0;
  if (res) memset(res, 0, sizeof(*res));
  if (e->round == 0) return DRB_OK;  // nothing sent yet
  drb::WireArgs a;
  memset(&a, 0, sizeof(a));
  a.from = from_slot;
  a.to = to_slot;
  a.buf = (uint32_t)(e->round & 1);
  a.round_tag = (uint32_t)e->round;
  a.deployment_id = cfg->deployment_id;
  a.max_batch = cfg->max_batch_bytes ? cfg->max_batch_bytes
                                     : (uint64_t)64 * 1024 * 1024;
  a.bin_ver = cfg->bin_ver;
  a.src_len = cfg->source_len;
  a.trailer = 1 + drb::sov64(a.deployment_id) + 1 + drb::sov64(a.src_len) +
              a.src_len + 1 + drb::sov64(a.bin_ver);
  if (a.src_len)
    HIPCHK(hipMemcpyAsync(w->src, cfg->source_address, a.src_len,
                          hipMemcpyHostToDevice, e->stream));
  const uint64_t G = w->G;
  const unsigned gb = (unsigned)((G + 255) / 256);
  drb::k_wire_measure<<<gb, 256, 0, e->stream>>>(e->v, a, w->cnt, w->bytes,
                                                 w->upper);
  HIPCHK(hipGetLastError());
  const uint64_t nb = (G + drb::SCAN_TILE - 1) / drb::SCAN_TILE;
  drb::k_scan3_up<<<(unsigned)nb, 256, 0, e->stream>>>(w->cnt, w->bytes,
                                                       w->upper, G, w->bsum);
  drb::k_scan3_top<<<1, 256, 0, e->stream>>>(w->bsum, nb, w->tot);
  drb::k_scan3_down<<<(unsigned)nb, 256, 0, e->stream>>>(w->cnt, w->bytes,
                                                         w->upper, G, w->bsum);
  drb::k_wire_plan<<<1, 64, 0, e->stream>>>(e->v, a, w->cnt, w->bytes,
                                           w->upper, w->tot, w->frames,
                                           w->plan);
  HIPCHK(hipGetLastError());
  drb::WirePlan plan;
  HIPCHK(hipMemcpyAsync(&plan, w->plan, sizeof(plan), hipMemcpyDeviceToHost,
                        e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (plan.overflow) return DRB_ERANGE;
  if (plan.total_bytes > w->out_cap) {
    if (w->out) HIPCHK(hipFree(w->out));
    w->out = nullptr;
    const uint64_t cap = (plan.total_bytes + (1 << 20)) & ~15ull;
    HIPCHK(hipMalloc(&w->out, cap));
    w->out_cap = cap;
  }
  if (plan.n_frames) {
    drb::k_wire_encode<<<gb, 256, 0, e->stream>>>(e->v, a, w->cnt, w->bytes,
                                                  w->frames, w->plan, w->out);
    HIPCHK(hipGetLastError());
    drb::k_wire_finish<<<(unsigned)((plan.n_frames + 63) / 64), 64, 0,
                         e->stream>>>(a, w->src, w->frames, w->plan, w->out);
    HIPCHK(hipGetLastError());
  }
  w->out_len = plan.total_bytes;
  w->n_frames = plan.n_frames;
  if (res) {
    res->n_msgs = plan.n_msgs;
    res->n_frames = plan.n_frames;
    res->n_bytes = plan.total_bytes;
  }
  return DRB_OK;
}

extern "C" int drb_wire_buffer(drb_engine *e, const uint8_t **dev,
                               uint64_t *len) {
  if (!e || !dev || !len) return DRB_EINVAL;
  *dev = e->wire ? e->wire->out : nullptr;
  *len = e->wire ? e->wire->out_len : 0;
  return DRB_OK;
}

extern "C" int drb_export_wire(drb_engine *e, uint8_t *out, size_t cap,
                               size_t *len) {
  if (!e || (!out && cap)) return DRB_EINVAL;
  const uint64_t n = e->wire ? e->wire->out_len : 0;
  if (len) *len = n;
  if (n > cap) return DRB_ERANGE;
  if (n) {
    HIPCHK(hipMemcpyAsync(out, e->wire->out, n, hipMemcpyDeviceToHost,
                          e->stream));
  }
  HIPCHK(hipStreamSynchronize(e->stream));
  return DRB_OK;
}
