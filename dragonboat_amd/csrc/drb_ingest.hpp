// drb_ingest.hpp -- the inbound wire path on the GPU (SURVEY 8(f) F1,
// receive half): the TCP byte stream a peer NodeHost wrote
// (tcp.go:142-178, transport.go:443-508) taken into the engine's mailbox.
//
//   tcp.go readMessage (:180-237)      magic, requestHeader + its CRC
//                                      (host: 20 B a frame), payload CRC32
//                                      (GPU: 16 KB chunks, combined per
//                                      frame with crc32_combine algebra)
//   MessageBatch.Unmarshal             top-level field walk (host, one
//     (raft_optimized.go:1056-1207)    thread per frame): where each
//                                      Requests element starts
//   Message.Unmarshal (:659-983),      GPU, one lane per message, two
//     colfer Entry (:308-656)          passes (entry counts, then the
//                                      decode into SoA records)
//   Transport.handleRequest's          DeploymentId / BinVer per frame
//     filter (transport.go:305-316)
//   IMessageHandler.HandleMessageBatch GPU: messages sorted by (group,
//     -> MessageQueue.Add (node.go,    sender, receiver) plane (a stable
//     internal/server/message.go:      radix sort keeps stream order), one
//     105-123), drb_ingest semantics   lane per plane placing its records,
//                                      entries, header, max-append word
//                                      and the receiver's round-tag byte
//
// Error behaviour follows the host transport: a frame whose header or
// payload CRC fails, or whose batch does not decode, is ErrBadMessage --
// the frames before it are delivered, it and the rest are not
// (drb_wire_in.bad, .consumed); a stream that ends inside a sound frame is
// not bad: .consumed stops before it, for the transport to hand in again
// with the bytes that follow; a snapshot chunk frame (method 200) and an
// InstallSnapshot message are counted for the CPU path.
#pragma once

#include <hipcub/hipcub.hpp>

#include <atomic>
#include <thread>

namespace drb {

// one decoded pb.Message (raftpb/message.go:6-20) of an ingested stream
struct DecMsg {
  uint64_t shard, from, to, term, log_term, log_index, commit, hint,
      hint_high;
  uint64_t ent0;   // its first entry in the decoded entry array
  uint32_t type, reject, n_ent, err;  // err: ING_*
};
constexpr uint32_t ING_OK = 0, ING_BAD = 1, ING_SNAPSHOT = 2, ING_BIG = 3;

// A lane's byte cursor over the uploaded stream: one load per byte, which
// hit the L1 (a 16 B register window measured 2-4 % slower on the C3
// plane, profiles/r04_ingest)
struct Bytes {
  const uint8_t *p;
  __device__ explicit Bytes(const uint8_t *d) : p(d) {}
  __device__ inline uint32_t operator[](uint64_t i) const { return p[i]; }
};

// (every index below is from the message's first byte; d_entry's from the
// entry's, at offset e0)
template <class B>
__device__ inline bool d_varint(B &d, uint32_t n, uint32_t &i,
                                uint64_t &v) {
  v = 0;
  for (uint32_t s = 0; s < 70; s += 7) {
    if (i >= n) return false;
    const uint32_t b = d[i++];
    v |= (uint64_t)(b & 0x7fu) << s;
    if (b < 0x80u) return true;
  }
  return false;
}

// skipRaft (raft.pb.go): an unknown field
template <class B>
__device__ inline bool d_skip(B &d, uint32_t n, uint32_t &i,
                              uint64_t wire) {
  uint64_t x;
  switch (wire & 7) {
    case 0: return d_varint(d, n, i, x);
    case 1: i += 8; return i <= n;
    case 2:
      if (!d_varint(d, n, i, x) || x > n - i) return false;
      i += (uint32_t)x;
      return true;
    case 5: i += 4; return i <= n;
    default: return false;  // groups are not used by raftpb
  }
}

// colfer u64 field body (raft_optimized.go:316-350): varint whose 9th
// byte is taken whole, or 8 bytes big endian after a 0x80-flagged tag
template <class B>
__device__ inline bool d_colfer_u64(B &d, uint32_t e0, uint32_t n,
                                    uint32_t &i, bool flag, uint64_t &v) {
  if (flag) {
    if (i + 8 >= n) return false;
    v = 0;
    for (int k = 0; k < 8; ++k) v = (v << 8) | d[e0 + i + k];
    i += 8;
    return true;
  }
  v = 0;
  for (uint32_t s = 0;; s += 7) {
    if (i + 1 >= n) return false;
    const uint64_t b = d[e0 + i++];
    if (s == 56 || b < 0x80) {
      v |= b << s;
      return true;
    }
    v |= (b & 0x7f) << s;
  }
}

// colfer Entry.Unmarshal (raft_optimized.go:308-656) of the n bytes at e0;
// cmd_off is the Cmd's offset from e0
template <class B>
__device__ inline bool d_entry(B &d, uint32_t e0, uint32_t n,
                               drb_entry &e) {
  e.term = e.index = e.key = e.client_id = e.series_id = e.responded_to = 0;
  e.type = e.cmd_len = 0;
  e.cmd_off = 0;
  if (n == 0) return false;
  uint32_t i = 1;
  uint32_t h = d[e0];
  for (uint32_t tag = 0; tag < 7; ++tag) {
    if ((h & 0x7fu) != tag || h == 0x7fu) continue;
    if (tag == 2) {  // Type: uint32 varint, 0x80 flag = negated
      uint64_t x = 0;
      for (uint32_t s = 0;; s += 7) {
        if (i + 1 >= n) return false;
        const uint64_t b = d[e0 + i++];
        x |= (b & 0x7f) << s;
        if (b < 0x80) break;
        if (s > 28) return false;
      }
      e.type = (h & 0x80u) ? (uint32_t)(~(uint32_t)x + 1) : (uint32_t)x;
    } else {
      uint64_t x;
      if (!d_colfer_u64(d, e0, n, i, (h & 0x80u) != 0, x)) return false;
      switch (tag) {
        case 0: e.term = x; break;
        case 1: e.index = x; break;
        case 3: e.key = x; break;
        case 4: e.client_id = x; break;
        case 5: e.series_id = x; break;
        default: e.responded_to = x; break;
      }
    }
    h = d[e0 + i++];
  }
  if (h == 7) {  // Cmd (raft_optimized.go:603-641)
    uint64_t x = 0;
    for (uint32_t s = 0;; s += 7) {
      if (i >= n) return false;
      const uint64_t b = d[e0 + i++];
      x |= (b & 0x7f) << s;
      if (b < 0x80) break;
      if (s > 56) return false;
    }
    if (x > 16 * 1024 * 1024 || x >= n - i) return false;  // ColferSizeMax
    e.cmd_off = i;
    e.cmd_len = (uint32_t)x;
    i += (uint32_t)x;
    h = d[e0 + i++];
  }
  return h == 0x7fu && i == n;
}

__constant__ uint8_t c_empty_snapshot[24] = {
    0x12, 0, 0x18, 0, 0x20, 0, 0x28, 0, 0x32, 2, 0x08, 0,
    0x48, 0, 0x50, 0, 0x58, 0, 0x60, 0, 0x68, 0, 0x70, 0};

// Message.Unmarshal (raft_optimized.go:659-983).  ents == nullptr: count
// the entries only.  Returns ING_*; *big when a Cmd exceeds cmd_cap.
__device__ inline uint32_t d_message(const uint8_t *msg, uint32_t n,
                                     DecMsg &m, drb_entry *ents,
                                     uint64_t base, uint32_t cmd_cap,
                                     bool &big) {
  Bytes d(msg);
  m.shard = m.from = m.to = m.term = m.log_term = m.log_index = m.commit = 0;
  m.hint = m.hint_high = 0;
  m.type = m.reject = m.n_ent = 0;
  uint32_t i = 0;
  while (i < n) {
    uint64_t wire, v;
    if (!d_varint(d, n, i, wire)) return ING_BAD;
    const uint64_t field = wire >> 3;
    const uint32_t wt = (uint32_t)(wire & 7);
    if (field == 0) return ING_BAD;
    if ((field >= 1 && field <= 10) || field == 13) {
      if (wt != 0 || !d_varint(d, n, i, v)) return ING_BAD;
      switch (field) {
        case 1: m.type = (uint32_t)v; break;
        case 2: m.to = v; break;
        case 3: m.from = v; break;
        case 4: m.shard = v; break;
        case 5: m.term = v; break;
        case 6: m.log_term = v; break;
        case 7: m.log_index = v; break;
        case 8: m.commit = v; break;
        case 9: m.reject = v != 0; break;
        case 10: m.hint = v; break;
        default: m.hint_high = v; break;
      }
    } else if (field == 11 || field == 12) {
      uint64_t l;
      if (wt != 2 || !d_varint(d, n, i, l) || l > n - i) return ING_BAD;
      if (field == 11) {
        drb_entry e;
        if (!d_entry(d, i, (uint32_t)l, e)) return ING_BAD;
        if (e.cmd_len > cmd_cap) big = true;
        if (ents) {
          e.cmd_off += base + i;  // the Cmd's offset in the stream
          ents[m.n_ent] = e;
        }
        m.n_ent++;
      } else {
        bool empty = l == 24;
        for (uint32_t k = 0; empty && k < 24; ++k)
          empty = d[i + k] == c_empty_snapshot[k];
        if (!empty) return ING_SNAPSHOT;  // InstallSnapshot: the CPU path
      }
      i += (uint32_t)l;
    } else if (!d_skip(d, n, i, wire)) {
      return ING_BAD;
    }
  }
  return ING_OK;
}

// The payload CRC of a frame in 16 KB chunks, a workgroup per chunk:
// thread t takes the 64 bytes that end 64 * (255 - t) bytes before the
// chunk's end (a shorter chunk is right-aligned: the pieces before its
// start are empty), runs the register-only CRC over them (init 0, no final
// xor: f(piece), linear over GF(2)) and shifts it past the bytes after it,
// f * x^(8 * 64 * (255 - t)) mod P (c_crc_k64, zlib's multmodp); the
// chunk's f is the XOR of the 256 pieces' (f is blind to leading zeros).
// The host combines the chunks of a frame with crc32_combine and applies
// the CRC's ~0 conditioning once per frame.  Coalesced (a wave reads 4 KB
// contiguous) with one chunk per workgroup, where the one-lane-per-chunk
// kernel ran a handful of waves each walking 16 KB alone.
__constant__ uint32_t c_crc_k64[256];
__global__ __launch_bounds__(256) void k_crc_chunks(const uint8_t *data,
                                                     const uint64_t *off,
                                                     const uint32_t *len,
                                                     uint32_t *fraw) {
  __shared__ uint32_t t[8][256];
  __shared__ uint32_t red[4];
  for (uint32_t i = threadIdx.x; i < 8 * 256; i += blockDim.x)
    t[i >> 8][i & 255] = c_crc_tab[i >> 8][i & 255];
  __syncthreads();
  const uint64_t b = blockIdx.x;
  const int64_t L = len[b];
  const int64_t e = L - 64 * (int64_t)(255 - threadIdx.x);
  const int64_t s0 = e > 64 ? e - 64 : 0;
  uint32_t c = 0;
  if (e > 0) {
    const uint8_t *p = data + off[b] + s0;
    uint32_t l = (uint32_t)(e - s0);
    while (l && ((uintptr_t)p & 7)) {
      c = t[0][(c ^ *p++) & 0xff] ^ (c >> 8);
      l--;
    }
    while (l >= 8) {
      const uint64_t w = *(const uint64_t *)p;
      const uint32_t lo = (uint32_t)w ^ c, hi = (uint32_t)(w >> 32);
      c = t[7][lo & 0xff] ^ t[6][(lo >> 8) & 0xff] ^ t[5][(lo >> 16) & 0xff] ^
          t[4][lo >> 24] ^ t[3][hi & 0xff] ^ t[2][(hi >> 8) & 0xff] ^
          t[1][(hi >> 16) & 0xff] ^ t[0][hi >> 24];
      p += 8;
      l -= 8;
    }
    while (l--) c = t[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    if (c) c = gf2_multmodp(c_crc_k64[threadIdx.x], c);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c ^= (uint32_t)__shfl_xor((int)c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) fraw[b] = red[0] ^ red[1] ^ red[2] ^ red[3];
}

// A pull over PCIe from mapped pinned host memory: 16 B loads, four in
// flight a lane.  dst and src share their alignment mod 16 (the caller
// checks), n bytes.  (drb_ingest_wire pulls the frames' element steps this
// way; the stream itself goes up by DMA, which measured ~56 GB/s against
// the pull's ~45 and leaves the CUs free)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_zc_pull(uint8_t *dst,
                                                 const uint8_t *src,
                                                 uint64_t n) {
  const uint64_t gt = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t head = (16 - ((uintptr_t)dst & 15)) & 15;
  const uint64_t h = head < n ? head : n;
  if (gt < h) dst[gt] = src[gt];
  const uint64_t nv = (n - h) >> 4;
  u32x4 *d = (u32x4 *)(dst + h);
  const u32x4 *s = (const u32x4 *)(src + h);
  const uint64_t stride = gridDim.x * 256ull;
  constexpr int U = 4;
  for (uint64_t i = gt; i < nv; i += stride * U) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < nv) x[u] = __builtin_nontemporal_load(s + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < nv) d[i + u * stride] = x[u];
  }
  const uint64_t t0 = h + (nv << 4);
  if (gt < n - t0) dst[t0 + gt] = src[t0 + gt];
}

// pass 1: entry counts and errors, and the record of every message (the
// decode pass parses again only the messages with entries); the frame of a
// malformed message is marked (the host stops the stream there)
__global__ void k_ing_count(const uint8_t *s, const uint64_t *moff,
                            const uint32_t *mlen, const uint32_t *mframe,
                            uint32_t *n_ent, uint32_t *err,
                            uint32_t *frame_bad, DecMsg *out, uint64_t n,
                            uint32_t cmd_cap, uint64_t i0 = 0) {
  const uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DecMsg m;
  bool big = false;
  uint32_t r = d_message(s + moff[i], mlen[i], m, nullptr, 0, cmd_cap, big);
  if (r == ING_OK && big) r = ING_BIG;
  n_ent[i] = r == ING_OK ? m.n_ent : 0;
  err[i] = r;
  m.err = r;
  m.ent0 = 0;
  out[i] = m;
  if (r == ING_BAD) atomicOr(&frame_bad[mframe[i]], 1u);
}

// the steps as they went up: 2 B each when every step fits (the common
// case: half the PCIe bytes), else 4 B
__global__ void k_widen_step(const void *in, uint64_t *out, uint64_t n,
                             bool narrow) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    out[i] = narrow ? ((const uint16_t *)in)[i] : ((const uint32_t *)in)[i];
}

// Requests element i: its tag at the frame's payload offset plus the
// in-frame inclusive sum of the steps (scan minus the frame's start), then
// its tag and length varints (the host walk validated both)
__global__ void k_ing_elems(const uint8_t *s, const uint64_t *scan,
                            const uint64_t *mbase, const uint64_t *foff,
                            const uint32_t *mframe, uint64_t *moff,
                            uint32_t *mlen, uint64_t n, uint64_t i0 = 0) {
  const uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t f = mframe[i];
  const uint64_t first = mbase[f];
  uint64_t at = foff[f] + scan[i] - (first ? scan[first - 1] : 0);
  uint32_t sh = 0;
  while (s[at++] & 0x80u) {}  // the tag (field 1, wire type 2)
  uint64_t l = 0;
  for (;; sh += 7) {
    const uint32_t b = s[at++];
    l |= (uint64_t)(b & 0x7fu) << sh;
    if (b < 0x80u) break;
  }
  moff[i] = at;
  mlen[i] = (uint32_t)l;
}

// the frame of each message: the last frame whose first message is <= i
__global__ void k_ing_frames(const uint64_t *mbase, uint32_t nf,
                             uint32_t *mframe, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t lo = 0, hi = nf;  // mbase[lo] <= i < mbase[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (mbase[mid] <= i) lo = mid; else hi = mid;
  }
  mframe[i] = lo;
}

// the outcome of each message once the host decided which frames are
// delivered (fstate: 0 past the stream's end, 1 delivered, 2 filtered by
// DeploymentId / BinVer): its entry count for the decode's scan, and the
// drb_wire_in tallies (ctr[2] snapshots, [3] messages, [4] filtered,
// [5] entries), one atomic per wave and counter
constexpr uint32_t ING_TALLY_ROWS = 64;
// drb_ingest_wire uploads the stream in pieces of whole frames of at least
// this many bytes; each piece's CRC and count kernels start when it lands
constexpr size_t ING_PIECE = 32u << 20;
__global__ void k_ing_tally(const uint32_t *mframe, const uint8_t *fstate,
                            const uint32_t *err, const uint32_t *n_ent,
                            uint32_t *nsc, uint8_t *deliver, uint64_t n,
                            unsigned long long *ctr, DecMsg *dm,
                            bool restore = false, uint64_t i0 = 0) {
  const uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t st = 0, r = ING_BAD, ne = 0;
  if (i < n) {
    st = fstate[mframe[i]];
    r = err[i];
    ne = n_ent[i];
  }
  // (a message with a Cmd over cmd_cap is delivered undecoded: its
  // placement diverts it to the CPU path, ING_BIG)
  const bool dl = st == 1 && (r == ING_OK || r == ING_BIG);
  if (i < n) {
    nsc[i] = dl && r == ING_OK ? ne : 0u;
    deliver[i] = dl ? 1 : 0;
    if (!dl)
      dm[i].err = ING_BAD;  // not delivered: sorts last
    else if (restore)       // after a speculation that did not hold
      dm[i].err = r;
  }
  const bool snap = st != 0 && r == ING_SNAPSHOT;
  const bool msg = st == 1 && r != ING_SNAPSHOT;
  const bool filt = st == 2 && r != ING_SNAPSHOT;
  const uint64_t b0 = __ballot(snap), b1 = __ballot(msg), b2 = __ballot(filt);
  uint32_t e = dl && r == ING_OK ? ne : 0u;
  for (int o = 32; o > 0; o >>= 1) e += __shfl_xor(e, o);
  // per workgroup, then one of ING_TALLY_ROWS counter rows (64 B apart):
  // ~25k workgroups adding to one line serialised at its L2 channel
  __shared__ unsigned long long part[4];
  if (threadIdx.x < 4) part[threadIdx.x] = 0;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    if (b0) atomicAdd(&part[0], (unsigned long long)__popcll(b0));
    if (b1) atomicAdd(&part[1], (unsigned long long)__popcll(b1));
    if (b2) atomicAdd(&part[2], (unsigned long long)__popcll(b2));
    if (e) atomicAdd(&part[3], (unsigned long long)e);
  }
  __syncthreads();
  if (threadIdx.x < 4 && part[threadIdx.x])
    atomicAdd(&ctr[(blockIdx.x % ING_TALLY_ROWS) * 8 + 2 + threadIdx.x],
              part[threadIdx.x]);
}

// pass 2: the entries of the messages to deliver (their records are pass
// 1's); a message not delivered is marked so that it sorts last
__global__ void k_ing_decode(const uint8_t *s, const uint64_t *moff,
                             const uint32_t *mlen, const uint32_t *ent0,
                             const uint32_t *n_ent, DecMsg *out,
                             drb_entry *ents, uint64_t n, uint32_t cmd_cap,
                             uint64_t ecap, unsigned long long *ctr,
                             uint64_t i0 = 0) {
  // (a compacted list of these messages, one lane each, measured slower:
  // 0.80 ms against 0.62, profiles/r04_ingest)
  const uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || n_ent[i] == 0) return;  // pass 1's record is complete
  // (k_ing_tally marked the messages not delivered)
  if ((uint64_t)ent0[i] + n_ent[i] > ecap) {  // the speculative pass's
    atomicOr(&ctr[7], 1ull);                 // buffer: decoded again
    return;
  }
  DecMsg m;
  bool big = false;
  m.err = d_message(s + moff[i], mlen[i], m, ents + ent0[i], moff[i],
                    cmd_cap, big);
  m.ent0 = ent0[i];
  out[i] = m;
}

// a piece's entry bases: its local exclusive sums plus the entries of the
// delivered messages before it (the previous piece's bases are final)
__global__ void k_ing_carry(uint32_t *ent0, const uint32_t *nsc, uint64_t m0,
                            uint64_t m1) {
  const uint64_t i = m0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m1 || m0 == 0) return;
  ent0[i] += ent0[m0 - 1] + nsc[m0 - 1];
}

// plane keys (group, sender slot, receiver slot); messages for a shard or
// replica this engine does not host (dropped, nodehost.go:2089-2098), or not
// delivered, sort last (~0)
__global__ void k_ing_keys(const View v, const DecMsg *dm, uint32_t *key,
                           uint32_t *val, uint64_t n,
                           unsigned long long *ctr, uint64_t i0 = 0) {
  const uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const DecMsg m = dm[i];
  uint32_t k = ~0u;
  if (m.err == ING_OK || m.err == ING_BIG) {
    uint64_t g;
    if (ing_target(v, m.shard, m.from, m.to, &g))
      k = (uint32_t)((g * v.R + (m.from - 1)) * v.R + (m.to - 1));
    else
      atomicAdd(&ctr[1], 1ull);  // dropped
  }
  key[i] = k;
  val[i] = (uint32_t)i;
}

// the CPU path's messages of a drb_ingest_wire call (drb_wire_cpu), in no
// particular order (the host sorts them by offset)
DRB_DEV void ing_cpu_push(drb_wire_cpu *cpu, unsigned long long *cpu_n,
                          uint64_t cap, uint64_t off, uint32_t len,
                          uint32_t fate) {
  const unsigned long long q = atomicAdd(cpu_n, 1ull);
  if (q < cap) {
    cpu[q].offset = off;
    cpu[q].length = len;
    cpu[q].fate = fate;
  }
}

// the InstallSnapshot messages of the delivered frames (the CPU path's)
__global__ void k_ing_snaps(const uint32_t *mframe, const uint8_t *fstate,
                            const uint32_t *err, const uint64_t *moff,
                            const uint32_t *mlen, uint64_t n,
                            drb_wire_cpu *cpu, unsigned long long *cpu_n,
                            uint64_t cap) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && err[i] == ING_SNAPSHOT && fstate[mframe[i]] == 1)
    ing_cpu_push(cpu, cpu_n, cap, moff[i], mlen[i], DRB_ING_SNAPSHOT);
}

// one lane per plane (the head of a run of equal keys): MessageQueue.Add of
// its messages in stream order (drb_engine.hip drb_ingest_ex, restated): a
// message the plane cannot hold -- its records, a second Propose or one the
// forward rows cannot take, a Replicate beyond a remote plane's entry rows
// or the window, a Cmd over cmd_cap -- sends the receiver to the CPU path
// (ing_flag_capacity) with it and the plane's later messages; a receiver
// already off the fast path takes none (the CPU raft.Peer's)
__global__ void k_ing_place(const View v, const uint8_t *s, const DecMsg *dm,
                            const drb_entry *ents, const uint32_t *key,
                            const uint32_t *idx, uint64_t n, uint32_t buf,
                            uint32_t tag, unsigned long long *ctr,
                            const uint64_t *moff, const uint32_t *mlen,
                            drb_wire_cpu *cpu, unsigned long long *cpu_n,
                            uint64_t cpu_cap, uint64_t round) {
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 >= n) return;
  const uint32_t k = key[i0];
  if (k == ~0u || (i0 > 0 && key[i0 - 1] == k)) return;
  const uint32_t to = k % v.R, from = (k / v.R) % v.R;
  const uint64_t g = (uint64_t)(k / v.R) / v.R;
  uint64_t i1 = i0 + 1;
  while (i1 < n && key[i1] == k) ++i1;
  // placement C4: a plane whose sender slot lives on another rank is read
  // from the inbound copies (mbox_in, ...), entries from its entry rows
  const bool rm = pair_remote(v, from, to);
  uint4 *const mbox = rm ? v.mbox_in : v.mbox;
  uint4 *const mmeta = rm ? v.meta_in : v.mbox_meta;
  uint64_t *const mmax = rm ? v.maxapp_in : v.mbox_maxapp;
  uint64_t *const rterm = rm ? v.rterm_in : v.rterm;
  unsigned long long *row = ctr + (blockIdx.x % ING_TALLY_ROWS) * 8;
  const uint32_t ft = v.u32[u32_ix(v, W_FLAGS, to, g)];
  // (co-resident senders step here; another rank's lane holds another group)
  const uint32_t ff = rm ? 0u : v.u32[u32_ix(v, W_FLAGS, from, g)];
  const bool from_hosted =
      (ff & DRB_F_HOSTED) && !(ff & (DRB_F_FALLBACK | DRB_F_ERROR));
  if (!(ft & DRB_F_HOSTED) || from_hosted) {
    // the transport delivers remote senders to hosted replicas only
    atomicAdd(&row[1], (unsigned long long)(i1 - i0));
    return;
  }
  // a receiver off the fast path: every message is the CPU path's
  bool div = (ft & (DRB_F_FALLBACK | DRB_F_ERROR)) != 0;
  const bool was_off = div;
  uint4 cur = mmeta[mmeta_ix(v, buf, from, to, g)];
  uint64_t maxapp = mmax[mmeta_ix(v, buf, from, to, g)];
  if (!tag_is(cur.x, tag)) {  // nothing there yet this round
    cur = make_uint4(tag & MQ_TAG, 0, 0, 0);
  }
  bool maxapp_valid = mi_nrep(cur.y) > 0;
  // remote planes: the first entry index of the plane's entry rows (set by
  // the round's first Replicate with entries placed here; 0: none yet)
  uint64_t elo = maxapp_valid && rm ? v.elo_in[mmeta_ix(v, buf, from, to, g)]
                                    : 0;
  uint64_t acc = 0, ndiv = 0;
  for (uint64_t j = i0; j < i1; ++j) {
    const uint32_t mi = idx[j];
    const DecMsg m = dm[mi];
    const bool rep = m.type == DRB_MSG_REPLICATE;
    if (!div) {
      if (m.type == DRB_MSG_QUIESCE) {  // node-level: a header bit
        cur.x |= MQ_QUIESCE;
        acc++;
        continue;
      }
      bool fit = m.err == ING_OK && mi_count(cur.y) < v.MB;
      if (fit && m.type == DRB_MSG_PROPOSE) {
        // handleFollowerPropose's message from another NodeHost: its
        // entries go to the sender's forward rows, one Propose per plane and
        // round (drb_config.forward_proposals)
        fit = v.fwd_props && !rm && !(cur.y & MI_PROP) &&
              m.n_ent <= v.max_props;
        for (uint32_t x = 0; fit && x < m.n_ent; ++x)
          fit = ents[m.ent0 + x].cmd_len <= v.C16 * 16;
      }
      if (fit && rep && m.n_ent > v.W) fit = false;  // (the window rows)
      if (fit && rep && rm && m.n_ent) {
        // entry rows [elo, elo + E), elo set by the round's first
        // Replicate that carries entries (a commit-only one needs none)
        const uint64_t e0 = elo ? elo : m.log_index + 1;
        fit = m.log_index + 1 >= e0 && m.log_index + m.n_ent - e0 < v.E;
        if (fit) elo = e0;
      }
      div = !fit;
    }
    if (div) {  // the CPU path's, in stream order after what was placed
      ing_cpu_push(cpu, cpu_n, cpu_cap, moff[mi], mlen[mi], DRB_ING_DIVERTED);
      ndiv++;
      continue;
    }
    const uint32_t kk =
        rep ? mi_nrep(cur.y) : rec_pos(false, mi_noth(cur.y), v.MB);
    if (m.type == DRB_MSG_PROPOSE) {
      const uint32_t fw = fwd_ps(v, buf, from);
      for (uint32_t x = 0; x < m.n_ent; ++x) {
        const drb_entry en = ents[m.ent0 + x];
        const uint32_t b0 = en.cmd_len ? s[en.cmd_off] : 0u;
        v.props[prop_ix(v, fw, x, 0, g)] = make_uint4(
            (uint32_t)en.key, (uint32_t)(en.key >> 32), (uint32_t)en.client_id,
            (uint32_t)(en.client_id >> 32));
        v.props[prop_ix(v, fw, x, 1, g)] = make_uint4(
            (uint32_t)en.series_id, (uint32_t)(en.series_id >> 32),
            (uint32_t)en.responded_to, (uint32_t)(en.responded_to >> 32));
        v.props[prop_ix(v, fw, x, 2, g)] = make_uint4(
            en.type, en.cmd_len,
            prop_fast(en.type, en.client_id, en.series_id, en.cmd_len, b0), 0);
        for (uint32_t cc = 0; cc < v.C16; ++cc) {
          uint32_t w[4] = {0, 0, 0, 0};
          for (uint32_t b = 0; b < 16 && cc * 16 + b < en.cmd_len; ++b)
            w[b >> 2] |= (uint32_t)s[en.cmd_off + cc * 16 + b] << (8 * (b & 3));
          v.props[prop_ix(v, fw, x, PROP_META + cc, g)] =
              make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
    }
    if (rep && m.n_ent) {
      // the entries travel in the sender's (unhosted) window slot, or in the
      // plane's entry rows when the plane is remote
      for (uint32_t x = 0; x < m.n_ent; ++x) {
        const drb_entry en = ents[m.ent0 + x];
        const uint64_t index = m.log_index + 1 + x;
        uint4 ch[ENT_META];
        ch[0] = make_uint4((uint32_t)en.term, (uint32_t)(en.term >> 32),
                           (uint32_t)en.key, (uint32_t)(en.key >> 32));
        ch[1] = make_uint4(
            (uint32_t)en.client_id, (uint32_t)(en.client_id >> 32),
            (uint32_t)en.series_id, (uint32_t)(en.series_id >> 32));
        ch[2] = make_uint4((uint32_t)en.responded_to,
                           (uint32_t)(en.responded_to >> 32), en.type,
                           en.cmd_len);
        for (uint32_t c = 0; c < ENT_META + v.C16; ++c) {
          uint4 q;
          if (c < ENT_META) {
            q = ch[c];
          } else {
            const uint32_t cc = c - ENT_META;
            uint32_t w[4] = {0, 0, 0, 0};
            for (uint32_t b = 0; b < 16 && cc * 16 + b < en.cmd_len; ++b)
              w[b >> 2] |= (uint32_t)s[en.cmd_off + cc * 16 + b]
                           << (8 * (b & 3));
            q = make_uint4(w[0], w[1], w[2], w[3]);
          }
          if (rm)
            v.embox_in[embox_ix(v, buf, from, to, (uint32_t)(index - elo), c,
                                g)] = q;
          else
            v.ring[ring_ix(v, from, index, c, g)] = q;
        }
      }
    }
    Msg mm;
    mm.type = m.type;
    mm.reject = m.reject ? 1 : 0;
    mm.n = m.n_ent;
    mm.term = m.term;
    mm.log_index = m.log_index;
    mm.log_term = m.log_term;
    mm.commit = m.commit;
    mm.hint = m.hint;
    mm.hint_high = m.hint_high;
    uint4 c0, c1;
    msg_encode(mm, to, nullptr, c0, c1);
    // the sender's term is stored once per (sender, receiver, round) in the
    // header; a record whose term differs makes the receiver fall back
    const bool zero = (c0.x & MF_TERM_ZERO) != 0;
    bool other = false;
    if (!zero) {
      // a pre-vote record carries a term of its own (r.term + 1 or the
      // granted one, not the sender's): it never seeds the header's term
      // and always travels with its own (as the GPU's emit writes them)
      const bool pv = is_prevote_type(m.type);
      if (!pv && !(cur.y & MI_TERM)) {
        cur.z = (uint32_t)m.term;
        cur.w = (uint32_t)(m.term >> 32);
      } else if (pv || q_hi(cur) != m.term) {
        other = true;
        c0.x |= MF_TERM_OTHER;
        if (rterm) rterm[rterm_ix(v, buf, from, to, kk, g)] = m.term;
      }
    }
    mbox[mbox_ix(v, buf, from, to, kk, 0, g)] = c0;
    mbox[mbox_ix(v, buf, from, to, kk, 1, g)] = c1;
    const uint32_t inf = msg_info(m.type, zero, m.reject != 0, m.n_ent) |
                         (other ? MI_TERM_OTHER : 0u);
    cur.y = (cur.y + (inf & MI_CNTS)) | (inf & ~MI_CNTS);
    if (rep) {
      const uint64_t ma = m.log_index + m.n_ent;
      maxapp = maxapp_valid ? umax64(maxapp, ma) : ma;
      maxapp_valid = true;
    }
    acc++;
  }
  if (acc) {
    mmeta[mmeta_ix(v, buf, from, to, g)] = cur;
    mmax[mmeta_ix(v, buf, from, to, g)] = maxapp;
    if (rm && maxapp_valid) v.elo_in[mmeta_ix(v, buf, from, to, g)] = elo;
    if (!rm && (mi_count(cur.y) || (cur.x & MQ_QUIESCE)))  // its tag byte
      ((uint8_t *)&v.inbox_tag[((uint64_t)buf * v.R + to) * v.G + g])[from] =
          tag_byte(tag, cur.y);
  }
  if (ndiv && !was_off) ing_flag_capacity(v, g, to, round);
  // (a lane per plane: the adds spread over the counter rows)
  if (acc) atomicAdd(&row[0], (unsigned long long)acc);
  if (ndiv) atomicAdd(&row[6], (unsigned long long)ndiv);
}

}  // namespace drb

// ------------------------------------------------------------ host side
// the host's part of the walk: frame headers, the MessageBatch top-level
// scan, the CRC combine algebra, the step packing (drb_wirehost.hpp: plain
// C++, also built under AddressSanitizer / UBSan by tests/test_wirehost.py)
#include "drb_wirehost.hpp"

// device buffers of drb_ingest_wire (grow-only, under ingest_mu)
struct IngestBuf {
  void *p = nullptr;
  size_t cap = 0;
};
static int ing_grow(IngestBuf &b, size_t need) {
  if (need <= b.cap) return DRB_OK;
  if (b.p) HIPCHK(hipFree(b.p));
  b.p = nullptr;
  HIPCHK(hipMalloc(&b.p, need));
  b.cap = need;
  return DRB_OK;
}
struct IngestState {
  IngestBuf stream, msgs, ents, sort, misc, chunks, cpu;
  // the CPU path's messages of the last call, in stream order
  std::vector<drb_wire_cpu> cpu_msgs;
  bool k64_ready = false;     // c_crc_k64 uploaded
  uint8_t *pinned = nullptr;  // drb_ingest_buffer (hipHostMalloc)
  size_t pinned_cap = 0;
  // the frames' element steps gathered for one DMA (grow-only, pinned)
  uint32_t *steps = nullptr;
  size_t steps_cap = 0;
  // the frames of the last call; their Requests vectors keep their
  // capacity, so a warm call neither faults nor unmaps ~12 B per message
  std::vector<wirehost::Frame> frames;
  // the stream goes up in pieces on its own stream, one event each, so the
  // CRC and count kernels of a piece run while the later pieces upload
  hipStream_t up = nullptr;
  std::vector<hipEvent_t> ev;  // per piece: uploaded
  hipEvent_t evv = nullptr;  // the verdicts' inputs are down (speculation)
};
static void ingest_free(IngestState *st) {
  if (!st) return;
  for (hipEvent_t x : st->ev) (void)hipEventDestroy(x);
  if (st->evv) (void)hipEventDestroy(st->evv);
  if (st->up) (void)hipStreamDestroy(st->up);
  if (st->pinned) (void)hipHostFree(st->pinned);
  if (st->steps) (void)hipHostFree(st->steps);
  for (IngestBuf *b : {&st->stream, &st->msgs, &st->ents, &st->sort,
                       &st->misc, &st->chunks, &st->cpu})
    if (b->p) (void)hipFree(b->p);
  delete st;
}

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// DRB_INGEST_TRACE=1: per-phase wall times on stderr (each mark waits for
// the engine stream, so a traced call is slower than an untraced one)
#include <chrono>
struct IngestTrace {
  bool on;
  hipStream_t s;
  std::chrono::steady_clock::time_point t;
  explicit IngestTrace(hipStream_t st) : s(st) {
    const char *e = getenv("DRB_INGEST_TRACE");
    on = e && e[0] == '1';
    t = std::chrono::steady_clock::now();
  }
  ~IngestTrace() { mark("return"); }
  void mark(const char *what) {
    if (!on) return;
    (void)hipStreamSynchronize(s);
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "ingest %-10s %8.3f ms\n", what,
            std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

// A transport's own pinned receive buffer (one per connection / thread):
// drb_ingest_wire reads it while the caller holds it, and no other caller
// can grow or free it.
extern "C" int drb_ingest_buffer_alloc(drb_engine *e, size_t cap,
                                       uint8_t **buf) {
  if (!e || !buf || !cap) return DRB_EINVAL;
  *buf = nullptr;
  HIPCHK(hipSetDevice(e->cfg.device));
  HIPCHK(hipHostMalloc((void **)buf, cap, hipHostMallocDefault));
  return DRB_OK;
}

extern "C" int drb_ingest_buffer_free(drb_engine *e, uint8_t *buf) {
  if (!e) return DRB_EINVAL;
  if (buf) {
    // a drb_ingest_wire of this buffer has synchronised before returning
    HIPCHK(hipHostFree(buf));
  }
  return DRB_OK;
}

extern "C" int drb_ingest_buffer(drb_engine *e, size_t cap, uint8_t **buf) {
  if (!e || !buf) return DRB_EINVAL;
  std::lock_guard<std::mutex> lock(e->ingest_mu);
  if (!e->ingest) e->ingest = new IngestState();
  IngestState &st = *e->ingest;
  if (cap > st.pinned_cap) {
    if (st.pinned) HIPCHK(hipHostFree(st.pinned));
    st.pinned = nullptr;
    st.pinned_cap = 0;
    HIPCHK(hipHostMalloc((void **)&st.pinned, cap, hipHostMallocDefault));
    st.pinned_cap = cap;
  }
  *buf = st.pinned;
  return DRB_OK;
}

extern "C" int drb_ingest_wire(drb_engine *e, const uint8_t *stream,
                               size_t len, uint64_t deployment_id,
                               drb_wire_in *out) {
  using namespace drb;
  if (!e || (!stream && len)) return DRB_EINVAL;
  if (!e->bound.empty()) return DRB_EINVAL;  // (drb_ingest_ex)
  wirehost::crc_init();
  std::lock_guard<std::mutex> lock(e->ingest_mu);
  // replicas spread over ranks: not between a round and its exchange
  // (drb_exchange_mark, include/drb_engine.h)
  if (e->v.remote_mask && e->exchanged_round != e->round) return DRB_EAGAIN;
  if (!e->ingest) e->ingest = new IngestState();
  IngestState &st = *e->ingest;
  const View &v = e->v;
  drb_wire_in res;
  memset(&res, 0, sizeof(res));
  st.cpu_msgs.clear();
  IngestTrace tr(e->stream);
  // 1. frames: magic + requestHeader + its CRC (tcp.go:64-112, 180-237)
  std::vector<wirehost::Frame> &fr = st.frames;
  bool bad_header = false;  // ErrBadMessage: the connection is closed
  const size_t walked = wirehost::walk_frames(stream, len, fr, &bad_header);
  tr.mark("headers");
  const size_t sb = al256(walked + 16);
  if (ing_grow(st.stream, sb)) return DRB_EDEVICE;
  uint8_t *ds = (uint8_t *)st.stream.p;
  hipStream_t sm = e->stream;
  // once the upload is enqueued, every return waits for the engine stream
  // first: the caller may reuse or refill `stream` (a pinned buffer is
  // read by the DMA engine asynchronously) as soon as this call returns
  struct SyncOnReturn {
    hipStream_t s;
    IngestState *st;
    ~SyncOnReturn() {
      if (st->up) (void)hipStreamSynchronize(st->up);
      (void)hipStreamSynchronize(s);
    }
  } sync_on_return{e->stream, &st};
  // 2. the stream goes up (its own host thread: a pageable source makes
  // the copy synchronous) while Requests boundaries are found, one host
  // thread per frame (a frame holds up to 64 MiB of messages), at most 16
  // the CRC tables, before the first CRC kernel (the upload thread's)
  if (!e->crc_tab_ready) {
    uint32_t tab[8][256];
    for (uint32_t a = 0; a < 256; ++a) tab[0][a] = wirehost::crc_tab[a];
    for (uint32_t a = 0; a < 256; ++a)
      for (int s = 1; s < 8; ++s)
        tab[s][a] = tab[0][tab[s - 1][a] & 0xff] ^ (tab[s - 1][a] >> 8);
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_tab), tab, sizeof(tab)));
    e->crc_tab_ready = true;
  }
  if (!st.k64_ready) {  // x^(8 * 64 * (255 - t)) mod P
    uint32_t k64[256];
    for (int t = 0; t < 256; ++t)
      k64[t] = wirehost::crc32_combine(1u << 31, 0, 64ull * (255 - t));
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_k64), k64, sizeof(k64)));
    st.k64_ready = true;
  }
  // the payload CRCs in 16 KB chunks (the chunk lists go up first)
  constexpr uint64_t CH = 16384;
  std::vector<uint64_t> coff;
  std::vector<uint32_t> clen;
  std::vector<uint32_t> cfirst(fr.size() + 1, 0);
  for (size_t f = 0; f < fr.size(); ++f) {
    cfirst[f] = (uint32_t)coff.size();
    for (uint64_t o = 0; o < fr[f].size; o += CH) {
      coff.push_back(fr[f].off + o);
      clen.push_back((uint32_t)std::min<uint64_t>(CH, fr[f].size - o));
    }
  }
  cfirst[fr.size()] = (uint32_t)coff.size();
  const size_t nc = coff.size();
  if (ing_grow(st.chunks, al256(nc * 8 + 8) + 2 * al256(nc * 4 + 4)))
    return DRB_EDEVICE;
  uint64_t *d_coff = (uint64_t *)st.chunks.p;
  uint32_t *d_clen = (uint32_t *)((uint8_t *)st.chunks.p + al256(nc * 8 + 8));
  uint32_t *d_ccrc = (uint32_t *)((uint8_t *)d_clen + al256(nc * 4 + 4));
  // pieces: runs of whole frames of at least ING_PIECE bytes
  std::vector<size_t> pf;  // first frame of each piece, then nf
  for (size_t f = 0, acc = 0; f < fr.size(); ++f) {
    if (pf.empty() || acc >= ING_PIECE) {
      pf.push_back(f);
      acc = 0;
    }
    acc += 20 + (size_t)fr[f].size;
  }
  pf.push_back(fr.size());
  const size_t np = pf.size() - 1;
  if (!st.up &&
      hipStreamCreateWithFlags(&st.up, hipStreamNonBlocking) != hipSuccess)
    return DRB_EDEVICE;
  while (st.ev.size() < (np ? np : 1)) {  // (ev[0] also for the start)
    hipEvent_t x;
    if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess)
      return DRB_EDEVICE;
    st.ev.push_back(x);
  }
  // the upload starts behind what the engine stream has enqueued (the
  // device buffers may still be read by an earlier call)
  HIPCHK(hipEventRecord(st.ev[0], sm));
  HIPCHK(hipStreamWaitEvent(st.up, st.ev[0], 0));
  // (the payload CRCs run on the engine stream per piece, after its bytes
  // landed; on a stream of their own as each piece lands they measured no
  // faster)
  if (nc) {
    HIPCHK(hipMemcpyAsync(d_coff, coff.data(), nc * 8, hipMemcpyHostToDevice,
                          sm));
    HIPCHK(hipMemcpyAsync(d_clen, clen.data(), nc * 4, hipMemcpyHostToDevice,
                          sm));
  }
  {
    hipError_t up_err = hipSuccess;
    std::thread up([&]() {
      up_err = hipSetDevice(e->cfg.device);  // (the current device is per thread)
      for (size_t q = 0; q < np && up_err == hipSuccess; ++q) {
        const size_t a = q ? fr[pf[q]].off - 20 : 0;
        const size_t b = pf[q + 1] < fr.size() ? fr[pf[q + 1]].off - 20
                                                : walked;
        if (b > a)
          up_err = hipMemcpyAsync(ds + a, stream + a, b - a,
                                  hipMemcpyHostToDevice, st.up);
        if (up_err == hipSuccess) up_err = hipEventRecord(st.ev[q], st.up);
      }
    });
    const size_t nt = std::min<size_t>(16, fr.size());
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt; ++t)
      th.emplace_back([&, t]() {
        for (size_t f = t; f < fr.size(); f += nt)
          if (fr[f].method == 100) wirehost::scan_batch(stream, fr[f]);
      });
    for (auto &x : th) x.join();
    up.join();
    HIPCHK(up_err);
  }
  uint64_t nm = 0;
  for (const auto &f : fr) nm += f.step.size();
  tr.mark("up+scan");
  // 3. the stream up (its payload CRCs ran per piece)
  // misc: chunk offsets/lens/crcs, message offsets/lens/frames, counts,
  // errors, entry bases, deliver flags, per-frame error, 2 counters
  const size_t m1 = nm ? nm : 1;
  const size_t nf = fr.size();
  size_t scan_tb = 0;
  HIPCHK(hipcub::DeviceScan::InclusiveSum(nullptr, scan_tb, (uint64_t *)nullptr,
                                          (uint64_t *)nullptr, (int)m1, sm));
  const size_t mb = al256(m1 * 8) * 3 +
                    al256(m1 * 4) * 7 + al256(m1) +
                    al256((nf + 1) * 4) + al256((nf + 1) * 8) * 2 +
                    al256(nf + 1) + ING_TALLY_ROWS * 64 + al256(scan_tb);
  if (ing_grow(st.misc, mb)) return DRB_EDEVICE;
  uint8_t *q = (uint8_t *)st.misc.p;
  auto take = [&](size_t b) {
    uint8_t *r = q;
    q += al256(b);
    return r;
  };
  uint64_t *d_moff = (uint64_t *)take(m1 * 8);
  uint32_t *d_mlen = (uint32_t *)take(m1 * 4);
  uint32_t *d_mframe = (uint32_t *)take(m1 * 4);
  uint32_t *d_nent = (uint32_t *)take(m1 * 4);
  uint32_t *d_err = (uint32_t *)take(m1 * 4);
  uint32_t *d_nsc = (uint32_t *)take(m1 * 4);
  uint32_t *d_ent0 = (uint32_t *)take(m1 * 4);
  uint8_t *d_deliver = take(m1);
  uint32_t *d_fbad = (uint32_t *)take((nf + 1) * 4);
  uint64_t *d_mbase = (uint64_t *)take((nf + 1) * 8);
  uint64_t *d_foff = (uint64_t *)take((nf + 1) * 8);
  uint32_t *d_step = (uint32_t *)take(m1 * 4);
  uint64_t *d_step64 = (uint64_t *)take(m1 * 8);
  uint64_t *d_scan = (uint64_t *)take(m1 * 8);
  void *d_scan_tmp = take(scan_tb);
  uint8_t *d_fstate = take(nf + 1);
  unsigned long long *d_ctr =
      (unsigned long long *)take(ING_TALLY_ROWS * 8 * 8);
  // each frame's Requests go up straight from its scan vectors
  std::vector<uint64_t> mbase(nf + 1, 0);
  for (size_t f = 0; f < nf; ++f) mbase[f + 1] = mbase[f] + fr[f].step.size();
  HIPCHK(hipMemsetAsync(d_fbad, 0, (fr.size() + 1) * 4, sm));
  HIPCHK(hipMemsetAsync(d_ctr, 0, ING_TALLY_ROWS * 8 * 8, sm));
  const uint32_t cmd_cap = v.C16 * 16;
  if (nm) {
    std::vector<uint64_t> foff(nf + 1, 0);
    for (size_t f = 0; f < nf; ++f) foff[f] = fr[f].off;
    // the frames' steps into one pinned buffer (host threads, one DMA):
    // per-frame pageable copies ran ~2 ms for a C3 plane's 25 MB
    if (nm > st.steps_cap) {
      if (st.steps) HIPCHK(hipHostFree(st.steps));
      st.steps = nullptr;
      st.steps_cap = 0;
      HIPCHK(hipHostMalloc((void **)&st.steps, nm * 4, hipHostMallocDefault));
      st.steps_cap = nm;
    }
    // 2 B steps when every one fits (a message under 64 KB), else 4 B
    std::atomic<bool> wide{false};
    {
      const size_t nt = std::min<size_t>(16, nf);
      std::vector<std::thread> th;
      uint16_t *s16 = (uint16_t *)st.steps;
      for (size_t t = 0; t < nt; ++t)
        th.emplace_back([&, t]() {
          for (size_t f = t; f < nf && !wide.load(std::memory_order_relaxed);
               f += nt)
            if (!wirehost::pack_steps16(fr[f], s16 + mbase[f]))
              wide.store(true);
        });
      for (auto &x : th) x.join();
    }
    if (wide) {
      const size_t nt = std::min<size_t>(16, nf);
      std::vector<std::thread> th;
      for (size_t t = 0; t < nt; ++t)
        th.emplace_back([&, t]() {
          for (size_t f = t; f < nf; f += nt)
            if (!fr[f].step.empty())
              memcpy(st.steps + mbase[f], fr[f].step.data(),
                     fr[f].step.size() * 4);
        });
      for (auto &x : th) x.join();
    }
    const uint64_t step_bytes = nm * (wide ? 4 : 2);
    // pulled by a kernel from the mapped pinned buffer, not DMA'd: a copy
    // queued here waits on the copy engine behind the stream's remaining
    // pieces, and the per-piece counts below need it (profiles/r04_ingest)
    void *hsteps = nullptr;
    if (hipHostGetDevicePointer(&hsteps, st.steps, 0) == hipSuccess &&
        hsteps && ((uintptr_t)hsteps & 15) == 0) {
      const uint64_t nv = step_bytes / 16 + 1;
      k_zc_pull<<<(unsigned)std::min<uint64_t>(1024, (nv + 1023) / 1024), 256,
                  0, sm>>>((uint8_t *)d_step, (const uint8_t *)hsteps,
                           step_bytes);
      HIPCHK(hipGetLastError());
    } else {
      (void)hipGetLastError();
      HIPCHK(hipMemcpyAsync(d_step, st.steps, step_bytes,
                            hipMemcpyHostToDevice, sm));
    }
    HIPCHK(hipMemcpyAsync(d_mbase, mbase.data(), (nf + 1) * 8,
                          hipMemcpyHostToDevice, sm));
    HIPCHK(hipMemcpyAsync(d_foff, foff.data(), (nf + 1) * 8,
                          hipMemcpyHostToDevice, sm));
    k_ing_frames<<<(unsigned)((nm + 255) / 256), 256, 0, sm>>>(
        d_mbase, (uint32_t)nf, d_mframe, nm);
    // offsets and lengths from the elements' steps: a scan, then each
    // element's tag and length varints read from the uploaded stream
    k_widen_step<<<(unsigned)((nm + 255) / 256), 256, 0, sm>>>(
        d_step, d_step64, nm, !wide);
    HIPCHK(hipcub::DeviceScan::InclusiveSum(d_scan_tmp, scan_tb, d_step64,
                                            d_scan, (int)nm, sm));
    if (ing_grow(st.msgs, al256(nm * sizeof(DecMsg)))) return DRB_EDEVICE;
  }
  // sort / scan temporary storage and the key arrays (the speculative
  // pass below uses them per piece)
  size_t tb = 0, tb2 = 0;
  uint8_t *sp = nullptr;
  void *tmp = nullptr;
  uint32_t *kin = nullptr, *kout = nullptr, *vin = nullptr, *vout = nullptr;
  DecMsg *dm = (DecMsg *)st.msgs.p;
  if (nm) {
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, vin,
                                              vout, (int)nm, 0, 32, sm));
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, d_nsc, d_ent0,
                                            (int)nm, sm));
    tb = std::max(tb, tb2);
    const size_t sbytes = al256(nm * 4) * 4 + al256(tb);
    if (ing_grow(st.sort, sbytes)) return DRB_EDEVICE;
    sp = (uint8_t *)st.sort.p;
    tmp = sp + 4 * al256(nm * 4);
    kin = (uint32_t *)sp;
    kout = (uint32_t *)(sp + al256(nm * 4));
    vin = (uint32_t *)(sp + 2 * al256(nm * 4));
    vout = (uint32_t *)(sp + 3 * al256(nm * 4));
  }
  // Speculation: every frame the host walk accepted is delivered (no bad
  // CRC, no malformed message -- the verdicts below confirm it).  Then each
  // piece's tally, entry bases, decode and plane keys run as it lands,
  // beside the upload of the rest, into the entry buffer as the last call
  // left it; a speculation that does not hold (or an entry buffer too
  // small) is redone after the verdicts, as without it.
  const bool spec = nm != 0;
  std::vector<uint8_t> fspec(nf + 1, 0);
  const uint64_t ecap = st.ents.cap / sizeof(drb_entry);
  if (spec) {
    for (size_t f = 0; f < nf; ++f)
      fspec[f] = fr[f].method == 200 ? 0
                 : fr[f].did == deployment_id && fr[f].bv == 210 ? 1 : 2;
    HIPCHK(hipMemcpyAsync(d_fstate, fspec.data(), nf + 1,
                          hipMemcpyHostToDevice, sm));
  }
  // per piece, once its bytes are up (and CRC'd): its messages' element
  // boundaries and counts
  for (size_t q = 0; q < np; ++q) {
    HIPCHK(hipStreamWaitEvent(sm, st.ev[q], 0));
    const uint32_t c0 = cfirst[pf[q]], c1 = cfirst[pf[q + 1]];
    if (c1 > c0)
      k_crc_chunks<<<c1 - c0, 256, 0, sm>>>(ds, d_coff + c0, d_clen + c0,
                                            d_ccrc + c0);
    const uint64_t m0 = mbase[pf[q]], m1 = mbase[pf[q + 1]];
    if (m1 > m0) {
      const unsigned gb = (unsigned)((m1 - m0 + 255) / 256);
      k_ing_elems<<<gb, 256, 0, sm>>>(ds, d_scan, d_mbase, d_foff, d_mframe,
                                      d_moff, d_mlen, m1, m0);
      k_ing_count<<<gb, 256, 0, sm>>>(
          ds, d_moff, d_mlen, d_mframe, d_nent, d_err, d_fbad, dm, m1,
          cmd_cap, m0);
      if (spec) {
        k_ing_tally<<<gb, 256, 0, sm>>>(d_mframe, d_fstate, d_err, d_nent,
                                        d_nsc, d_deliver, m1, d_ctr, dm, false,
                                        m0);
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, d_nsc + m0,
                                                d_ent0 + m0, (int)(m1 - m0),
                                                sm));
        k_ing_carry<<<gb, 256, 0, sm>>>(d_ent0, d_nsc, m0, m1);
        k_ing_decode<<<gb, 256, 0, sm>>>(
            ds, d_moff, d_mlen, d_ent0, d_nsc, dm, (drb_entry *)st.ents.p, m1,
            cmd_cap, ecap, d_ctr, m0);
        k_ing_keys<<<gb, 256, 0, sm>>>(v, dm, kin, vin, m1, d_ctr, m0);
      }
    }
    HIPCHK(hipGetLastError());
  }
  std::vector<uint32_t> ccrc(nc), fbad(fr.size() + 1);
  unsigned long long rows[ING_TALLY_ROWS * 8];
  if (nc)
    HIPCHK(hipMemcpyAsync(ccrc.data(), d_ccrc, nc * 4, hipMemcpyDeviceToHost, sm));
  HIPCHK(hipMemcpyAsync(fbad.data(), d_fbad, (fr.size() + 1) * 4,
                        hipMemcpyDeviceToHost, sm));
  // the key bits that can differ: plane keys < G·R·R, and the ~0 of a
  // refused message keeps all ones in those bits, so it still sorts last
  int kbits = 1;
  while (kbits < 32 && ((uint64_t)1 << kbits) <= (uint64_t)v.G * v.R * v.R)
    ++kbits;
  if (spec) {
    // the plane sort of the speculative keys runs while the host checks
    // the verdicts
    HIPCHK(hipMemcpyAsync(rows, d_ctr, sizeof(rows), hipMemcpyDeviceToHost,
                          sm));
    if (!st.evv &&
        hipEventCreateWithFlags(&st.evv, hipEventDisableTiming) != hipSuccess)
      return DRB_EDEVICE;
    HIPCHK(hipEventRecord(st.evv, sm));
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kin, kout, vin, vout,
                                              (int)nm, 0, kbits, sm));
    HIPCHK(hipEventSynchronize(st.evv));
  } else {
    HIPCHK(hipStreamSynchronize(sm));
  }
  tr.mark("crc+cnt");
  // 4. the frames delivered: up to the first with a bad CRC or a batch that
  // does not decode (ErrBadMessage closes the connection, tcp.go:528-530)
  std::vector<uint8_t> fstate(nf + 1, 0);
  size_t consumed = 0;
  bool any_deliver = false;
  {
    size_t mi = 0;
    for (size_t f = 0; f < nf; ++f) {
      // the chunks' register-only CRCs combined, then the ~0 conditioning
      const uint32_t c = wirehost::fold_frame_crc(
          ccrc.data() + cfirst[f], clen.data() + cfirst[f],
          cfirst[f + 1] - cfirst[f], fr[f].size);
      const size_t nmf = fr[f].step.size();
      if (c != fr[f].pcrc || !fr[f].scan_ok || (fbad[f] & 1u)) {
        res.bad = 1;
        break;
      }
      res.frames++;
      consumed = fr[f].off + fr[f].size;
      if (fr[f].method == 200) {  // a snapshot Chunk (tcp.go:532-540)
        res.snapshots++;
        mi += nmf;
        continue;
      }
      const bool keep = fr[f].did == deployment_id && fr[f].bv == 210;
      fstate[f] = keep ? 1 : 2;
      any_deliver |= keep && nmf;
      mi += nmf;
    }
  }
  if (bad_header && !res.bad) res.bad = 1;
  res.consumed = consumed;
  bool spec_ok = spec && fstate == fspec;
  if (spec_ok) {
    unsigned long long ovf = 0;
    for (uint32_t q = 0; q < ING_TALLY_ROWS; ++q) ovf |= rows[q * 8 + 7];
    spec_ok = ovf == 0;
  }
  // per-message outcomes (snapshot / delivered / filtered), the entry bases
  if (nm) {
    unsigned long long c0[6] = {0, 0, 0, 0, 0, 0};
    if (!spec_ok) {
      if (spec)  // the speculative pass's tallies and drops start over
        HIPCHK(hipMemsetAsync(d_ctr, 0, ING_TALLY_ROWS * 8 * 8, sm));
      HIPCHK(hipMemcpyAsync(d_fstate, fstate.data(), nf + 1,
                            hipMemcpyHostToDevice, sm));
      k_ing_tally<<<(unsigned)((nm + 255) / 256), 256, 0, sm>>>(
          d_mframe, d_fstate, d_err, d_nent, d_nsc, d_deliver, nm, d_ctr, dm,
          spec);
      HIPCHK(hipGetLastError());
      HIPCHK(hipcub::DeviceScan::ExclusiveSum(tmp, tb2, d_nsc, d_ent0,
                                              (int)nm, sm));
      HIPCHK(hipMemcpyAsync(rows, d_ctr, sizeof(rows), hipMemcpyDeviceToHost,
                            sm));
      HIPCHK(hipStreamSynchronize(sm));
    }
    for (uint32_t q = 0; q < ING_TALLY_ROWS; ++q)
      for (int k = 2; k < 6; ++k) c0[k] += rows[q * 8 + k];
    res.snapshots += c0[2];
    res.messages = c0[3];
    res.dropped += c0[4];
    const uint64_t tot = c0[5];
    // the CPU path's messages: InstallSnapshots, and what placement diverts
    if (ing_grow(st.cpu, al256(8) + nm * sizeof(drb_wire_cpu)))
      return DRB_EDEVICE;
    unsigned long long *d_cpu_n = (unsigned long long *)st.cpu.p;
    drb_wire_cpu *d_cpu = (drb_wire_cpu *)((uint8_t *)st.cpu.p + al256(8));
    HIPCHK(hipMemsetAsync(d_cpu_n, 0, 8, sm));
    if (c0[2])
      k_ing_snaps<<<(unsigned)((nm + 255) / 256), 256, 0, sm>>>(
          d_mframe, d_fstate, d_err, d_moff, d_mlen, nm, d_cpu, d_cpu_n, nm);
    if (any_deliver) {
      if (!spec_ok) {
        const size_t eb = al256((tot ? tot : 1) * sizeof(drb_entry));
        if (ing_grow(st.ents, eb)) return DRB_EDEVICE;
        k_ing_decode<<<(unsigned)((nm + 255) / 256), 256, 0, sm>>>(
            ds, d_moff, d_mlen, d_ent0, d_nsc, dm, (drb_entry *)st.ents.p, nm,
            cmd_cap, st.ents.cap / sizeof(drb_entry), d_ctr, 0);
        HIPCHK(hipGetLastError());
        tr.mark("decode");
        // 5. planes: keys, a stable radix sort, one lane per plane
        k_ing_keys<<<(unsigned)((nm + 255) / 256), 256, 0, sm>>>(
            v, dm, kin, vin, nm, d_ctr);
        HIPCHK(hipGetLastError());
      }
      if (!spec_ok)
        HIPCHK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kin, kout, vin,
                                                  vout, (int)nm, 0, kbits, sm));
      k_ing_place<<<(unsigned)((nm + 255) / 256), 256, 0, sm>>>(
          v, ds, dm, (const drb_entry *)st.ents.p, kout, vout, nm,
          (uint32_t)(e->round & 1), (uint32_t)e->round, d_ctr, d_moff,
          d_mlen, d_cpu, d_cpu_n, nm, e->round);
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(rows, d_ctr, sizeof(rows), hipMemcpyDeviceToHost,
                            sm));
    }
    unsigned long long ncpu = 0;
    HIPCHK(hipMemcpyAsync(&ncpu, d_cpu_n, 8, hipMemcpyDeviceToHost, sm));
    HIPCHK(hipStreamSynchronize(sm));
    if (any_deliver)
      for (uint32_t q = 0; q < ING_TALLY_ROWS; ++q) {
        res.accepted += rows[q * 8];
        res.dropped += rows[q * 8 + 1];
        res.diverted += rows[q * 8 + 6];
      }
    if (ncpu) {
      st.cpu_msgs.resize(std::min<uint64_t>(ncpu, nm));
      HIPCHK(hipMemcpyAsync(st.cpu_msgs.data(), d_cpu,
                            st.cpu_msgs.size() * sizeof(drb_wire_cpu),
                            hipMemcpyDeviceToHost, sm));
      HIPCHK(hipStreamSynchronize(sm));
      std::sort(st.cpu_msgs.begin(), st.cpu_msgs.end(),
                [](const drb_wire_cpu &a, const drb_wire_cpu &b) {
                  return a.offset < b.offset;
                });
    }
  }
  tr.mark("place");
  if (out) *out = res;
  return DRB_OK;
}

extern "C" int drb_ingest_wire_cpu(drb_engine *e, drb_wire_cpu *out,
                                   size_t cap, size_t *n_out) {
  if (!e || (cap && !out)) return DRB_EINVAL;
  std::lock_guard<std::mutex> lock(e->ingest_mu);
  const size_t n = e->ingest ? e->ingest->cpu_msgs.size() : 0;
  if (n_out) *n_out = n;
  if (n > cap) return DRB_ERANGE;
  if (n) memcpy(out, e->ingest->cpu_msgs.data(), n * sizeof(drb_wire_cpu));
  return DRB_OK;
}
