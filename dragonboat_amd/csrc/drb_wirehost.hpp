// drb_wirehost.hpp -- the host's part of drb_ingest_wire (drb_ingest.hpp):
// plain C++ with no HIP dependency, so that tests/test_wirehost.py builds it
// with AddressSanitizer and UBSan and runs streams through it on the CPU.
//
//   tcp.go readMessage (:180-237)     walk_frames: the 2-byte magic, the
//                                     18-byte requestHeader (method, size,
//                                     header CRC32, payload CRC32) and its
//                                     CRC; a bad header stops the stream
//   MessageBatch.Unmarshal            scan_batch: the batch's top-level
//     (raft_optimized.go:1056-1207)   fields -- where each Requests element
//                                     starts (as the distance from the
//                                     previous one), DeploymentId, BinVer
//   the element steps' upload         pack_steps16: 2 B per step when every
//                                     element is under 64 KB
//   hash/crc32 + zlib's crc32_combine the payload CRC folded from 16 KB
//                                     chunk CRCs (the GPU computes those)
#pragma once

#include <stdint.h>
#include <string.h>

#include <mutex>
#include <vector>

namespace wirehost {

constexpr uint32_t POLY = 0xEDB88320u;  // CRC-32/IEEE, reflected

// a * b mod P over GF(2), reflected (zlib's multmodp)
static inline uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = b & 1 ? (b >> 1) ^ POLY : b >> 1;
  }
  return p;
}

static uint32_t crc_tab[256];
static uint32_t x2n[32];  // x^(2^k) mod P (zlib x2n_table)
// the shift over one 16 KB payload chunk, multmodp(x^(8 * 16384), a), as
// four byte tables (the operator is linear in a): a chunk's CRC folds into
// its frame's in four lookups instead of two multmodp loops
static uint32_t sh16k[4][256];
static std::once_flag crc_once;

static void crc_build() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? POLY ^ (c >> 1) : c >> 1;
    crc_tab[i] = c;
  }
  uint32_t p = 1u << 30;  // x^1
  x2n[0] = p;
  for (int n = 1; n < 32; ++n) x2n[n] = p = multmodp(p, p);
  uint32_t op = 1u << 31;  // x^0, then x^(8 * 16384)
  uint32_t k = 3;
  for (uint64_t n = 16384; n; n >>= 1, ++k)
    if (n & 1) op = multmodp(x2n[k & 31], op);
  for (int b = 0; b < 4; ++b)
    for (uint32_t v = 0; v < 256; ++v)
      sh16k[b][v] = multmodp(op, v << (8 * b));
}
// thread-safe: transport threads may call drb_ingest_wire concurrently
static void crc_init() { std::call_once(crc_once, crc_build); }

static uint32_t crc32_small(const uint8_t *p, size_t n) {
  uint32_t c = 0xffffffffu;
  while (n--) c = crc_tab[(c ^ *p++) & 0xff] ^ (c >> 8);
  return c ^ 0xffffffffu;
}

// crc32_combine(a, b, len_b) (zlib): CRC(A|B) from CRC(A), CRC(B), |B|
static uint32_t crc32_combine(uint32_t a, uint32_t b, uint64_t len_b) {
  uint32_t p = 1u << 31;  // x^0
  uint32_t k = 3;         // 8 * len_b = len_b * 2^3
  for (uint64_t n = len_b; n; n >>= 1, ++k)
    if (n & 1) p = multmodp(x2n[k & 31], p);
  return multmodp(p, a) ^ b;
}

// crc32_combine(a, b, 16384)
static inline uint32_t crc32_combine16k(uint32_t a, uint32_t b) {
  return sh16k[0][a & 0xff] ^ sh16k[1][(a >> 8) & 0xff] ^
         sh16k[2][(a >> 16) & 0xff] ^ sh16k[3][a >> 24] ^ b;
}

// the raw CRC of a chunk as the GPU's k_crc_chunks leaves it: init 0, no
// final xor (linear over GF(2)); the host folds a frame's chunks and
// applies the ~0 conditioning once: CRC(M) = f(M) ^ (~0 * x^(8|M|)) ^ ~0
static uint32_t crc_raw(const uint8_t *p, size_t n) {
  uint32_t c = 0;
  while (n--) c = crc_tab[(c ^ *p++) & 0xff] ^ (c >> 8);
  return c;
}
static uint32_t fold_frame_crc(const uint32_t *chunk_raw, const uint32_t *len,
                               size_t n, uint64_t frame_size) {
  uint32_t c = 0;
  for (size_t k = 0; k < n; ++k)
    c = len[k] == 16384 ? crc32_combine16k(c, chunk_raw[k])
                        : crc32_combine(c, chunk_raw[k], len[k]);
  return c ^ crc32_combine(0xffffffffu, 0, frame_size) ^ 0xffffffffu;
}

static uint64_t be(const uint8_t *p, int n) {
  uint64_t x = 0;
  for (int k = 0; k < n; ++k) x = (x << 8) | p[k];
  return x;
}

static bool varint(const uint8_t *d, size_t n, size_t &i, uint64_t &v) {
  v = 0;
  for (unsigned s = 0; s < 70; s += 7) {
    if (i >= n) return false;
    const uint8_t b = d[i++];
    v |= (uint64_t)(b & 0x7f) << s;
    if (b < 0x80) return true;
  }
  return false;
}

static bool skip(const uint8_t *d, size_t n, size_t &i, uint64_t wire) {
  uint64_t x;
  switch (wire & 7) {
    case 0: return varint(d, n, i, x);
    case 1:
      if (n - i < 8) return false;
      i += 8;
      return true;
    case 2:
      if (!varint(d, n, i, x) || x > n - i) return false;
      i += (size_t)x;
      return true;
    case 5:
      if (n - i < 4) return false;
      i += 4;
      return true;
    default: return false;
  }
}

struct Frame {
  uint64_t off;   // payload offset in the stream
  uint64_t size;  // payload bytes
  uint32_t method, pcrc;
  bool scan_ok = true;
  uint64_t did = 0, bv = 0;
  // Requests elements: where each element's tag starts, as the distance
  // from the previous element's tag (the first: from the payload start);
  // the GPU rebuilds offsets and lengths from these (k_ing_elems), so 2-4 B
  // per message cross the link instead of a u64 offset and a u32 length
  std::vector<uint32_t> step;
};

// the whole frames of a stream (tcp.go:64-112, 180-237), reusing fr's
// vectors (a warm call neither faults nor frees); returns the bytes of the
// whole frames, *bad set when a header is malformed or its CRC fails (the
// frames before it are kept: ErrBadMessage closes the connection there).
// A stream that ends inside a frame whose bytes so far are sound -- the
// magic's first bytes, or a whole header whose payload has not all arrived
// -- is not bad: readMessage would still be waiting for the rest
// (io.ReadFull), so the walk stops before it and the transport hands those
// bytes in again with what follows.
static size_t walk_frames(const uint8_t *stream, size_t len,
                          std::vector<Frame> &fr, bool *bad) {
  size_t nfr = 0, i = 0;
  *bad = false;
  while (i < len) {
    if (len - i < 20) {  // a header still arriving, if its magic is sound
      *bad = stream[i] != 0xAE || (len - i > 1 && stream[i + 1] != 0x7D);
      break;
    }
    if (stream[i] != 0xAE || stream[i + 1] != 0x7D) {
      *bad = true;
      break;
    }
    uint8_t h[18];
    memcpy(h, stream + i + 2, 18);
    const uint32_t hcrc = (uint32_t)be(h + 10, 4);
    memset(h + 10, 0, 4);
    const uint32_t method = (uint32_t)be(h, 2);
    const uint64_t size = be(h + 2, 8);
    if (crc32_small(h, 18) != hcrc || (method != 100 && method != 200) ||
        size == 0) {
      *bad = true;
      break;
    }
    if (size > len - i - 20) break;  // its payload still arriving
    if (nfr == fr.size()) fr.emplace_back();
    Frame &f = fr[nfr++];
    f.off = i + 20;
    f.size = size;
    f.method = method;
    f.pcrc = (uint32_t)be(h + 14, 4);
    f.scan_ok = true;
    f.did = f.bv = 0;
    f.step.clear();
    i += 20 + (size_t)size;
  }
  fr.resize(nfr);
  return i;
}

// MessageBatch.Unmarshal's top-level walk (raft_optimized.go:1056-1207):
// where each Requests element (field 1) lies; DeploymentId, BinVer
static void scan_batch(const uint8_t *stream, Frame &f) {
  const uint8_t *p = stream + f.off;
  const size_t n = (size_t)f.size;
  size_t j = 0, prev = 0;
  f.step.reserve(n / 32);
  while (j < n) {
    uint64_t wire, v;
    // the common element: tag 0x0a and a one- or two-byte length
    if (p[j] == 0x0a && n - j >= 3) {
      uint32_t l = p[j + 1];
      size_t h = 2;
      if (l >= 0x80) {
        l = (l & 0x7f) | ((uint32_t)p[j + 2] << 7);
        h = 3;
      }
      if (l < (1u << 14) && l <= n - j - h) {
        f.step.push_back((uint32_t)(j - prev));
        prev = j;
        j += h + l;
        continue;
      }
    }
    const size_t tag_at = j;
    if (!varint(p, n, j, wire) || (wire >> 3) == 0) {
      f.scan_ok = false;
      return;
    }
    const uint64_t field = wire >> 3;
    if (field == 1) {
      uint64_t l;
      if ((wire & 7) != 2 || !varint(p, n, j, l) || l > n - j) {
        f.scan_ok = false;
        return;
      }
      if (l > 0xffffffffull || tag_at - prev > 0xffffffffull) {
        f.scan_ok = false;
        return;
      }
      f.step.push_back((uint32_t)(tag_at - prev));
      prev = tag_at;
      j += (size_t)l;
    } else if (field == 2 || field == 4) {
      if ((wire & 7) != 0 || !varint(p, n, j, v)) {
        f.scan_ok = false;
        return;
      }
      (field == 2 ? f.did : f.bv) = v;
    } else if (!skip(p, n, j, wire)) {
      f.scan_ok = false;
      return;
    }
  }
}

// one frame's steps as 2 B each; false (the caller uploads 4 B steps) when
// one does not fit
static bool pack_steps16(const Frame &f, uint16_t *out) {
  uint32_t any = 0;
  const uint32_t *a = f.step.data();
  for (size_t k = 0, n = f.step.size(); k < n; ++k) {
    any |= a[k];
    out[k] = (uint16_t)a[k];
  }
  return (any >> 16) == 0;
}

}  // namespace wirehost
