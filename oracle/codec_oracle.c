/*
 * codec_oracle.c -- CPU restatement of the raftpb codecs on this path.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 *   Entry colfer codec      raftpb/raft_optimized.go:77-656
 *   EntryBatch gogo codec   raftpb/entrybatch.go:25-146
 *   varint helpers          raftpb/common.go:11-30
 *   ConfigChange marshal    raftpb/configchange.go:28-71
 *   PBKV codec              internal/tests/kvpb/kv.go:26-283
 *   CRC32-IEEE              Go hash/crc32 ChecksumIEEE (stdlib, go 1.23),
 *                           used at internal/transport/tcp.go:87,98,146,232
 */
#include <stdio.h>
#include <string.h>

#include "oracle_internal.h"

#define COLFER_SIZE_MAX (8ull * 1024 * 1024 * 1024 * 1024)

/* ---- Entry.Size (raft_optimized.go:84-158) ---------------------------- */
static size_t u64_field_size(uint64_t x) {
  if (x >= (1ull << 49)) return 9;
  if (x == 0) return 0;
  size_t l = 2;
  for (; x >= 0x80; l++) x >>= 7;
  return l;
}

size_t orc_entry_size(const drb_entry *e) {
  size_t l = 1;
  l += u64_field_size(e->term);
  l += u64_field_size(e->index);
  if (e->type != 0) {
    uint32_t x = e->type; /* EntryType is int32; values here are >= 0 */
    size_t k = 2;
    for (; x >= 0x80; k++) x >>= 7;
    l += k;
  }
  l += u64_field_size(e->key);
  l += u64_field_size(e->client_id);
  l += u64_field_size(e->series_id);
  l += u64_field_size(e->responded_to);
  if (e->cmd_len != 0) {
    uint64_t x = e->cmd_len;
    l += x + 2;
    for (; x >= 0x80; l++) x >>= 7;
  }
  return l;
}

/* ---- Entry.marshalTo (raft_optimized.go:166-300) ---------------------- */
static size_t put_u64_field(uint8_t *buf, size_t i, uint8_t tag, uint64_t x) {
  if (x >= (1ull << 49)) {
    buf[i] = tag | 0x80;
    for (int k = 0; k < 8; k++) buf[i + 1 + k] = (uint8_t)(x >> (56 - 8 * k));
    return i + 9;
  }
  if (x != 0) {
    buf[i++] = tag;
    while (x >= 0x80) {
      buf[i++] = (uint8_t)(x | 0x80);
      x >>= 7;
    }
    buf[i++] = (uint8_t)x;
  }
  return i;
}

size_t orc_entry_marshal(const drb_entry *e, const uint8_t *pool,
                         uint8_t *buf) {
  size_t i = 0;
  i = put_u64_field(buf, i, 0, e->term);
  i = put_u64_field(buf, i, 1, e->index);
  if (e->type != 0) {
    uint32_t x = e->type;
    buf[i++] = 2;
    while (x >= 0x80) {
      buf[i++] = (uint8_t)(x | 0x80);
      x >>= 7;
    }
    buf[i++] = (uint8_t)x;
  }
  i = put_u64_field(buf, i, 3, e->key);
  i = put_u64_field(buf, i, 4, e->client_id);
  i = put_u64_field(buf, i, 5, e->series_id);
  i = put_u64_field(buf, i, 6, e->responded_to);
  if (e->cmd_len != 0) {
    buf[i++] = 7;
    uint64_t x = e->cmd_len;
    while (x >= 0x80) {
      buf[i++] = (uint8_t)(x | 0x80);
      x >>= 7;
    }
    buf[i++] = (uint8_t)x;
    memcpy(buf + i, pool + e->cmd_off, e->cmd_len);
    i += e->cmd_len;
  }
  buf[i++] = 0x7f;
  return i;
}

/* ---- Entry.unmarshal (raft_optimized.go:308-656) ---------------------- */
/* u64 field: 7-bit groups, the 9th byte (shift 56) taken whole. */
static int get_u64_field(const uint8_t *d, size_t n, size_t *pi, uint8_t *hdr,
                         uint8_t tag, uint64_t *out) {
  size_t i = *pi;
  if (*hdr == tag) {
    size_t start = i;
    i++;
    if (i >= n) return -1;
    uint64_t x = d[start];
    if (x >= 0x80) {
      x &= 0x7f;
      for (unsigned shift = 7;; shift += 7) {
        uint64_t b = d[i];
        i++;
        if (i >= n) return -1;
        if (b < 0x80 || shift == 56) {
          x |= b << shift;
          break;
        }
        x |= (b & 0x7f) << shift;
      }
    }
    *out = x;
    *hdr = d[i];
    i++;
  } else if (*hdr == (tag | 0x80)) {
    size_t start = i;
    i += 8;
    if (i >= n) return -1;
    uint64_t x = 0;
    for (int k = 0; k < 8; k++) x = (x << 8) | d[start + k];
    *out = x;
    *hdr = d[i];
    i++;
  }
  *pi = i;
  return 0;
}

long orc_entry_unmarshal(const uint8_t *d, size_t n, drb_entry *e,
                         uint8_t *pool, size_t pool_cap, size_t *pool_used) {
  memset(e, 0, sizeof(*e));
  if (n == 0) return -1;
  uint8_t hdr = d[0];
  size_t i = 1;
  if (get_u64_field(d, n, &i, &hdr, 0, &e->term)) return -1;
  if (get_u64_field(d, n, &i, &hdr, 1, &e->index)) return -1;
  if (hdr == 2 || hdr == (2 | 0x80)) {
    int neg = (hdr & 0x80) != 0;
    if (i + 1 >= n) return -1;
    uint32_t x = d[i];
    i++;
    if (x >= 0x80) {
      x &= 0x7f;
      for (unsigned shift = 7;; shift += 7) {
        uint32_t b = d[i];
        i++;
        if (i >= n) return -1;
        if (b < 0x80) {
          x |= b << shift;
          break;
        }
        x |= (b & 0x7f) << shift;
      }
    }
    e->type = neg ? (~x + 1) : x;
    hdr = d[i];
    i++;
  }
  if (get_u64_field(d, n, &i, &hdr, 3, &e->key)) return -1;
  if (get_u64_field(d, n, &i, &hdr, 4, &e->client_id)) return -1;
  if (get_u64_field(d, n, &i, &hdr, 5, &e->series_id)) return -1;
  if (get_u64_field(d, n, &i, &hdr, 6, &e->responded_to)) return -1;
  if (hdr == 7) {
    if (i >= n) return -1;
    uint64_t x = d[i];
    i++;
    if (x >= 0x80) {
      x &= 0x7f;
      for (unsigned shift = 7;; shift += 7) {
        if (i >= n) return -1;
        uint64_t b = d[i];
        i++;
        if (b < 0x80) {
          x |= b << shift;
          break;
        }
        x |= (b & 0x7f) << shift;
      }
    }
    if (x > COLFER_SIZE_MAX) return -1;
    size_t start = i;
    i += (size_t)x;
    if (i >= n) return -1;
    if (*pool_used + x > pool_cap) return -1;
    memcpy(pool + *pool_used, d + start, (size_t)x);
    e->cmd_off = *pool_used;
    e->cmd_len = (uint32_t)x;
    *pool_used += (size_t)x;
    hdr = d[i];
    i++;
  }
  if (hdr != 0x7f) return -1;
  return (long)i;
}

/* ---- varints (common.go:11-30) ---------------------------------------- */
static size_t put_varint(uint8_t *d, size_t off, uint64_t v) {
  while (v >= 0x80) {
    d[off++] = (uint8_t)((v & 0x7f) | 0x80);
    v >>= 7;
  }
  d[off++] = (uint8_t)v;
  return off;
}

static size_t sov(uint64_t x) {
  size_t n = 0;
  do {
    n++;
    x >>= 7;
  } while (x);
  return n;
}

static int get_varint(const uint8_t *d, size_t n, size_t *pi, uint64_t *v) {
  uint64_t x = 0;
  for (unsigned shift = 0;; shift += 7) {
    if (shift >= 64) return -1;
    if (*pi >= n) return -1;
    uint8_t b = d[(*pi)++];
    x |= (uint64_t)(b & 0x7f) << shift;
    if (b < 0x80) break;
  }
  *v = x;
  return 0;
}

/* ---- EntryBatch (entrybatch.go:25-58) --------------------------------- */
size_t orc_entrybatch_size(const drb_entry *e, size_t n) {
  size_t s = 0;
  for (size_t i = 0; i < n; i++) {
    size_t l = orc_entry_size(&e[i]);
    s += 1 + l + sov(l);
  }
  return s;
}

size_t orc_entrybatch_marshal(const drb_entry *e, size_t n,
                              const uint8_t *pool, uint8_t *buf) {
  size_t i = 0;
  for (size_t k = 0; k < n; k++) {
    buf[i++] = 0x0a;
    i = put_varint(buf, i, orc_entry_size(&e[k]));
    i += orc_entry_marshal(&e[k], pool, buf + i);
  }
  return i;
}

/* skipRaft (common.go:37-117) for wire types 0,1,2,5 */
static int skip_field(const uint8_t *d, size_t n, size_t *pi) {
  uint64_t wire;
  if (get_varint(d, n, pi, &wire)) return -1;
  switch (wire & 7) {
    case 0: {
      uint64_t v;
      return get_varint(d, n, pi, &v);
    }
    case 1:
      *pi += 8;
      return *pi > n ? -1 : 0;
    case 2: {
      uint64_t l;
      if (get_varint(d, n, pi, &l)) return -1;
      *pi += (size_t)l;
      return *pi > n ? -1 : 0;
    }
    case 5:
      *pi += 4;
      return *pi > n ? -1 : 0;
    default:
      return -1;
  }
}

/* EntryBatch.Unmarshal (entrybatch.go:60-146) */
long orc_entrybatch_unmarshal(const uint8_t *d, size_t n, drb_entry *out,
                              size_t cap, uint8_t *pool, size_t pool_cap) {
  size_t i = 0, cnt = 0, pu = 0;
  while (i < n) {
    size_t pre = i;
    uint64_t wire;
    if (get_varint(d, n, &i, &wire)) return -1;
    uint64_t field = wire >> 3;
    int wt = (int)(wire & 7);
    if (wt == 4 || field == 0) return -1;
    if (field == 1) {
      if (wt != 2) return -1;
      uint64_t ml;
      if (get_varint(d, n, &i, &ml)) return -1;
      size_t post = i + (size_t)ml;
      if (post > n) return -1;
      if (cnt >= cap) return -1;
      if (orc_entry_unmarshal(d + i, (size_t)ml, &out[cnt], pool, pool_cap,
                              &pu) < 0)
        return -1;
      cnt++;
      i = post;
    } else {
      i = pre;
      if (skip_field(d, n, &i)) return -1;
    }
  }
  return (long)cnt;
}

/* ---- ConfigChange.MarshalTo (configchange.go:28-56) ------------------- */
size_t orc_configchange_marshal_addnode(uint64_t replica_id,
                                        const char *address, uint8_t *buf) {
  size_t i = 0;
  size_t al = strlen(address);
  buf[i++] = 0x08;
  i = put_varint(buf, i, 0); /* ConfigChangeId */
  buf[i++] = 0x10;
  i = put_varint(buf, i, 0); /* Type = AddNode */
  buf[i++] = 0x18;
  i = put_varint(buf, i, replica_id);
  buf[i++] = 0x22;
  i = put_varint(buf, i, al);
  memcpy(buf + i, address, al);
  i += al;
  buf[i++] = 0x28;
  buf[i++] = 1; /* Initialize (bootstrap, peer.go:412-417) */
  return i;
}

/* ---- PBKV (internal/tests/kvpb/kv.go) --------------------------------- */
size_t orc_pbkv_marshal(const uint8_t *key, uint32_t klen, const uint8_t *val,
                        uint32_t vlen, uint8_t *buf) {
  size_t i = 0;
  buf[i++] = 0x0a;
  i = put_varint(buf, i, klen);
  memcpy(buf + i, key, klen);
  i += klen;
  buf[i++] = 0x12;
  i = put_varint(buf, i, vlen);
  memcpy(buf + i, val, vlen);
  i += vlen;
  return i;
}

/* PBKV.Unmarshal (kv.go:76-283) for a message with fields 1 and 2; later
 * occurrences overwrite earlier ones, unknown fields are skipped.  Returns
 * -1 on a decode error (KVTest.Update panics on it, kvtest.go:155-157). */
int orc_pbkv_unmarshal(const uint8_t *d, size_t n, const uint8_t **key,
                       uint32_t *klen, const uint8_t **val, uint32_t *vlen) {
  size_t i = 0;
  *key = d;
  *klen = 0;
  *val = d;
  *vlen = 0;
  while (i < n) {
    size_t pre = i;
    uint64_t wire;
    if (get_varint(d, n, &i, &wire)) return -1;
    uint64_t field = wire >> 3;
    int wt = (int)(wire & 7);
    if (wt == 4 || field == 0) return -1;
    if (field == 1 || field == 2) {
      if (wt != 2) return -1;
      uint64_t l;
      if (get_varint(d, n, &i, &l)) return -1;
      size_t post = i + (size_t)l;
      if (post > n) return -1;
      if (field == 1) {
        *key = d + i;
        *klen = (uint32_t)l;
      } else {
        *val = d + i;
        *vlen = (uint32_t)l;
      }
      i = post;
    } else {
      i = pre;
      if (skip_field(d, n, &i)) return -1;
    }
  }
  return 0;
}

/* ---- CRC32-IEEE (reflected polynomial 0xEDB88320) --------------------- */
static uint32_t crc_table[256];
static int crc_init_done;

static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (0xEDB88320u ^ (c >> 1)) : (c >> 1);
    crc_table[i] = c;
  }
  crc_init_done = 1;
}

uint32_t orc_crc32_ieee(const uint8_t *p, size_t n) {
  if (!crc_init_done) crc_init();
  uint32_t c = 0xffffffffu;
  for (size_t i = 0; i < n; i++) c = crc_table[(c ^ p[i]) & 0xff] ^ (c >> 8);
  return c ^ 0xffffffffu;
}
