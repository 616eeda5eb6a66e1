/*
 * codec_oracle.c -- CPU restatement of the raftpb codecs on this path.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 *   Entry colfer codec      raftpb/raft_optimized.go:77-656
 *   EntryBatch gogo codec   raftpb/entrybatch.go:25-146
 *   varint helpers          raftpb/common.go:11-30
 *   ConfigChange marshal    raftpb/configchange.go:28-71
 *   PBKV codec              internal/tests/kvpb/kv.go:26-283
 *   Message / MessageBatch  raftpb/message.go:32-124, messagebatch.go:23-70,
 *                           raft_optimized.go:659-1207
 *   TCP request framing     internal/transport/tcp.go:64-112,142-178
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

/* ---- pb.Message (raftpb/message.go:32-124) ---------------------------- */
/* the empty pb.Snapshot every fast-path message embeds
 * (snapshot.go:72-150: Filepath "", FileSize, Index, Term 0, Membership
 * {ConfigChangeId 0} (membership.go:29-148), Dummy, ShardID, Type,
 * Imported, OnDiskIndex, Witness all zero) */
static const uint8_t EMPTY_SNAPSHOT[24] = {
    0x12, 0x00, 0x18, 0x00, 0x20, 0x00, 0x28, 0x00, 0x32, 0x02, 0x08, 0x00,
    0x48, 0x00, 0x50, 0x00, 0x58, 0x00, 0x60, 0x00, 0x68, 0x00, 0x70, 0x00};

size_t orc_message_size(const drb_message *m, const drb_entry *ents) {
  size_t n = 0;
  n += 1 + sov(m->type) + 1 + sov(m->to) + 1 + sov(m->from);
  n += 1 + sov(m->shard_id) + 1 + sov(m->term) + 1 + sov(m->log_term);
  n += 1 + sov(m->log_index) + 1 + sov(m->commit) + 2 + 1 + sov(m->hint);
  for (uint64_t k = 0; k < m->n_entries; k++) {
    size_t l = orc_entry_size(&ents[m->entries_off + k]);
    n += 1 + l + sov(l);
  }
  n += 1 + sizeof(EMPTY_SNAPSHOT) + sov(sizeof(EMPTY_SNAPSHOT));
  n += 1 + sov(m->hint_high);
  return n;
}

size_t orc_message_marshal(const drb_message *m, const drb_entry *ents,
                           const uint8_t *pool, uint8_t *d) {
  size_t i = 0;
  d[i++] = 0x08;
  i = put_varint(d, i, m->type);
  d[i++] = 0x10;
  i = put_varint(d, i, m->to);
  d[i++] = 0x18;
  i = put_varint(d, i, m->from);
  d[i++] = 0x20;
  i = put_varint(d, i, m->shard_id);
  d[i++] = 0x28;
  i = put_varint(d, i, m->term);
  d[i++] = 0x30;
  i = put_varint(d, i, m->log_term);
  d[i++] = 0x38;
  i = put_varint(d, i, m->log_index);
  d[i++] = 0x40;
  i = put_varint(d, i, m->commit);
  d[i++] = 0x48;
  d[i++] = m->reject ? 1 : 0;
  d[i++] = 0x50;
  i = put_varint(d, i, m->hint);
  for (uint64_t k = 0; k < m->n_entries; k++) {
    const drb_entry *e = &ents[m->entries_off + k];
    d[i++] = 0x5a;
    i = put_varint(d, i, orc_entry_size(e));
    i += orc_entry_marshal(e, pool, d + i);
  }
  d[i++] = 0x62;
  i = put_varint(d, i, sizeof(EMPTY_SNAPSHOT));
  memcpy(d + i, EMPTY_SNAPSHOT, sizeof(EMPTY_SNAPSHOT));
  i += sizeof(EMPTY_SNAPSHOT);
  d[i++] = 0x68;
  i = put_varint(d, i, m->hint_high);
  return i;
}

/* Message.Unmarshal (raft_optimized.go:659-983): varint fields 1-10 and 13,
 * Entries (11, colfer Entry), Snapshot (12, must be the empty one here:
 * returns -2 for any other).  Entries go to ents[*n_ents...], Cmds to
 * pool. */
long orc_message_unmarshal(const uint8_t *d, size_t n, drb_message *m,
                           drb_entry *ents, size_t ent_cap, size_t *n_ents,
                           uint8_t *pool, size_t pool_cap, size_t *pool_used) {
  size_t i = 0;
  memset(m, 0, sizeof(*m));
  m->entries_off = *n_ents;
  while (i < n) {
    size_t pre = i;
    uint64_t wire, v;
    if (get_varint(d, n, &i, &wire)) return -1;
    uint64_t field = wire >> 3;
    int wt = (int)(wire & 7);
    if (wt == 4 || field == 0) return -1;
    if ((field >= 1 && field <= 10) || field == 13) {
      if (wt != 0) return -1;
      if (get_varint(d, n, &i, &v)) return -1;
      switch (field) {
        case 1: m->type = (uint32_t)v; break;
        case 2: m->to = v; break;
        case 3: m->from = v; break;
        case 4: m->shard_id = v; break;
        case 5: m->term = v; break;
        case 6: m->log_term = v; break;
        case 7: m->log_index = v; break;
        case 8: m->commit = v; break;
        case 9: m->reject = v != 0; break;
        case 10: m->hint = v; break;
        default: m->hint_high = v; break;
      }
    } else if (field == 11 || field == 12) {
      if (wt != 2) return -1;
      uint64_t l;
      if (get_varint(d, n, &i, &l)) return -1;
      if (i + l > n) return -1;
      if (field == 11) {
        if (*n_ents >= ent_cap) return -1;
        if (orc_entry_unmarshal(d + i, (size_t)l, &ents[*n_ents], pool,
                                pool_cap, pool_used) < 0)
          return -1;
        (*n_ents)++;
        m->n_entries++;
      } else if (l != sizeof(EMPTY_SNAPSHOT) ||
                 memcmp(d + i, EMPTY_SNAPSHOT, sizeof(EMPTY_SNAPSHOT))) {
        return -2;
      }
      i += (size_t)l;
    } else {
      i = pre;
      if (skip_field(d, n, &i)) return -1;
    }
  }
  return (long)i;
}

/* ---- pb.MessageBatch (raftpb/messagebatch.go:23-70) ------------------- */
size_t orc_messagebatch_marshal(const drb_message *ms, size_t n,
                                const drb_entry *ents, const uint8_t *pool,
                                uint64_t deployment_id, const char *src,
                                size_t src_len, uint32_t bin_ver,
                                uint8_t *d) {
  size_t i = 0;
  for (size_t k = 0; k < n; k++) {
    d[i++] = 0x0a;
    i = put_varint(d, i, orc_message_size(&ms[k], ents));
    i += orc_message_marshal(&ms[k], ents, pool, d + i);
  }
  d[i++] = 0x10;
  i = put_varint(d, i, deployment_id);
  d[i++] = 0x1a;
  i = put_varint(d, i, src_len);
  memcpy(d + i, src, src_len);
  i += src_len;
  d[i++] = 0x20;
  i = put_varint(d, i, bin_ver);
  return i;
}

/* MessageBatch.Unmarshal (raft_optimized.go:1056-1207).  Returns the
 * message count, -1 on a malformed batch, -2 on a non-empty Snapshot. */
long orc_messagebatch_unmarshal(const uint8_t *d, size_t n, drb_message *ms,
                                size_t cap, drb_entry *ents, size_t ent_cap,
                                uint8_t *pool, size_t pool_cap,
                                uint64_t *deployment_id, uint32_t *bin_ver,
                                char *src, size_t src_cap, size_t *src_len) {
  size_t i = 0, cnt = 0, ne = 0, pu = 0;
  *deployment_id = 0;
  *bin_ver = 0;
  *src_len = 0;
  while (i < n) {
    size_t pre = i;
    uint64_t wire, v;
    if (get_varint(d, n, &i, &wire)) return -1;
    uint64_t field = wire >> 3;
    int wt = (int)(wire & 7);
    if (wt == 4 || field == 0) return -1;
    if (field == 1 || field == 3) {
      if (wt != 2) return -1;
      uint64_t l;
      if (get_varint(d, n, &i, &l)) return -1;
      if (i + l > n) return -1;
      if (field == 1) {
        if (cnt >= cap) return -1;
        long rc = orc_message_unmarshal(d + i, (size_t)l, &ms[cnt], ents,
                                        ent_cap, &ne, pool, pool_cap, &pu);
        if (rc < 0) return rc;
        cnt++;
      } else {
        if (l > src_cap) return -1;
        memcpy(src, d + i, (size_t)l);
        *src_len = (size_t)l;
      }
      i += (size_t)l;
    } else if (field == 2 || field == 4) {
      if (wt != 0) return -1;
      if (get_varint(d, n, &i, &v)) return -1;
      if (field == 2)
        *deployment_id = v;
      else
        *bin_ver = (uint32_t)v;
    } else {
      i = pre;
      if (skip_field(d, n, &i)) return -1;
    }
  }
  return (long)cnt;
}

/* ---- TCP framing (internal/transport/tcp.go:64-112,142-178) ----------- */
/* requestHeader.encode: method BE16, size BE64, header CRC BE32 (over the
 * 18 bytes with this field zero), payload CRC BE32 */
void orc_request_header_encode(uint16_t method, uint64_t size, uint32_t crc,
                               uint8_t *b) {
  b[0] = (uint8_t)(method >> 8);
  b[1] = (uint8_t)method;
  for (int k = 0; k < 8; k++) b[2 + k] = (uint8_t)(size >> (56 - 8 * k));
  memset(b + 10, 0, 4);
  for (int k = 0; k < 4; k++) b[14 + k] = (uint8_t)(crc >> (24 - 8 * k));
  uint32_t h = orc_crc32_ieee(b, 18);
  for (int k = 0; k < 4; k++) b[10 + k] = (uint8_t)(h >> (24 - 8 * k));
}

/* requestHeader.decode: 0 when the header CRC matches and the method is
 * raftType (100) or snapshotType (200) */
int orc_request_header_decode(const uint8_t *b, uint16_t *method,
                              uint64_t *size, uint32_t *crc) {
  uint8_t t[18];
  memcpy(t, b, 18);
  uint32_t in = ((uint32_t)t[10] << 24) | ((uint32_t)t[11] << 16) |
                ((uint32_t)t[12] << 8) | t[13];
  memset(t + 10, 0, 4);
  if (orc_crc32_ieee(t, 18) != in) return -1;
  uint16_t me = (uint16_t)((t[0] << 8) | t[1]);
  if (me != 100 && me != 200) return -1;
  uint64_t s = 0;
  for (int k = 0; k < 8; k++) s = (s << 8) | t[2 + k];
  uint32_t c = 0;
  for (int k = 0; k < 4; k++) c = (c << 8) | t[14 + k];
  *method = me;
  *size = s;
  *crc = c;
  return 0;
}

/* writeMessage (tcp.go:142-178): magic {0xAE, 0x7D} || header || payload */
size_t orc_wire_frame(const uint8_t *payload, size_t n, uint8_t *out) {
  out[0] = 0xAE;
  out[1] = 0x7D;
  orc_request_header_encode(100, n, orc_crc32_ieee(payload, n), out + 2);
  memcpy(out + 20, payload, n);
  return n + 20;
}
