/*
 * tan_oracle.c -- CPU restatement of the tan LogDB's write path: one
 * replica's log in the regular tan (one log per raft node,
 * internal/tan/logdb.go:103-109, the plugin/tan Factory).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 *   getCRC = uint32(xxhash.Sum64(b))   internal/tan/crc.go:21-23
 *   xxhash.Sum64  github.com/cespare/xxhash/v2 v2.1.2 (go.mod:5): XXH64
 *                 with seed 0.  The module is not in /root/reference; this
 *                 follows the published XXH64 algorithm and is pinned
 *                 against the python xxhash package (tests/test_oracle_tan.py)
 *   writer        internal/tan/record.go:414-653 (fillHeader :468-487,
 *                 writeBlock :491-497, writePending :501-511, getNext
 *                 :548-573, writeRecord :577-591, size :594-599,
 *                 lastRecordOffset :613-621, singleWriter.Write :628-653)
 *   reader        record.go:163-311 (nextChunk :203-295, next :300-311),
 *                 legacy chunks, no recovery -- what the tests read back
 *   Update.MarshalTo   raftpb/update.go:128-169 (empty Snapshot)
 *   State.MarshalTo    raftpb/state.go:27-42
 *   db.write           internal/tan/db.go:97-116, doWriteLocked :118-130,
 *                      stateSyncChange :88-90, makeRoomForWrite :175-180,
 *                      createNewLog open.go:171-198 (a new writer at
 *                      offset 0), MaxLogFileSize options.go:29
 *   nodeStates.getState / setState   internal/tan/node_states.go:44-59
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle_internal.h"

/* ---- XXH64 ----------------------------------------------------------- */
#define XP1 0x9E3779B185EBCA87ull
#define XP2 0xC2B2AE3D27D4EB4Full
#define XP3 0x165667B19E3779F9ull
#define XP4 0x85EBCA77C2B2AE63ull
#define XP5 0x27D4EB2F165667C5ull

static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t rd64(const uint8_t *p) {
  uint64_t x = 0;
  for (int k = 7; k >= 0; k--) x = (x << 8) | p[k];
  return x;
}
static uint32_t rd32(const uint8_t *p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 |
         (uint32_t)p[3] << 24;
}
static uint64_t xround(uint64_t acc, uint64_t in) {
  acc += in * XP2;
  acc = rotl64(acc, 31);
  return acc * XP1;
}
static uint64_t xmerge(uint64_t acc, uint64_t v) {
  acc ^= xround(0, v);
  return acc * XP1 + XP4;
}

uint64_t orc_xxh64(const uint8_t *p, size_t n) {
  const uint8_t *b = p;
  size_t left = n;
  uint64_t h;
  if (n >= 32) {
    uint64_t v1 = XP1 + XP2, v2 = XP2, v3 = 0, v4 = (uint64_t)0 - XP1;
    while (left >= 32) {
      v1 = xround(v1, rd64(b));
      v2 = xround(v2, rd64(b + 8));
      v3 = xround(v3, rd64(b + 16));
      v4 = xround(v4, rd64(b + 24));
      b += 32;
      left -= 32;
    }
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xmerge(h, v1);
    h = xmerge(h, v2);
    h = xmerge(h, v3);
    h = xmerge(h, v4);
  } else {
    h = XP5;
  }
  h += (uint64_t)n;
  while (left >= 8) {
    h ^= xround(0, rd64(b));
    h = rotl64(h, 27) * XP1 + XP4;
    b += 8;
    left -= 8;
  }
  if (left >= 4) {
    h ^= (uint64_t)rd32(b) * XP1;
    h = rotl64(h, 23) * XP2 + XP3;
    b += 4;
    left -= 4;
  }
  while (left > 0) {
    h ^= (uint64_t)(*b) * XP5;
    h = rotl64(h, 11) * XP1;
    b++;
    left--;
  }
  h ^= h >> 33;
  h *= XP2;
  h ^= h >> 29;
  h *= XP3;
  h ^= h >> 32;
  return h;
}

/* getCRC (crc.go:21-23) */
static uint32_t tan_crc(const uint8_t *p, size_t n) {
  return (uint32_t)orc_xxh64(p, n);
}

/* ---- record writer (record.go) ---------------------------------------- */
#define TAN_BLOCK 32768
#define TAN_HDR 7 /* legacyHeaderSize */
enum { FULL_CHUNK = 1, FIRST_CHUNK = 2, MIDDLE_CHUNK = 3, LAST_CHUNK = 4 };

typedef struct tan_file {
  uint8_t *p;
  size_t n, cap;
} tan_file;

static void file_write(tan_file *f, const uint8_t *p, size_t n) {
  if (f->n + n > f->cap) {
    size_t c = f->cap ? f->cap : 4096;
    while (c < f->n + n) c *= 2;
    f->p = (uint8_t *)realloc(f->p, c);
    f->cap = c;
  }
  memcpy(f->p + f->n, p, n);
  f->n += n;
}

struct orc_tanw {
  tan_file *f; /* the underlying io.Writer */
  int own;     /* f allocated by orc_tanw_new */
  int64_t block_number;
  int i, j, written;
  int first, pending;
  int64_t last_offset; /* -1: no record yet */
  int closed;
  uint8_t buf[TAN_BLOCK];
};

static void tw_init(orc_tanw *w, tan_file *f) {
  memset(w, 0, sizeof(*w));
  w->f = f;
  w->last_offset = -1;
}

/* fillHeader (record.go:468-487) */
static void tw_fill_header(orc_tanw *w, int last) {
  if (w->i + TAN_HDR > w->j || w->j > TAN_BLOCK)
    orc_panic("pebble/record: bad writer state");
  if (last)
    w->buf[w->i + 6] = w->first ? FULL_CHUNK : LAST_CHUNK;
  else
    w->buf[w->i + 6] = w->first ? FIRST_CHUNK : MIDDLE_CHUNK;
  const uint32_t c = tan_crc(w->buf + w->i + 6, (size_t)(w->j - w->i - 6));
  const uint32_t len = (uint32_t)(w->j - w->i - TAN_HDR);
  for (int k = 0; k < 4; k++) w->buf[w->i + k] = (uint8_t)(c >> (8 * k));
  w->buf[w->i + 4] = (uint8_t)len;
  w->buf[w->i + 5] = (uint8_t)(len >> 8);
}

/* writeBlock (record.go:491-497) */
static void tw_write_block(orc_tanw *w) {
  file_write(w->f, w->buf + w->written, (size_t)(TAN_BLOCK - w->written));
  w->i = 0;
  w->j = TAN_HDR;
  w->written = 0;
  w->block_number++;
}

/* writePending (record.go:501-511) */
static void tw_write_pending(orc_tanw *w) {
  if (w->pending) {
    tw_fill_header(w, 1);
    w->pending = 0;
  }
  file_write(w->f, w->buf + w->written, (size_t)(w->j - w->written));
  w->written = w->j;
}

/* getNext (record.go:548-573) */
static void tw_get_next(orc_tanw *w) {
  if (w->pending) tw_fill_header(w, 1);
  w->i = w->j;
  w->j = w->j + TAN_HDR;
  if (w->j > TAN_BLOCK) {
    for (int k = w->i; k < TAN_BLOCK; k++) w->buf[k] = 0;
    tw_write_block(w);
  }
  w->last_offset = w->block_number * TAN_BLOCK + w->i;
  w->first = 1;
  w->pending = 1;
}

/* singleWriter.Write (record.go:628-653) */
static void tw_write(orc_tanw *w, const uint8_t *p, size_t n) {
  while (n > 0) {
    if (w->j == TAN_BLOCK) {
      tw_fill_header(w, 0);
      tw_write_block(w);
      w->first = 0;
    }
    size_t k = (size_t)(TAN_BLOCK - w->j);
    if (k > n) k = n;
    memcpy(w->buf + w->j, p, k);
    w->j += (int)k;
    p += k;
    n -= k;
  }
}

/* writeRecord (record.go:577-591): the offset just past the record */
static int64_t tw_write_record(orc_tanw *w, const uint8_t *p, size_t n) {
  tw_get_next(w);
  tw_write(w, p, n);
  tw_write_pending(w);
  return w->block_number * TAN_BLOCK + w->j;
}

orc_tanw *orc_tanw_new(void) {
  orc_tanw *w = (orc_tanw *)malloc(sizeof(orc_tanw));
  tan_file *f = (tan_file *)calloc(1, sizeof(tan_file));
  tw_init(w, f);
  w->own = 1;
  return w;
}

void orc_tanw_free(orc_tanw *w) {
  if (!w) return;
  if (w->own) {
    free(w->f->p);
    free(w->f);
  }
  free(w);
}

int64_t orc_tanw_write_record(orc_tanw *w, const uint8_t *p, size_t n) {
  if (w->closed) return -1;
  ORC_TRY(-1);
  int64_t off = tw_write_record(w, p, n);
  ORC_END;
  return off;
}

/* flush (record.go:526-537) / close (:514-522) finish the pending record */
int orc_tanw_flush(orc_tanw *w, int close) {
  if (w->closed) return -1;
  ORC_TRY(-1);
  tw_write_pending(w);
  ORC_END;
  if (close) w->closed = 1;
  return 0;
}

/* size (record.go:594-599) */
int64_t orc_tanw_size(const orc_tanw *w) {
  return w->block_number * TAN_BLOCK + w->j;
}

/* lastRecordOffset (record.go:613-621): -1 ErrNoLastRecord */
int64_t orc_tanw_last_record_offset(const orc_tanw *w) {
  return w->last_offset;
}

/* the bytes written to the underlying io.Writer so far */
long orc_tanw_bytes(const orc_tanw *w, uint8_t *buf, size_t cap) {
  if (buf && cap >= w->f->n) memcpy(buf, w->f->p, w->f->n);
  return (long)w->f->n;
}

/* ---- record reader (record.go:163-311) --------------------------------- */
/* Reads the records of a log written from offset 0.  Returns the record
 * count, or ORC_TAN_ZEROED / ORC_TAN_INVALID / ORC_TAN_CRC /
 * ORC_TAN_UNEXPECTED_EOF (io.ErrUnexpectedEOF); offsets[k] = reader.offset()
 * before record k, lens[k] = its length, data gets the payloads back to
 * back (when cap allows). */
long orc_tan_read(const uint8_t *file, size_t size, int64_t *offsets,
                  size_t *lens, size_t max_recs, uint8_t *data,
                  size_t data_cap) {
  int64_t block_num = -1;
  size_t pos = 0; /* bytes of file consumed into blocks */
  const uint8_t *buf = NULL;
  int n = 0, begin = 0, end = 0, last = 0;
  long nrec = 0;
  size_t dn = 0;
  for (;;) {
    /* next (record.go:300-311): nextChunk(wantFirst = true) */
    const int64_t rec_off = block_num < 0 ? 0 : block_num * TAN_BLOCK + end;
    size_t rlen = 0;
    int want_first = 1;
    begin = end;
    for (;;) {
      /* nextChunk (record.go:203-295) */
      int got = 0;
      while (!got) {
        if (end + TAN_HDR <= n) {
          const uint32_t checksum = rd32(buf + end);
          const uint32_t length = (uint32_t)buf[end + 4] |
                                  (uint32_t)buf[end + 5] << 8;
          const uint8_t type = buf[end + 6];
          if (checksum == 0 && length == 0 && type == 0) {
            if (end + TAN_HDR + 4 > n) {
              end = n;  /* skip the rest of the block */
              continue;
            }
            return ORC_TAN_ZEROED;
          }
          if (type >= 5 && type <= 8) return ORC_TAN_INVALID; /* recyclable:
                                                  never written by tan */
          begin = end + TAN_HDR;
          end = begin + (int)length;
          if (end > n) return ORC_TAN_INVALID;
          if (checksum != tan_crc(buf + begin - 1, (size_t)(end - begin + 1)))
            return ORC_TAN_CRC;
          if (want_first && type != FULL_CHUNK && type != FIRST_CHUNK)
            continue;
          last = type == FULL_CHUNK || type == LAST_CHUNK;
          got = 1;
          break;
        }
        if (n < TAN_BLOCK && block_num >= 0) {
          if (!want_first || end != n) return ORC_TAN_INVALID;
          goto done; /* io.EOF */
        }
        /* io.ReadFull of the next block */
        if (pos >= size) {
          if (!want_first) return ORC_TAN_UNEXPECTED_EOF;
          goto done;
        }
        buf = file + pos;
        n = (int)(size - pos < TAN_BLOCK ? size - pos : TAN_BLOCK);
        pos += (size_t)n;
        begin = end = 0;
        block_num++;
      }
      /* singleReader.Read: this chunk's payload */
      const size_t k = (size_t)(end - begin);
      if (data && dn + k <= data_cap) memcpy(data + dn, buf + begin, k);
      dn += k;
      rlen += k;
      begin = end;
      if (last) break;
      want_first = 0;
    }
    if ((size_t)nrec < max_recs) {
      if (offsets) offsets[nrec] = rec_off;
      if (lens) lens[nrec] = rlen;
    }
    nrec++;
  }
done:
  return nrec;
}

/* ---- pb.Update as tan stores it (update.go:128-169) --------------------- */
static size_t put_uvarint(uint8_t *b, uint64_t x) {
  size_t i = 0;
  while (x >= 0x80) {
    b[i++] = (uint8_t)(x | 0x80);
    x >>= 7;
  }
  b[i++] = (uint8_t)x;
  return i;
}
static void put_le32(uint8_t *b, uint32_t x) {
  for (int k = 0; k < 4; k++) b[k] = (uint8_t)(x >> (8 * k));
}

/* State.MarshalTo (state.go:27-42) */
static size_t state_marshal(uint64_t term, uint64_t vote, uint64_t commit,
                            uint8_t *b) {
  size_t i = 0;
  b[i++] = 0x08;
  i += put_uvarint(b + i, term);
  b[i++] = 0x10;
  i += put_uvarint(b + i, vote);
  b[i++] = 0x18;
  i += put_uvarint(b + i, commit);
  return i;
}

/* Update.SizeUpperLimit-style bound of the marshalled form */
size_t orc_update_size_bound(const drb_entry *ents, size_t n) {
  size_t sz = 10 + 10 + 1 + 4 + 33 + 4 + 1;
  for (size_t i = 0; i < n; i++) sz += 4 + 64 + ents[i].cmd_len + 16;
  return sz;
}

/* Update.MarshalTo with an empty Snapshot; term = vote = commit = 0 is the
 * empty State (IsEmptyState, raftpb/raft.go:44-46) */
size_t orc_update_marshal(uint64_t shard, uint64_t replica, uint64_t term,
                          uint64_t vote, uint64_t commit,
                          const drb_entry *ents, size_t n,
                          const uint8_t *pool, uint8_t *buf) {
  size_t off = put_uvarint(buf, shard);
  off += put_uvarint(buf + off, replica);
  if (term == 0 && vote == 0 && commit == 0) {
    buf[off++] = 0;
  } else {
    buf[off++] = 1;
    const size_t k = state_marshal(term, vote, commit, buf + off + 4);
    put_le32(buf + off, (uint32_t)k);
    off += 4 + k;
  }
  put_le32(buf + off, (uint32_t)n);
  off += 4;
  for (size_t i = 0; i < n; i++) {
    const size_t k = orc_entry_marshal(&ents[i], pool, buf + off + 4);
    put_le32(buf + off, (uint32_t)k);
    off += 4 + k;
  }
  buf[off++] = 0; /* IsEmptySnapshot */
  return off;
}

/* ---- db (db.go): one replica's (regular) or many shards' (multiplexed) */
struct orc_tandb {
  orc_tanw w;
  tan_file *files; /* one per log created, in order */
  size_t nfiles;
  int64_t offset;      /* db.mu.offset */
  int64_t max_log;     /* MaxLogFileSize */
  /* nodeStates (db.go:108, 128): the last stored State per (shard,
   * replica) -- one node in the regular tan, the nodes of every shard
   * with the same key in the multiplexed one (db_keeper.go:84-123) */
  struct tan_node {
    uint64_t shard, replica, term, vote, commit;
  } *nodes;
  size_t nnodes;
  /* the last orc_tandb_write */
  int64_t last_off;   /* file offset its bytes start at */
  size_t last_len;    /* bytes it appended (zero padding included) */
  int last_sync, last_new_log;
};

/* createNewLog (open.go:171-198): a new log file and writer, offset 0 */
static void db_create_new_log(orc_tandb *db) {
  db->files = (tan_file *)realloc(db->files,
                                  (db->nfiles + 1) * sizeof(tan_file));
  memset(&db->files[db->nfiles], 0, sizeof(tan_file));
  db->nfiles++;
  /* files may have moved: the writer always targets the newest */
  tw_init(&db->w, &db->files[db->nfiles - 1]);
  db->offset = 0;
}

orc_tandb *orc_tandb_new(int64_t max_log_size) {
  orc_tandb *db = (orc_tandb *)calloc(1, sizeof(orc_tandb));
  db->max_log = max_log_size > 0 ? max_log_size : (int64_t)64 << 20;
  db_create_new_log(db);
  return db;
}

void orc_tandb_free(orc_tandb *db) {
  if (!db) return;
  for (size_t i = 0; i < db->nfiles; i++) free(db->files[i].p);
  free(db->files);
  free(db->nodes);
  free(db);
}

/* db.write (db.go:97-130) of one Update {shard, replica, State, ents}:
 * 1 written (sync in *sync), 0 nothing to write, -1 error */
int orc_tandb_write(orc_tandb *db, uint64_t shard, uint64_t replica,
                    uint64_t term, uint64_t vote, uint64_t commit,
                    const drb_entry *ents, size_t n, const uint8_t *pool,
                    int *sync) {
  db->last_len = 0;
  db->last_sync = 0;
  db->last_new_log = 0;
  db->last_off = db->offset;
  if (sync) *sync = 0;
  struct tan_node *nd = NULL;
  for (size_t k = 0; k < db->nnodes && !nd; k++)
    if (db->nodes[k].shard == shard && db->nodes[k].replica == replica)
      nd = &db->nodes[k];
  if (!nd) { /* getState of a node never written: the empty State */
    db->nodes = (struct tan_node *)realloc(
        db->nodes, (db->nnodes + 1) * sizeof(struct tan_node));
    nd = &db->nodes[db->nnodes++];
    memset(nd, 0, sizeof(*nd));
    nd->shard = shard;
    nd->replica = replica;
  }
  if (term == nd->term && vote == nd->vote && commit == nd->commit && n == 0)
    return 0;
  /* stateSyncChange (db.go:88-90) */
  const int s = n > 0 || term != nd->term || vote != nd->vote;
  uint8_t *buf = (uint8_t *)malloc(orc_update_size_bound(ents, n));
  const size_t len =
      orc_update_marshal(shard, replica, term, vote, commit, ents, n, pool, buf);
  ORC_TRY(-1);
  /* makeRoomForWrite (db.go:175-180) */
  if (db->offset >= db->max_log) {
    db_create_new_log(db);
    db->last_new_log = 1;
  }
  const size_t before = db->files[db->nfiles - 1].n;
  db->offset = tw_write_record(&db->w, buf, len);
  ORC_END;
  free(buf);
  db->last_off = (int64_t)before;
  db->last_len = db->files[db->nfiles - 1].n - before;
  nd->term = term;
  nd->vote = vote;
  nd->commit = commit;
  db->last_sync = s;
  if (sync) *sync = s;
  return 1;
}

/* the last write: out[0] file offset of its bytes, out[1] byte count,
 * out[2] sync, out[3] switched to a new log first, out[4] log number
 * (0 = the first log), out[5] db offset after it */
void orc_tandb_last(const orc_tandb *db, int64_t *out6) {
  out6[0] = db->last_off;
  out6[1] = (int64_t)db->last_len;
  out6[2] = db->last_sync;
  out6[3] = db->last_new_log;
  out6[4] = (int64_t)db->nfiles - 1;
  out6[5] = db->offset;
}

/* bytes [off, off + len) of log `log` (cap permitting); returns the log's
 * size or -1 */
long orc_tandb_file(const orc_tandb *db, size_t log, uint8_t *buf,
                    size_t cap) {
  if (log >= db->nfiles) return -1;
  const tan_file *f = &db->files[log];
  if (buf && cap >= f->n) memcpy(buf, f->p, f->n);
  return (long)f->n;
}
