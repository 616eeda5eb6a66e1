/*
 * logdb_oracle.c -- CPU restatement of the batched LogDB record path for
 * EntriesToSave.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 *   getBatchID                    internal/logdb/batch.go:64-66
 *   getBatchIDRange               batch.go:76-83
 *   restoreBatchFields            batch.go:86-98
 *   compactBatchFields            batch.go:100-113
 *   getMergedFirstBatch           batch.go:115-141
 *   batchedEntries.recordBatch    batch.go:288-314
 *   batchedEntries.record         batch.go:316-346
 *   batchedEntries.getLastBatch   batch.go:369-380
 *   batchedEntries.getMergedFirstBatch (method)  batch.go:382-393
 *   cache.setLastBatch / getLastBatch   internal/logdb/cache.go:108-135
 *   batchSize = LogDBEntryBatchSize = 48 (internal/settings/hard.go:125)
 *
 * The key-value store under the records is a per-(shard, replica) map of
 * batch id -> the last value Put, which getBatchFromDB (batch.go:348-366)
 * decodes and restores.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle_internal.h"

#define ORC_BATCH_SIZE 48u

static uint64_t batch_id(uint64_t index) { return index / ORC_BATCH_SIZE; }

/* getBatchIDRange (batch.go:76-83) */
void orc_batch_id_range(uint64_t low, uint64_t high, uint64_t *lo_id,
                        uint64_t *hi_id) {
  *lo_id = batch_id(low);
  *hi_id = batch_id(high) + (high % ORC_BATCH_SIZE == 0 ? 0 : 1);
}

/* compactBatchFields (batch.go:100-113), in place */
static void compact_fields(orc_evec *eb) {
  if (eb->n <= 1) orc_panic("compact called on small batch");
  const uint64_t exp_last = eb->v[0].index + (uint64_t)(eb->n - 1);
  if (eb->v[0].term == eb->v[eb->n - 1].term &&
      exp_last == eb->v[eb->n - 1].index) {
    for (size_t i = 1; i < eb->n; i++) {
      eb->v[i].term = 0;
      eb->v[i].index = 0;
    }
  }
}

/* restoreBatchFields (batch.go:86-98), in place */
static void restore_fields(orc_evec *eb) {
  if (eb->n <= 1) orc_panic("restore called on small batch");
  if (eb->v[eb->n - 1].term == 0) {
    const uint64_t term = eb->v[0].term, idx = eb->v[0].index;
    for (size_t i = 1; i < eb->n; i++) {
      eb->v[i].term = term;
      eb->v[i].index = idx + i;
    }
  }
}

/* getMergedFirstBatch (batch.go:115-141): the merged batch into out */
static void merged_first(const orc_evec *eb, const orc_evec *lb,
                         orc_evec *out) {
  if (eb->n == 0 || lb->n == 0)
    orc_panic("getMergedFirstBatch called on empty batch");
  const uint64_t b = batch_id(eb->v[0].index);
  if (b < batch_id(lb->v[0].index)) orc_panic("eb batch < lb batch");
  ev_truncate(out, 0);
  if (b > batch_id(lb->v[0].index)) {
    ev_copy_range(out, eb->v, eb->n);
    return;
  }
  const uint64_t first = eb->v[0].index;
  if (first > lb->v[0].index) {
    size_t keep = lb->n;
    if (first <= lb->v[lb->n - 1].index) {
      for (keep = 0; keep < lb->n; keep++)
        if (lb->v[keep].index >= first) break;
    }
    ev_copy_range(out, lb->v, keep);
    ev_copy_range(out, eb->v, eb->n);
    return;
  }
  ev_copy_range(out, eb->v, eb->n);
}

/* ---- the store ------------------------------------------------------- */
typedef struct kv_rec {
  uint64_t batch;
  uint8_t *val;
  size_t len;
} kv_rec;

typedef struct node_db {
  uint64_t shard, replica;
  int has_lb;
  orc_evec lb; /* cache.lastEntryBatch (full form, copied) */
  kv_rec *recs;
  size_t nrec, caprec;
} node_db;

struct orc_batchdb {
  node_db *nodes;
  size_t n, cap;
  /* the records Put by the last orc_batchdb_record call */
  uint64_t *out_batch;
  uint8_t **out_val;
  size_t *out_len;
  size_t nout, capout;
};

orc_batchdb *orc_batchdb_new(void) {
  return (orc_batchdb *)calloc(1, sizeof(orc_batchdb));
}

static void clear_out(orc_batchdb *db) {
  for (size_t i = 0; i < db->nout; i++) free(db->out_val[i]);
  db->nout = 0;
}

void orc_batchdb_free(orc_batchdb *db) {
  if (!db) return;
  for (size_t i = 0; i < db->n; i++) {
    node_db *nd = &db->nodes[i];
    ev_free(&nd->lb);
    for (size_t k = 0; k < nd->nrec; k++) free(nd->recs[k].val);
    free(nd->recs);
  }
  free(db->nodes);
  clear_out(db);
  free(db->out_batch);
  free(db->out_val);
  free(db->out_len);
  free(db);
}

static node_db *node_of(orc_batchdb *db, uint64_t shard, uint64_t replica) {
  for (size_t i = 0; i < db->n; i++)
    if (db->nodes[i].shard == shard && db->nodes[i].replica == replica)
      return &db->nodes[i];
  if (db->n == db->cap) {
    db->cap = db->cap ? 2 * db->cap : 8;
    db->nodes = (node_db *)realloc(db->nodes, db->cap * sizeof(node_db));
  }
  node_db *nd = &db->nodes[db->n++];
  memset(nd, 0, sizeof(*nd));
  nd->shard = shard;
  nd->replica = replica;
  return nd;
}

static kv_rec *rec_of(node_db *nd, uint64_t batch) {
  for (size_t k = 0; k < nd->nrec; k++)
    if (nd->recs[k].batch == batch) return &nd->recs[k];
  return NULL;
}

/* marshal an evec as an EntryBatch (raftpb/entrybatch.go:25-58) */
static uint8_t *marshal_batch(const orc_evec *eb, size_t *len) {
  size_t pool_cap = 0;
  for (size_t i = 0; i < eb->n; i++)
    pool_cap += eb->v[i].cmd ? eb->v[i].cmd->len : 0;
  drb_entry *views = (drb_entry *)calloc(eb->n ? eb->n : 1, sizeof(drb_entry));
  uint8_t *pool = (uint8_t *)malloc(pool_cap ? pool_cap : 1);
  size_t used = 0;
  for (size_t i = 0; i < eb->n; i++)
    entry_to_view(&eb->v[i], &views[i], pool, pool_cap, &used);
  const size_t n = orc_entrybatch_size(views, eb->n);
  uint8_t *buf = (uint8_t *)malloc(n ? n : 1);
  *len = orc_entrybatch_marshal(views, eb->n, pool, buf);
  free(views);
  free(pool);
  return buf;
}

/* getBatchFromDB (batch.go:348-366): the stored value, decoded, with its
 * compacted fields restored */
static int batch_from_db(node_db *nd, uint64_t batch, orc_evec *out) {
  kv_rec *r = rec_of(nd, batch);
  if (!r) return 0;
  const size_t cap = r->len; /* >= entries and >= Cmd bytes */
  drb_entry *views = (drb_entry *)calloc(cap ? cap : 1, sizeof(drb_entry));
  uint8_t *pool = (uint8_t *)malloc(cap ? cap : 1);
  const long n = orc_entrybatch_unmarshal(r->val, r->len, views, cap, pool,
                                          cap);
  if (n < 0) orc_panic("stored batch does not decode");
  ev_truncate(out, 0);
  for (long i = 0; i < n; i++) {
    orc_entry e = entry_from_view(&views[i], pool);
    ev_push(out, &e);
    blob_unref(e.cmd);
  }
  free(views);
  free(pool);
  if (out->n > 1) restore_fields(out);
  return 1;
}

/* recordBatch (batch.go:288-314) */
static void record_batch(orc_batchdb *db, node_db *nd, const orc_evec *eb,
                         uint64_t first_id, uint64_t last_id) {
  if (eb->n == 0) return;
  const uint64_t b = batch_id(eb->v[0].index);
  orc_evec meb = {0};
  if (first_id == b) {
    /* the getMergedFirstBatch method (batch.go:382-393) */
    int merged = 0;
    if (eb->v[0].index % ORC_BATCH_SIZE != 0) {
      /* getLastBatch (batch.go:369-380) */
      orc_evec lb = {0};
      int ok = nd->has_lb;
      if (ok) ev_copy_range(&lb, nd->lb.v, nd->lb.n);
      if (!ok || b < batch_id(lb.v[0].index)) ok = batch_from_db(nd, b, &lb);
      if (ok) {
        merged_first(eb, &lb, &meb);
        merged = 1;
      }
      ev_free(&lb);
    }
    if (!merged) ev_copy_range(&meb, eb->v, eb->n);
  } else {
    ev_copy_range(&meb, eb->v, eb->n);
  }
  if (last_id == b) { /* cache.setLastBatch copies the entries */
    ev_truncate(&nd->lb, 0);
    ev_copy_range(&nd->lb, meb.v, meb.n);
    nd->has_lb = 1;
  }
  if (meb.n > 1) compact_fields(&meb);
  size_t len;
  uint8_t *val = marshal_batch(&meb, &len);
  ev_free(&meb);
  /* wb.Put(EntryBatchKey(shard, replica, batch), value) */
  kv_rec *r = rec_of(nd, b);
  if (!r) {
    if (nd->nrec == nd->caprec) {
      nd->caprec = nd->caprec ? 2 * nd->caprec : 8;
      nd->recs = (kv_rec *)realloc(nd->recs, nd->caprec * sizeof(kv_rec));
    }
    r = &nd->recs[nd->nrec++];
    r->batch = b;
    r->val = NULL;
  }
  free(r->val);
  r->val = (uint8_t *)malloc(len ? len : 1);
  memcpy(r->val, val, len);
  r->len = len;
  if (db->nout == db->capout) {
    db->capout = db->capout ? 2 * db->capout : 8;
    db->out_batch =
        (uint64_t *)realloc(db->out_batch, db->capout * sizeof(uint64_t));
    db->out_val = (uint8_t **)realloc(db->out_val, db->capout * sizeof(void *));
    db->out_len = (size_t *)realloc(db->out_len, db->capout * sizeof(size_t));
  }
  db->out_batch[db->nout] = b;
  db->out_val[db->nout] = val;
  db->out_len[db->nout] = len;
  db->nout++;
}

/* record (batch.go:316-346) of one Update's EntriesToSave.  Returns the
 * number of records Put (orc_batchdb_out), -1 panic. */
long orc_batchdb_record(orc_batchdb *db, uint64_t shard, uint64_t replica,
                        const drb_entry *ents, size_t n, const uint8_t *pool) {
  clear_out(db);
  orc_evec in = {0}, eb = {0};
  for (size_t i = 0; i < n; i++) {
    orc_entry e = entry_from_view(&ents[i], pool);
    ev_push(&in, &e);
    blob_unref(e.cmd);
  }
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    ev_free(&in);
    ev_free(&eb);
    return -1;
  }
  if (n == 0) orc_panic("empty entries");
  node_db *nd = node_of(db, shard, replica);
  const uint64_t first_id = batch_id(in.v[0].index);
  const uint64_t last_id = batch_id(in.v[in.n - 1].index);
  uint64_t cur = UINT64_MAX;
  for (size_t i = 0; i < in.n; i++) {
    const uint64_t b = batch_id(in.v[i].index);
    if (b != cur) {
      record_batch(db, nd, &eb, first_id, last_id);
      ev_truncate(&eb, 0);
      cur = b;
    }
    ev_push(&eb, &in.v[i]);
  }
  if (eb.n > 0) record_batch(db, nd, &eb, first_id, last_id);
  orc_jb = prev;
  ev_free(&in);
  ev_free(&eb);
  return (long)db->nout;
}

/* record i of the last orc_batchdb_record call: its batch id and value */
long orc_batchdb_out(orc_batchdb *db, size_t i, uint64_t *batch, uint8_t *buf,
                     size_t cap) {
  if (i >= db->nout) return -1;
  *batch = db->out_batch[i];
  if (db->out_len[i] > cap) return -(long)db->out_len[i] - 2;
  memcpy(buf, db->out_val[i], db->out_len[i]);
  return (long)db->out_len[i];
}

/* ---- KAT hooks over drb_entry arrays (batch_test.go) ------------------ */
static void views_in(const drb_entry *e, size_t n, orc_evec *out) {
  for (size_t i = 0; i < n; i++) {
    orc_entry x = entry_from_view(&e[i], NULL);
    ev_push(out, &x);
  }
}
static void views_out(const orc_evec *in, drb_entry *e) {
  for (size_t i = 0; i < in->n; i++) {
    size_t used = 0;
    entry_to_view(&in->v[i], &e[i], NULL, 0, &used);
  }
}

/* compactBatchFields / restoreBatchFields in place: 0, -1 panic */
int orc_batch_compact(drb_entry *e, size_t n, int restore) {
  orc_evec v = {0};
  views_in(e, n, &v);
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    ev_free(&v);
    return -1;
  }
  if (restore)
    restore_fields(&v);
  else
    compact_fields(&v);
  orc_jb = prev;
  views_out(&v, e);
  ev_free(&v);
  return 0;
}

/* getMergedFirstBatch: the merged count (out must hold ne + nl), -1 panic */
long orc_batch_merged_first(const drb_entry *eb, size_t ne,
                            const drb_entry *lb, size_t nl, drb_entry *out) {
  orc_evec a = {0}, b = {0}, m = {0};
  views_in(eb, ne, &a);
  views_in(lb, nl, &b);
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    ev_free(&a);
    ev_free(&b);
    ev_free(&m);
    return -1;
  }
  merged_first(&a, &b, &m);
  orc_jb = prev;
  views_out(&m, out);
  const long n = (long)m.n;
  ev_free(&a);
  ev_free(&b);
  ev_free(&m);
  return n;
}
