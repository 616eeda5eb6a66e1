/*
 * raft_oracle.c -- CPU restatement of dragonboat internal/raft for the
 * replication fast path.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Every function names the reference function it restates; line numbers
 * refer to /root/reference (dragonboat v4 @ 2025-08-15).
 */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle_internal.h"

/* ------------------------------------------------------------------ */
/* panic -> longjmp to the API entry                                    */
/* ------------------------------------------------------------------ */
__thread jmp_buf *orc_jb;
static __thread char orc_err[512];

const char *orc_last_error(void) { return orc_err; }

void orc_panic(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(orc_err, sizeof(orc_err), fmt, ap);
  va_end(ap);
  if (orc_jb) longjmp(*orc_jb, 1);
  fprintf(stderr, "oracle panic outside API: %s\n", orc_err);
  abort();
}

/* ------------------------------------------------------------------ */
/* blobs, entries, vectors                                              */
/* ------------------------------------------------------------------ */
orc_blob *blob_new(const uint8_t *p, uint32_t len) {
  if (len == 0) return NULL;
  orc_blob *b = (orc_blob *)malloc(sizeof(orc_blob) + len);
  b->refs = 1;
  b->len = len;
  memcpy(b->data, p, len);
  return b;
}

void ev_push(orc_evec *v, const orc_entry *e) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 16;
    v->v = (orc_entry *)realloc(v->v, v->cap * sizeof(orc_entry));
  }
  v->v[v->n] = *e;
  blob_ref(e->cmd);
  v->n++;
}

void ev_truncate(orc_evec *v, size_t n) {
  for (size_t i = n; i < v->n; i++) blob_unref(v->v[i].cmd);
  if (n < v->n) v->n = n;
}

void ev_drop_front(orc_evec *v, size_t k) {
  if (k == 0) return;
  for (size_t i = 0; i < k; i++) blob_unref(v->v[i].cmd);
  memmove(v->v, v->v + k, (v->n - k) * sizeof(orc_entry));
  v->n -= k;
}

void ev_free(orc_evec *v) {
  ev_truncate(v, 0);
  free(v->v);
  v->v = NULL;
  v->cap = 0;
}

void ev_copy_range(orc_evec *dst, const orc_entry *src, size_t n) {
  for (size_t i = 0; i < n; i++) ev_push(dst, &src[i]);
}

void msg_free(orc_msg *m) { ev_free(&m->ents); }

void mv_push(orc_mvec *v, const orc_msg *m) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 8;
    v->v = (orc_msg *)realloc(v->v, v->cap * sizeof(orc_msg));
  }
  v->v[v->n++] = *m; /* takes ownership of m->ents */
}

void mv_clear(orc_mvec *v) {
  for (size_t i = 0; i < v->n; i++) msg_free(&v->v[i]);
  v->n = 0;
}

void mv_free(orc_mvec *v) {
  mv_clear(v);
  free(v->v);
  v->v = NULL;
  v->cap = 0;
}

orc_entry entry_from_view(const drb_entry *e, const uint8_t *pool) {
  orc_entry o;
  o.term = e->term;
  o.index = e->index;
  o.key = e->key;
  o.client_id = e->client_id;
  o.series_id = e->series_id;
  o.responded_to = e->responded_to;
  o.type = e->type;
  o.cmd = (e->cmd_len && pool) ? blob_new(pool + e->cmd_off, e->cmd_len)
                               : NULL;
  return o;
}

/* the view does not retain a reference; pool receives the bytes */
int entry_to_view(const orc_entry *e, drb_entry *out, uint8_t *pool,
                  size_t pool_cap, size_t *pool_used) {
  out->term = e->term;
  out->index = e->index;
  out->key = e->key;
  out->client_id = e->client_id;
  out->series_id = e->series_id;
  out->responded_to = e->responded_to;
  out->type = e->type;
  out->cmd_len = e->cmd ? e->cmd->len : 0;
  out->cmd_off = *pool_used;
  if (out->cmd_len) {
    if (!pool || *pool_used + out->cmd_len > pool_cap) return -1;
    memcpy(pool + *pool_used, e->cmd->data, out->cmd_len);
    *pool_used += out->cmd_len;
  }
  return 0;
}

static inline uint64_t umin(uint64_t a, uint64_t b) { return a < b ? a : b; }
static inline uint64_t umax(uint64_t a, uint64_t b) { return a > b ? a : b; }

/* Entry.SizeUpperLimit (raft_optimized.go:77-81) */
static uint64_t entry_size_upper_limit(const orc_entry *e) {
  return 128 /* settings.EntryNonCmdFieldsSize, soft.go:20 */ +
         (e->cmd ? e->cmd->len : 0);
}

/* limitSize (entryutils.go:50-63): returns the count to keep */
static size_t limit_size(const orc_entry *ents, size_t n, uint64_t limit) {
  if (n == 0) return 0;
  uint64_t total = entry_size_upper_limit(&ents[0]);
  size_t inc;
  for (inc = 1; inc < n; inc++) {
    total += entry_size_upper_limit(&ents[inc]);
    if (total > limit) break;
  }
  return inc;
}

/* checkEntriesToAppend (entryutils.go:36-48) */
static void check_entries_to_append(const orc_entry *ents, size_t n,
                                    const orc_entry *app, size_t an) {
  if (n == 0 || an == 0) return;
  if (ents[n - 1].index + 1 != app[0].index)
    orc_panic("found a hole, last %llu, first to append %llu",
              (unsigned long long)ents[n - 1].index,
              (unsigned long long)app[0].index);
  if (ents[n - 1].term > app[0].term)
    orc_panic("term value not expected, %llu vs %llu",
              (unsigned long long)ents[n - 1].term,
              (unsigned long long)app[0].term);
}

/* ------------------------------------------------------------------ */
/* remote (remote.go)                                                   */
/* ------------------------------------------------------------------ */
/* reset (remote.go:99-101) */
static void remote_reset(orc_remote *r) { r->snapshot_index = 0; }

/* becomeRetry (remote.go:103-111) */
void orc_remote_become_retry(orc_remote *r) {
  if (r->state == DRB_REMOTE_SNAPSHOT)
    r->next = umax(r->match + 1, r->snapshot_index + 1);
  else
    r->next = r->match + 1;
  remote_reset(r);
  r->state = DRB_REMOTE_RETRY;
}

/* retryToWait (remote.go:113-117) */
void orc_remote_retry_to_wait(orc_remote *r) {
  if (r->state == DRB_REMOTE_RETRY) r->state = DRB_REMOTE_WAIT;
}

/* waitToRetry (remote.go:119-123) */
void orc_remote_wait_to_retry(orc_remote *r) {
  if (r->state == DRB_REMOTE_WAIT) r->state = DRB_REMOTE_RETRY;
}

/* becomeWait (remote.go:125-129); clearSnapshotAck has no state here */
void orc_remote_become_wait(orc_remote *r) {
  orc_remote_become_retry(r);
  orc_remote_retry_to_wait(r);
}

/* becomeReplicate (remote.go:131-135) */
void orc_remote_become_replicate(orc_remote *r) {
  r->next = r->match + 1;
  remote_reset(r);
  r->state = DRB_REMOTE_REPLICATE;
}

/* becomeSnapshot (remote.go:137-141) */
void orc_remote_become_snapshot(orc_remote *r, uint64_t index) {
  remote_reset(r);
  r->snapshot_index = index;
  r->state = DRB_REMOTE_SNAPSHOT;
}

/* tryUpdate (remote.go:147-157) */
int orc_remote_try_update(orc_remote *r, uint64_t index) {
  if (r->next < index + 1) r->next = index + 1;
  if (r->match < index) {
    orc_remote_wait_to_retry(r);
    r->match = index;
    return 1;
  }
  return 0;
}

/* progress (remote.go:159-168) */
static void remote_progress(orc_remote *r, uint64_t last_index) {
  switch (r->state) {
    case DRB_REMOTE_REPLICATE:
      r->next = last_index + 1;
      break;
    case DRB_REMOTE_RETRY:
      orc_remote_retry_to_wait(r);
      break;
    default:
      orc_panic("unexpected remote state");
  }
}

/* respondedTo (remote.go:170-180) */
void orc_remote_responded_to(orc_remote *r) {
  switch (r->state) {
    case DRB_REMOTE_RETRY:
      orc_remote_become_replicate(r);
      break;
    case DRB_REMOTE_SNAPSHOT:
      if (r->match >= r->snapshot_index) orc_remote_become_retry(r);
      break;
    default:
      break;
  }
}

/* decreaseTo (remote.go:182-198) */
int orc_remote_decrease_to(orc_remote *r, uint64_t rejected, uint64_t last) {
  if (r->state == DRB_REMOTE_REPLICATE) {
    if (rejected <= r->match) return 0;
    r->next = r->match + 1;
    return 1;
  }
  if (r->next - 1 != rejected) return 0;
  orc_remote_wait_to_retry(r);
  r->next = umax(1, umin(rejected, last + 1));
  return 1;
}

/* isPaused (remote.go:200-213) */
static int remote_is_paused(const orc_remote *r) {
  switch (r->state) {
    case DRB_REMOTE_RETRY:
      return 0;
    case DRB_REMOTE_WAIT:
      return 1;
    case DRB_REMOTE_REPLICATE:
      return 0;
    case DRB_REMOTE_SNAPSHOT:
      return 1;
    default:
      orc_panic("unexpected remote state");
  }
  return 0;
}

int orc_remote_progress(orc_remote *r, uint64_t last_index) {
  ORC_TRY(-1);
  remote_progress(r, last_index);
  ORC_END;
  return 0;
}

int orc_remote_is_paused(orc_remote *r) {
  ORC_TRY(-1);
  int p = remote_is_paused(r);
  ORC_END;
  return p;
}

/* ------------------------------------------------------------------ */
/* readIndex (readindex.go)                                             */
/* ------------------------------------------------------------------ */
static int ctx_eq(orc_ctx a, orc_ctx b) {
  return a.low == b.low && a.high == b.high;
}

static long ri_find(const orc_readindex *r, orc_ctx ctx) {
  for (size_t i = 0; i < r->n; i++)
    if (ctx_eq(r->q[i].ctx, ctx)) return (long)i;
  return -1;
}

/* addRequest (readindex.go:43-66) */
void ri_add_request(orc_readindex *r, uint64_t index, orc_ctx ctx,
                    uint64_t from) {
  if (ri_find(r, ctx) >= 0) return;
  if (r->n > 0) {
    /* p, ok := r.pending[r.peepCtx()]; the raw-queue test hook may make
     * the queue tail a ctx with no pending status */
    orc_rstatus *p = &r->q[r->n - 1];
    if (p->index == UINT64_MAX) orc_panic("inconsistent pending and queue");
    if (index < p->index)
      orc_panic("index moved backward in readIndex, %llu:%llu",
                (unsigned long long)index, (unsigned long long)p->index);
  }
  if (r->n == r->cap) {
    r->cap = r->cap ? r->cap * 2 : 4;
    r->q = (orc_rstatus *)realloc(r->q, r->cap * sizeof(orc_rstatus));
  }
  orc_rstatus *s = &r->q[r->n++];
  memset(s, 0, sizeof(*s));
  s->ctx = ctx;
  s->index = index;
  s->from = from;
}

/* hasPendingRequest / peepCtx (readindex.go:68-75) */
static int ri_has_pending(const orc_readindex *r) { return r->n > 0; }
static orc_ctx ri_peep(const orc_readindex *r) { return r->q[r->n - 1].ctx; }

/* confirm (readindex.go:77-115).  Released statuses are copied to out. */
size_t ri_confirm(orc_readindex *r, orc_ctx ctx, uint64_t from, int quorum,
                  orc_rstatus *out, size_t out_cap) {
  long pi = ri_find(r, ctx);
  if (pi < 0) return 0;
  orc_rstatus *p = &r->q[pi];
  if (p->index == UINT64_MAX) return 0; /* raw queue entry, not pending */
  int seen = 0;
  for (int i = 0; i < p->nconfirmed; i++)
    if (p->confirmed[i] == from) seen = 1;
  if (!seen) {
    if (p->nconfirmed >= ORC_MAX_PEERS) orc_panic("too many confirmations");
    p->confirmed[p->nconfirmed++] = from;
  }
  if (p->nconfirmed + 1 < quorum) return 0;
  size_t done = 0;
  for (size_t i = 0; i < r->n; i++) {
    done++;
    if (r->q[i].index == UINT64_MAX)
      orc_panic("inconsistent pending and queue content");
    if (ctx_eq(r->q[i].ctx, ctx)) {
      uint64_t sidx = r->q[i].index;
      for (size_t j = 0; j <= i; j++) {
        if (r->q[j].index > sidx) orc_panic("v.index > s.index is unexpected");
        r->q[j].index = sidx;
      }
      if (done > out_cap) orc_panic("confirm output overflow");
      memcpy(out, r->q, done * sizeof(orc_rstatus));
      memmove(r->q, r->q + done, (r->n - done) * sizeof(orc_rstatus));
      r->n -= done;
      return done;
    }
  }
  return 0;
}

orc_readindex *orc_readindex_new(void) {
  return (orc_readindex *)calloc(1, sizeof(orc_readindex));
}

void orc_readindex_free(orc_readindex *r) {
  if (!r) return;
  free(r->q);
  free(r);
}

int orc_readindex_add_request(orc_readindex *r, uint64_t index, uint64_t low,
                              uint64_t high, uint64_t from) {
  ORC_TRY(-1);
  orc_ctx c = {low, high};
  ri_add_request(r, index, c, from);
  ORC_END;
  return 0;
}

size_t orc_readindex_len(orc_readindex *r) { return r->n; }

int orc_readindex_get(orc_readindex *r, size_t i, uint64_t *low,
                      uint64_t *high, uint64_t *index, uint64_t *from) {
  if (i >= r->n) return -1;
  *low = r->q[i].ctx.low;
  *high = r->q[i].ctx.high;
  *index = r->q[i].index;
  *from = r->q[i].from;
  return 0;
}

int orc_readindex_confirm(orc_readindex *r, uint64_t low, uint64_t high,
                          uint64_t from, int quorum, uint64_t *out_low,
                          uint64_t *out_high, uint64_t *out_index,
                          uint64_t *out_from, int out_cap) {
  ORC_TRY(-1);
  orc_rstatus tmp[64];
  orc_ctx c = {low, high};
  size_t n = ri_confirm(r, c, from, quorum, tmp, 64);
  for (size_t i = 0; i < n && (int)i < out_cap; i++) {
    out_low[i] = tmp[i].ctx.low;
    out_high[i] = tmp[i].ctx.high;
    out_index[i] = tmp[i].index;
    out_from[i] = tmp[i].from;
  }
  ORC_END;
  return (int)n;
}

/* A ctx present in queue but not in pending: modelled with index
 * UINT64_MAX (used only by the reference's inconsistency tests). */
int orc_readindex_push_raw_queue(orc_readindex *r, uint64_t low, uint64_t high,
                                 int front) {
  if (r->n == r->cap) {
    r->cap = r->cap ? r->cap * 2 : 4;
    r->q = (orc_rstatus *)realloc(r->q, r->cap * sizeof(orc_rstatus));
  }
  orc_rstatus s;
  memset(&s, 0, sizeof(s));
  s.ctx.low = low;
  s.ctx.high = high;
  s.index = UINT64_MAX;
  if (front) {
    memmove(r->q + 1, r->q, r->n * sizeof(orc_rstatus));
    r->q[0] = s;
  } else {
    r->q[r->n] = s;
  }
  r->n++;
  return 0;
}

/* ------------------------------------------------------------------ */
/* TestLogDB (internal/raft/logdb_test.go)                              */
/* ------------------------------------------------------------------ */
static uint64_t db_first(const orc_logdb *db) { return db->marker_index + 1; }
static uint64_t db_last(const orc_logdb *db) {
  return db->marker_index + db->ents.n;
}

/* Entries (logdb_test.go:143-156).  *out points into db storage. */
static int db_entries(const orc_logdb *db, uint64_t low, uint64_t high,
                      uint64_t max_size, const orc_entry **out, size_t *n) {
  if (low <= db->marker_index) return ORC_ERR_COMPACTED;
  if (high > db_last(db) + 1) return ORC_ERR_UNAVAILABLE;
  if (db->ents.n == 0) return ORC_ERR_UNAVAILABLE;
  const orc_entry *e = db->ents.v + (low - db->marker_index - 1);
  size_t cnt = (size_t)(high - low);
  *out = e;
  *n = limit_size(e, cnt, max_size);
  return 0;
}

/* Term (logdb_test.go:91-102) */
static int db_term(const orc_logdb *db, uint64_t index, uint64_t *term) {
  if (index == db->marker_index) {
    *term = db->marker_term;
    return 0;
  }
  const orc_entry *e;
  size_t n;
  int err = db_entries(db, index, index + 1, UINT64_MAX, &e, &n);
  if (err) return err;
  *term = n ? e[0].term : 0;
  return 0;
}

/* Append (logdb_test.go:104-125) */
void db_append(orc_logdb *db, const orc_entry *ents, size_t n) {
  if (n == 0) return;
  uint64_t first = db_first(db);
  if (db->marker_index + n < first) return;
  if (first > ents[0].index) {
    size_t cut = (size_t)(first - ents[0].index);
    ents += cut;
    n -= cut;
  }
  uint64_t offset = ents[0].index - db->marker_index;
  if ((uint64_t)db->ents.n + 1 > offset)
    ev_truncate(&db->ents, (size_t)(offset - 1));
  else if ((uint64_t)db->ents.n + 1 < offset)
    orc_panic("found a hole last index %llu, first incoming index %llu",
              (unsigned long long)db_last(db),
              (unsigned long long)ents[0].index);
  ev_copy_range(&db->ents, ents, n);
}

/* Compact (logdb_test.go:158-176) */
static int db_compact(orc_logdb *db, uint64_t index) {
  if (index <= db->marker_index) return ORC_ERR_COMPACTED;
  if (index > db_last(db)) return ORC_ERR_UNAVAILABLE;
  if (db->ents.n == 0) return ORC_ERR_UNAVAILABLE;
  uint64_t term;
  int err = db_term(db, index, &term);
  if (err) return err;
  ev_drop_front(&db->ents, (size_t)(index - db->marker_index));
  db->marker_index = index;
  db->marker_term = term;
  return 0;
}

orc_logdb *orc_logdb_new(void) {
  return (orc_logdb *)calloc(1, sizeof(orc_logdb));
}

void orc_logdb_free(orc_logdb *db) {
  if (!db) return;
  ev_free(&db->ents);
  free(db);
}

int orc_logdb_append(orc_logdb *db, const drb_entry *ents, size_t n,
                     const uint8_t *pool) {
  ORC_TRY(-1);
  orc_evec tmp = {0};
  for (size_t i = 0; i < n; i++) {
    orc_entry e = entry_from_view(&ents[i], pool);
    ev_push(&tmp, &e);
    blob_unref(e.cmd);
  }
  db_append(db, tmp.v, tmp.n);
  ev_free(&tmp);
  ORC_END;
  return 0;
}

int orc_logdb_compact(orc_logdb *db, uint64_t index) {
  return db_compact(db, index);
}

void orc_logdb_set_state(orc_logdb *db, uint64_t term, uint64_t vote,
                         uint64_t commit) {
  db->st_term = term;
  db->st_vote = vote;
  db->st_commit = commit;
}

/* ------------------------------------------------------------------ */
/* inMemory (inmemory.go)                                               */
/* ------------------------------------------------------------------ */
/* newInMemory (inmemory.go:41-50) */
static void im_init(orc_inmem *im, uint64_t last_index) {
  memset(im, 0, sizeof(*im));
  im->marker_index = last_index + 1;
  im->saved_to = last_index;
}

/* checkMarkerIndex (inmemory.go:52-59) */
static void im_check_marker(const orc_inmem *im) {
  if (im->ents.n > 0 && im->ents.v[0].index != im->marker_index)
    orc_panic("marker index %llu, first index %llu",
              (unsigned long long)im->marker_index,
              (unsigned long long)im->ents.v[0].index);
}

/* getEntries (inmemory.go:61-72) */
static const orc_entry *im_get_entries(const orc_inmem *im, uint64_t low,
                                       uint64_t high, size_t *n) {
  uint64_t upper = im->marker_index + im->ents.n;
  if (low > high || low < im->marker_index)
    orc_panic("invalid low value %llu, high %llu, marker index %llu",
              (unsigned long long)low, (unsigned long long)high,
              (unsigned long long)im->marker_index);
  if (high > upper)
    orc_panic("invalid high value %llu, upperBound %llu",
              (unsigned long long)high, (unsigned long long)upper);
  *n = (size_t)(high - low);
  return im->ents.v + (low - im->marker_index);
}

/* getLastIndex (inmemory.go:81-86); no snapshot on this path */
static int im_last_index(const orc_inmem *im, uint64_t *idx) {
  if (im->ents.n > 0) {
    *idx = im->ents.v[im->ents.n - 1].index;
    return 1;
  }
  return 0;
}

/* getTerm (inmemory.go:88-106) */
static int im_get_term(const orc_inmem *im, uint64_t index, uint64_t *term) {
  if (index > 0 && index == im->applied_to_index) {
    if (im->applied_to_term == 0)
      orc_panic("im.appliedToTerm == 0, index %llu", (unsigned long long)index);
    *term = im->applied_to_term;
    return 1;
  }
  if (index < im->marker_index) return 0;
  uint64_t last;
  if (im_last_index(im, &last) && index <= last) {
    *term = im->ents.v[index - im->marker_index].term;
    return 1;
  }
  return 0;
}

/* entriesToSave (inmemory.go:116-122) */
static const orc_entry *im_entries_to_save(const orc_inmem *im, size_t *n) {
  uint64_t idx = im->saved_to + 1;
  if (idx - im->marker_index > (uint64_t)im->ents.n) {
    *n = 0;
    return NULL;
  }
  *n = im->ents.n - (size_t)(idx - im->marker_index);
  return im->ents.v + (idx - im->marker_index);
}

/* savedLogTo (inmemory.go:124-136) */
static void im_saved_log_to(orc_inmem *im, uint64_t index, uint64_t term) {
  if (index < im->marker_index) return;
  if (im->ents.n == 0) return;
  if (index > im->ents.v[im->ents.n - 1].index ||
      term != im->ents.v[index - im->marker_index].term)
    return;
  im->saved_to = index;
}

/* appliedLogTo (inmemory.go:138-164) */
static void im_applied_log_to(orc_inmem *im, uint64_t index) {
  if (index < im->marker_index) return;
  if (im->ents.n == 0) return;
  if (index > im->ents.v[im->ents.n - 1].index) return;
  const orc_entry *last = &im->ents.v[index - im->marker_index];
  if (last->index != index) orc_panic("lastEntry.Index != index");
  im->applied_to_index = last->index;
  im->applied_to_term = last->term;
  uint64_t nm = index + 1;
  im->shrunk = 1;
  ev_drop_front(&im->ents, (size_t)(nm - im->marker_index));
  im->marker_index = nm;
  /* resizeEntrySlice (inmemory.go:185-190) changes capacity only */
  im_check_marker(im);
}

/* commitUpdate (inmemory.go:107-114) */
static void im_commit_update(orc_inmem *im, uint64_t stable_log_to,
                             uint64_t stable_log_term) {
  if (stable_log_to > 0) im_saved_log_to(im, stable_log_to, stable_log_term);
}

/* merge (inmemory.go:199-230) */
static void im_merge(orc_inmem *im, const orc_entry *ents, size_t n) {
  uint64_t first_new = ents[0].index;
  if (first_new == im->marker_index + im->ents.n) {
    check_entries_to_append(im->ents.v, im->ents.n, ents, n);
    ev_copy_range(&im->ents, ents, n);
  } else if (first_new <= im->marker_index) {
    im->marker_index = first_new;
    im->shrunk = 0;
    ev_truncate(&im->ents, 0);
    ev_copy_range(&im->ents, ents, n);
    im->saved_to = first_new - 1;
  } else {
    size_t en;
    im_get_entries(im, im->marker_index, first_new, &en);
    check_entries_to_append(im->ents.v, en, ents, n);
    im->shrunk = 0;
    ev_truncate(&im->ents, en);
    ev_copy_range(&im->ents, ents, n);
    im->saved_to = umin(im->saved_to, first_new - 1);
  }
  im_check_marker(im);
}

/* ------------------------------------------------------------------ */
/* entryLog (logentry.go)                                               */
/* ------------------------------------------------------------------ */
/* newEntryLog (logentry.go:86-95) */
static void log_init(orc_log *l, orc_logdb *db) {
  l->db = db;
  uint64_t first = db_first(db), last = db_last(db);
  im_init(&l->im, last);
  l->committed = first - 1;
  l->processed = first - 1;
}

/* firstIndex (logentry.go:97-105) */
static uint64_t log_first(const orc_log *l) { return db_first(l->db); }

/* lastIndex (logentry.go:107-114) */
uint64_t log_last(const orc_log *l) {
  uint64_t idx;
  if (im_last_index(&l->im, &idx)) return idx;
  return db_last(l->db);
}

/* term (logentry.go:142-155) */
int log_term(const orc_log *l, uint64_t index, uint64_t *term) {
  uint64_t first = log_first(l) - 1, last = log_last(l);
  if (index < first || index > last) {
    *term = 0;
    return 0;
  }
  if (im_get_term(&l->im, index, term)) return 0;
  return db_term(l->db, index, term);
}

/* checkBound (logentry.go:157-173) */
static int log_check_bound(const orc_log *l, uint64_t low, uint64_t high) {
  if (low > high)
    orc_panic("input low %llu > high %llu", (unsigned long long)low,
              (unsigned long long)high);
  uint64_t first = log_first(l), last = log_last(l);
  if (low < first) return ORC_ERR_COMPACTED;
  if (high > last + 1)
    orc_panic("requested range [%llu,%llu) is out of bound [%llu,%llu]",
              (unsigned long long)low, (unsigned long long)high,
              (unsigned long long)first, (unsigned long long)last);
  return 0;
}

/* getEntries (logentry.go:214-231) = getEntriesFromLogDB (:180-195) +
 * getEntriesFromInMem (:197-212) + limitSize; the result is appended to
 * out (caller-owned evec) */
static int log_get_entries(const orc_log *l, uint64_t low, uint64_t high,
                           uint64_t max_size, orc_evec *out) {
  int err = log_check_bound(l, low, high);
  if (err) return err;
  if (low == high) return 0;
  orc_evec tmp = {0};
  int check_inmem = 1;
  if (low < l->im.marker_index) {
    uint64_t upper = umin(high, l->im.marker_index);
    const orc_entry *e;
    size_t n;
    err = db_entries(l->db, low, upper, max_size, &e, &n);
    if (err) return err;
    if ((uint64_t)n > upper - low) orc_panic("uint64(len(ents)) > upperBound-low");
    ev_copy_range(&tmp, e, n);
    check_inmem = ((uint64_t)n == upper - low);
  }
  if (!check_inmem) {
    ev_copy_range(out, tmp.v, tmp.n);
    ev_free(&tmp);
    return 0;
  }
  if (high > l->im.marker_index) {
    uint64_t lower = umax(low, l->im.marker_index);
    size_t n;
    const orc_entry *e = im_get_entries(&l->im, lower, high, &n);
    if (n > 0) {
      if (tmp.n > 0) check_entries_to_append(tmp.v, tmp.n, e, n);
      ev_copy_range(&tmp, e, n);
    }
  }
  size_t keep = limit_size(tmp.v, tmp.n, max_size);
  ev_copy_range(out, tmp.v, keep);
  ev_free(&tmp);
  return 0;
}

/* entries (logentry.go:233-238) */
static int log_entries(const orc_log *l, uint64_t start, uint64_t max_size,
                       orc_evec *out) {
  if (start > log_last(l)) return 0;
  return log_get_entries(l, start, log_last(l) + 1, max_size, out);
}

/* firstNotAppliedIndex / toApplyIndexLimit / hasEntriesToApply
 * (logentry.go:248-258) */
static uint64_t log_first_not_applied(const orc_log *l) {
  return umax(l->processed + 1, log_first(l));
}
int log_has_entries_to_apply(const orc_log *l) {
  return l->committed + 1 > log_first_not_applied(l);
}

/* entriesToApply (logentry.go:264-278), maxEntriesToApplySize = 64 MiB */
int log_entries_to_apply(const orc_log *l, orc_evec *out) {
  if (log_has_entries_to_apply(l))
    return log_get_entries(l, log_first_not_applied(l), l->committed + 1,
                           64ull * 1024 * 1024, out);
  return 0;
}

/* append (logentry.go:312-321) */
static void log_append(orc_log *l, const orc_entry *ents, size_t n) {
  if (n == 0) return;
  if (ents[0].index <= l->committed)
    orc_panic("committed entries being changed, committed %llu, first idx %llu",
              (unsigned long long)l->committed,
              (unsigned long long)ents[0].index);
  im_merge(&l->im, ents, n);
}

/* matchTerm (logentry.go:373-379) */
static int log_match_term(const orc_log *l, uint64_t index, uint64_t term,
                          int *match) {
  uint64_t lt;
  int err = log_term(l, index, &lt);
  if (err) return err;
  *match = (lt == term);
  return 0;
}

/* getConflictIndex (logentry.go:323-334) */
static int log_conflict_index(const orc_log *l, const orc_entry *ents,
                              size_t n, uint64_t *ci) {
  for (size_t i = 0; i < n; i++) {
    int match;
    int err = log_match_term(l, ents[i].index, ents[i].term, &match);
    if (err) return err;
    if (!match) {
      *ci = ents[i].index;
      return 0;
    }
  }
  *ci = 0;
  return 0;
}

/* tryAppend (logentry.go:296-310) */
static int log_try_append(orc_log *l, uint64_t index, const orc_entry *ents,
                          size_t n, int *appended) {
  uint64_t ci;
  int err = log_conflict_index(l, ents, n, &ci);
  if (err) return err;
  *appended = 0;
  if (ci != 0) {
    if (ci <= l->committed)
      orc_panic("entry %llu conflicts with committed entry, committed %llu",
                (unsigned long long)ci, (unsigned long long)l->committed);
    size_t off = (size_t)(ci - index - 1);
    log_append(l, ents + off, n - off);
    *appended = 1;
  }
  return 0;
}

/* commitTo (logentry.go:336-349) */
void log_commit_to(orc_log *l, uint64_t index) {
  if (index <= l->committed) return;
  if (index > log_last(l))
    orc_panic("invalid commitTo index %llu, lastIndex() %llu",
              (unsigned long long)index, (unsigned long long)log_last(l));
  l->committed = index;
}

/* commitUpdate (logentry.go:351-371) */
void log_commit_update(orc_log *l, uint64_t stable_log_to,
                       uint64_t stable_log_term, uint64_t processed,
                       uint64_t last_applied) {
  im_commit_update(&l->im, stable_log_to, stable_log_term);
  if (processed > 0) {
    if (processed < l->processed || processed > l->committed)
      orc_panic("invalid ApplyReturnedTo %llu, current applied %llu, "
                "committed %llu",
                (unsigned long long)processed,
                (unsigned long long)l->processed,
                (unsigned long long)l->committed);
    l->processed = processed;
  }
  if (last_applied > 0) {
    if (last_applied > l->committed)
      orc_panic("invalid last applied %llu, committed %llu",
                (unsigned long long)last_applied,
                (unsigned long long)l->committed);
    if (last_applied > l->processed)
      orc_panic("invalid last applied %llu, processed %llu",
                (unsigned long long)last_applied,
                (unsigned long long)l->processed);
    im_applied_log_to(&l->im, last_applied);
  }
}

/* upToDate (logentry.go:381-393) */
static int log_up_to_date(const orc_log *l, uint64_t index, uint64_t term,
                          int *ok) {
  uint64_t lt;
  int err = log_term(l, log_last(l), &lt);
  if (err) return err;
  if (term >= lt) {
    *ok = (term > lt) ? 1 : (index >= log_last(l));
    return 0;
  }
  *ok = 0;
  return 0;
}

/* tryCommit (logentry.go:395-410) */
static int log_try_commit(orc_log *l, uint64_t index, uint64_t term,
                          int *committed) {
  *committed = 0;
  if (index <= l->committed) return 0;
  uint64_t lterm;
  int err = log_term(l, index, &lterm);
  if (err == ORC_ERR_COMPACTED)
    lterm = 0;
  else if (err)
    return err;
  if (index > l->committed && lterm == term) {
    log_commit_to(l, index);
    *committed = 1;
  }
  return 0;
}

static void log_free(orc_log *l) { ev_free(&l->im.ents); }

/* ------------------------------------------------------------------ */
/* raft (raft.go)                                                       */
/* ------------------------------------------------------------------ */
static uint64_t splitmix64(uint64_t *s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int raft_rem_idx(const orc_raft *r, uint64_t id) {
  for (int i = 0; i < r->nrem; i++)
    if (r->rem_id[i] == id) return i;
  return -1;
}

static void raft_set_remote(orc_raft *r, uint64_t id, uint64_t match,
                            uint64_t next) {
  int i = raft_rem_idx(r, id);
  if (i < 0) {
    if (r->nrem >= ORC_MAX_PEERS) orc_panic("too many remotes");
    i = r->nrem;
    while (i > 0 && r->rem_id[i - 1] > id) {
      r->rem_id[i] = r->rem_id[i - 1];
      r->rem[i] = r->rem[i - 1];
      r->rem_kind[i] = r->rem_kind[i - 1];
      i--;
    }
    r->nrem++;
    r->rem_id[i] = id;
    r->rem_kind[i] = ORC_VOTING;
  }
  memset(&r->rem[i], 0, sizeof(orc_remote));
  r->rem[i].match = match;
  r->rem[i].next = next;
}

/* the member kind of replica id (0: none of them) */
static int raft_is_kind(const orc_raft *r, uint64_t id, int kind) {
  const int i = raft_rem_idx(r, id);
  return i >= 0 && r->rem_kind[i] == kind;
}

/* numVotingMembers / quorum (raft.go:383-389): remotes and witnesses */
static int raft_num_voting(const orc_raft *r) {
  int n = 0;
  for (int i = 0; i < r->nrem; i++) n += r->rem_kind[i] != ORC_NONVOTING;
  return n;
}
static int raft_quorum(const orc_raft *r) { return raft_num_voting(r) / 2 + 1; }
static int raft_single_node_quorum(const orc_raft *r) {
  return raft_quorum(r) == 1;
}

/* resetMatchValueArray (raft.go:315-317) */
static void raft_reset_matched(orc_raft *r) {
  r->nmatched = raft_num_voting(r);
  memset(r->matched, 0, sizeof(r->matched));
}

/* setLeaderID (raft.go:354-373) */
static void raft_set_leader_id(orc_raft *r, uint64_t leader) {
  r->leader_id = leader;
  r->leader_update = 1;
}

/* setRandomizedElectionTimeout (raft.go:658-661) */
static void raft_set_rand_timeout(orc_raft *r) {
  r->randomized_election_timeout =
      r->election_timeout + splitmix64(&r->rng) % r->election_timeout;
}

/* resetRemotes (raft.go:1088-1097) */
static void raft_reset_remotes(orc_raft *r) {
  uint64_t last = log_last(&r->log);
  for (int i = 0; i < r->nrem; i++) {
    memset(&r->rem[i], 0, sizeof(orc_remote));
    r->rem[i].next = last + 1;
    if (r->rem_id[i] == r->replica_id) r->rem[i].match = last;
  }
}

/* reset (raft.go:1052-1073) */
static void raft_reset(orc_raft *r, uint64_t term, int reset_election) {
  if (r->term != term) {
    r->term = term;
    r->vote = 0;
  }
  if (reset_election) {
    r->election_tick = 0;
    raft_set_rand_timeout(r);
  }
  r->nvotes = 0;
  r->heartbeat_tick = 0;
  r->ri.n = 0;
  r->pending_config_change = 0;
  r->leader_transfer_target = 0;
  raft_reset_remotes(r);
  raft_reset_matched(r);
}

/* finalizeMessageTerm + send (raft.go:667-687) */
static int is_request_message(uint32_t t) {
  return t == DRB_MSG_PROPOSE || t == DRB_MSG_READ_INDEX ||
         t == DRB_MSG_LEADER_TRANSFER;
}
static int is_request_vote_message(uint32_t t) {
  return t == DRB_MSG_REQUEST_VOTE || t == DRB_MSG_REQUEST_PREVOTE;
}
static int is_leader_message(uint32_t t) {
  return t == DRB_MSG_REPLICATE || t == DRB_MSG_INSTALL_SNAPSHOT ||
         t == DRB_MSG_HEARTBEAT || t == DRB_MSG_TIMEOUT_NOW ||
         t == DRB_MSG_READ_INDEX_RESP;
}

static void raft_send(orc_raft *r, orc_msg *m) {
  m->from = r->replica_id;
  if (m->term == 0 && m->type == DRB_MSG_REQUEST_VOTE)
    orc_panic("sending RequestVote with 0 term");
  if (m->term > 0 && !is_request_vote_message(m->type) &&
      m->type != DRB_MSG_REQUEST_PREVOTE_RESP)
    orc_panic("term unexpectedly set for message type %u", m->type);
  if (!is_request_message(m->type) && !is_request_vote_message(m->type) &&
      m->type != DRB_MSG_REQUEST_PREVOTE_RESP)
    m->term = r->term;
  mv_push(&r->msgs, m);
}

static orc_msg new_msg(uint32_t type, uint64_t to) {
  orc_msg m;
  memset(&m, 0, sizeof(m));
  m.type = type;
  m.to = to;
  return m;
}

/* makeReplicateMessage (raft.go:738-769); returns log error code */
static int raft_make_replicate(orc_raft *r, uint64_t to, uint64_t next,
                               uint64_t max_size, orc_msg *m) {
  uint64_t term;
  int err = log_term(&r->log, next - 1, &term);
  if (err) return err;
  orc_evec ents = {0};
  err = log_entries(&r->log, next, max_size, &ents);
  if (err) {
    ev_free(&ents);
    return err;
  }
  if (ents.n > 0) {
    uint64_t li = ents.v[ents.n - 1].index, exp = next - 1 + ents.n;
    if (li != exp)
      orc_panic("expected last index in Replicate %llu, got %llu",
                (unsigned long long)exp, (unsigned long long)li);
  }
  /* a witness is sent metadata entries (makeMetadataEntries, raft.go:
   * 756-785): Index and Term of each, config changes as they are */
  if (raft_is_kind(r, to, ORC_WITNESS))
    for (size_t i = 0; i < ents.n; i++) {
      orc_entry *e = &ents.v[i];
      if (e->type == DRB_ENTRY_CONFIG_CHANGE) continue;
      const uint64_t t = e->term, x = e->index;
      blob_unref(e->cmd);
      memset(e, 0, sizeof(*e));
      e->type = DRB_ENTRY_METADATA;
      e->term = t;
      e->index = x;
    }
  *m = new_msg(DRB_MSG_REPLICATE, to);
  m->log_index = next - 1;
  m->log_term = term;
  m->ents = ents;
  m->commit = r->log.committed;
  return 0;
}

/* sendReplicateMessage (raft.go:787-819) */
static void raft_send_replicate(orc_raft *r, uint64_t to) {
  int i = raft_rem_idx(r, to);
  if (i < 0) orc_panic("failed to get the remote instance");
  orc_remote *rp = &r->rem[i];
  if (remote_is_paused(rp)) return;
  orc_msg m;
  int err = raft_make_replicate(r, to, rp->next,
                                64ull * 1024 * 1024 /* maxEntrySize */, &m);
  if (err) {
    /* log compacted: InstallSnapshot path -- not on this path */
    orc_panic("snapshot required for replica %llu (not on the fast path)",
              (unsigned long long)to);
  } else if (m.ents.n > 0) {
    remote_progress(rp, m.ents.v[m.ents.n - 1].index);
  }
  raft_send(r, &m);
}

/* broadcastReplicateMessage (raft.go:821-833) */
static void raft_broadcast_replicate(orc_raft *r) {
  if (r->state != DRB_LEADER) orc_panic("is not leader");
  for (int i = 0; i < r->nrem; i++)
    if (r->rem_id[i] != r->replica_id) raft_send_replicate(r, r->rem_id[i]);
}

/* sendHeartbeatMessage (raft.go:835-845) */
static void raft_send_heartbeat(orc_raft *r, uint64_t to, orc_ctx hint,
                                uint64_t match) {
  orc_msg m = new_msg(DRB_MSG_HEARTBEAT, to);
  m.commit = umin(match, r->log.committed);
  m.hint = hint.low;
  m.hint_high = hint.high;
  raft_send(r, &m);
}

/* broadcastHeartbeatMessageWithHint (raft.go:859-871): the voting members
 * (remotes and witnesses) with the ctx, the nonVotings only without one */
static void raft_broadcast_heartbeat_hint(orc_raft *r, orc_ctx ctx) {
  for (int i = 0; i < r->nrem; i++)
    if (r->rem_id[i] != r->replica_id && r->rem_kind[i] != ORC_NONVOTING)
      raft_send_heartbeat(r, r->rem_id[i], ctx, r->rem[i].match);
  if (ctx.low == 0 && ctx.high == 0) {
    orc_ctx zero = {0, 0};
    for (int i = 0; i < r->nrem; i++)
      if (r->rem_kind[i] == ORC_NONVOTING)
        raft_send_heartbeat(r, r->rem_id[i], zero, r->rem[i].match);
  }
}

/* broadcastHeartbeatMessage (raft.go:849-857) */
static void raft_broadcast_heartbeat(orc_raft *r) {
  if (r->state != DRB_LEADER) orc_panic("is not leader");
  orc_ctx zero = {0, 0};
  if (ri_has_pending(&r->ri))
    raft_broadcast_heartbeat_hint(r, ri_peep(&r->ri));
  else
    raft_broadcast_heartbeat_hint(r, zero);
}

/* sortMatchValues (raft.go:884-909) */
void orc_sort_match_values(uint64_t *v, int n) {
  if (n == 3) {
    uint64_t t;
    if (v[0] > v[1]) { t = v[0]; v[0] = v[1]; v[1] = t; }
    if (v[1] > v[2]) { t = v[1]; v[1] = v[2]; v[2] = t; }
    if (v[0] > v[1]) { t = v[0]; v[0] = v[1]; v[1] = t; }
  } else if (n == 1) {
    return;
  } else {
    for (int i = 1; i < n; i++) {
      uint64_t x = v[i];
      int j = i - 1;
      while (j >= 0 && v[j] > x) {
        v[j + 1] = v[j];
        j--;
      }
      v[j + 1] = x;
    }
  }
}

/* tryCommit (raft.go:911-942) */
static int raft_try_commit(orc_raft *r) {
  if (r->state != DRB_LEADER) orc_panic("is not leader");
  if (raft_num_voting(r) != r->nmatched) raft_reset_matched(r);
  /* the remotes' and the witnesses' matches */
  for (int i = 0, k = 0; i < r->nrem; i++)
    if (r->rem_kind[i] != ORC_NONVOTING) r->matched[k++] = r->rem[i].match;
  orc_sort_match_values(r->matched, r->nmatched);
  uint64_t q = r->matched[raft_num_voting(r) - raft_quorum(r)];
  int ok;
  int err = log_try_commit(&r->log, q, r->term, &ok);
  if (err) orc_panic("tryCommit: log error %d", err);
  return ok;
}

/* appendEntries (raft.go:944-955); ents are modified in place */
static void raft_append_entries(orc_raft *r, orc_entry *ents, size_t n) {
  uint64_t last = log_last(&r->log);
  for (size_t i = 0; i < n; i++) {
    ents[i].term = r->term;
    ents[i].index = last + 1 + i;
  }
  log_append(&r->log, ents, n);
  int si = raft_rem_idx(r, r->replica_id);
  if (si < 0) orc_panic("self remote missing");
  orc_remote_try_update(&r->rem[si], log_last(&r->log));
  if (raft_single_node_quorum(r)) raft_try_commit(r);
}

/* toFollowerState / becomeFollower (raft.go:961-999) */
static void raft_to_follower(orc_raft *r, uint64_t term, uint64_t leader,
                             int reset_election) {
  r->state = DRB_FOLLOWER;
  raft_reset(r, term, reset_election);
  raft_set_leader_id(r, leader);
}

/* becomeCandidate (raft.go:1020-1036) */
static void raft_become_candidate(orc_raft *r) {
  if (r->state == DRB_LEADER)
    orc_panic("transitioning to candidate state from leader");
  if (r->state == DRB_NONVOTING) orc_panic("nonVoting is becoming candidate");
  if (r->state == DRB_WITNESS) orc_panic("witness is becoming candidate");
  r->state = DRB_CANDIDATE;
  raft_reset(r, r->term + 1, 1);
  raft_set_leader_id(r, 0);
  r->vote = r->replica_id;
}

/* getPendingConfigChangeCount (raft.go:1380-1398): config change entries
 * in (committed, last] */
static int raft_pending_config_change_count(orc_raft *r) {
  const uint64_t lo = r->log.committed + 1, last = log_last(&r->log);
  if (lo > last) return 0;
  orc_evec ents = {0};
  if (log_get_entries(&r->log, lo, last + 1, UINT64_MAX, &ents))
    orc_panic("failed to get entries");
  int n = 0;
  for (size_t i = 0; i < ents.n; i++)
    if (ents.v[i].type == DRB_ENTRY_CONFIG_CHANGE) n++;
  ev_free(&ents);
  return n;
}

/* becomeLeader (raft.go:1038-1050) + preLeaderPromotionHandleConfigChange
 * (raft.go:1075-1083) */
static void raft_become_leader(orc_raft *r) {
  if (r->state != DRB_LEADER && r->state != DRB_CANDIDATE)
    orc_panic("transitioning to leader state from %u", r->state);
  r->state = DRB_LEADER;
  raft_reset(r, r->term, 1);
  raft_set_leader_id(r, r->replica_id);
  const int pcc = raft_pending_config_change_count(r);
  if (pcc > 1) orc_panic("multiple uncommitted config change entries");
  if (pcc == 1) r->pending_config_change = 1;
  orc_entry e;
  memset(&e, 0, sizeof(e));
  e.type = DRB_ENTRY_APPLICATION;
  raft_append_entries(r, &e, 1);
}

/* handleVoteResp (raft.go:1125-1147) */
static int raft_handle_vote_resp(orc_raft *r, uint64_t from, int rejected) {
  int found = 0;
  for (int i = 0; i < r->nvotes; i++)
    if (r->vote_id[i] == from) found = 1;
  if (!found) {
    r->vote_id[r->nvotes] = from;
    r->vote_ok[r->nvotes] = !rejected;
    r->nvotes++;
  }
  int c = 0;
  for (int i = 0; i < r->nvotes; i++) c += r->vote_ok[i];
  return c;
}

/* campaign (raft.go:1176-1217) */
static void raft_campaign(orc_raft *r) {
  raft_become_candidate(r);
  uint64_t term = r->term;
  raft_handle_vote_resp(r, r->replica_id, 0);
  if (raft_single_node_quorum(r)) {
    raft_become_leader(r);
    return;
  }
  uint64_t hint = 0; /* the transfer target names itself (raft.go:1192) */
  if (r->is_leader_transfer_target) {
    hint = r->replica_id;
    r->is_leader_transfer_target = 0;
  }
  uint64_t index = log_last(&r->log);
  uint64_t last_term;
  if (log_term(&r->log, index, &last_term)) orc_panic("campaign: log error");
  for (int i = 0; i < r->nrem; i++) {  /* votingMembers (raft.go:1202) */
    if (r->rem_id[i] == r->replica_id || r->rem_kind[i] == ORC_NONVOTING)
      continue;
    orc_msg m = new_msg(DRB_MSG_REQUEST_VOTE, r->rem_id[i]);
    m.term = term;
    m.log_index = index;
    m.log_term = last_term;
    m.hint = hint;
    raft_send(r, &m);
  }
}

/* becomePreVoteCandidate (raft.go:1001-1018) */
static void raft_become_pre_vote_candidate(orc_raft *r) {
  if (!r->pre_vote) orc_panic("becomePreVoteCandidate: preVote not enabled");
  if (r->state == DRB_LEADER)
    orc_panic("transitioning to candidate state from leader");
  if (r->state == DRB_NONVOTING) orc_panic("nonVoting is becoming candidate");
  if (r->state == DRB_WITNESS) orc_panic("witness is becoming candidate");
  r->state = DRB_PREVOTE_CANDIDATE;
  raft_reset(r, r->term, 1);
  raft_set_leader_id(r, 0);
}

/* preVoteCampaign (raft.go:1149-1174): RequestPreVote at term + 1, the
 * term itself unchanged */
static void raft_pre_vote_campaign(orc_raft *r) {
  raft_become_pre_vote_candidate(r);
  raft_handle_vote_resp(r, r->replica_id, 0);
  if (raft_single_node_quorum(r)) {
    raft_campaign(r);
    return;
  }
  uint64_t index = log_last(&r->log);
  uint64_t last_term;
  if (log_term(&r->log, index, &last_term))
    orc_panic("preVoteCampaign: log error");
  for (int i = 0; i < r->nrem; i++) {  /* votingMembers (raft.go:1160) */
    if (r->rem_id[i] == r->replica_id || r->rem_kind[i] == ORC_NONVOTING)
      continue;
    orc_msg m = new_msg(DRB_MSG_REQUEST_PREVOTE, r->rem_id[i]);
    m.term = r->term + 1;
    m.log_index = index;
    m.log_term = last_term;
    raft_send(r, &m);
  }
}

/* handleHeartbeatMessage (raft.go:1400-1409) */
static void raft_handle_heartbeat_message(orc_raft *r, const orc_msg *m) {
  log_commit_to(&r->log, m->commit);
  orc_msg resp = new_msg(DRB_MSG_HEARTBEAT_RESP, m->from);
  resp.hint = m->hint;
  resp.hint_high = m->hint_high;
  raft_send(r, &resp);
}

/* handleReplicateMessage (raft.go:1444-1484) */
static void raft_handle_replicate_message(orc_raft *r, const orc_msg *m) {
  orc_msg resp = new_msg(DRB_MSG_REPLICATE_RESP, m->from);
  if (m->log_index < r->log.committed) {
    resp.log_index = r->log.committed;
    raft_send(r, &resp);
    return;
  }
  int ok;
  if (log_match_term(&r->log, m->log_index, m->log_term, &ok))
    orc_panic("handleReplicateMessage: log error");
  if (ok) {
    int appended;
    if (log_try_append(&r->log, m->log_index, m->ents.v, m->ents.n,
                       &appended))
      orc_panic("tryAppend: log error");
    uint64_t last_idx = m->log_index + m->ents.n;
    log_commit_to(&r->log, umin(last_idx, m->commit));
    resp.log_index = last_idx;
  } else {
    resp.reject = 1;
    resp.log_index = m->log_index;
    resp.hint = log_last(&r->log);
  }
  raft_send(r, &resp);
}

/* dropRequestVoteFromHighTermNode (raft.go:1507-1529) */
static int raft_drop_request_vote(orc_raft *r, const orc_msg *m) {
  if (!is_request_vote_message(m->type) || !r->check_quorum ||
      m->term <= r->term)
    return 0;
  if (m->hint == m->from) return 0;
  if (r->state == DRB_LEADER && !r->quiesce &&
      r->election_tick >= r->election_timeout)
    orc_panic("r.electionTick >= r.electionTimeout on leader");
  if (r->leader_id != 0 && r->election_tick < r->election_timeout) return 1;
  return 0;
}

/* onMessageTermNotMatched (raft.go:1540-1590) */
static int raft_term_not_matched(orc_raft *r, const orc_msg *m) {
  if (m->term == 0 || m->term == r->term) return 0;
  if (raft_drop_request_vote(r, m)) return 1;
  if (m->term > r->term) {
    int prevote_higher = m->type == DRB_MSG_REQUEST_PREVOTE ||
                         (m->type == DRB_MSG_REQUEST_PREVOTE_RESP && !m->reject);
    if (!prevote_higher) {
      uint64_t leader = is_leader_message(m->type) ? m->from : 0;
      if (r->state == DRB_NONVOTING || r->state == DRB_WITNESS) {
        /* becomeNonVoting / becomeWitness (raft.go:973-999) */
        raft_reset(r, m->term, 1);
        raft_set_leader_id(r, leader);
      } else if (m->type == DRB_MSG_REQUEST_VOTE) {
        raft_to_follower(r, m->term, leader, 0); /* becomeFollowerKE */
      } else {
        raft_to_follower(r, m->term, leader, 1);
      }
    }
  } else if (m->term < r->term) {
    if (m->type == DRB_MSG_REQUEST_PREVOTE ||
        (is_leader_message(m->type) && (r->check_quorum || r->pre_vote))) {
      orc_msg resp = new_msg(DRB_MSG_NOOP, m->from);
      raft_send(r, &resp);
    }
    return 1;
  }
  return 0;
}

/* hasCommittedEntryAtCurrentTerm (raft.go:1818-1827) */
static int raft_has_committed_at_term(orc_raft *r) {
  if (r->term == 0) orc_panic("not suppose to reach here");
  uint64_t t;
  int err = log_term(&r->log, r->log.committed, &t);
  if (err && err != ORC_ERR_COMPACTED) orc_panic("failed to get term");
  if (err) t = 0;
  return t == r->term;
}

/* addReadyToRead (raft.go:1833-1839) */
static void raft_add_ready(orc_raft *r, uint64_t index, orc_ctx ctx) {
  if (r->nrtr == r->caprtr) {
    r->caprtr = r->caprtr ? r->caprtr * 2 : 4;
    r->rtr = (orc_rtr *)realloc(r->rtr, r->caprtr * sizeof(orc_rtr));
  }
  r->rtr[r->nrtr].index = index;
  r->rtr[r->nrtr].ctx = ctx;
  r->nrtr++;
}

/* reportDroppedReadIndex (raft.go:2294-2307) */
static void raft_report_dropped_ri(orc_raft *r, const orc_msg *m) {
  if (r->ndropped_ri == r->capdropped_ri) {
    r->capdropped_ri = r->capdropped_ri ? r->capdropped_ri * 2 : 4;
    r->dropped_ri =
        (orc_ctx *)realloc(r->dropped_ri, r->capdropped_ri * sizeof(orc_ctx));
  }
  r->dropped_ri[r->ndropped_ri].low = m->hint;
  r->dropped_ri[r->ndropped_ri].high = m->hint_high;
  r->ndropped_ri++;
}

/* leaderHasQuorum (raft.go:395-405): over the voting members */
static int raft_leader_has_quorum(orc_raft *r) {
  int c = 0;
  for (int i = 0; i < r->nrem; i++) {
    if (r->rem_kind[i] == ORC_NONVOTING) continue;
    if (r->rem_id[i] == r->replica_id || r->rem[i].active) {
      c++;
      r->rem[i].active = 0;
    }
  }
  return c >= raft_quorum(r);
}

/* ---- handlers (raft.go:1762-2233) --------------------------------- */
static int raft_handle(orc_raft *r, orc_msg *m);

/* tick / leaderTick / nonLeaderTick / quiescedTick (raft.go:571-656) */
static void raft_tick(orc_raft *r) {
  r->quiesce = 0;
  r->tick_count++;
  /* timeForInMemGC -> inmem.tryResize changes capacity only */
  if (r->state == DRB_LEADER) {
    r->election_tick++;
    int abort_transfer = r->leader_transfer_target != 0 &&
                         r->election_tick >= r->election_timeout;
    if (r->election_tick >= r->election_timeout) {
      r->election_tick = 0;
      if (r->check_quorum) {
        orc_msg cq = new_msg(DRB_MSG_CHECK_QUORUM, 0);
        cq.from = r->replica_id;
        raft_handle(r, &cq);
      }
    }
    if (abort_transfer) r->leader_transfer_target = 0;
    r->heartbeat_tick++;
    if (r->heartbeat_tick >= r->heartbeat_timeout) {
      r->heartbeat_tick = 0;
      orc_msg hb = new_msg(DRB_MSG_LEADER_HEARTBEAT, 0);
      hb.from = r->replica_id;
      raft_handle(r, &hb);
    }
    return;
  }
  r->election_tick++;
  /* a nonVoting or witness replica takes no part in elections (raft.go:
   * 596-600) */
  if (r->state == DRB_NONVOTING || r->state == DRB_WITNESS) return;
  if (r->election_tick >= r->randomized_election_timeout) {
    r->election_tick = 0;
    orc_msg el = new_msg(DRB_MSG_ELECTION, 0);
    el.from = r->replica_id;
    raft_handle(r, &el);
  }
}

static void raft_quiesced_tick(orc_raft *r) {
  if (!r->quiesce) r->quiesce = 1;
  r->election_tick++;
}

/* leaderTransfering / abortLeaderTransfer (raft.go:375-381) */
static int raft_leader_transfering(const orc_raft *r) {
  return r->leader_transfer_target != 0 && r->state == DRB_LEADER;
}

/* sendTimeoutNowMessage (raft.go:873-878) */
static void raft_send_timeout_now(orc_raft *r, uint64_t to) {
  orc_msg m = new_msg(DRB_MSG_TIMEOUT_NOW, to);
  raft_send(r, &m);
}

/* handleLeaderReplicateResp (raft.go:1878-1908) */
static void handle_leader_replicate_resp(orc_raft *r, const orc_msg *m,
                                         orc_remote *rp) {
  rp->active = 1;
  if (!m->reject) {
    int paused = remote_is_paused(rp);
    if (orc_remote_try_update(rp, m->log_index)) {
      orc_remote_responded_to(rp);
      if (raft_try_commit(r))
        raft_broadcast_replicate(r);
      else if (paused)
        raft_send_replicate(r, m->from);
      /* the leadership transfer protocol, p29 of the raft thesis
       * (raft.go:1890-1895): the target caught up */
      if (raft_leader_transfering(r) && m->from == r->leader_transfer_target &&
          log_last(&r->log) == rp->match)
        raft_send_timeout_now(r, r->leader_transfer_target);
    }
  } else {
    if (orc_remote_decrease_to(rp, m->log_index, m->hint)) {
      /* enterRetryState (raft.go:2013-2017) */
      if (rp->state == DRB_REMOTE_REPLICATE) orc_remote_become_retry(rp);
      raft_send_replicate(r, m->from);
    }
  }
}

/* handleReadIndexLeaderConfirmation (raft.go:1955-1974) */
static void handle_ri_confirmation(orc_raft *r, const orc_msg *m) {
  orc_ctx ctx = {m->hint, m->hint_high};
  orc_rstatus ris[64];
  size_t n = ri_confirm(&r->ri, ctx, m->from, raft_quorum(r), ris, 64);
  for (size_t i = 0; i < n; i++) {
    if (ris[i].from == 0 || ris[i].from == r->replica_id) {
      raft_add_ready(r, ris[i].index, ris[i].ctx);
    } else {
      orc_msg resp = new_msg(DRB_MSG_READ_INDEX_RESP, ris[i].from);
      resp.log_index = ris[i].index;
      resp.hint = m->hint;
      resp.hint_high = m->hint_high;
      raft_send(r, &resp);
    }
  }
}

/* handleLeaderHeartbeatResp (raft.go:1910-1923) */
static void handle_leader_heartbeat_resp(orc_raft *r, const orc_msg *m,
                                         orc_remote *rp) {
  rp->active = 1;
  orc_remote_wait_to_retry(rp);
  if (rp->match < log_last(&r->log)) raft_send_replicate(r, m->from);
  if (m->hint != 0) handle_ri_confirmation(r, m);
}

/* handleLeaderReadIndex (raft.go:1842-1876) */
static void handle_leader_read_index(orc_raft *r, const orc_msg *m) {
  orc_ctx ctx = {m->hint, m->hint_high};
  if (raft_is_kind(r, m->from, ORC_WITNESS)) {
    return; /* dropped: a witness node (raft.go:1848-1849) */
  } else if (!raft_single_node_quorum(r)) {
    if (!raft_has_committed_at_term(r)) {
      raft_report_dropped_ri(r, m);
      return;
    }
    ri_add_request(&r->ri, r->log.committed, ctx, m->from);
    raft_broadcast_heartbeat_hint(r, ctx);
  } else {
    raft_add_ready(r, r->log.committed, ctx);
    if (m->from != r->replica_id &&
        raft_is_kind(r, m->from, ORC_NONVOTING)) {  /* raft.go:1863-1872 */
      orc_msg resp = new_msg(DRB_MSG_READ_INDEX_RESP, m->from);
      resp.log_index = r->log.committed;
      resp.hint = m->hint;
      resp.hint_high = m->hint_high;
      resp.commit = m->commit;
      raft_send(r, &resp);
    }
  }
}

/* handleLeaderPropose (raft.go:1794-1815) */
static void handle_leader_propose(orc_raft *r, orc_msg *m) {
  if (raft_leader_transfering(r)) { /* raft.go:1796-1800 */
    r->ndropped_entries += m->ents.n;
    return;
  }
  for (size_t i = 0; i < m->ents.n; i++)
    if (m->ents.v[i].type == DRB_ENTRY_CONFIG_CHANGE) {
      if (r->pending_config_change) {
        /* reportDroppedConfigChange: the entry becomes an empty
         * application entry */
        blob_unref(m->ents.v[i].cmd);
        memset(&m->ents.v[i], 0, sizeof(orc_entry));
        m->ents.v[i].type = DRB_ENTRY_APPLICATION;
      }
      r->pending_config_change = 1; /* setPendingConfigChange */
    }
  raft_append_entries(r, m->ents.v, m->ents.n);
  raft_broadcast_replicate(r);
}

/* handleLeaderTransfer (raft.go:1925-1953) */
static void handle_leader_transfer(orc_raft *r, const orc_msg *m) {
  uint64_t target = m->hint;
  if (target == 0) orc_panic("leader transfer target not set");
  if (raft_leader_transfering(r)) return; /* a transfer is ongoing */
  if (r->replica_id == target) return;    /* pointing to itself */
  int i = raft_rem_idx(r, target);
  if (i < 0 || r->rem_kind[i] != ORC_VOTING) return; /* unknown target */
  r->leader_transfer_target = target;
  r->election_tick = 0;
  /* fast path, or wait for the target to catch up (p29, raft thesis) */
  if (r->rem[i].match == log_last(&r->log))
    raft_send_timeout_now(r, target);
}

/* handleFollowerTimeoutNow (raft.go:2172-2185): the clock moving forward
 * quickly, campaigning without a pre-vote round */
static void handle_follower_timeout_now(orc_raft *r) {
  r->election_tick = r->randomized_election_timeout;
  r->is_leader_transfer_target = 1;
  raft_tick(r);
  r->is_leader_transfer_target = 0;
}

/* handleLeaderCheckQuorum (raft.go:1785-1792) */
static void handle_leader_check_quorum(orc_raft *r) {
  if (!raft_leader_has_quorum(r)) raft_to_follower(r, r->term, 0, 1);
}

/* handleNodeRequestVote (raft.go:1697-1722) */
static void handle_node_request_vote(orc_raft *r, const orc_msg *m) {
  orc_msg resp = new_msg(DRB_MSG_REQUEST_VOTE_RESP, m->from);
  int can_grant = r->vote == 0 || r->vote == m->from || m->term > r->term;
  int utd;
  if (log_up_to_date(&r->log, m->log_index, m->log_term, &utd))
    orc_panic("upToDate: log error");
  if (can_grant && utd) {
    r->election_tick = 0;
    r->vote = m->from;
  } else {
    resp.reject = 1;
  }
  raft_send(r, &resp);
}

/* handleNodeRequestPreVote (raft.go:1670-1695) */
static void handle_node_request_pre_vote(orc_raft *r, const orc_msg *m) {
  orc_msg resp = new_msg(DRB_MSG_REQUEST_PREVOTE_RESP, m->from);
  int utd;
  if (log_up_to_date(&r->log, m->log_index, m->log_term, &utd))
    orc_panic("upToDate: log error");
  if (m->term < r->term) orc_panic("m.term < r.term");
  if (m->term > r->term && utd) {
    resp.term = m->term;
  } else {
    resp.term = r->term;
    resp.reject = 1;
  }
  raft_send(r, &resp);
}

/* handlePreVoteCandidateRequestPreVoteResp (raft.go:2259-2276) */
static void handle_pre_vote_candidate_resp(orc_raft *r, const orc_msg *m) {
  int count = raft_handle_vote_resp(r, m->from, m->reject);
  if (count == raft_quorum(r)) {
    raft_campaign(r);
  } else if (r->nvotes - count == raft_quorum(r)) {
    raft_to_follower(r, r->term, 0, 1);
  }
}

/* handleCandidateRequestVoteResp (raft.go:2235-2253) */
static void handle_candidate_vote_resp(orc_raft *r, const orc_msg *m) {
  int count = raft_handle_vote_resp(r, m->from, m->reject);
  if (count == raft_quorum(r)) {
    raft_become_leader(r);
    raft_broadcast_replicate(r);
  } else if (r->nvotes - count == raft_quorum(r)) {
    raft_to_follower(r, r->term, 0, 1);
  }
}

/* handleNodeElection (raft.go:1632-1668) */
static void handle_node_election(orc_raft *r) {
  if (r->state != DRB_LEADER) {
    if (!r->test_has_config_change_hook && r->log.committed > r->applied)
      return; /* hasConfigChangeToApply (raft.go:1611-1622) */
    if (r->pre_vote && !r->is_leader_transfer_target) {
      raft_pre_vote_campaign(r);
      return;
    }
    raft_campaign(r);
  }
}

/* defaultHandle over the handler table (raft.go:2325-2417), restricted to
 * the follower / candidate / leader states and the message types of this
 * path plus the election used for setup. */
static void raft_dispatch(orc_raft *r, orc_msg *m) {
  uint32_t t = m->type;
  switch (r->state) {
    case DRB_LEADER:
      switch (t) {
        case DRB_MSG_LEADER_HEARTBEAT:
          raft_broadcast_heartbeat(r);
          return;
        case DRB_MSG_CHECK_QUORUM:
          handle_leader_check_quorum(r);
          return;
        case DRB_MSG_PROPOSE:
          handle_leader_propose(r, m);
          return;
        case DRB_MSG_READ_INDEX:
          handle_leader_read_index(r, m);
          return;
        case DRB_MSG_REPLICATE_RESP:
        case DRB_MSG_HEARTBEAT_RESP: {
          int i = raft_rem_idx(r, m->from); /* lw (raft.go:2309-2323) */
          if (i < 0) return;
          if (t == DRB_MSG_REPLICATE_RESP)
            handle_leader_replicate_resp(r, m, &r->rem[i]);
          else
            handle_leader_heartbeat_resp(r, m, &r->rem[i]);
          return;
        }
        case DRB_MSG_ELECTION:
          handle_node_election(r);
          return;
        case DRB_MSG_REQUEST_VOTE:
          handle_node_request_vote(r, m);
          return;
        case DRB_MSG_REQUEST_PREVOTE:
          handle_node_request_pre_vote(r, m);
          return;
        case DRB_MSG_LEADER_TRANSFER:
          handle_leader_transfer(r, m);
          return;
        case DRB_MSG_LOCAL_TICK:
          if (m->reject)
            raft_quiesced_tick(r);
          else
            raft_tick(r);
          return;
        default:
          return;
      }
    case DRB_FOLLOWER:
      switch (t) {
        case DRB_MSG_REPLICATE: /* handleFollowerReplicate (raft.go:2122) */
          r->election_tick = 0;
          raft_set_leader_id(r, m->from);
          raft_handle_replicate_message(r, m);
          return;
        case DRB_MSG_HEARTBEAT: /* handleFollowerHeartbeat (raft.go:2128) */
          r->election_tick = 0;
          raft_set_leader_id(r, m->from);
          raft_handle_heartbeat_message(r, m);
          return;
        case DRB_MSG_READ_INDEX: /* handleFollowerReadIndex (raft.go:2134) */
          if (r->leader_id == 0) {
            raft_report_dropped_ri(r, m);
            return;
          }
          {
            orc_msg fwd = new_msg(DRB_MSG_READ_INDEX, r->leader_id);
            fwd.hint = m->hint;
            fwd.hint_high = m->hint_high;
            fwd.commit = m->commit;
            raft_send(r, &fwd);
          }
          return;
        case DRB_MSG_READ_INDEX_RESP: { /* raft.go:2155-2164 */
          orc_ctx ctx = {m->hint, m->hint_high};
          r->election_tick = 0;
          raft_set_leader_id(r, m->from);
          raft_add_ready(r, m->log_index, ctx);
          return;
        }
        case DRB_MSG_PROPOSE: /* handleFollowerPropose (raft.go:2103-2116) */
          if (r->leader_id == 0) {
            r->ndropped_entries += m->ents.n; /* reportDroppedProposal */
            return;
          }
          {
            orc_msg fwd = *m;
            memset(&fwd.ents, 0, sizeof(fwd.ents));
            ev_copy_range(&fwd.ents, m->ents.v, m->ents.n);
            fwd.to = r->leader_id;
            raft_send(r, &fwd);
          }
          return;
        case DRB_MSG_ELECTION:
          handle_node_election(r);
          return;
        case DRB_MSG_REQUEST_VOTE:
          handle_node_request_vote(r, m);
          return;
        case DRB_MSG_REQUEST_PREVOTE:
          handle_node_request_pre_vote(r, m);
          return;
        case DRB_MSG_LEADER_TRANSFER: /* handleFollowerLeaderTransfer */
          if (r->leader_id == 0) return; /* raft.go:2145-2153 */
          {
            orc_msg fwd = new_msg(DRB_MSG_LEADER_TRANSFER, r->leader_id);
            fwd.hint = m->hint;
            raft_send(r, &fwd);
          }
          return;
        case DRB_MSG_TIMEOUT_NOW:
          handle_follower_timeout_now(r);
          return;
        case DRB_MSG_LOCAL_TICK:
          if (m->reject)
            raft_quiesced_tick(r);
          else
            raft_tick(r);
          return;
        default:
          return;
      }
    case DRB_CANDIDATE:
      switch (t) {
        case DRB_MSG_REPLICATE: /* handleCandidateReplicate (raft.go:2220) */
          raft_to_follower(r, r->term, m->from, 1);
          raft_handle_replicate_message(r, m);
          return;
        case DRB_MSG_HEARTBEAT:
          raft_to_follower(r, r->term, m->from, 1);
          raft_handle_heartbeat_message(r, m);
          return;
        case DRB_MSG_REQUEST_VOTE_RESP:
          handle_candidate_vote_resp(r, m);
          return;
        case DRB_MSG_REQUEST_VOTE:
          handle_node_request_vote(r, m);
          return;
        case DRB_MSG_REQUEST_PREVOTE:
          handle_node_request_pre_vote(r, m);
          return;
        case DRB_MSG_ELECTION:
          handle_node_election(r);
          return;
        case DRB_MSG_READ_INDEX: /* handleCandidateReadIndex (2203) */
          raft_report_dropped_ri(r, m);
          return;
        case DRB_MSG_PROPOSE: /* handleCandidatePropose (2197) */
          r->ndropped_entries += m->ents.n;
          return;
        case DRB_MSG_LOCAL_TICK:
          if (m->reject)
            raft_quiesced_tick(r);
          else
            raft_tick(r);
          return;
        default:
          return;
      }
    case DRB_PREVOTE_CANDIDATE: /* raft.go:2348-2360 */
      switch (t) {
        case DRB_MSG_REPLICATE:
          raft_to_follower(r, r->term, m->from, 1);
          raft_handle_replicate_message(r, m);
          return;
        case DRB_MSG_HEARTBEAT:
          raft_to_follower(r, r->term, m->from, 1);
          raft_handle_heartbeat_message(r, m);
          return;
        case DRB_MSG_REQUEST_PREVOTE_RESP:
          handle_pre_vote_candidate_resp(r, m);
          return;
        case DRB_MSG_REQUEST_VOTE:
          handle_node_request_vote(r, m);
          return;
        case DRB_MSG_REQUEST_PREVOTE:
          handle_node_request_pre_vote(r, m);
          return;
        case DRB_MSG_ELECTION:
          handle_node_election(r);
          return;
        case DRB_MSG_READ_INDEX:
          raft_report_dropped_ri(r, m);
          return;
        case DRB_MSG_PROPOSE:
          r->ndropped_entries += m->ents.n;
          return;
        case DRB_MSG_LOCAL_TICK:
          if (m->reject)
            raft_quiesced_tick(r);
          else
            raft_tick(r);
          return;
        default:
          return;
      }
    case DRB_NONVOTING: /* raft.go:2396-2407, re-routed to the follower's */
    case DRB_WITNESS:   /* raft.go:2409-2416 */
      switch (t) {
        case DRB_MSG_REPLICATE: /* handleNonVoting/WitnessReplicate */
          r->election_tick = 0;
          raft_set_leader_id(r, m->from);
          raft_handle_replicate_message(r, m);
          return;
        case DRB_MSG_HEARTBEAT:
          r->election_tick = 0;
          raft_set_leader_id(r, m->from);
          raft_handle_heartbeat_message(r, m);
          return;
        case DRB_MSG_REQUEST_VOTE:
          handle_node_request_vote(r, m);
          return;
        case DRB_MSG_REQUEST_PREVOTE:
          handle_node_request_pre_vote(r, m);
          return;
        case DRB_MSG_LOCAL_TICK:
          if (m->reject)
            raft_quiesced_tick(r);
          else
            raft_tick(r);
          return;
        default:
          break;
      }
      if (r->state == DRB_WITNESS) return; /* no other handlers */
      switch (t) {
        case DRB_MSG_PROPOSE: /* handleNonVotingPropose (raft.go:2071) */
          if (r->leader_id == 0) {
            r->ndropped_entries += m->ents.n;
            return;
          }
          {
            orc_msg fwd = *m;
            memset(&fwd.ents, 0, sizeof(fwd.ents));
            ev_copy_range(&fwd.ents, m->ents.v, m->ents.n);
            fwd.to = r->leader_id;
            raft_send(r, &fwd);
          }
          return;
        case DRB_MSG_READ_INDEX: /* handleNonVotingReadIndex (raft.go:2075) */
          if (r->leader_id == 0) {
            raft_report_dropped_ri(r, m);
            return;
          }
          {
            orc_msg fwd = new_msg(DRB_MSG_READ_INDEX, r->leader_id);
            fwd.hint = m->hint;
            fwd.hint_high = m->hint_high;
            fwd.commit = m->commit;
            raft_send(r, &fwd);
          }
          return;
        case DRB_MSG_READ_INDEX_RESP: { /* raft.go:2079-2085 */
          orc_ctx ctx = {m->hint, m->hint_high};
          r->election_tick = 0;
          raft_set_leader_id(r, m->from);
          raft_add_ready(r, m->log_index, ctx);
          return;
        }
        default:
          return;
      }
    default:
      orc_panic("raft state %u not on this path", r->state);
  }
}

/* Handle (raft.go:1596-1609) */
static int raft_handle(orc_raft *r, orc_msg *m) {
  const int pv = m->type == DRB_MSG_REQUEST_PREVOTE ||
                 m->type == DRB_MSG_REQUEST_PREVOTE_RESP;
  if (pv && !r->pre_vote) /* inconsistentRaftConfig (raft.go:1592-1594) */
    orc_panic("received preVote message when preVote is not enabled");
  if (!raft_term_not_matched(r, m)) {
    if (!pv && m->term != 0 && r->term != m->term)
      orc_panic("mismatched term found");
    raft_dispatch(r, m);
  }
  return 0;
}

int raft_handle_msg(orc_raft *r, orc_msg *m) { return raft_handle(r, m); }
void raft_tick_public(orc_raft *r, int quiesced) {
  orc_msg t = new_msg(DRB_MSG_LOCAL_TICK, 0);
  t.reject = quiesced;
  raft_handle(r, &t);
}

/* Peer.Handle (peer.go:184-195) */
static int is_local_message_type(uint32_t t) {
  return t == DRB_MSG_ELECTION || t == DRB_MSG_LEADER_HEARTBEAT ||
         t == DRB_MSG_UNREACHABLE || t == DRB_MSG_SNAPSHOT_STATUS ||
         t == DRB_MSG_CHECK_QUORUM || t == DRB_MSG_LOCAL_TICK ||
         t == DRB_MSG_BATCHED_READ_INDEX;
}
static int is_response_message_type(uint32_t t) {
  return t == DRB_MSG_REPLICATE_RESP || t == DRB_MSG_REQUEST_VOTE_RESP ||
         t == DRB_MSG_HEARTBEAT_RESP || t == DRB_MSG_READ_INDEX_RESP ||
         t == DRB_MSG_UNREACHABLE || t == DRB_MSG_SNAPSHOT_STATUS ||
         t == DRB_MSG_LEADER_TRANSFER;
}

void peer_handle(orc_raft *r, orc_msg *m) {
  if (is_local_message_type(m->type)) orc_panic("local message sent to Step");
  if (raft_rem_idx(r, m->from) >= 0 || !is_response_message_type(m->type))
    raft_handle(r, m);
}

/* newRaft (raft.go:241-297): no membership in the logdb on this path, so
 * remotes start empty; loadState (raft.go:446-454); becomeFollower. */
orc_raft *raft_new(uint64_t shard, uint64_t id, uint64_t election,
                   uint64_t heartbeat, int check_quorum, orc_logdb *db,
                   uint64_t seed) {
  orc_raft *r = (orc_raft *)calloc(1, sizeof(orc_raft));
  r->shard_id = shard;
  r->replica_id = id;
  r->leader_id = 0;
  r->election_timeout = election;
  r->heartbeat_timeout = heartbeat;
  r->check_quorum = check_quorum;
  r->rng = seed;
  log_init(&r->log, db);
  raft_reset_matched(r);
  if (db->st_term || db->st_vote || db->st_commit) {
    if (db->st_commit < r->log.committed ||
        db->st_commit > log_last(&r->log))
      orc_panic("got out of range state");
    r->log.committed = db->st_commit;
    r->term = db->st_term;
    r->vote = db->st_vote;
  }
  raft_to_follower(r, r->term, 0, 1);
  return r;
}

/* setTestPeers / newTestRaft (raft.go:299-305, raft_etcd_test.go:3071) */
void raft_set_test_peers(orc_raft *r, const uint64_t *peers, int npeers) {
  if (r->nrem == 0)
    for (int i = 0; i < npeers; i++) raft_set_remote(r, peers[i], 0, 1);
}

/* addNode (raft.go:1236-1258) for a replica not yet known */
void raft_add_node(orc_raft *r, uint64_t id) {
  r->pending_config_change = 0;
  if (raft_rem_idx(r, id) >= 0) return;
  raft_set_remote(r, id, 0, log_last(&r->log) + 1);
}

/* bootstrap (peer.go:404-428): one ConfigChangeEntry per member at term 1,
 * committed; cmd bytes are supplied by the caller (pb.ConfigChange
 * encoding, see codec_oracle.c). */
void raft_bootstrap(orc_raft *r, const uint64_t *ids, int n,
                    orc_blob *const *cmds) {
  orc_entry ents[ORC_MAX_PEERS];
  memset(ents, 0, sizeof(ents));
  for (int i = 0; i < n; i++) {
    ents[i].type = DRB_ENTRY_CONFIG_CHANGE;
    ents[i].term = 1;
    ents[i].index = (uint64_t)i + 1;
    ents[i].cmd = cmds ? cmds[i] : NULL;
  }
  log_append(&r->log, ents, (size_t)n);
  r->log.committed = (uint64_t)n;
  for (int i = 0; i < n; i++) raft_add_node(r, ids[i]);
}

void raft_free(orc_raft *r) {
  if (!r) return;
  log_free(&r->log);
  free(r->ri.q);
  mv_free(&r->msgs);
  free(r->rtr);
  free(r->dropped_ri);
  free(r);
}

/* ---- public KAT API -------------------------------------------------- */
static orc_msg msg_from_view(const drb_message *v, const drb_entry *ents,
                             const uint8_t *pool) {
  orc_msg m;
  memset(&m, 0, sizeof(m));
  m.type = v->type;
  m.reject = v->reject;
  m.to = v->to;
  m.from = v->from;
  m.shard_id = v->shard_id;
  m.term = v->term;
  m.log_term = v->log_term;
  m.log_index = v->log_index;
  m.commit = v->commit;
  m.hint = v->hint;
  m.hint_high = v->hint_high;
  for (uint64_t i = 0; i < v->n_entries; i++) {
    orc_entry e = entry_from_view(&ents[v->entries_off + i], pool);
    ev_push(&m.ents, &e);
    blob_unref(e.cmd);
  }
  return m;
}

orc_msg orc_msg_from_view(const drb_message *v, const drb_entry *ents,
                          const uint8_t *pool) {
  return msg_from_view(v, ents, pool);
}

int msg_to_view(const orc_msg *m, drb_message *out, drb_entry *ents,
                size_t ent_cap, size_t *ent_used, uint8_t *pool,
                size_t pool_cap, size_t *pool_used) {
  memset(out, 0, sizeof(*out));
  out->type = m->type;
  out->reject = m->reject;
  out->to = m->to;
  out->from = m->from;
  out->shard_id = m->shard_id;
  out->term = m->term;
  out->log_term = m->log_term;
  out->log_index = m->log_index;
  out->commit = m->commit;
  out->hint = m->hint;
  out->hint_high = m->hint_high;
  out->n_entries = m->ents.n;
  out->entries_off = *ent_used;
  if (*ent_used + m->ents.n > ent_cap) return -1;
  for (size_t i = 0; i < m->ents.n; i++)
    if (entry_to_view(&m->ents.v[i], &ents[(*ent_used)++], pool, pool_cap,
                      pool_used))
      return -1;
  return 0;
}

orc_raft *orc_raft_new_test(uint64_t id, const uint64_t *peers, int npeers,
                            uint64_t election, uint64_t heartbeat,
                            orc_logdb *db) {
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    return NULL;
  }
  orc_raft *r =
      raft_new(0, id, election, heartbeat, 0, db, 0x5EEDD8B0ull ^ id);
  raft_set_test_peers(r, peers, npeers);
  r->test_has_config_change_hook = 1;
  orc_jb = prev;
  return r;
}

void orc_raft_free(orc_raft *r) { raft_free(r); }

int orc_raft_handle(orc_raft *r, const drb_message *m, const drb_entry *ents,
                    const uint8_t *pool) {
  orc_msg mm = msg_from_view(m, ents, pool);
  ORC_TRY(-1);
  raft_handle(r, &mm);
  ORC_END;
  msg_free(&mm);
  return 0;
}

int orc_raft_peer_handle(orc_raft *r, const drb_message *m,
                         const drb_entry *ents, const uint8_t *pool) {
  orc_msg mm = msg_from_view(m, ents, pool);
  ORC_TRY(-1);
  peer_handle(r, &mm);
  ORC_END;
  msg_free(&mm);
  return 0;
}

int orc_raft_become_follower(orc_raft *r, uint64_t term, uint64_t leader) {
  ORC_TRY(-1);
  raft_to_follower(r, term, leader, 1);
  ORC_END;
  return 0;
}

int orc_raft_become_candidate(orc_raft *r) {
  ORC_TRY(-1);
  raft_become_candidate(r);
  ORC_END;
  return 0;
}

int orc_raft_become_leader(orc_raft *r) {
  ORC_TRY(-1);
  raft_become_leader(r);
  ORC_END;
  return 0;
}

int orc_raft_load_state(orc_raft *r, uint64_t term, uint64_t vote,
                        uint64_t commit) {
  ORC_TRY(-1);
  if (commit < r->log.committed || commit > log_last(&r->log))
    orc_panic("got out of range state, st.commit %llu",
              (unsigned long long)commit);
  r->log.committed = commit;
  r->term = term;
  r->vote = vote;
  ORC_END;
  return 0;
}

int orc_raft_broadcast_replicate(orc_raft *r) {
  ORC_TRY(-1);
  raft_broadcast_replicate(r);
  ORC_END;
  return 0;
}

int orc_raft_broadcast_heartbeat(orc_raft *r) {
  ORC_TRY(-1);
  raft_broadcast_heartbeat(r);
  ORC_END;
  return 0;
}

int orc_raft_try_commit(orc_raft *r) {
  ORC_TRY(-1);
  int ok = raft_try_commit(r);
  ORC_END;
  return ok;
}

int orc_raft_tick(orc_raft *r) {
  ORC_TRY(-1);
  raft_tick(r);
  ORC_END;
  return 0;
}

int orc_raft_campaign(orc_raft *r) {
  ORC_TRY(-1);
  raft_campaign(r);
  ORC_END;
  return 0;
}

/* the test harness's r.checkQuorum = ... (raft_etcd_test.go) */
void orc_raft_set_check_quorum(orc_raft *r, int on) { r->check_quorum = on; }
void orc_raft_set_pre_vote(orc_raft *r, int on) { r->pre_vote = on; }

void orc_raft_set_randomized_election_timeout(orc_raft *r, uint64_t v) {
  r->randomized_election_timeout = v;
}

long orc_raft_read_messages(orc_raft *r, drb_message *out, size_t cap,
                            drb_entry *ents, size_t ent_cap, uint8_t *pool,
                            size_t pool_cap) {
  size_t n = r->msgs.n;
  if (n > cap) return (long)n;
  size_t eu = 0, pu = 0;
  for (size_t i = 0; i < n; i++)
    if (msg_to_view(&r->msgs.v[i], &out[i], ents, ent_cap, &eu, pool, pool_cap,
                    &pu))
      return -2;
  mv_clear(&r->msgs);
  return (long)n;
}

long orc_raft_log_entries(orc_raft *r, int which, drb_entry *out, size_t cap,
                          uint8_t *pool, size_t pool_cap) {
  orc_evec v = {0};
  long ret = 0;
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    ev_free(&v);
    return -1;
  }
  if (which == 0) {
    if (log_entries_to_apply(&r->log, &v)) ret = -3;
  } else if (which == 1) {
    size_t n;
    const orc_entry *e = im_entries_to_save(&r->log.im, &n);
    ev_copy_range(&v, e, n);
  } else {
    if (log_entries(&r->log, log_first(&r->log), UINT64_MAX, &v)) ret = -3;
  }
  orc_jb = prev;
  if (ret == 0) {
    if (v.n > cap) {
      ret = (long)v.n;
    } else {
      size_t pu = 0;
      for (size_t i = 0; i < v.n; i++)
        if (entry_to_view(&v.v[i], &out[i], pool, pool_cap, &pu)) ret = -2;
      if (ret == 0) ret = (long)v.n;
    }
  }
  ev_free(&v);
  return ret;
}

int orc_raft_log_term(orc_raft *r, uint64_t index, uint64_t *term) {
  ORC_TRY(-1);
  int err = log_term(&r->log, index, term);
  ORC_END;
  return err;
}

void orc_raft_info(orc_raft *r, drb_replica_state *st) {
  memset(st, 0, sizeof(*st));
  st->shard_id = r->shard_id;
  st->replica_id = r->replica_id;
  st->term = r->term;
  st->vote = r->vote;
  st->leader_id = r->leader_id;
  st->applied = r->applied;
  st->election_tick = r->election_tick;
  st->heartbeat_tick = r->heartbeat_tick;
  st->randomized_election_timeout = r->randomized_election_timeout;
  st->tick_count = r->tick_count;
  st->committed = r->log.committed;
  st->processed = r->log.processed;
  st->last_index = log_last(&r->log);
  st->marker_index = r->log.im.marker_index;
  st->saved_to = r->log.im.saved_to;
  st->applied_to_index = r->log.im.applied_to_index;
  st->applied_to_term = r->log.im.applied_to_term;
  st->role = r->state;
  st->rng = r->rng;
  st->transfer = (uint32_t)r->leader_transfer_target;
  /* raft.votes as answered | granted << 8, bit (ID - 1) */
  for (int i = 0; i < r->nvotes; i++) {
    const uint64_t id = r->vote_id[i];
    if (id < 1 || id > 8) continue;
    st->votes |= 1u << (id - 1);
    if (r->vote_ok[i]) st->votes |= 1u << (8 + id - 1);
  }
  for (int i = 0; i < r->nrem && i < DRB_MAX_REPLICAS; i++) {
    uint64_t id = r->rem_id[i];
    if (id == 0 || id > DRB_MAX_REPLICAS) continue;
    drb_remote_state *d = &st->remotes[id - 1];
    d->match = r->rem[i].match;
    d->next = r->rem[i].next;
    d->state = r->rem[i].state;
    d->active = (uint32_t)r->rem[i].active;
  }
  st->ri_count = (uint32_t)(r->ri.n < DRB_RI_DEPTH ? r->ri.n : DRB_RI_DEPTH);
  for (uint32_t i = 0; i < st->ri_count; i++) {
    st->ri[i].ctx_low = r->ri.q[i].ctx.low;
    st->ri[i].ctx_high = r->ri.q[i].ctx.high;
    st->ri[i].index = r->ri.q[i].index;
    st->ri[i].from = r->ri.q[i].from;
    uint32_t mask = 0;
    for (int k = 0; k < r->ri.q[i].nconfirmed; k++) {
      uint64_t id = r->ri.q[i].confirmed[k];
      if (id >= 1 && id <= DRB_MAX_REPLICAS) mask |= 1u << (id - 1);
    }
    st->ri[i].confirmed = mask;
  }
}

int orc_raft_remote(orc_raft *r, uint64_t id, orc_remote *out) {
  int i = raft_rem_idx(r, id);
  if (i < 0) return -1;
  *out = r->rem[i];
  return 0;
}

int orc_raft_set_remote(orc_raft *r, uint64_t id, const orc_remote *in) {
  int i = raft_rem_idx(r, id);
  if (i < 0) return -1;
  r->rem[i] = *in;
  return 0;
}

size_t orc_raft_ready_to_read(orc_raft *r, uint64_t *index, uint64_t *low,
                              uint64_t *high, size_t cap) {
  size_t n = r->nrtr < cap ? r->nrtr : cap;
  for (size_t i = 0; i < n; i++) {
    index[i] = r->rtr[i].index;
    low[i] = r->rtr[i].ctx.low;
    high[i] = r->rtr[i].ctx.high;
  }
  return r->nrtr;
}

size_t orc_raft_dropped_read_indexes(orc_raft *r) { return r->ndropped_ri; }

int orc_log_commit_to(orc_raft *r, uint64_t index) {
  ORC_TRY(-1);
  log_commit_to(&r->log, index);
  ORC_END;
  return 0;
}

int orc_log_try_commit(orc_raft *r, uint64_t index, uint64_t term) {
  ORC_TRY(-1);
  int ok;
  if (log_try_commit(&r->log, index, term, &ok)) ok = -2;
  ORC_END;
  return ok;
}

int orc_log_match_term(orc_raft *r, uint64_t index, uint64_t term) {
  ORC_TRY(-1);
  int ok;
  if (log_match_term(&r->log, index, term, &ok)) ok = -2;
  ORC_END;
  return ok;
}

int orc_log_up_to_date(orc_raft *r, uint64_t index, uint64_t term) {
  ORC_TRY(-1);
  int ok;
  if (log_up_to_date(&r->log, index, term, &ok)) ok = -2;
  ORC_END;
  return ok;
}

long orc_log_conflict_index(orc_raft *r, const drb_entry *ents, size_t n) {
  orc_evec tmp = {0};
  for (size_t i = 0; i < n; i++) {
    orc_entry e = entry_from_view(&ents[i], NULL);
    ev_push(&tmp, &e);
  }
  long ret;
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    ev_free(&tmp);
    return -1;
  }
  uint64_t ci;
  ret = log_conflict_index(&r->log, tmp.v, tmp.n, &ci) ? -2 : (long)ci;
  orc_jb = prev;
  ev_free(&tmp);
  return ret;
}

static int views_to_evec(const drb_entry *ents, size_t n, const uint8_t *pool,
                         orc_evec *out) {
  for (size_t i = 0; i < n; i++) {
    orc_entry e = entry_from_view(&ents[i], pool);
    ev_push(out, &e);
    blob_unref(e.cmd);
  }
  return 0;
}

int orc_log_try_append(orc_raft *r, uint64_t index, const drb_entry *ents,
                       size_t n, const uint8_t *pool) {
  orc_evec tmp = {0};
  views_to_evec(ents, n, pool, &tmp);
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    ev_free(&tmp);
    return -1;
  }
  int appended = 0;
  int err = log_try_append(&r->log, index, tmp.v, tmp.n, &appended);
  orc_jb = prev;
  ev_free(&tmp);
  return err ? -2 : appended;
}

int orc_log_append(orc_raft *r, const drb_entry *ents, size_t n,
                   const uint8_t *pool) {
  orc_evec tmp = {0};
  views_to_evec(ents, n, pool, &tmp);
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    ev_free(&tmp);
    return -1;
  }
  log_append(&r->log, tmp.v, tmp.n);
  orc_jb = prev;
  ev_free(&tmp);
  return 0;
}

int orc_log_commit_update(orc_raft *r, uint64_t stable_log_to,
                          uint64_t stable_log_term, uint64_t processed,
                          uint64_t last_applied) {
  ORC_TRY(-1);
  log_commit_update(&r->log, stable_log_to, stable_log_term, processed,
                    last_applied);
  ORC_END;
  return 0;
}

/* makeReplicateMessage with an explicit maxSize (raft_test.go:1578-1611).
 * Returns the entry count; -1 panic, -2 log error, -3 out of capacity. */
long orc_raft_make_replicate(orc_raft *r, uint64_t to, uint64_t next,
                             uint64_t max_size, drb_message *out,
                             drb_entry *ents, size_t ent_cap, uint8_t *pool,
                             size_t pool_cap) {
  ORC_TRY(-1);
  orc_msg m;
  long rc;
  if (raft_make_replicate(r, to, next, max_size, &m)) {
    rc = -2;
  } else {
    size_t eu = 0, pu = 0;
    rc = msg_to_view(&m, out, ents, ent_cap, &eu, pool, pool_cap, &pu)
             ? -3
             : (long)m.ents.n;
    msg_free(&m);
  }
  ORC_END;
  return rc;
}

/* raft.appendEntries (raft.go:944-955) */
int orc_raft_append_entries(orc_raft *r, const drb_entry *ents, size_t n,
                            const uint8_t *pool) {
  orc_evec tmp = {0};
  views_to_evec(ents, n, pool, &tmp);
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    ev_free(&tmp);
    return -1;
  }
  raft_append_entries(r, tmp.v, tmp.n);
  orc_jb = prev;
  ev_free(&tmp);
  return 0;
}

/* broadcastHeartbeatMessageWithHint (raft.go:859-867) */
int orc_raft_broadcast_heartbeat_hint(orc_raft *r, uint64_t low,
                                      uint64_t high) {
  ORC_TRY(-1);
  orc_ctx ctx = {low, high};
  raft_broadcast_heartbeat_hint(r, ctx);
  ORC_END;
  return 0;
}

/* hasCommittedEntryAtCurrentTerm (raft.go:1818-1827) */
int orc_raft_has_committed_entry_at_current_term(orc_raft *r) {
  ORC_TRY(-1);
  int ok = raft_has_committed_at_term(r);
  ORC_END;
  return ok;
}

/* readIndex.pending / queue sizes: one queue in this restatement, so both
 * lengths are the same (readindex.go:32-36) */
size_t orc_raft_read_index_len(orc_raft *r) { return r->ri.n; }

/* ---- inMemory KAT hooks (inmemory_test.go:260-548) ------------------ */
/* restore (inmemory.go:232-243); the snapshot record itself is not kept */
static void im_restore(orc_inmem *im, uint64_t ss_index, uint64_t ss_term) {
  im->marker_index = ss_index + 1;
  im->applied_to_index = ss_index;
  im->applied_to_term = ss_term;
  im->shrunk = 0;
  ev_truncate(&im->ents, 0);
  im->saved_to = ss_index;
}

orc_inmem *orc_inmem_new(uint64_t marker_index, const drb_entry *ents,
                         size_t n, uint64_t saved_to, int shrunk) {
  orc_inmem *im = (orc_inmem *)calloc(1, sizeof(orc_inmem));
  im->marker_index = marker_index;
  im->saved_to = saved_to;
  im->shrunk = shrunk;
  views_to_evec(ents, n, NULL, &im->ents);
  return im;
}

void orc_inmem_free(orc_inmem *im) {
  if (!im) return;
  ev_free(&im->ents);
  free(im);
}

int orc_inmem_merge(orc_inmem *im, const drb_entry *ents, size_t n) {
  orc_evec tmp = {0};
  views_to_evec(ents, n, NULL, &tmp);
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    ev_free(&tmp);
    return -1;
  }
  im_merge(im, tmp.v, tmp.n);
  orc_jb = prev;
  ev_free(&tmp);
  return 0;
}

int orc_inmem_saved_log_to(orc_inmem *im, uint64_t index, uint64_t term) {
  ORC_TRY(-1);
  im_saved_log_to(im, index, term);
  ORC_END;
  return 0;
}

int orc_inmem_applied_log_to(orc_inmem *im, uint64_t index) {
  ORC_TRY(-1);
  im_applied_log_to(im, index);
  ORC_END;
  return 0;
}

void orc_inmem_restore(orc_inmem *im, uint64_t ss_index, uint64_t ss_term) {
  im_restore(im, ss_index, ss_term);
}

/* entriesToSave: count, first index in *first (0 when none) */
long orc_inmem_entries_to_save(orc_inmem *im, uint64_t *first) {
  size_t n;
  const orc_entry *e = im_entries_to_save(im, &n);
  *first = n ? e[0].index : 0;
  return (long)n;
}

/* getLastIndex / getTerm: 1 ok, 0 not found, -1 panic */
int orc_inmem_last_index(orc_inmem *im, uint64_t *idx) {
  return im_last_index(im, idx);
}

int orc_inmem_get_term(orc_inmem *im, uint64_t index, uint64_t *term) {
  ORC_TRY(-1);
  int ok = im_get_term(im, index, term);
  ORC_END;
  return ok;
}

/* marker index, savedTo, shrunk, len(entries), entries[0].Index */
void orc_inmem_info(orc_inmem *im, uint64_t *out5) {
  out5[0] = im->marker_index;
  out5[1] = im->saved_to;
  out5[2] = (uint64_t)im->shrunk;
  out5[3] = im->ents.n;
  out5[4] = im->ents.n ? im->ents.v[0].index : 0;
}

/* helpers used by node_oracle.c */
const orc_entry *log_entries_to_save(const orc_log *l, size_t *n) {
  return im_entries_to_save(&l->im, n);
}
void raft_clear_msgs(orc_raft *r) { mv_clear(&r->msgs); }
void raft_become_follower(orc_raft *r, uint64_t term, uint64_t leader) {
  raft_to_follower(r, term, leader, 1);
}

/* newNetworkWithConfig for a *raft peer (raft_etcd_test.go:2931-2954):
 * replicaID = id, every address a fresh remote, then reset(term, true). */
/* newNetworkWithConfig for a *raft (raft_etcd_test.go:2932-2957): the
 * remotes become ids 1..n, each keeping the kind it had (nonVoting,
 * witness, else voting) */
int orc_raft_network_reset(orc_raft *r, uint64_t id, const uint64_t *ids,
                           int n) {
  ORC_TRY(-1);
  uint8_t kind[ORC_MAX_PEERS];
  for (int i = 0; i < n; i++) {
    const int k = raft_rem_idx(r, ids[i]);
    kind[i] = k >= 0 ? r->rem_kind[k] : ORC_VOTING;
  }
  r->replica_id = id;
  r->nrem = 0;
  for (int i = 0; i < n; i++) {
    raft_set_remote(r, ids[i], 0, 0);
    r->rem_kind[raft_rem_idx(r, ids[i])] = kind[i];
  }
  raft_reset(r, r->term, 1);
  ORC_END;
  return 0;
}

/* newTestNonVoting / newTestWitness (raft_etcd_test.go:3099-3140): the
 * raft starts as a nonVoting (witness) with the given remotes and
 * nonVotings (witnesses) */
orc_raft *orc_raft_new_test_kind(uint64_t id, const uint64_t *peers,
                                 int npeers, const uint64_t *others,
                                 int nothers, int kind, uint64_t election,
                                 uint64_t heartbeat, orc_logdb *db) {
  orc_raft *r = orc_raft_new_test(id, peers, npeers, election, heartbeat, db);
  if (!r) return NULL;
  r->state = kind == ORC_NONVOTING ? DRB_NONVOTING : DRB_WITNESS;
  for (int i = 0; i < nothers; i++) {
    raft_set_remote(r, others[i], 0, 1);
    r->rem_kind[raft_rem_idx(r, others[i])] = (uint8_t)kind;
  }
  return r;
}

/* addNode / addNonVoting / addWitness (raft.go:1236-1282) */
int orc_raft_add_member(orc_raft *r, uint64_t id, int kind) {
  ORC_TRY(-1);
  r->pending_config_change = 0;  /* clearPendingConfigChange */
  const int i = raft_rem_idx(r, id);
  if (kind == ORC_VOTING) {
    if (id == r->replica_id && r->state == DRB_WITNESS)
      orc_panic("is witness");
    if (i >= 0 && r->rem_kind[i] == ORC_VOTING) {
      /* already a voting member */
    } else if (i >= 0 && r->rem_kind[i] == ORC_NONVOTING) {
      /* promoting to full member with inherited progress info */
      r->rem_kind[i] = ORC_VOTING;
      if (id == r->replica_id) {  /* local peer promoted: becomeFollower */
        r->state = DRB_FOLLOWER;
        raft_reset(r, r->term, 1);
        raft_set_leader_id(r, r->leader_id);
      }
    } else if (i >= 0) {
      orc_panic("could not promote witness to full member");
    } else {
      raft_set_remote(r, id, 0, log_last(&r->log) + 1);
    }
  } else {
    if (id == r->replica_id &&
        r->state != (kind == ORC_NONVOTING ? DRB_NONVOTING : DRB_WITNESS))
      orc_panic("is not a %s", kind == ORC_NONVOTING ? "nonVoting" : "witness");
    if (i < 0 || r->rem_kind[i] != kind) {
      raft_set_remote(r, id, 0, log_last(&r->log) + 1);
      r->rem_kind[raft_rem_idx(r, id)] = (uint8_t)kind;
    }
  }
  ORC_END;
  return 0;
}

int orc_raft_remote_kind(orc_raft *r, uint64_t id) {
  const int i = raft_rem_idx(r, id);
  return i < 0 ? -1 : r->rem_kind[i];
}

/* ---- election KAT hooks (raft_etcd_test.go, raft_test.go) ------------- */
/* the raft fields the reference's tests assign directly (sm.state = ...,
 * r.term = ..., r.electionTick = ..., r.log.committed = ...,
 * r.hasNotAppliedConfigChange = nil) */
int orc_raft_poke(orc_raft *r, int field, uint64_t v) {
  switch (field) {
    case ORC_POKE_STATE: r->state = (uint32_t)v; break;
    case ORC_POKE_TERM: r->term = v; break;
    case ORC_POKE_VOTE: r->vote = v; break;
    case ORC_POKE_ELECTION_TICK: r->election_tick = v; break;
    case ORC_POKE_ELECTION_TIMEOUT: r->election_timeout = v; break;
    case ORC_POKE_COMMITTED: r->log.committed = v; break;
    case ORC_POKE_APPLIED: r->applied = v; break;
    case ORC_POKE_CONFIG_CHANGE_HOOK: r->test_has_config_change_hook = (int)v;
      break;
    /* abortLeaderTransfer (raft.go:379-381) is a poke of 0 */
    case ORC_POKE_LEADER_TRANSFER_TARGET: r->leader_transfer_target = v; break;
    case ORC_POKE_IS_LEADER_TRANSFER_TARGET:
      r->is_leader_transfer_target = (int)v;
      break;
    default: return -1;
  }
  return 0;
}

uint64_t orc_raft_peek(orc_raft *r, int field) {
  switch (field) {
    case ORC_POKE_STATE: return r->state;
    case ORC_POKE_TERM: return r->term;
    case ORC_POKE_VOTE: return r->vote;
    case ORC_POKE_ELECTION_TICK: return r->election_tick;
    case ORC_POKE_ELECTION_TIMEOUT: return r->election_timeout;
    case ORC_POKE_COMMITTED: return r->log.committed;
    case ORC_POKE_APPLIED: return r->applied;
    case ORC_POKE_CONFIG_CHANGE_HOOK: return (uint64_t)r->test_has_config_change_hook;
    case ORC_POKE_LEADER_TRANSFER_TARGET: return r->leader_transfer_target;
    case ORC_POKE_IS_LEADER_TRANSFER_TARGET:
      return (uint64_t)r->is_leader_transfer_target;
    default: return ~0ull;
  }
}

/* reset(term, true) (raft.go:1052-1073), as entsWithConfig /
 * votedWithConfig call it (raft_etcd_test.go:2865-2893) */
int orc_raft_reset(orc_raft *r, uint64_t term) {
  ORC_TRY(-1);
  raft_reset(r, term, 1);
  ORC_END;
  return 0;
}

int orc_raft_become_pre_vote_candidate(orc_raft *r) {
  ORC_TRY(-1);
  raft_become_pre_vote_candidate(r);
  ORC_END;
  return 0;
}

/* setRandomizedElectionTimeout (raft.go:658-661) + timeForElection
 * (raft.go:602-604): TestPastElectionTimeout draws the timeout and asks */
int orc_raft_draw_timeout_time_for_election(orc_raft *r) {
  raft_set_rand_timeout(r);
  return r->election_tick >= r->randomized_election_timeout;
}

/* onMessageTermNotMatched (raft.go:1540-1590) alone: 1 when the message is
 * dropped there */
int orc_raft_term_not_matched(orc_raft *r, const drb_message *m,
                              const drb_entry *ents, const uint8_t *pool) {
  orc_msg mm = msg_from_view(m, ents, pool);
  ORC_TRY(-1);
  int rc = raft_term_not_matched(r, &mm);
  ORC_END;
  msg_free(&mm);
  return rc;
}
