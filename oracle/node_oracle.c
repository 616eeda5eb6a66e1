/*
 * node_oracle.c -- CPU restatement of the node-level step round, the rsm
 * apply path and the KVTest state machine.  TEST INFRASTRUCTURE ONLY.
 *
 *   node.handleEvents            node.go:1161-1223
 *   node.handleReadIndex         node.go:1296-1307
 *   node.handleReceivedMessages  node.go:1347-1377 (+ handleMessage 1379)
 *   node.handleProposals         node.go:1275-1294
 *   node.tick                    node.go:1562-1579
 *   node.getUpdate               node.go:1025-1042
 *   Peer.HasUpdate/GetUpdate     peer.go:198-289, getUpdate 333-379,
 *                                getUpdateCommit 432-449
 *   Peer.Commit                  peer.go:292-305
 *   step() loop                  node_test.go:274-353
 *   quiesceState                 quiesce.go:23-120 (node.go:195-200,
 *                                993-1005, 1148-1150, 1339-1345, 1385)
 *   StateMachine.Handle/handle   internal/rsm/statemachine.go:599-906
 *   handleEntry/update/noop      statemachine.go:935-1103
 *   setApplied/setLastApplied    statemachine.go:716-760
 *   GetPayload/getDecodedPayload internal/rsm/encoded.go:55-170
 *   snappy block decode          github.com/golang/snappy v0.0.4 (go.mod:8,
 *                                not vendored; dio.DecompressSnappyBlock
 *                                internal/utils/dio/io.go:199-209)
 *   KVTest.Update                internal/tests/kvtest.go:145-162,311
 *   pb.EntriesToApply            raftpb/entry.go:27-47
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle_internal.h"

/* ------------------------------------------------------------------ */
/* KVTest: map[string]string + Count                                    */
/* ------------------------------------------------------------------ */
typedef struct kv_item {
  uint8_t *key;
  uint8_t *val;
  uint32_t klen, vlen;
  int used;
} kv_item;

typedef struct orc_kv {
  kv_item *t;
  size_t cap, n;
  uint64_t count;
} orc_kv;

static uint64_t fnv1a(const uint8_t *p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; i++) h = (h ^ p[i]) * 0x100000001b3ull;
  return h;
}

static void kv_insert_raw(orc_kv *kv, uint8_t *key, uint32_t klen, uint8_t *val,
                          uint32_t vlen) {
  size_t m = kv->cap - 1;
  size_t i = (size_t)fnv1a(key, klen) & m;
  while (kv->t[i].used) {
    if (kv->t[i].klen == klen && memcmp(kv->t[i].key, key, klen) == 0) {
      free(kv->t[i].val);
      free(key);
      kv->t[i].val = val;
      kv->t[i].vlen = vlen;
      return;
    }
    i = (i + 1) & m;
  }
  kv->t[i].used = 1;
  kv->t[i].key = key;
  kv->t[i].klen = klen;
  kv->t[i].val = val;
  kv->t[i].vlen = vlen;
  kv->n++;
}

static void kv_grow(orc_kv *kv) {
  size_t oc = kv->cap;
  kv_item *ot = kv->t;
  kv->cap = oc ? oc * 2 : 16;
  kv->t = (kv_item *)calloc(kv->cap, sizeof(kv_item));
  kv->n = 0;
  for (size_t i = 0; i < oc; i++)
    if (ot[i].used)
      kv_insert_raw(kv, ot[i].key, ot[i].klen, ot[i].val, ot[i].vlen);
  free(ot);
}

static uint8_t *dupbytes(const uint8_t *p, uint32_t n) {
  uint8_t *d = (uint8_t *)malloc(n ? n : 1);
  if (n) memcpy(d, p, n);
  return d;
}

/* updateStore (kvtest.go:311-313): s.KVStore[key] = value */
static void kv_update_store(orc_kv *kv, const uint8_t *key, uint32_t klen,
                            const uint8_t *val, uint32_t vlen) {
  if ((kv->n + 1) * 2 > kv->cap) kv_grow(kv);
  kv_insert_raw(kv, dupbytes(key, klen), klen, dupbytes(val, vlen), vlen);
}

static const kv_item *kv_find(const orc_kv *kv, const uint8_t *key,
                              uint32_t klen) {
  if (!kv->cap) return NULL;
  size_t m = kv->cap - 1;
  size_t i = (size_t)fnv1a(key, klen) & m;
  while (kv->t[i].used) {
    if (kv->t[i].klen == klen && memcmp(kv->t[i].key, key, klen) == 0)
      return &kv->t[i];
    i = (i + 1) & m;
  }
  return NULL;
}

static void kv_free(orc_kv *kv) {
  for (size_t i = 0; i < kv->cap; i++)
    if (kv->t[i].used) {
      free(kv->t[i].key);
      free(kv->t[i].val);
    }
  free(kv->t);
  memset(kv, 0, sizeof(*kv));
}

/* ------------------------------------------------------------------ */
/* node                                                                 */
/* ------------------------------------------------------------------ */
/* quiesceState (quiesce.go:23-33) */
typedef struct orc_qs {
  uint64_t current_tick, election_tick, quiesced_since, idle_since,
      exit_quiesce_tick;
  int enabled, new_flag;
} orc_qs;

typedef struct orc_node {
  orc_raft *r;
  orc_qs qs;
  uint32_t quiesce_to; /* Quiesce messages of this round, bit per slot */
  orc_logdb *db;
  orc_kv kv;
  uint64_t sm_index, sm_term; /* StateMachine.index/term */
  uint64_t la_index, la_term; /* StateMachine.lastApplied */
  uint64_t applied_index, confirmed_index, pushed_index;
  uint64_t prev_term, prev_vote, prev_commit; /* Peer.prevState */
  uint64_t current_tick;
  orc_mvec inbox;  /* MessageQueue contents */
  uint32_t *inbox_from_slot;
  size_t inbox_from_cap;
  orc_evec props; /* incomingProposals */
  int has_ri;
  orc_ctx ri;
  uint64_t xfer; /* pendingLeaderTransfer: a requested target, 0 none */
  int hosted;
  orc_mvec out;   /* ud.Messages of the last round */
  orc_rtr *rtr;   /* ud.ReadyToReads of the last round */
  size_t nrtr, caprtr;
  orc_evec applyq; /* tasks pushed for the apply worker */
  orc_evec saved;  /* ud.EntriesToSave of the last round (SaveRaftState) */
  int upd_have;    /* the last round produced a pb.Update for SaveRaftState */
  uint64_t upd_st[3]; /* its State {Term, Vote, Commit}, zero when empty */
} orc_node;

struct orc_cluster {
  orc_cluster_cfg cfg;
  uint64_t *gids; /* [num_groups] global group ids */
  orc_node *nodes; /* [g * R + slot] */
  uint64_t round;
};

static orc_node *node_at(orc_cluster *c, uint64_t g, uint32_t s) {
  return &c->nodes[g * c->cfg.num_replicas + s];
}

static void msg_clone(orc_msg *dst, const orc_msg *src) {
  *dst = *src;
  memset(&dst->ents, 0, sizeof(dst->ents));
  ev_copy_range(&dst->ents, src->ents.v, src->ents.n);
}

/* MessageQueue.Add (internal/server/message.go:105-123) */
static void node_enqueue(orc_node *n, const orc_msg *m, uint32_t from_slot) {
  orc_msg cp;
  msg_clone(&cp, m);
  if (n->inbox.n == n->inbox_from_cap) {
    n->inbox_from_cap = n->inbox_from_cap ? n->inbox_from_cap * 2 : 8;
    n->inbox_from_slot = (uint32_t *)realloc(
        n->inbox_from_slot, n->inbox_from_cap * sizeof(uint32_t));
  }
  n->inbox_from_slot[n->inbox.n] = from_slot;
  mv_push(&n->inbox, &cp);
}

/* ---- rsm apply (statemachine.go) ------------------------------------ */
/* setApplied (statemachine.go:716-725) */
static void sm_set_applied(orc_node *n, uint64_t index, uint64_t term) {
  if (n->sm_index + 1 != index)
    orc_panic("applied index %llu, new index %llu",
              (unsigned long long)n->sm_index, (unsigned long long)index);
  if (n->sm_term > term)
    orc_panic("applied term %llu, new term %llu",
              (unsigned long long)n->sm_term, (unsigned long long)term);
  n->sm_index = index;
  n->sm_term = term;
}

/* golang/snappy v0.0.4 Decode, restated from the published block format
 * (the module is a go.mod dependency absent from /root/reference): a
 * uvarint decoded length, then literal (tag&3 == 0) and copy elements with
 * 1-, 2- or 4-byte offsets.  dlen is the exact decoded length
 * (DecompressSnappyBlock panics on a mismatch).  0 ok, -1 corrupt. */
static int snappy_decode(const uint8_t *s, size_t n, uint8_t *d, size_t dlen) {
  size_t i = 0, o = 0;
  uint64_t want = 0;
  for (int sh = 0;; sh += 7) {
    if (i >= n || sh > 63) return -1;
    uint8_t b = s[i++];
    want |= (uint64_t)(b & 0x7f) << sh;
    if (!(b & 0x80)) break;
  }
  if (want != dlen) orc_panic("corrupted decodedLen in header");
  while (i < n) {
    uint8_t tag = s[i++];
    size_t len, off;
    switch (tag & 3) {
      case 0: {
        len = tag >> 2;
        if (len >= 60) {
          size_t nb = len - 59;
          if (i + nb > n) return -1;
          len = 0;
          for (size_t k = 0; k < nb; k++) len |= (size_t)s[i + k] << (8 * k);
          i += nb;
        }
        len += 1;
        if (len > n - i || len > dlen - o) return -1;
        memcpy(d + o, s + i, len);
        i += len;
        o += len;
        continue;
      }
      case 1:
        if (i >= n) return -1;
        len = 4 + ((tag >> 2) & 7);
        off = ((size_t)(tag >> 5) << 8) | s[i++];
        break;
      case 2:
        if (i + 2 > n) return -1;
        len = 1 + (tag >> 2);
        off = (size_t)s[i] | ((size_t)s[i + 1] << 8);
        i += 2;
        break;
      default:
        if (i + 4 > n) return -1;
        len = 1 + (tag >> 2);
        off = (size_t)s[i] | ((size_t)s[i + 1] << 8) |
              ((size_t)s[i + 2] << 16) | ((size_t)s[i + 3] << 24);
        i += 4;
        break;
    }
    if (off == 0 || off > o || len > dlen - o) return -1;
    for (size_t k = 0; k < len; k++, o++) d[o] = d[o - off]; /* may overlap */
  }
  return o == dlen ? 0 : -1;
}

/* GetPayload (encoded.go:55-66) -> getDecodedPayload (encoded.go:127-160).
 * *owned receives a malloc'd buffer when the payload was decompressed. */
static const uint8_t *get_payload(uint32_t type, const uint8_t *cmd,
                                  uint32_t clen, uint32_t *plen,
                                  uint8_t **owned) {
  *owned = NULL;
  switch (type) {
    case DRB_ENTRY_APPLICATION:
    case DRB_ENTRY_CONFIG_CHANGE:
      *plen = clen;
      return clen ? cmd : NULL;
    case DRB_ENTRY_ENCODED:
      break;
    default:
      orc_panic("unknown entry type");
  }
  if (clen == 0) orc_panic("index out of range [0] with length 0");
  uint8_t h = cmd[0]; /* parseEncodedHeader (encoded.go:119-125) */
  uint8_t ver = h & 0xf0, ct = h & 0x0e;
  if (ver != 0) orc_panic("unknown cmd encoding version");
  if (h & 1) orc_panic("v0 cmd has session info");
  if (ct == 0) { /* getV0NoCompressPayload (encoded.go:162-164) */
    *plen = clen - 1;
    return cmd + 1;
  }
  if (ct != 2) orc_panic("unknown compression type %d", ct);
  /* getV0PayloadUncompressedSize (encoded.go:166-168): binary.Uvarint */
  uint64_t sz = 0;
  int ok = 0;
  for (uint32_t i = 1, sh = 0; i < clen && i <= 10; i++, sh += 7) {
    sz |= (uint64_t)(cmd[i] & 0x7f) << sh;
    if (!(cmd[i] & 0x80)) {
      ok = 1;
      break;
    }
  }
  if (!ok) sz = 0; /* Uvarint n <= 0: size 0 */
  if (sz == 0) orc_panic("empty uncompressed size found");
  uint8_t *buf = (uint8_t *)malloc((size_t)sz);
  if (snappy_decode(cmd + 1, clen - 1, buf, (size_t)sz)) {
    free(buf);
    orc_panic("snappy: corrupt input"); /* the apply error stops the node */
  }
  *owned = buf;
  *plen = (uint32_t)sz;
  return buf;
}

static int entry_is_session_managed(const orc_entry *e) {
  /* IsSessionManaged (raftpb/raft.go:90-99) */
  if (e->type == DRB_ENTRY_CONFIG_CHANGE) return 0;
  return e->client_id != 0;
}

/* handleEntry (statemachine.go:935-969) -> update (1057-1103) ->
 * KVTest.Update (kvtest.go:145-162).  Returns 1 if the KV was updated. */
static int sm_handle_entry(orc_node *n, const orc_entry *e) {
  uint32_t clen = e->cmd ? e->cmd->len : 0;
  if (e->type == DRB_ENTRY_CONFIG_CHANGE) {
    /* configChange (statemachine.go:1006-1019): membership is not on the
     * fast path; the bootstrap AddNode entries name existing members so
     * node.ApplyConfigChange only clears pendingConfigChange. */
    sm_set_applied(n, e->index, e->term);
    n->r->pending_config_change = 0;
    return 0;
  }
  if (!entry_is_session_managed(e)) {
    if (clen == 0) { /* noop (statemachine.go:1047-1054) */
      sm_set_applied(n, e->index, e->term);
      return 0;
    }
    orc_panic("not session managed, not empty");
  }
  /* IsNewSessionRequest / IsEndOfSessionRequest (raftpb/raft.go:108-126) */
  if (clen == 0 && (e->series_id == UINT64_MAX - 1 ||
                    e->series_id == UINT64_MAX))
    orc_panic("session management is not on the fast path");
  if (e->series_id != 0)
    orc_panic("regular client sessions are not on the fast path");
  /* update(): NoOP session -> GetPayload -> sm.Update; setApplied deferred.
   * (The GPU path falls back before appending a Snappy entry; the oracle
   * decodes it, as the CPU raft.Peer + rsm would.) */
  uint8_t *owned;
  uint32_t plen;
  const uint8_t *payload = get_payload(e->type, clen ? e->cmd->data : NULL,
                                       clen, &plen, &owned);
  /* KVTest.Update */
  n->kv.count++;
  const uint8_t *k, *v;
  uint32_t kl, vl;
  if (orc_pbkv_unmarshal(payload, plen, &k, &kl, &v, &vl)) {
    free(owned);
    orc_panic("PBKV unmarshal failed");
  }
  kv_update_store(&n->kv, k, kl, v, vl);
  free(owned);
  sm_set_applied(n, e->index, e->term);
  return 1;
}

/* pb.EntriesToApply (raftpb/entry.go:27-47): index of the first entry to
 * keep, or n when none */
static size_t entries_to_apply_off(const orc_entry *ents, size_t n,
                                   uint64_t applied, int strict) {
  if (n == 0) return 0;
  uint64_t last = ents[n - 1].index, first = ents[0].index;
  if (last <= applied) {
    if (strict)
      orc_panic("got entries [%llu-%llu] older than current state %llu",
                (unsigned long long)first, (unsigned long long)last,
                (unsigned long long)applied);
    return n;
  }
  if (first > applied + 1)
    orc_panic("entry hole found: %llu, want: %llu", (unsigned long long)first,
              (unsigned long long)(applied + 1));
  if (applied - first + 1 < (uint64_t)n) return (size_t)(applied - first + 1);
  return n;
}

/* StateMachine.Handle -> handle (statemachine.go:599-645, 877-906) for the
 * pushed tasks (one task per round here), then setLastApplied. */
static void sm_handle(orc_node *n, int is_leader, drb_round_out *out) {
  if (n->applyq.n == 0) return;
  size_t off = entries_to_apply_off(n->applyq.v, n->applyq.n, n->sm_index, 0);
  const orc_entry *e = n->applyq.v + off;
  size_t cnt = n->applyq.n - off;
  for (size_t i = 0; i < cnt; i++) {
    int upd = sm_handle_entry(n, &e[i]);
    if (out) {
      out->applied_entries++;
      if (is_leader && upd) out->committed_entries++;
    }
  }
  /* setLastApplied (statemachine.go:727-760) */
  if (cnt > 0) {
    for (size_t i = 1; i < cnt; i++) {
      if (e[i].index != e[i - 1].index + 1) orc_panic("index gap found");
      if (e[i].term < e[i - 1].term) orc_panic("term moving backward");
    }
    if (n->la_index + 1 != e[0].index) orc_panic("gap between batches");
    if (n->la_term > e[0].term) orc_panic("invalid term");
    n->la_index = e[cnt - 1].index;
    n->la_term = e[cnt - 1].term;
  }
  ev_truncate(&n->applyq, 0);
}

/* ---- quiesceState (quiesce.go) ------------------------------------- */
static int qs_quiesced(const orc_qs *q) {
  return q->enabled && q->quiesced_since > 0;
}
static uint64_t qs_threshold(const orc_qs *q) { return q->election_tick * 10; }
/* enterQuiesce (quiesce.go:104-109) */
static void qs_enter(orc_qs *q) {
  q->quiesced_since = q->current_tick;
  q->idle_since = q->current_tick;
  q->new_flag = 1;
}
/* exitQuiesce (quiesce.go:111-114) */
static void qs_exit(orc_qs *q) {
  q->quiesced_since = 0;
  q->exit_quiesce_tick = q->current_tick;
}
/* tick (quiesce.go:40-51) */
static void qs_tick(orc_qs *q) {
  if (!q->enabled) return;
  uint64_t threshold = qs_threshold(q);
  q->current_tick++;
  if (!qs_quiesced(q) && q->current_tick - q->idle_since > threshold)
    qs_enter(q);
}
/* newToQuiesce (quiesce.go:80-85) */
static int qs_new_to_quiesce(const orc_qs *q) {
  if (!qs_quiesced(q)) return 0;
  return q->current_tick - q->quiesced_since < q->election_tick;
}
/* justExitedQuiesce (quiesce.go:87-92) */
static int qs_just_exited(const orc_qs *q) {
  if (qs_quiesced(q)) return 0;
  return q->current_tick - q->exit_quiesce_tick < qs_threshold(q);
}
/* record (quiesce.go:56-74) */
static void qs_record(orc_qs *q, uint32_t type) {
  if (!q->enabled) return;
  if (type == DRB_MSG_HEARTBEAT || type == DRB_MSG_HEARTBEAT_RESP) {
    if (!qs_quiesced(q)) return;
    if (qs_new_to_quiesce(q)) return;
  }
  q->idle_since = q->current_tick;
  if (qs_quiesced(q)) qs_exit(q);
}
/* tryEnterQuiesce (quiesce.go:94-102) */
static void qs_try_enter(orc_qs *q) {
  if (qs_just_exited(q)) return;
  if (!qs_quiesced(q)) qs_enter(q);
}
/* newQuiesceState (quiesce.go:39-41) */
static int qs_take_new(orc_qs *q) {
  int f = q->new_flag;
  q->new_flag = 0;
  return f;
}

/* ---- node-level event handling -------------------------------------- */
static void node_tick(orc_node *n) {
  /* node.tick (node.go:1562-1579) */
  n->current_tick++;
  qs_tick(&n->qs);
  raft_tick_public(n->r, qs_quiesced(&n->qs));
}

/* node.recordMessage (node.go:1339-1345) */
static void node_record_message(orc_node *n, const orc_msg *m) {
  if ((m->type == DRB_MSG_HEARTBEAT || m->type == DRB_MSG_HEARTBEAT_RESP) &&
      m->hint > 0)
    qs_record(&n->qs, DRB_MSG_READ_INDEX);
  else
    qs_record(&n->qs, m->type);
}

/* stable order: all Replicate messages by sender slot, then every other
 * message by sender slot (node_test.go:311-339 delivery order) */
static void node_sort_inbox(orc_node *n) {
  size_t cnt = n->inbox.n;
  if (cnt < 2) return;
  orc_msg *tmp = (orc_msg *)malloc(cnt * sizeof(orc_msg));
  uint32_t *ts = (uint32_t *)malloc(cnt * sizeof(uint32_t));
  size_t k = 0;
  for (int pass = 0; pass < 2; pass++)
    for (uint32_t s = 0; s <= ORC_MAX_PEERS; s++)
      for (size_t i = 0; i < cnt; i++) {
        int isrep = n->inbox.v[i].type == DRB_MSG_REPLICATE;
        if ((pass == 0) != isrep) continue;
        if (n->inbox_from_slot[i] != s) continue;
        tmp[k] = n->inbox.v[i];
        ts[k] = s;
        k++;
      }
  memcpy(n->inbox.v, tmp, cnt * sizeof(orc_msg));
  memcpy(n->inbox_from_slot, ts, cnt * sizeof(uint32_t));
  free(tmp);
  free(ts);
}

/* handleEvents (node.go:1161-1223) */
static int node_handle_events(orc_node *n, int tick) {
  orc_raft *r = n->r;
  int has_event = 0;
  /* updateAppliedIndex (node.go:1133-1137) */
  n->applied_index = n->la_index;
  r->applied = n->applied_index;
  if (n->applied_index != n->confirmed_index) has_event = 1;
  if (log_has_entries_to_apply(&r->log)) has_event = 1;
  /* handleReadIndex (node.go:1296-1307) -> Peer.ReadIndex (peer.go:309) */
  if (n->has_ri) {
    qs_record(&n->qs, DRB_MSG_READ_INDEX);
    orc_msg m;
    memset(&m, 0, sizeof(m));
    m.type = DRB_MSG_READ_INDEX;
    m.hint = n->ri.low;
    m.hint_high = n->ri.high;
    raft_handle_msg(r, &m);
    n->has_ri = 0;
    has_event = 1;
  }
  /* handleReceivedMessages (node.go:1347-1377) */
  node_sort_inbox(n);
  if (tick) {
    orc_msg t;
    memset(&t, 0, sizeof(t));
    t.type = DRB_MSG_LOCAL_TICK;
    node_enqueue(n, &t, ORC_MAX_PEERS + 1);
  }
  size_t cnt = n->inbox.n;
  for (size_t i = 0; i < cnt; i++) {
    orc_msg *m = &n->inbox.v[i];
    /* node.handleMessage (node.go:1379-1401), else recordMessage +
     * Peer.Handle */
    if (m->type == DRB_MSG_LOCAL_TICK) {
      node_tick(n);
    } else if (m->type == DRB_MSG_QUIESCE) {
      qs_try_enter(&n->qs);
    } else {
      node_record_message(n, m);
      peer_handle(r, m);
    }
  }
  if (cnt > 0) has_event = 1;
  mv_clear(&n->inbox);
  /* handleProposals (node.go:1275-1294) -> Peer.ProposeEntries */
  if (n->props.n > 0) {
    orc_msg m;
    memset(&m, 0, sizeof(m));
    m.type = DRB_MSG_PROPOSE;
    m.from = r->replica_id;
    m.ents = n->props;
    memset(&n->props, 0, sizeof(n->props));
    raft_handle_msg(r, &m);
    msg_free(&m);
    has_event = 1;
  }
  /* handleLeaderTransfer (node.go:1249-1257) -> Peer.RequestLeaderTransfer
   * (peer.go:106-113) */
  if (n->xfer) {
    orc_msg m;
    memset(&m, 0, sizeof(m));
    m.type = DRB_MSG_LEADER_TRANSFER;
    m.to = r->replica_id;
    m.hint = n->xfer;
    n->xfer = 0;
    raft_handle_msg(r, &m);
    has_event = 1;
  }
  return has_event;
}

typedef struct orc_update {
  orc_evec save;
  orc_evec committed;
  orc_mvec msgs;
  uint64_t last_applied;
  int has_state;
  uint64_t st_term, st_vote, st_commit;
  size_t nrtr;
  uint64_t uc_ready, uc_last_applied, uc_processed, uc_stable_to,
      uc_stable_term;
} orc_update;

/* Peer.HasUpdate (peer.go:254-289) with moreToApply = true */
static int peer_has_update(orc_node *n) {
  orc_raft *r = n->r;
  size_t ns;
  log_entries_to_save(&r->log, &ns);
  if (ns > 0) return 1;
  if (r->leader_update) return 1;
  if (r->msgs.n > 0) return 1;
  if (log_has_entries_to_apply(&r->log)) return 1;
  uint64_t t = r->term, v = r->vote, c = r->log.committed;
  if (!(t == 0 && v == 0 && c == 0) &&
      !(t == n->prev_term && v == n->prev_vote && c == n->prev_commit))
    return 1;
  if (r->nrtr != 0) return 1;
  if (r->ndropped_entries > 0) return 1;
  if (r->ndropped_ri > 0) return 1;
  return 0;
}

/* node.getUpdate (node.go:1025-1042) -> Peer.GetUpdate (peer.go:198-208) */
static int node_get_update(orc_node *n, orc_update *ud) {
  orc_raft *r = n->r;
  if (!(peer_has_update(n) || n->confirmed_index != n->applied_index))
    return 0;
  memset(ud, 0, sizeof(*ud));
  size_t ns;
  const orc_entry *s = log_entries_to_save(&r->log, &ns);
  ev_copy_range(&ud->save, s, ns);
  ud->msgs = r->msgs;
  memset(&r->msgs, 0, sizeof(r->msgs));
  for (size_t i = 0; i < ud->msgs.n; i++) ud->msgs.v[i].shard_id = r->shard_id;
  ud->last_applied = n->applied_index;
  if (log_entries_to_apply(&r->log, &ud->committed))
    orc_panic("entriesToApply: log error");
  if (!(r->term == n->prev_term && r->vote == n->prev_vote &&
        r->log.committed == n->prev_commit)) {
    ud->has_state = 1;
    ud->st_term = r->term;
    ud->st_vote = r->vote;
    ud->st_commit = r->log.committed;
  }
  ud->nrtr = r->nrtr;
  /* validateUpdate (peer.go:228-245) */
  if (r->log.committed > 0 && ud->committed.n > 0 &&
      ud->committed.v[ud->committed.n - 1].index > r->log.committed)
    orc_panic("trying to apply not committed entry");
  if (ud->committed.n > 0 && ud->save.n > 0 &&
      ud->committed.v[ud->committed.n - 1].index >
          ud->save.v[ud->save.n - 1].index)
    orc_panic("trying to apply not saved entry");
  /* getUpdateCommit (peer.go:432-449) */
  ud->uc_ready = ud->nrtr;
  ud->uc_last_applied = ud->last_applied;
  if (ud->committed.n > 0)
    ud->uc_processed = ud->committed.v[ud->committed.n - 1].index;
  if (ud->save.n > 0) {
    ud->uc_stable_to = ud->save.v[ud->save.n - 1].index;
    ud->uc_stable_term = ud->save.v[ud->save.n - 1].term;
  }
  n->confirmed_index = n->applied_index;
  return 1;
}

/* Peer.Commit (peer.go:292-305) */
static void peer_commit(orc_node *n, orc_update *ud) {
  orc_raft *r = n->r;
  raft_clear_msgs(r);
  r->leader_update = 0;
  r->ndropped_entries = 0;
  r->ndropped_ri = 0;
  if (ud->has_state && !(ud->st_term == 0 && ud->st_vote == 0 &&
                         ud->st_commit == 0)) {
    n->prev_term = ud->st_term;
    n->prev_vote = ud->st_vote;
    n->prev_commit = ud->st_commit;
  }
  if (ud->uc_ready > 0) r->nrtr = 0; /* clearReadyToRead */
  log_commit_update(&r->log, ud->uc_stable_to, ud->uc_stable_term,
                    ud->uc_processed, ud->uc_last_applied);
}

static void update_free(orc_update *ud) {
  ev_free(&ud->save);
  ev_free(&ud->committed);
  mv_free(&ud->msgs);
}

/* deliver one message to its target replica of the same group */
static void deliver(orc_cluster *c, uint64_t g, uint32_t from_slot,
                    const orc_msg *m) {
  if (m->to < 1 || m->to > c->cfg.num_replicas) return;
  /* an unhosted target is served by the outbound boundary; what sits in
   * its queue is dropped unless it is hosted again for the next round
   * (the device mailbox has the same lifetime) */
  node_enqueue(node_at(c, g, (uint32_t)(m->to - 1)), m, from_slot);
}

/* one step() (node_test.go:274-353) for group g */
static void group_round(orc_cluster *c, uint64_t g, int tick,
                        drb_round_out *out) {
  uint32_t R = c->cfg.num_replicas;
  orc_update uds[ORC_MAX_PEERS];
  int have[ORC_MAX_PEERS];
  memset(have, 0, sizeof(have));
  for (uint32_t s = 0; s < R; s++) {
    orc_node *n = node_at(c, g, s);
    mv_clear(&n->out);
    n->nrtr = 0;
    n->saved.n = 0;
    n->upd_have = 0;
    n->quiesce_to = 0;
    if (!n->hosted) {
      mv_clear(&n->inbox);
      continue;
    }
    if (node_handle_events(n, tick)) {
      /* stepNode: newQuiesceState -> sendEnterQuiesceMessages
       * (node.go:1148-1150, 993-1005), ahead of the Update's messages */
      if (qs_take_new(&n->qs))
        n->quiesce_to = ((1u << R) - 1u) & ~(1u << s);
      have[s] = node_get_update(n, &uds[s]);
    }
  }
  for (uint32_t s = 0; s < R; s++) {
    orc_node *n = node_at(c, g, s);
    for (uint32_t t = 0; t < R; t++) {
      if (!((n->quiesce_to >> t) & 1u)) continue;
      orc_msg q;
      memset(&q, 0, sizeof(q));
      q.type = DRB_MSG_QUIESCE;
      q.from = s + 1;
      q.to = t + 1;
      q.shard_id = n->r->shard_id;
      deliver(c, g, s, &q);
      mv_push(&n->out, &q); /* this round's outbox, first */
      if (out) out->messages++;
    }
  }
  /* applyRaftUpdates / sendReplicateMessages / processReadyToRead */
  for (uint32_t s = 0; s < R; s++) {
    if (!have[s]) continue;
    orc_node *n = node_at(c, g, s);
    orc_update *ud = &uds[s];
    size_t off = entries_to_apply_off(ud->committed.v, ud->committed.n,
                                      n->pushed_index, 1);
    if (off < ud->committed.n) {
      ev_copy_range(&n->applyq, ud->committed.v + off, ud->committed.n - off);
      n->pushed_index = ud->committed.v[ud->committed.n - 1].index;
    }
    for (size_t i = 0; i < ud->msgs.n; i++)
      if (ud->msgs.v[i].type == DRB_MSG_REPLICATE)
        deliver(c, g, s, &ud->msgs.v[i]);
    orc_raft *r = n->r;
    if (ud->nrtr) {
      if (n->caprtr < ud->nrtr) {
        n->caprtr = ud->nrtr;
        n->rtr = (orc_rtr *)realloc(n->rtr, n->caprtr * sizeof(orc_rtr));
      }
      memcpy(n->rtr, r->rtr, ud->nrtr * sizeof(orc_rtr));
      n->nrtr = ud->nrtr;
      if (out) out->ready_to_reads += ud->nrtr;
    }
    if (out) {
      out->messages += ud->msgs.n;
      out->dropped_read_indexes += r->ndropped_ri;
      out->dropped_proposals += r->ndropped_entries;
    }
  }
  /* SaveRaftState, processRaftUpdate, commitRaftUpdate, sm.Handle */
  for (uint32_t s = 0; s < R; s++) {
    if (!have[s]) continue;
    orc_node *n = node_at(c, g, s);
    orc_update *ud = &uds[s];
    db_append(n->db, ud->save.v, ud->save.n); /* LogReader.Append */
    ev_copy_range(&n->saved, ud->save.v, ud->save.n);
    n->upd_have = 1;
    n->upd_st[0] = ud->has_state ? ud->st_term : 0;
    n->upd_st[1] = ud->has_state ? ud->st_vote : 0;
    n->upd_st[2] = ud->has_state ? ud->st_commit : 0;
    for (size_t i = 0; i < ud->msgs.n; i++)
      if (ud->msgs.v[i].type != DRB_MSG_REPLICATE)
        deliver(c, g, s, &ud->msgs.v[i]);
    peer_commit(n, ud);
    sm_handle(n, n->r->state == DRB_LEADER, out);
    if (c->cfg.logdb_keep && n->db->ents.n > 2 * c->cfg.logdb_keep) {
      uint64_t keep_from = n->r->log.processed;
      uint64_t lim = n->db->marker_index + n->db->ents.n - c->cfg.logdb_keep;
      if (keep_from > lim) keep_from = lim;
      if (keep_from > n->db->marker_index) orc_logdb_compact(n->db, keep_from);
    }
    /* the outbox of this round in send order: the Quiesce messages, the
     * Replicates (sendReplicateMessages, node.go:1016-1023), then the
     * rest (processRaftUpdate -> sendMessages, node.go:1104-1108) */
    for (int pass = 0; pass < 2; pass++)
      for (size_t i = 0; i < ud->msgs.n; i++)
        if ((ud->msgs.v[i].type == DRB_MSG_REPLICATE) == (pass == 0))
          mv_push(&n->out, &ud->msgs.v[i]);
    ud->msgs.n = 0;
    update_free(ud);
  }
}

/* ------------------------------------------------------------------ */
/* cluster API                                                          */
/* ------------------------------------------------------------------ */
static uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

orc_cluster *orc_cluster_new(const orc_cluster_cfg *cfg) {
  if (cfg->num_replicas < 1 || cfg->num_replicas > DRB_MAX_REPLICAS)
    return NULL;
  orc_cluster *c = (orc_cluster *)calloc(1, sizeof(orc_cluster));
  c->cfg = *cfg;
  c->gids = (uint64_t *)malloc((cfg->num_groups ? cfg->num_groups : 1) *
                               sizeof(uint64_t));
  for (uint64_t g = 0; g < cfg->num_groups; g++)
    c->gids[g] = cfg->gids ? cfg->gids[g] : g;
  c->cfg.gids = c->gids;
  uint64_t R = cfg->num_replicas;
  c->nodes = (orc_node *)calloc(cfg->num_groups * R, sizeof(orc_node));
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    return NULL;
  }
  for (uint64_t g = 0; g < cfg->num_groups; g++)
    for (uint32_t s = 0; s < R; s++) {
      orc_node *n = node_at(c, g, s);
      n->db = orc_logdb_new();
      const uint64_t gid = c->gids[g];
      n->r = raft_new(cfg->first_shard_id + gid, s + 1, cfg->election_rtt,
                      cfg->heartbeat_rtt, (int)cfg->check_quorum, n->db,
                      mix64(cfg->seed ^ (gid * R + s)));
      n->r->pre_vote = cfg->pre_vote != 0;
      n->hosted = 1;
      /* quiesceState{electionTick: ElectionRTT * 2} (node.go:195-200) */
      n->qs.election_tick = 2ull * cfg->election_rtt;
      n->qs.enabled = cfg->quiesce != 0;
    }
  orc_jb = prev;
  return c;
}

void orc_cluster_free(orc_cluster *c) {
  if (!c) return;
  uint64_t N = c->cfg.num_groups * c->cfg.num_replicas;
  for (uint64_t i = 0; i < N; i++) {
    orc_node *n = &c->nodes[i];
    raft_free(n->r);
    orc_logdb_free(n->db);
    kv_free(&n->kv);
    mv_free(&n->inbox);
    free(n->inbox_from_slot);
    ev_free(&n->props);
    mv_free(&n->out);
    free(n->rtr);
    ev_free(&n->applyq);
    ev_free(&n->saved);
  }
  free(c->nodes);
  free(c->gids);
  free(c);
}

/* Launch (peer.go:64-79) with initial && newNode, then bootstrap, then an
 * election of leader_slot (its election timer fired), then rounds until
 * no messages move.  The randomized election timeouts are finally set to
 * a documented formula so the device-side initialiser can reproduce them
 * (they are random in the reference: raft.go:658-661). */
int orc_cluster_setup_steady(orc_cluster *c, uint32_t leader_slot) {
  ORC_TRY(-1);
  uint32_t R = c->cfg.num_replicas;
  if (leader_slot >= R) orc_panic("bad leader slot");
  uint64_t ids[ORC_MAX_PEERS];
  orc_blob *cmds[ORC_MAX_PEERS];
  for (uint32_t s = 0; s < R; s++) {
    ids[s] = s + 1;
    char addr[32];
    uint8_t buf[64];
    snprintf(addr, sizeof(addr), "localhost:%u", 26000 + s);
    size_t l = orc_configchange_marshal_addnode(s + 1, addr, buf);
    cmds[s] = blob_new(buf, (uint32_t)l);
  }
  for (uint64_t g = 0; g < c->cfg.num_groups; g++)
    for (uint32_t s = 0; s < R; s++) {
      orc_node *n = node_at(c, g, s);
      /* Launch: becomeFollower(1, NoLeader) then bootstrap */
      raft_become_follower(n->r, 1, 0);
      raft_bootstrap(n->r, ids, (int)R, cmds);
    }
  for (uint32_t s = 0; s < R; s++) blob_unref(cmds[s]);
  ORC_END;
  /* round: apply the bootstrap entries */
  drb_round_out o;
  memset(&o, 0, sizeof(o));
  if (orc_cluster_round(c, 0, &o)) return -1;
  /* leader's election timer fires on the next tick */
  for (uint64_t g = 0; g < c->cfg.num_groups; g++) {
    orc_raft *r = node_at(c, g, leader_slot)->r;
    r->election_tick = r->randomized_election_timeout - 1;
  }
  if (orc_cluster_round(c, 1, &o)) return -1;
  for (int i = 0; i < 64; i++) {
    memset(&o, 0, sizeof(o));
    if (orc_cluster_round(c, 0, &o)) return -1;
    if (o.messages == 0) break;
  }
  for (uint64_t g = 0; g < c->cfg.num_groups; g++)
    for (uint32_t s = 0; s < R; s++) {
      orc_raft *r = node_at(c, g, s)->r;
      uint64_t e = c->cfg.election_rtt;
      r->randomized_election_timeout =
          e + mix64(c->cfg.seed ^ (0xE1ull << 56) ^ (c->gids[g] * R + s)) % e;
      /* raft.rand restarts from a per-replica seed the engine derives the
       * same way (k_init_steady), so later resets draw the same timeouts */
      r->rng = mix64(c->cfg.seed ^ (0xE2ull << 56) ^ (c->gids[g] * R + s));
    }
  return 0;
}

/* Member kinds (the shard's membership, pb.Membership's NonVotings and
 * Witnesses): replica slot s is a nonVoting when bit s of nonvoting_mask is
 * set, a witness when bit s of witness_mask is; every replica's raft gets
 * them in its remotes' kinds (r.nonVotings / r.witnesses, raft.go:199-239)
 * and those replicas their states.  The harness sets the membership after
 * setup_steady, as a membership restored from a snapshot would be; the
 * leader must be a voting member. */
int orc_cluster_set_member_kinds(orc_cluster *c, uint32_t nonvoting_mask,
                                 uint32_t witness_mask) {
  const uint32_t R = c->cfg.num_replicas;
  if (nonvoting_mask & witness_mask) return -1;
  for (uint64_t g = 0; g < c->cfg.num_groups; g++)
    for (uint32_t s = 0; s < R; s++) {
      orc_raft *r = node_at(c, g, s)->r;
      for (uint32_t t = 0; t < R; t++) {
        const int kind = (nonvoting_mask >> t) & 1u   ? ORC_NONVOTING
                         : (witness_mask >> t) & 1u ? ORC_WITNESS
                                                     : ORC_VOTING;
        const int i = raft_rem_idx(r, t + 1);
        if (i < 0) return -1;
        r->rem_kind[i] = (uint8_t)kind;
        if (t == s && kind != ORC_VOTING) {
          if (r->state == DRB_LEADER) return -1;
          r->state = kind == ORC_NONVOTING ? DRB_NONVOTING : DRB_WITNESS;
        }
      }
    }
  return 0;
}

int orc_cluster_stage_proposals(orc_cluster *c, const uint32_t *counts,
                                uint32_t max_per_group, const drb_entry *ents,
                                const uint8_t *pool) {
  return orc_cluster_stage_proposals_at(c, counts, max_per_group, ents, pool,
                                        0);
}

/* NodeHost.Propose -> node.propose -> entryQueue.add (queue.go:60) at
 * replica ID `replica` of every group (0: the group's leader replica, the
 * NodeHost holding it); node.handleProposals hands the queue to
 * Peer.ProposeEntries (node.go:1275-1294), and a follower forwards it to
 * its leader (handleFollowerPropose, raft.go:2103-2116) */
int orc_cluster_stage_proposals_at(orc_cluster *c, const uint32_t *counts,
                                   uint32_t max_per_group,
                                   const drb_entry *ents, const uint8_t *pool,
                                   uint32_t replica) {
  uint32_t R = c->cfg.num_replicas;
  for (uint64_t g = 0; g < c->cfg.num_groups; g++) {
    if (!counts[g]) continue;
    orc_node *ln = NULL;
    for (uint32_t s = 0; s < R; s++) {
      orc_node *n = node_at(c, g, s);
      const int here = replica ? s + 1 == replica
                               : n->r->state == DRB_LEADER;
      if (n->hosted && here) ln = n;
    }
    if (!ln) continue;
    for (uint32_t j = 0; j < counts[g]; j++) {
      orc_entry e = entry_from_view(&ents[g * max_per_group + j], pool);
      e.term = 0;
      e.index = 0;
      ev_push(&ln->props, &e);
      blob_unref(e.cmd);
    }
  }
  return 0;
}

int orc_cluster_stage_read_index(orc_cluster *c, const uint64_t *low,
                                 const uint64_t *high) {
  return orc_cluster_stage_read_index_at(c, low, high, 0);
}

/* node.read / handleReadIndex (node.go:1296-1307) at replica ID `replica`
 * (0: the group's leader) */
int orc_cluster_stage_read_index_at(orc_cluster *c, const uint64_t *low,
                                    const uint64_t *high, uint32_t replica) {
  uint32_t R = c->cfg.num_replicas;
  for (uint64_t g = 0; g < c->cfg.num_groups; g++) {
    if (!low[g]) continue;
    for (uint32_t s = 0; s < R; s++) {
      orc_node *n = node_at(c, g, s);
      const int here = replica ? s + 1 == replica
                               : n->r->state == DRB_LEADER;
      if (n->hosted && here) {
        n->has_ri = 1;
        n->ri.low = low[g];
        n->ri.high = high[g];
      }
    }
  }
  return 0;
}

/* NodeHost.RequestLeaderTransfer (nodehost.go:1238-1251) ->
 * node.requestLeaderTransfer -> pendingLeaderTransfer.request (a channel of
 * one: a second request before the node takes the first is ErrSystemBusy)
 * at replica slot `slot` of every group with targets[g] != 0.  Returns the
 * number of busy refusals. */
int64_t orc_cluster_request_leader_transfer(orc_cluster *c, uint32_t slot,
                                            const uint32_t *targets) {
  if (slot >= c->cfg.num_replicas) return -1;
  int64_t busy = 0;
  for (uint64_t g = 0; g < c->cfg.num_groups; g++) {
    if (!targets[g]) continue;
    orc_node *n = node_at(c, g, slot);
    if (!n->hosted) continue;
    if (n->xfer)
      busy++;
    else
      n->xfer = targets[g];
  }
  return busy;
}

int orc_cluster_ingest(orc_cluster *c, const drb_message *m, size_t n,
                       const drb_entry *ents, const uint8_t *pool) {
  for (size_t i = 0; i < n; i++) {
    uint64_t g = m[i].shard_id - c->cfg.first_shard_id;
    if (g >= c->cfg.num_groups) continue;
    if (m[i].to < 1 || m[i].to > c->cfg.num_replicas) continue;
    if (m[i].from < 1 || m[i].from > c->cfg.num_replicas) continue;
    orc_node *t = node_at(c, g, (uint32_t)(m[i].to - 1));
    if (!t->hosted) continue;
    if (node_at(c, g, (uint32_t)(m[i].from - 1))->hosted) continue;
    orc_msg mm = orc_msg_from_view(&m[i], ents, pool);
    node_enqueue(t, &mm, (uint32_t)(m[i].from - 1));
    msg_free(&mm);
  }
  return 0;
}

int orc_cluster_round_range(orc_cluster *c, int tick, uint64_t g0, uint64_t g1,
                            drb_round_out *out) {
  ORC_TRY(-1);
  for (uint64_t g = g0; g < g1 && g < c->cfg.num_groups; g++)
    group_round(c, g, tick, out);
  ORC_END;
  return 0;
}

int orc_cluster_end_round(orc_cluster *c) {
  c->round++;
  return 0;
}

int orc_cluster_round(orc_cluster *c, int tick, drb_round_out *out) {
  if (out) out->round = c->round;
  int rc = orc_cluster_round_range(c, tick, 0, c->cfg.num_groups, out);
  orc_cluster_end_round(c);
  return rc;
}

int orc_cluster_export(orc_cluster *c, uint64_t g, uint32_t slot,
                       drb_replica_state *st) {
  if (g >= c->cfg.num_groups || slot >= c->cfg.num_replicas) return -1;
  orc_node *n = node_at(c, g, slot);
  orc_raft_info(n->r, st);
  st->applied_index = n->applied_index;
  st->confirmed_index = n->confirmed_index;
  st->pushed_index = n->pushed_index;
  st->prev_term = n->prev_term;
  st->prev_vote = n->prev_vote;
  st->prev_commit = n->prev_commit;
  st->sm_index = n->sm_index;
  st->sm_term = n->sm_term;
  st->kv_count = n->kv.count;
  st->qs_current_tick = n->qs.current_tick;
  st->qs_idle_since = n->qs.idle_since;
  st->qs_quiesced_since = n->qs.quiesced_since;
  st->qs_exit_quiesce_tick = n->qs.exit_quiesce_tick;
  st->rng = n->r->rng;
  st->flags = n->hosted ? DRB_F_HOSTED : 0;
  return 0;
}

/* The inverse of orc_cluster_export plus the log: replica (g, slot) takes
 * the given state, as the engine's drb_import_replicas + drb_import_log do
 * -- raft.loadState over a LogDB (raft.go:1099-1117) and the inMemory
 * window (newEntryLog, logentry.go:86-95, with the markers the state
 * names).  ents hold [ents[0].index, st->last_index] contiguously: those
 * <= saved_to are the LogDB's (LogReader), those >= marker_index
 * inMemory's.  The KV keeps its contents (KVTest.Count is taken from st);
 * the inbox and the apply queue are emptied.  0 ok, -1 bad input. */
int orc_cluster_import(orc_cluster *c, uint64_t g, uint32_t slot,
                       const drb_replica_state *st, const drb_entry *ents,
                       size_t n, const uint8_t *pool) {
  if (g >= c->cfg.num_groups || slot >= c->cfg.num_replicas) return -1;
  if (st->ri_count) return -1; /* a readIndex queue is not imported */
  const uint64_t first = n ? ents[0].index : st->last_index + 1;
  if (first == 0 || first - 1 + n != st->last_index) return -1;
  if (st->marker_index < first || st->marker_index > st->last_index + 1 ||
      st->saved_to + 1 < first || st->saved_to > st->last_index)
    return -1;
  orc_node *nd = node_at(c, g, slot);
  orc_raft *r = nd->r;
  ORC_TRY(-1);
  orc_logdb *db = nd->db;
  ev_truncate(&db->ents, 0);
  db->marker_index = first - 1;
  db->marker_term = 0; /* first == 1 on this path: term(0) == 0 */
  orc_log *l = &r->log;
  ev_truncate(&l->im.ents, 0);
  for (size_t i = 0; i < n; i++) {
    orc_entry e = entry_from_view(&ents[i], pool);
    e.index = first + i;
    if (e.index <= st->saved_to) ev_push(&db->ents, &e);
    if (e.index >= st->marker_index) ev_push(&l->im.ents, &e);
    blob_unref(e.cmd);
  }
  l->im.marker_index = st->marker_index;
  l->im.saved_to = st->saved_to;
  l->im.applied_to_index = st->applied_to_index;
  l->im.applied_to_term = st->applied_to_term;
  l->im.shrunk = 0;
  l->committed = st->committed;
  l->processed = st->processed;
  r->term = st->term;
  r->vote = st->vote;
  r->leader_id = st->leader_id;
  r->applied = st->applied;
  r->election_tick = st->election_tick;
  r->heartbeat_tick = st->heartbeat_tick;
  r->randomized_election_timeout = st->randomized_election_timeout;
  r->tick_count = st->tick_count;
  r->state = st->role;
  r->rng = st->rng;
  r->leader_transfer_target = st->role == DRB_LEADER ? st->transfer : 0;
  r->is_leader_transfer_target = 0;
  r->nvotes = 0;
  for (uint32_t s = 0; s < DRB_MAX_REPLICAS; s++)
    if ((st->votes >> s) & 1u) {
      r->vote_id[r->nvotes] = s + 1;
      r->vote_ok[r->nvotes] = (int)((st->votes >> (8 + s)) & 1u);
      r->nvotes++;
    }
  for (int i = 0; i < r->nrem; i++) {
    const uint64_t id = r->rem_id[i];
    if (id < 1 || id > DRB_MAX_REPLICAS) continue;
    const drb_remote_state *d = &st->remotes[id - 1];
    r->rem[i].match = d->match;
    r->rem[i].next = d->next;
    r->rem[i].state = d->state;
    r->rem[i].active = (int)d->active;
  }
  r->ri.n = 0;
  raft_clear_msgs(r);
  nd->applied_index = st->applied_index;
  nd->confirmed_index = st->confirmed_index;
  nd->pushed_index = st->pushed_index;
  nd->prev_term = st->prev_term;
  nd->prev_vote = st->prev_vote;
  nd->prev_commit = st->prev_commit;
  nd->sm_index = nd->la_index = st->sm_index;
  nd->sm_term = nd->la_term = st->sm_term;
  nd->kv.count = st->kv_count;
  nd->qs.current_tick = st->qs_current_tick;
  nd->qs.idle_since = st->qs_idle_since;
  nd->qs.quiesced_since = st->qs_quiesced_since;
  nd->qs.exit_quiesce_tick = st->qs_exit_quiesce_tick;
  nd->hosted = (st->flags & DRB_F_HOSTED) != 0;
  mv_clear(&nd->inbox);
  ev_truncate(&nd->applyq, 0);
  ORC_END;
  return 0;
}

long orc_cluster_export_log(orc_cluster *c, uint64_t g, uint32_t slot,
                            uint64_t lo, uint64_t hi, drb_entry *out,
                            uint8_t *pool, size_t pool_cap) {
  orc_node *n = node_at(c, g, slot);
  orc_log *l = &n->r->log;
  size_t pu = 0, k = 0;
  for (uint64_t i = lo; i <= hi; i++) {
    const orc_entry *e = NULL;
    if (i >= l->im.marker_index && i < l->im.marker_index + l->im.ents.n)
      e = &l->im.ents.v[i - l->im.marker_index];
    else if (i > l->db->marker_index &&
             i <= l->db->marker_index + l->db->ents.n)
      e = &l->db->ents.v[i - l->db->marker_index - 1];
    if (!e) return -1;
    if (entry_to_view(e, &out[k++], pool, pool_cap, &pu)) return -2;
  }
  return (long)k;
}

long orc_cluster_export_outbox(orc_cluster *c, uint64_t g, uint32_t slot,
                               drb_message *out, size_t cap, drb_entry *ents,
                               size_t ent_cap, uint8_t *pool,
                               size_t pool_cap) {
  orc_node *n = node_at(c, g, slot);
  if (n->out.n > cap) return (long)n->out.n;
  size_t eu = 0, pu = 0;
  for (size_t i = 0; i < n->out.n; i++)
    if (msg_to_view(&n->out.v[i], &out[i], ents, ent_cap, &eu, pool, pool_cap,
                    &pu))
      return -2;
  return (long)n->out.n;
}

long orc_cluster_export_kv(orc_cluster *c, uint64_t g, uint32_t slot,
                           uint8_t *keys, uint32_t *klens, uint8_t *vals,
                           uint32_t *vlens, size_t cap, size_t key_cap,
                           size_t val_cap) {
  orc_node *n = node_at(c, g, slot);
  size_t k = 0;
  for (size_t i = 0; i < n->kv.cap; i++) {
    kv_item *it = &n->kv.t[i];
    if (!it->used) continue;
    if (k >= cap) return (long)n->kv.n;
    if (it->klen > key_cap || it->vlen > val_cap) return -2;
    memcpy(keys + k * key_cap, it->key, it->klen);
    klens[k] = it->klen;
    memcpy(vals + k * val_cap, it->val, it->vlen);
    vlens[k] = it->vlen;
    k++;
  }
  return (long)k;
}

long orc_cluster_export_ready(orc_cluster *c, uint64_t g, uint32_t slot,
                              drb_ready_to_read *out, size_t cap) {
  orc_node *n = node_at(c, g, slot);
  size_t k = n->nrtr < cap ? n->nrtr : cap;
  for (size_t i = 0; i < k; i++) {
    out[i].shard_id = n->r->shard_id;
    out[i].replica_id = n->r->replica_id;
    out[i].index = n->rtr[i].index;
    out[i].ctx_low = n->rtr[i].ctx.low;
    out[i].ctx_high = n->rtr[i].ctx.high;
  }
  return (long)n->nrtr;
}

/* The last round's EntriesToSave of one replica as the bytes
 * ILogDB.SaveRaftState persists: EntryBatch.MarshalTo (entrybatch.go:25-58)
 * of the colfer Entries (raft_optimized.go:166-300), and their
 * crc32.ChecksumIEEE.  Returns the byte count (0: nothing saved), or -1
 * when cap is too small. */
long orc_cluster_export_saved(orc_cluster *c, uint64_t g, uint32_t slot,
                              uint8_t *buf, size_t cap, uint32_t *crc) {
  orc_node *n = node_at(c, g, slot);
  const size_t ne = n->saved.n;
  if (crc) *crc = 0;
  if (ne == 0) return 0;
  drb_entry *de = (drb_entry *)calloc(ne, sizeof(drb_entry));
  size_t pool_n = 0;
  for (size_t i = 0; i < ne; i++)
    pool_n += n->saved.v[i].cmd ? n->saved.v[i].cmd->len : 0;
  uint8_t *pool = (uint8_t *)malloc(pool_n + 1);
  size_t off = 0;
  for (size_t i = 0; i < ne; i++) {
    const orc_entry *e = &n->saved.v[i];
    de[i].term = e->term;
    de[i].index = e->index;
    de[i].key = e->key;
    de[i].client_id = e->client_id;
    de[i].series_id = e->series_id;
    de[i].responded_to = e->responded_to;
    de[i].type = e->type;
    de[i].cmd_len = e->cmd ? e->cmd->len : 0;
    de[i].cmd_off = off;
    if (de[i].cmd_len) memcpy(pool + off, e->cmd->data, de[i].cmd_len);
    off += de[i].cmd_len;
  }
  long rc = -1;
  const size_t sz = orc_entrybatch_size(de, ne);
  if (sz <= cap) {
    orc_entrybatch_marshal(de, ne, pool, buf);
    if (crc) *crc = orc_crc32_ieee(buf, sz);
    rc = (long)sz;
  }
  free(de);
  free(pool);
  return rc;
}

/* SaveRaftState of the last round's pb.Update of replica (g, slot) into a
 * regular tan db (internal/tan/logdb.go:306-340 -> db.write, db.go:97):
 * 1 written, 0 no Update or nothing to write, -1 error */
int orc_cluster_tan_write(orc_cluster *c, uint64_t g, uint32_t slot,
                          orc_tandb *db, int *sync) {
  orc_node *n = node_at(c, g, slot);
  if (sync) *sync = 0;
  if (!n->upd_have) return 0;
  const size_t ne = n->saved.n;
  drb_entry *de = (drb_entry *)calloc(ne ? ne : 1, sizeof(drb_entry));
  size_t pool_n = 0;
  for (size_t i = 0; i < ne; i++)
    pool_n += n->saved.v[i].cmd ? n->saved.v[i].cmd->len : 0;
  uint8_t *pool = (uint8_t *)malloc(pool_n + 1);
  size_t used = 0;
  int rc = 0;
  for (size_t i = 0; i < ne && rc == 0; i++)
    rc = entry_to_view(&n->saved.v[i], &de[i], pool, pool_n + 1, &used);
  if (rc == 0)
    rc = orc_tandb_write(db, n->r->shard_id, n->r->replica_id, n->upd_st[0],
                         n->upd_st[1], n->upd_st[2], de, ne, pool, sync);
  else
    rc = -1;
  free(de);
  free(pool);
  return rc;
}

/* Config.PreVote of every replica (set after setup_steady's election) */
void orc_cluster_set_pre_vote(orc_cluster *c, int on) {
  for (uint64_t g = 0; g < c->cfg.num_groups; g++)
    for (uint32_t s = 0; s < c->cfg.num_replicas; s++)
      node_at(c, g, s)->r->pre_vote = on;
}

int orc_cluster_set_hosted(orc_cluster *c, uint64_t g, uint32_t slot,
                           int hosted) {
  node_at(c, g, slot)->hosted = hosted;
  return 0;
}

/* ReadLocalNode for the reads behind each replica's ReadyToReads of the
 * last round: pendingReadIndex.applied releases a read once the replica
 * applied its index (request.go:930-953); the client's ReadLocalNode then
 * runs KVTest.Lookup (nodehost.go:849, kvtest.go:164-175).  Read j of ctx
 * {low, high} looks up LE64(mix64(low ^ (j+1)*GOLDEN) % key_space); results
 * fold into sums[g * R + slot] (drb_serve_reads in include/drb_engine.h). */
int orc_cluster_serve_reads(orc_cluster *c, uint32_t reads_per_ctx,
                            uint32_t key_space, uint64_t g0, uint64_t g1,
                            uint64_t *sums, uint64_t *served,
                            uint64_t *deferred) {
  const uint32_t R = c->cfg.num_replicas;
  uint64_t sv = 0, df = 0;
  if (g1 > c->cfg.num_groups) g1 = c->cfg.num_groups;
  for (uint64_t g = g0; g < g1; ++g)
    for (uint32_t s = 0; s < R; ++s) {
      orc_node *n = node_at(c, g, s);
      uint64_t sum = 0;
      if (!n->hosted) continue;
      for (size_t k = 0; k < n->nrtr; ++k) {
        if (n->rtr[k].index > n->sm_index) {
          df += reads_per_ctx;
          continue;
        }
        for (uint32_t j = 0; j < reads_per_ctx; ++j) {
          uint64_t key = mix64(n->rtr[k].ctx.low ^
                               ((uint64_t)(j + 1) * 0x9E3779B97F4A7C15ull)) %
                         key_space;
          uint8_t kb[8];
          for (int b = 0; b < 8; ++b) kb[b] = (uint8_t)(key >> (8 * b));
          const kv_item *it = kv_find(&n->kv, kb, 8);
          uint64_t word = ~0ull;
          if (it) {
            uint32_t v0 = 0;
            for (uint32_t b = 0; b < it->vlen && b < 4; ++b)
              v0 |= (uint32_t)it->val[b] << (8 * b);
            word = ((uint64_t)it->vlen << 32) | v0;
          }
          sum += mix64(word ^ key ^ ((uint64_t)j << 56));
          sv++;
        }
      }
      if (n->nrtr) sums[g * R + s] = sum;
    }
  if (served) *served = sv;
  if (deferred) *deferred = df;
  return 0;
}

int orc_cluster_kv_lookup(orc_cluster *c, uint64_t g, uint32_t slot,
                          const uint8_t *key, uint32_t klen, uint8_t *val,
                          uint32_t cap, uint32_t *vlen) {
  const kv_item *it = kv_find(&node_at(c, g, slot)->kv, key, klen);
  if (!it) return 1;
  *vlen = it->vlen;
  if (it->vlen > cap) return -1;
  memcpy(val, it->val, it->vlen);
  return 0;
}

/* ---- rsm KAT hooks (internal/rsm/statemachine_test.go, encoded_test.go) */
/* GetPayload: payload length copied to out; -1 panic, -3 out of capacity */
long orc_get_payload(uint32_t type, const uint8_t *cmd, size_t clen,
                     uint8_t *out, size_t cap) {
  ORC_TRY(-1);
  uint8_t *owned;
  uint32_t plen;
  const uint8_t *p = get_payload(type, cmd, (uint32_t)clen, &plen, &owned);
  long rc = plen > cap ? -3 : (long)plen;
  if (rc >= 0 && plen) memcpy(out, p, plen);
  free(owned);
  ORC_END;
  return rc;
}

/* A StateMachine over KVTest with sm.lastApplied.index = sm.index =
 * applied (the tests' setup, statemachine_test.go:348-349). */
void *orc_sm_new(uint64_t applied_index, uint64_t applied_term) {
  orc_node *n = (orc_node *)calloc(1, sizeof(orc_node));
  n->sm_index = n->la_index = applied_index;
  n->sm_term = n->la_term = applied_term;
  return n;
}

void orc_sm_free(void *h) {
  orc_node *n = (orc_node *)h;
  if (!n) return;
  kv_free(&n->kv);
  ev_free(&n->applyq);
  free(n);
}

/* taskQ.Add(Task{Entries}) + Handle (statemachine.go:599-645).  Returns
 * the number of entries that reached KVTest.Update; -1 panic. */
long orc_sm_handle(void *h, const drb_entry *ents, size_t cnt,
                   const uint8_t *pool) {
  orc_node *n = (orc_node *)h;
  for (size_t i = 0; i < cnt; i++) {
    orc_entry e = entry_from_view(&ents[i], pool);
    ev_push(&n->applyq, &e);
    blob_unref(e.cmd);
  }
  drb_round_out out;
  memset(&out, 0, sizeof(out));
  jmp_buf jb;
  jmp_buf *prev = orc_jb;
  orc_jb = &jb;
  if (setjmp(jb)) {
    orc_jb = prev;
    ev_truncate(&n->applyq, 0);
    return -1;
  }
  sm_handle(n, 1, &out);
  orc_jb = prev;
  return (long)out.committed_entries;
}

/* GetLastApplied (statemachine.go:380-385) and KVTest.Count */
uint64_t orc_sm_last_applied(void *h) { return ((orc_node *)h)->la_index; }
uint64_t orc_sm_count(void *h) { return ((orc_node *)h)->kv.count; }

/* Lookup (kvtest.go:120-130): 0 found, 1 missing, -1 out of capacity */
int orc_sm_lookup(void *h, const uint8_t *key, uint32_t klen, uint8_t *val,
                  uint32_t cap, uint32_t *vlen) {
  const kv_item *it = kv_find(&((orc_node *)h)->kv, key, klen);
  if (!it) return 1;
  *vlen = it->vlen;
  if (it->vlen > cap) return -1;
  memcpy(val, it->val, it->vlen);
  return 0;
}
