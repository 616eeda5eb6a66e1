/*
 * oracle_internal.h -- internals shared by the oracle translation units.
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 */
#ifndef ORC_ORACLE_INTERNAL_H
#define ORC_ORACLE_INTERNAL_H

#include <setjmp.h>
#include <stdlib.h>

#include "oracle.h"

#define ORC_ERR_COMPACTED 1   /* raft.ErrCompacted (logentry.go:31) */
#define ORC_ERR_UNAVAILABLE 2 /* raft.ErrUnavailable (logentry.go:40) */

extern __thread jmp_buf *orc_jb;
void orc_panic(const char *fmt, ...) __attribute__((noreturn, format(printf, 1, 2)));

#define ORC_TRY(errval)            \
  jmp_buf orc__jb;                 \
  jmp_buf *orc__prev = orc_jb;     \
  orc_jb = &orc__jb;               \
  if (setjmp(orc__jb)) {           \
    orc_jb = orc__prev;            \
    return errval;                 \
  }
#define ORC_END orc_jb = orc__prev

orc_blob *blob_new(const uint8_t *p, uint32_t len);
static inline orc_blob *blob_ref(orc_blob *b) {
  if (b) b->refs++;
  return b;
}
static inline void blob_unref(orc_blob *b) {
  if (b && --b->refs == 0) free(b);
}

void ev_push(orc_evec *v, const orc_entry *e);
void ev_truncate(orc_evec *v, size_t n);
void ev_drop_front(orc_evec *v, size_t k);
void ev_free(orc_evec *v);
void ev_copy_range(orc_evec *dst, const orc_entry *src, size_t n);
void msg_free(orc_msg *m);
void mv_push(orc_mvec *v, const orc_msg *m);
void mv_clear(orc_mvec *v);
void mv_free(orc_mvec *v);
orc_entry entry_from_view(const drb_entry *e, const uint8_t *pool);
int entry_to_view(const orc_entry *e, drb_entry *out, uint8_t *pool,
                  size_t pool_cap, size_t *pool_used);
orc_msg orc_msg_from_view(const drb_message *v, const drb_entry *ents,
                          const uint8_t *pool);
int msg_to_view(const orc_msg *m, drb_message *out, drb_entry *ents,
                size_t ent_cap, size_t *ent_used, uint8_t *pool,
                size_t pool_cap, size_t *pool_used);

/* logdb / log */
void db_append(orc_logdb *db, const orc_entry *ents, size_t n);
uint64_t log_last(const orc_log *l);
int log_term(const orc_log *l, uint64_t index, uint64_t *term);
int log_has_entries_to_apply(const orc_log *l);
int log_entries_to_apply(const orc_log *l, orc_evec *out);
const orc_entry *log_entries_to_save(const orc_log *l, size_t *n);
void log_commit_to(orc_log *l, uint64_t index);
void log_commit_update(orc_log *l, uint64_t stable_log_to,
                       uint64_t stable_log_term, uint64_t processed,
                       uint64_t last_applied);

/* raft */
orc_raft *raft_new(uint64_t shard, uint64_t id, uint64_t election,
                   uint64_t heartbeat, int check_quorum, orc_logdb *db,
                   uint64_t seed);
void raft_free(orc_raft *r);
void raft_set_test_peers(orc_raft *r, const uint64_t *peers, int npeers);
void raft_add_node(orc_raft *r, uint64_t id);
void raft_bootstrap(orc_raft *r, const uint64_t *ids, int n,
                    orc_blob *const *cmds);
int raft_handle_msg(orc_raft *r, orc_msg *m);
void raft_tick_public(orc_raft *r, int quiesced);
void peer_handle(orc_raft *r, orc_msg *m);
void raft_clear_msgs(orc_raft *r);
void raft_become_follower(orc_raft *r, uint64_t term, uint64_t leader);
int raft_rem_idx(const orc_raft *r, uint64_t id);

/* codecs */
size_t orc_configchange_marshal_addnode(uint64_t replica_id,
                                        const char *address, uint8_t *buf);

#endif
