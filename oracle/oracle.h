/*
 * oracle.h -- CPU restatement of dragonboat's replication fast path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in dragonboat_amd/ links, loads or
 * calls this code.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py use it, as the checker.
 *
 * It restates, function by function, the Go reference at
 * /root/reference (github.com/lni/dragonboat/v4): internal/raft
 * (remote.go, readindex.go, inmemory.go, logentry.go, entryutils.go,
 * raft.go, peer.go), the node-level step loop (node.go, node_test.go
 * step()), the rsm apply path (internal/rsm/statemachine.go, encoded.go),
 * the KVTest state machine (internal/tests/kvtest.go) and the raftpb
 * codecs (raft_optimized.go, entrybatch.go, message.go, messagebatch.go,
 * common.go).  Each function cites the file:line it follows.
 *
 * Parity pinning: the Go reference cannot be built here (no Go toolchain,
 * SURVEY.md 0/8c).  The restatement is pinned by the reference's own
 * known-answer tests, restated in tests/test_oracle_*.py, and by the
 * byte-level fixture tests/golden/ (see tests/golden/README.md).
 *
 * Error model: where the reference panics (plog.Panicf / panic) the oracle
 * longjmps back to the API entry, which returns -1 with orc_last_error()
 * describing the panic.
 */
#ifndef ORC_ORACLE_H
#define ORC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/drb_engine.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_PEERS 16
/* orc_raft.rem_kind: r.remotes, r.nonVotings, r.witnesses */
#define ORC_VOTING 0
#define ORC_NONVOTING 1
#define ORC_WITNESS 2

typedef struct orc_blob {
  uint32_t refs;
  uint32_t len;
  uint8_t data[];
} orc_blob;

/* pb.Entry (raftpb/entry.go:6-16) */
typedef struct orc_entry {
  uint64_t term, index, key, client_id, series_id, responded_to;
  uint32_t type;
  orc_blob *cmd; /* NULL == empty Cmd */
} orc_entry;

typedef struct orc_evec {
  orc_entry *v;
  size_t n, cap;
} orc_evec;

/* pb.Message (raftpb/message.go:6-20), Snapshot omitted (always empty) */
typedef struct orc_msg {
  uint32_t type, reject;
  uint64_t to, from, shard_id, term, log_term, log_index, commit, hint,
      hint_high;
  orc_evec ents;
} orc_msg;

typedef struct orc_mvec {
  orc_msg *v;
  size_t n, cap;
} orc_mvec;

/* remote (remote.go:72-80) */
typedef struct orc_remote {
  uint64_t match, next, snapshot_index;
  uint32_t state;
  int active;
} orc_remote;

typedef struct orc_ctx {
  uint64_t low, high;
} orc_ctx;

/* readStatus (readindex.go:21-26) */
typedef struct orc_rstatus {
  orc_ctx ctx;
  uint64_t index, from;
  uint64_t confirmed[ORC_MAX_PEERS];
  int nconfirmed;
} orc_rstatus;

/* readIndex (readindex.go:30-33); pending == queue (same ctx set) */
typedef struct orc_readindex {
  orc_rstatus *q;
  size_t n, cap;
} orc_readindex;

/* TestLogDB (internal/raft/logdb_test.go:24-170) -- the ILogDB the raft
 * core reads below inMemory.markerIndex; also models LogReader
 * (internal/logdb/logreader.go) which has the same range semantics. */
typedef struct orc_logdb {
  uint64_t marker_index, marker_term;
  orc_evec ents;
  uint64_t st_term, st_vote, st_commit;
} orc_logdb;

/* inMemory (inmemory.go:30-39); snapshots are not on this path */
typedef struct orc_inmem {
  orc_evec ents;
  uint64_t saved_to, marker_index, applied_to_index, applied_to_term;
  int shrunk;
} orc_inmem;

/* entryLog (logentry.go:78-84) */
typedef struct orc_log {
  orc_logdb *db;
  orc_inmem im;
  uint64_t committed, processed;
} orc_log;

typedef struct orc_rtr {
  uint64_t index;
  orc_ctx ctx;
} orc_rtr;

/* raft (raft.go:199-239), voting members only on this path */
typedef struct orc_raft {
  uint32_t state;
  uint64_t term, vote, leader_id, shard_id, replica_id, applied;
  uint64_t election_tick, heartbeat_tick, heartbeat_timeout, election_timeout;
  uint64_t randomized_election_timeout, tick_count;
  uint64_t leader_transfer_target;
  int check_quorum, pre_vote, quiesce, snapshotting, pending_config_change;
  int is_leader_transfer_target;
  int nrem;
  uint64_t rem_id[ORC_MAX_PEERS]; /* sorted ascending */
  orc_remote rem[ORC_MAX_PEERS];
  /* the member kind of each: r.remotes (0), r.nonVotings (1), r.witnesses
   * (2) (raft.go:199-239); the raft's own is its state (nonVoting / witness
   * replicas are in those states for good) */
  uint8_t rem_kind[ORC_MAX_PEERS];
  int nvotes;
  uint64_t vote_id[ORC_MAX_PEERS];
  int vote_ok[ORC_MAX_PEERS];
  int nmatched;
  uint64_t matched[ORC_MAX_PEERS];
  orc_log log;
  orc_readindex ri;
  orc_mvec msgs;
  orc_rtr *rtr;
  size_t nrtr, caprtr;
  orc_ctx *dropped_ri;
  size_t ndropped_ri, capdropped_ri;
  size_t ndropped_entries;
  int leader_update;
  uint64_t rng;
  int test_has_config_change_hook; /* 1: hasConfigChangeToApply() = false */
} orc_raft;

/* ---- error handling -------------------------------------------------- */
const char *orc_last_error(void);

/* ---- remote (remote.go) : KAT hooks ----------------------------------- */
void orc_remote_become_retry(orc_remote *r);
void orc_remote_retry_to_wait(orc_remote *r);
void orc_remote_wait_to_retry(orc_remote *r);
void orc_remote_become_wait(orc_remote *r);
void orc_remote_become_replicate(orc_remote *r);
void orc_remote_become_snapshot(orc_remote *r, uint64_t index);
int orc_remote_try_update(orc_remote *r, uint64_t index);
int orc_remote_progress(orc_remote *r, uint64_t last_index); /* -1 panic */
void orc_remote_responded_to(orc_remote *r);
int orc_remote_decrease_to(orc_remote *r, uint64_t rejected, uint64_t last);
int orc_remote_is_paused(orc_remote *r); /* -1 panic */

/* ---- readIndex (readindex.go) : KAT hooks ----------------------------- */
orc_readindex *orc_readindex_new(void);
void orc_readindex_free(orc_readindex *r);
int orc_readindex_add_request(orc_readindex *r, uint64_t index, uint64_t low,
                              uint64_t high, uint64_t from);
size_t orc_readindex_len(orc_readindex *r);
int orc_readindex_get(orc_readindex *r, size_t i, uint64_t *low,
                      uint64_t *high, uint64_t *index, uint64_t *from);
/* returns number of released statuses (written to out arrays), -1 panic */
int orc_readindex_confirm(orc_readindex *r, uint64_t low, uint64_t high,
                          uint64_t from, int quorum, uint64_t *out_low,
                          uint64_t *out_high, uint64_t *out_index,
                          uint64_t *out_from, int out_cap);
/* test-only corruption helper mirroring tests that poke r.queue */
int orc_readindex_push_raw_queue(orc_readindex *r, uint64_t low, uint64_t high,
                                 int front);

/* ---- sortMatchValues (raft.go:884-909) -------------------------------- */
void orc_sort_match_values(uint64_t *v, int n);

/* ---- TestLogDB / raft : harness for the reference's raft KATs --------- */
orc_logdb *orc_logdb_new(void);
void orc_logdb_free(orc_logdb *db);
int orc_logdb_append(orc_logdb *db, const drb_entry *ents, size_t n,
                     const uint8_t *pool);
int orc_logdb_compact(orc_logdb *db, uint64_t index);
void orc_logdb_set_state(orc_logdb *db, uint64_t term, uint64_t vote,
                         uint64_t commit);

/* newTestRaft (raft_etcd_test.go:3071); the raft does NOT own the logdb */
orc_raft *orc_raft_new_test(uint64_t id, const uint64_t *peers, int npeers,
                            uint64_t election, uint64_t heartbeat,
                            orc_logdb *db);
void orc_raft_free(orc_raft *r);
/* newTestNonVoting / newTestWitness: kind ORC_NONVOTING / ORC_WITNESS */
orc_raft *orc_raft_new_test_kind(uint64_t id, const uint64_t *peers,
                                 int npeers, const uint64_t *others,
                                 int nothers, int kind, uint64_t election,
                                 uint64_t heartbeat, orc_logdb *db);
/* addNode (kind ORC_VOTING) / addNonVoting / addWitness */
int orc_raft_add_member(orc_raft *r, uint64_t id, int kind);
/* the member kind of replica id (-1: unknown) */
int orc_raft_remote_kind(orc_raft *r, uint64_t id);
int orc_raft_handle(orc_raft *r, const drb_message *m, const drb_entry *ents,
                    const uint8_t *pool);
int orc_raft_peer_handle(orc_raft *r, const drb_message *m,
                         const drb_entry *ents, const uint8_t *pool);
int orc_raft_become_follower(orc_raft *r, uint64_t term, uint64_t leader);
int orc_raft_become_candidate(orc_raft *r);
int orc_raft_become_leader(orc_raft *r);
int orc_raft_load_state(orc_raft *r, uint64_t term, uint64_t vote,
                        uint64_t commit);
int orc_raft_broadcast_replicate(orc_raft *r);
int orc_raft_broadcast_heartbeat(orc_raft *r);
int orc_raft_try_commit(orc_raft *r);
int orc_raft_tick(orc_raft *r);
int orc_raft_campaign(orc_raft *r);
void orc_raft_set_check_quorum(orc_raft *r, int on);
void orc_raft_set_pre_vote(orc_raft *r, int on);
void orc_raft_set_randomized_election_timeout(orc_raft *r, uint64_t v);
int orc_raft_network_reset(orc_raft *r, uint64_t id, const uint64_t *ids,
                           int n);
/* readMessages(): copies (and clears) r.msgs.  Returns count; if more than
 * cap, returns the count without clearing.  Entries are appended to ents
 * and Cmd bytes to pool. */
long orc_raft_read_messages(orc_raft *r, drb_message *out, size_t cap,
                            drb_entry *ents, size_t ent_cap, uint8_t *pool,
                            size_t pool_cap);
/* entryLog views: which = 0 entriesToApply, 1 entriesToSave,
 * 2 all entries (getAllEntries, logentry_etcd_test.go:33) */
long orc_raft_log_entries(orc_raft *r, int which, drb_entry *out, size_t cap,
                          uint8_t *pool, size_t pool_cap);
int orc_raft_log_term(orc_raft *r, uint64_t index, uint64_t *term);
void orc_raft_info(orc_raft *r, drb_replica_state *st);
int orc_raft_remote(orc_raft *r, uint64_t id, orc_remote *out);
int orc_raft_set_remote(orc_raft *r, uint64_t id, const orc_remote *in);
size_t orc_raft_ready_to_read(orc_raft *r, uint64_t *index, uint64_t *low,
                              uint64_t *high, size_t cap);
size_t orc_raft_dropped_read_indexes(orc_raft *r);
/* election KAT hooks: fields the reference's tests assign directly */
enum {
  ORC_POKE_STATE = 0,
  ORC_POKE_TERM,
  ORC_POKE_VOTE,
  ORC_POKE_ELECTION_TICK,
  ORC_POKE_ELECTION_TIMEOUT,
  ORC_POKE_COMMITTED,
  ORC_POKE_APPLIED,
  ORC_POKE_CONFIG_CHANGE_HOOK, /* 1: hasNotAppliedConfigChange = test hook */
  ORC_POKE_LEADER_TRANSFER_TARGET,
  ORC_POKE_IS_LEADER_TRANSFER_TARGET
};
int orc_raft_poke(orc_raft *r, int field, uint64_t v);
uint64_t orc_raft_peek(orc_raft *r, int field);
int orc_raft_reset(orc_raft *r, uint64_t term);
int orc_raft_become_pre_vote_candidate(orc_raft *r);
int orc_raft_draw_timeout_time_for_election(orc_raft *r);
int orc_raft_term_not_matched(orc_raft *r, const drb_message *m,
                              const drb_entry *ents, const uint8_t *pool);
/* entryLog KAT hooks */
int orc_log_commit_to(orc_raft *r, uint64_t index);
int orc_log_try_commit(orc_raft *r, uint64_t index, uint64_t term);
int orc_log_match_term(orc_raft *r, uint64_t index, uint64_t term);
int orc_log_up_to_date(orc_raft *r, uint64_t index, uint64_t term);
long orc_log_conflict_index(orc_raft *r, const drb_entry *ents, size_t n);
int orc_log_try_append(orc_raft *r, uint64_t index, const drb_entry *ents,
                       size_t n, const uint8_t *pool);
int orc_log_append(orc_raft *r, const drb_entry *ents, size_t n,
                   const uint8_t *pool);
int orc_log_commit_update(orc_raft *r, uint64_t stable_log_to,
                          uint64_t stable_log_term, uint64_t processed,
                          uint64_t last_applied);
/* raft KAT hooks (raft_test.go:1578-1611, 2952-3037) */
long orc_raft_make_replicate(orc_raft *r, uint64_t to, uint64_t next,
                             uint64_t max_size, drb_message *out,
                             drb_entry *ents, size_t ent_cap, uint8_t *pool,
                             size_t pool_cap);
int orc_raft_append_entries(orc_raft *r, const drb_entry *ents, size_t n,
                            const uint8_t *pool);
int orc_raft_broadcast_heartbeat_hint(orc_raft *r, uint64_t low,
                                      uint64_t high);
int orc_raft_has_committed_entry_at_current_term(orc_raft *r);
size_t orc_raft_read_index_len(orc_raft *r);

/* ---- inMemory (inmemory.go) : KAT hooks (inmemory_test.go:260-548) ---- */
orc_inmem *orc_inmem_new(uint64_t marker_index, const drb_entry *ents,
                         size_t n, uint64_t saved_to, int shrunk);
void orc_inmem_free(orc_inmem *im);
int orc_inmem_merge(orc_inmem *im, const drb_entry *ents, size_t n);
int orc_inmem_saved_log_to(orc_inmem *im, uint64_t index, uint64_t term);
int orc_inmem_applied_log_to(orc_inmem *im, uint64_t index);
void orc_inmem_restore(orc_inmem *im, uint64_t ss_index, uint64_t ss_term);
long orc_inmem_entries_to_save(orc_inmem *im, uint64_t *first);
int orc_inmem_last_index(orc_inmem *im, uint64_t *idx);
int orc_inmem_get_term(orc_inmem *im, uint64_t index, uint64_t *term);
void orc_inmem_info(orc_inmem *im, uint64_t *out5);

/* ---- batched LogDB records (internal/logdb/batch.go) ------------------ */
typedef struct orc_batchdb orc_batchdb;
orc_batchdb *orc_batchdb_new(void);
void orc_batchdb_free(orc_batchdb *db);
/* batchedEntries.record of one Update's EntriesToSave: records Put, -1 */
long orc_batchdb_record(orc_batchdb *db, uint64_t shard, uint64_t replica,
                        const drb_entry *ents, size_t n, const uint8_t *pool);
/* record i of the last call: value length (copied to buf), -1 no such
 * record, < -1 buf too small (-(len) - 2) */
long orc_batchdb_out(orc_batchdb *db, size_t i, uint64_t *batch, uint8_t *buf,
                     size_t cap);
void orc_batch_id_range(uint64_t low, uint64_t high, uint64_t *lo_id,
                        uint64_t *hi_id);
int orc_batch_compact(drb_entry *e, size_t n, int restore);
long orc_batch_merged_first(const drb_entry *eb, size_t ne,
                            const drb_entry *lb, size_t nl, drb_entry *out);

/* ---- tan LogDB write path (internal/tan: record.go, db.go, crc.go) ---- */
/* xxhash.Sum64 (cespare/xxhash/v2 v2.1.2; tan getCRC = its low 32 bits) */
uint64_t orc_xxh64(const uint8_t *p, size_t n);
/* record writer (record.go:414-653) over an in-memory io.Writer */
typedef struct orc_tanw orc_tanw;
orc_tanw *orc_tanw_new(void);
void orc_tanw_free(orc_tanw *w);
int64_t orc_tanw_write_record(orc_tanw *w, const uint8_t *p, size_t n);
int orc_tanw_flush(orc_tanw *w, int close);
int64_t orc_tanw_size(const orc_tanw *w);
int64_t orc_tanw_last_record_offset(const orc_tanw *w);
long orc_tanw_bytes(const orc_tanw *w, uint8_t *buf, size_t cap);
/* record reader (record.go:163-311) over a whole log */
#define ORC_TAN_ZEROED (-2)         /* ErrZeroedChunk */
#define ORC_TAN_INVALID (-3)        /* ErrInvalidChunk */
#define ORC_TAN_CRC (-4)            /* ErrCRCMismatch */
#define ORC_TAN_UNEXPECTED_EOF (-5) /* io.ErrUnexpectedEOF */
long orc_tan_read(const uint8_t *file, size_t size, int64_t *offsets,
                  size_t *lens, size_t max_recs, uint8_t *data,
                  size_t data_cap);
/* Update.MarshalTo (raftpb/update.go:128-169), empty Snapshot */
size_t orc_update_size_bound(const drb_entry *ents, size_t n);
size_t orc_update_marshal(uint64_t shard, uint64_t replica, uint64_t term,
                          uint64_t vote, uint64_t commit,
                          const drb_entry *ents, size_t n,
                          const uint8_t *pool, uint8_t *buf);
/* one replica's tan db (db.go:97-130; max_log_size 0: 64 MiB) */
typedef struct orc_tandb orc_tandb;
orc_tandb *orc_tandb_new(int64_t max_log_size);
void orc_tandb_free(orc_tandb *db);
int orc_tandb_write(orc_tandb *db, uint64_t shard, uint64_t replica,
                    uint64_t term, uint64_t vote, uint64_t commit,
                    const drb_entry *ents, size_t n, const uint8_t *pool,
                    int *sync);
void orc_tandb_last(const orc_tandb *db, int64_t *out6);
long orc_tandb_file(const orc_tandb *db, size_t log, uint8_t *buf, size_t cap);

/* ---- rsm (statemachine.go, encoded.go) : KAT hooks -------------------- */
long orc_get_payload(uint32_t type, const uint8_t *cmd, size_t clen,
                     uint8_t *out, size_t cap);
void *orc_sm_new(uint64_t applied_index, uint64_t applied_term);
void orc_sm_free(void *h);
long orc_sm_handle(void *h, const drb_entry *ents, size_t cnt,
                   const uint8_t *pool);
uint64_t orc_sm_last_applied(void *h);
uint64_t orc_sm_count(void *h);
int orc_sm_lookup(void *h, const uint8_t *key, uint32_t klen, uint8_t *val,
                  uint32_t cap, uint32_t *vlen);

/* ---- BSP cluster: node_test.go step() over G groups x R replicas ------ */
typedef struct orc_cluster orc_cluster;

typedef struct orc_cluster_cfg {
  uint64_t num_groups;
  uint64_t first_shard_id;
  uint32_t num_replicas;
  uint32_t election_rtt, heartbeat_rtt, check_quorum;
  uint64_t seed;
  uint64_t logdb_keep; /* 0: keep every saved entry; else compact behind */
  uint32_t quiesce;    /* Config.Quiesce (config.go:195) */
  uint32_t pre_vote;   /* Config.PreVote (config.go:178-183) */
  /* NULL: group g is global group g.  Else group g of this cluster is
   * global group gids[g] (ShardID, seeds): a sample of a large engine's
   * groups, simulated alone (groups are independent) */
  const uint64_t *gids;
} orc_cluster_cfg;

orc_cluster *orc_cluster_new(const orc_cluster_cfg *cfg);
void orc_cluster_free(orc_cluster *c);
/* bootstrap + elect `leader_slot` at term 2 + settle */
int orc_cluster_setup_steady(orc_cluster *c, uint32_t leader_slot);
/* stage proposals (counts[g] from ents[g*max_per_group..]) for next round */
int orc_cluster_stage_proposals(orc_cluster *c, const uint32_t *counts,
                                uint32_t max_per_group, const drb_entry *ents,
                                const uint8_t *pool);
/* the same at replica ID `replica` of every group (0: the leader) */
int orc_cluster_stage_proposals_at(orc_cluster *c, const uint32_t *counts,
                                   uint32_t max_per_group,
                                   const drb_entry *ents, const uint8_t *pool,
                                   uint32_t replica);
/* replica slots that are nonVotings / witnesses in every group (after
 * setup_steady; the leader slot must be a voting member) */
int orc_cluster_set_member_kinds(orc_cluster *c, uint32_t nonvoting_mask,
                                 uint32_t witness_mask);
/* stage one ReadIndex ctx per group (low==0: none) for next round */
int orc_cluster_stage_read_index(orc_cluster *c, const uint64_t *low,
                                 const uint64_t *high);
int64_t orc_cluster_request_leader_transfer(orc_cluster *c, uint32_t slot,
                                            const uint32_t *targets);
int orc_cluster_stage_read_index_at(orc_cluster *c, const uint64_t *low,
                                    const uint64_t *high, uint32_t replica);
int orc_cluster_ingest(orc_cluster *c, const drb_message *m, size_t n,
                       const drb_entry *ents, const uint8_t *pool);
/* one step round; groups [g0, g1) only (for threaded timing) */
int orc_cluster_round(orc_cluster *c, int tick, drb_round_out *out);
int orc_cluster_round_range(orc_cluster *c, int tick, uint64_t g0, uint64_t g1,
                            drb_round_out *out);
int orc_cluster_end_round(orc_cluster *c);
int orc_cluster_export(orc_cluster *c, uint64_t g, uint32_t slot,
                       drb_replica_state *st);
/* replica (g, slot) takes state st and the log ents (drb_import_replicas +
 * drb_import_log on the engine side); see node_oracle.c */
int orc_cluster_import(orc_cluster *c, uint64_t g, uint32_t slot,
                       const drb_replica_state *st, const drb_entry *ents,
                       size_t n, const uint8_t *pool);
long orc_cluster_export_log(orc_cluster *c, uint64_t g, uint32_t slot,
                            uint64_t lo, uint64_t hi, drb_entry *out,
                            uint8_t *pool, size_t pool_cap);
long orc_cluster_export_outbox(orc_cluster *c, uint64_t g, uint32_t slot,
                               drb_message *out, size_t cap, drb_entry *ents,
                               size_t ent_cap, uint8_t *pool, size_t pool_cap);
long orc_cluster_export_kv(orc_cluster *c, uint64_t g, uint32_t slot,
                           uint8_t *keys, uint32_t *klens, uint8_t *vals,
                           uint32_t *vlens, size_t cap, size_t key_cap,
                           size_t val_cap);
long orc_cluster_export_ready(orc_cluster *c, uint64_t g, uint32_t slot,
                              drb_ready_to_read *out, size_t cap);
long orc_cluster_export_saved(orc_cluster *c, uint64_t g, uint32_t slot,
                              uint8_t *buf, size_t cap, uint32_t *crc);
int orc_cluster_tan_write(orc_cluster *c, uint64_t g, uint32_t slot,
                          orc_tandb *db, int *sync);
void orc_cluster_set_pre_vote(orc_cluster *c, int on);
int orc_cluster_set_hosted(orc_cluster *c, uint64_t g, uint32_t slot,
                           int hosted);
/* make an engine-importable image of replica (g,slot) */
int orc_cluster_serve_reads(orc_cluster *c, uint32_t reads_per_ctx,
                            uint32_t key_space, uint64_t g0, uint64_t g1,
                            uint64_t *sums, uint64_t *served,
                            uint64_t *deferred);
int orc_cluster_kv_lookup(orc_cluster *c, uint64_t g, uint32_t slot,
                          const uint8_t *key, uint32_t klen, uint8_t *val,
                          uint32_t cap, uint32_t *vlen);

/* ---- codecs (raftpb) -------------------------------------------------- */
/* Entry.Size (raft_optimized.go:84-158) */
size_t orc_entry_size(const drb_entry *e);
/* Entry.marshalTo (raft_optimized.go:166-300) */
size_t orc_entry_marshal(const drb_entry *e, const uint8_t *pool, uint8_t *buf);
/* Entry.unmarshal (raft_optimized.go:308-656); returns bytes consumed or -1 */
long orc_entry_unmarshal(const uint8_t *buf, size_t len, drb_entry *e,
                         uint8_t *pool, size_t pool_cap, size_t *pool_used);
/* EntryBatch.Size / MarshalTo (entrybatch.go:25-58) */
size_t orc_entrybatch_size(const drb_entry *e, size_t n);
size_t orc_entrybatch_marshal(const drb_entry *e, size_t n, const uint8_t *pool,
                              uint8_t *buf);
/* EntryBatch.Unmarshal (entrybatch.go:60-146); returns entry count or -1 */
long orc_entrybatch_unmarshal(const uint8_t *buf, size_t len, drb_entry *out,
                              size_t cap, uint8_t *pool, size_t pool_cap);
/* crc32.ChecksumIEEE (Go hash/crc32, tcp.go:146) */
uint32_t orc_crc32_ieee(const uint8_t *p, size_t n);
/* pb.Message Size / MarshalTo (message.go:32-124), the embedded Snapshot
 * empty; Unmarshal (raft_optimized.go:659-983): bytes consumed, -1
 * malformed, -2 non-empty Snapshot */
size_t orc_message_size(const drb_message *m, const drb_entry *ents);
size_t orc_message_marshal(const drb_message *m, const drb_entry *ents,
                           const uint8_t *pool, uint8_t *buf);
long orc_message_unmarshal(const uint8_t *buf, size_t len, drb_message *m,
                           drb_entry *ents, size_t ent_cap, size_t *n_ents,
                           uint8_t *pool, size_t pool_cap, size_t *pool_used);
/* pb.MessageBatch MarshalTo (messagebatch.go:23-70) / Unmarshal
 * (raft_optimized.go:1056-1207) */
size_t orc_messagebatch_marshal(const drb_message *ms, size_t n,
                                const drb_entry *ents, const uint8_t *pool,
                                uint64_t deployment_id, const char *src,
                                size_t src_len, uint32_t bin_ver,
                                uint8_t *buf);
long orc_messagebatch_unmarshal(const uint8_t *buf, size_t len,
                                drb_message *ms, size_t cap, drb_entry *ents,
                                size_t ent_cap, uint8_t *pool, size_t pool_cap,
                                uint64_t *deployment_id, uint32_t *bin_ver,
                                char *src, size_t src_cap, size_t *src_len);
/* requestHeader encode / decode (internal/transport/tcp.go:64-112) and the
 * writeMessage frame (tcp.go:142-178) */
void orc_request_header_encode(uint16_t method, uint64_t size, uint32_t crc,
                               uint8_t *buf18);
int orc_request_header_decode(const uint8_t *buf18, uint16_t *method,
                              uint64_t *size, uint32_t *crc);
size_t orc_wire_frame(const uint8_t *payload, size_t n, uint8_t *out);
/* PBKV codec (internal/tests/kvpb/kv.go) */
size_t orc_pbkv_marshal(const uint8_t *key, uint32_t klen, const uint8_t *val,
                        uint32_t vlen, uint8_t *buf);
int orc_pbkv_unmarshal(const uint8_t *buf, size_t len, const uint8_t **key,
                       uint32_t *klen, const uint8_t **val, uint32_t *vlen);

#ifdef __cplusplus
}
#endif
#endif
