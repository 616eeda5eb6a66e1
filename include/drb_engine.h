/*
 * drb_engine.h -- C ABI of the MI355X-native batched multi-group Raft
 * replication engine (dragonboat_amd).
 *
 * This header is the drop-in boundary.  Every entry point replaces one
 * interface on dragonboat's replication fast path; the reference interface
 * it stands in for is cited next to it (paths relative to the dragonboat
 * v4 source tree).  All types are plain C: fixed-width integers, plain
 * pointers and sizes.  No torch / HIP types cross this boundary.
 *
 * Execution model:
 *   One engine owns G Raft groups x R replica slots resident in HBM as
 *   structure-of-arrays.  Replica slot s of every group has replica ID s+1.
 *   drb_step_round() executes ONE step round for every hosted replica, with
 *   exactly the semantics of one iteration of dragonboat's step loop
 *   (node_test.go:274-353 / engine.go:1304-1364): each replica drains its
 *   inbox (messages sent in the previous round), handles its tick, ReadIndex
 *   batch and proposals, builds its Update, applies committed entries to
 *   its in-memory KV state machine and commits the Update; messages it
 *   sends are delivered at the end of the round.
 *
 * Error behaviour: functions return DRB_OK (0) or a negative DRB_E* code.
 * Conditions the reference reports with plog.Panicf mark the replica
 * DRB_F_ERROR; paths that stay on the reference CPU code (election,
 * membership change, snapshot, session management, higher/lower term
 * messages) mark it DRB_F_FALLBACK *before* it mutates any state, so the
 * pre-round state can be exported to the CPU raft.Peer.  One exception is
 * the state machine: the rsm applies committed entries after the raft
 * round (engine.go:1153 apply workers, statemachine.go:599), so an entry
 * the fast path cannot apply (KV table or value pool full, an entry a
 * proposal check could not see) stops the APPLY only: the replica is
 * marked DRB_F_FALLBACK | DRB_F_APPLY_STOPPED, its raft state is the
 * completed round's, and the committed entries (sm_index, pushed_index]
 * are pushed but unapplied -- the rsm task queue a CPU StateMachine
 * resumes from (drb_export_log reads them from the window).
 *
 * Threading: drb_ingest / drb_ingest_wire may be called from several
 * transport threads at once (each call stages under the engine's ingest
 * lock, which drb_step_round* also takes while it launches a round and
 * advances the round number, so a message lands either before a round's
 * launch -- read by that round -- or after it, read by the next); each
 * such thread reads its connection into a buffer of its own
 * (drb_ingest_buffer_alloc).  Every other entry point is driven by one
 * host thread, which is not re-entrant (the reference holds node.raftMu
 * across stepNode, node.go:1140).
 */
#ifndef DRB_ENGINE_H
#define DRB_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRB_MAX_REPLICAS 8
#define DRB_RI_DEPTH 4        /* device readIndex queue depth (readindex.go:30-33) */

/* status codes */
#define DRB_OK 0
#define DRB_EINVAL (-1)
#define DRB_EDEVICE (-2)
#define DRB_ENOMEM (-3)
#define DRB_ENOSYS (-4)
#define DRB_ERANGE (-5)
#define DRB_EAGAIN (-6)  /* retry later: the call would race a step in
                          * flight (drb_ingest before drb_exchange_*) */
#define DRB_EDIVERTED (-7) /* drb_ingest: messages were diverted to the CPU
                            * path; only drb_ingest_ex says which */

/* raftpb.MessageType (raftpb/types.go:8-37) */
enum drb_message_type {
  DRB_MSG_LOCAL_TICK = 0,
  DRB_MSG_ELECTION = 1,
  DRB_MSG_LEADER_HEARTBEAT = 2,
  DRB_MSG_CONFIG_CHANGE_EVENT = 3,
  DRB_MSG_NOOP = 4,
  DRB_MSG_PING = 5,
  DRB_MSG_PONG = 6,
  DRB_MSG_PROPOSE = 7,
  DRB_MSG_SNAPSHOT_STATUS = 8,
  DRB_MSG_UNREACHABLE = 9,
  DRB_MSG_CHECK_QUORUM = 10,
  DRB_MSG_BATCHED_READ_INDEX = 11,
  DRB_MSG_REPLICATE = 12,
  DRB_MSG_REPLICATE_RESP = 13,
  DRB_MSG_REQUEST_VOTE = 14,
  DRB_MSG_REQUEST_VOTE_RESP = 15,
  DRB_MSG_INSTALL_SNAPSHOT = 16,
  DRB_MSG_HEARTBEAT = 17,
  DRB_MSG_HEARTBEAT_RESP = 18,
  DRB_MSG_READ_INDEX = 19,
  DRB_MSG_READ_INDEX_RESP = 20,
  DRB_MSG_QUIESCE = 21,
  DRB_MSG_SNAPSHOT_RECEIVED = 22,
  DRB_MSG_LEADER_TRANSFER = 23,
  DRB_MSG_TIMEOUT_NOW = 24,
  DRB_MSG_RATE_LIMIT = 25,
  DRB_MSG_REQUEST_PREVOTE = 26,
  DRB_MSG_REQUEST_PREVOTE_RESP = 27,
  DRB_MSG_LOG_QUERY = 28
};

/* raftpb.EntryType (raftpb/types.go) */
enum drb_entry_type {
  DRB_ENTRY_APPLICATION = 0,
  DRB_ENTRY_CONFIG_CHANGE = 1,
  DRB_ENTRY_ENCODED = 2,
  DRB_ENTRY_METADATA = 3
};

/* raft.State (internal/raft/raft.go:63-71) */
enum drb_role {
  DRB_FOLLOWER = 0,
  DRB_CANDIDATE = 1,
  DRB_PREVOTE_CANDIDATE = 2,
  DRB_LEADER = 3,
  DRB_NONVOTING = 4,
  DRB_WITNESS = 5
};

/* remoteStateType (internal/raft/remote.go:54-59) */
enum drb_remote_fsm {
  DRB_REMOTE_RETRY = 0,
  DRB_REMOTE_WAIT = 1,
  DRB_REMOTE_REPLICATE = 2,
  DRB_REMOTE_SNAPSHOT = 3
};

/* drb_replica_state.flags */
#define DRB_F_HOSTED 1u    /* stepped by this engine */
#define DRB_F_FALLBACK 2u  /* handed back to the CPU raft.Peer, frozen here */
#define DRB_F_ERROR 4u     /* invariant violation (reference: plog.Panicf) */
#define DRB_F_APPLY_STOPPED 8u /* with FALLBACK: the raft round completed,
                                * the rsm apply stopped at sm_index + 1 */

/* drb_replica_state.fallback_reason */
enum drb_fallback_reason {
  DRB_FB_NONE = 0,
  DRB_FB_TERM_MISMATCH = 1,     /* raft.go:1540-1590 term gate not on fast path */
  DRB_FB_MESSAGE_TYPE = 2,      /* message type handled only on the CPU path */
  DRB_FB_ELECTION = 3,          /* raft.go:602 election timeout */
  DRB_FB_CHECK_QUORUM = 4,      /* raft.go:1785 leader lost quorum */
  DRB_FB_ENTRY_TYPE = 5,        /* config change / session / compressed entry */
  DRB_FB_CAPACITY = 6,          /* window / mailbox / readIndex capacity */
  DRB_FB_ROLE = 7,              /* candidate / non-voting / witness */
  DRB_FB_SNAPSHOT = 9,          /* a remote in the Snapshot state
                                 * (remote.go:54-59, 128-141) */
  DRB_ERR_LOG_RANGE = 100,      /* internal invariant: a read below the
                                 * resident window the pre-pass did not
                                 * predict (it falls back with CAPACITY) */
  DRB_ERR_COMMIT = 101,         /* logentry.go:336-349 commitTo panic */
  DRB_ERR_APPEND = 103,         /* entryutils.go:36-48 hole / term regress,
                                 * logentry.go:296-321 committed entry
                                 * changed */
  DRB_ERR_APPLY = 104,          /* statemachine.go:935-969 malformed entry */
  DRB_ERR_READINDEX = 105,      /* readindex.go:43-115 invariant */
  DRB_ERR_TRANSFER = 106,       /* raft.go:1929-1931 LeaderTransfer without
                                 * a target */
  DRB_ERR_PROPOSE = 107         /* internal invariant: proposals at a replica
                                 * that stepped down and knows a leader, with
                                 * no forward rows (the pre-pass routes that
                                 * round to the CPU path) */
};

/* remote (internal/raft/remote.go:72-80); remotes[] is indexed by slot. */
typedef struct drb_remote_state {
  uint64_t match;
  uint64_t next;
  uint32_t state;   /* drb_remote_fsm */
  uint32_t active;  /* remote.active (remote.go:215-225) */
} drb_remote_state;

/* readStatus (internal/raft/readindex.go:21-26), kept in queue order. */
typedef struct drb_read_status {
  uint64_t ctx_low;    /* pb.SystemCtx.Low */
  uint64_t ctx_high;   /* pb.SystemCtx.High */
  uint64_t index;
  uint64_t from;
  uint32_t confirmed;  /* bit s set: replica slot s confirmed */
  uint32_t pad;
} drb_read_status;

/*
 * Per-replica state: the fields of raft (raft.go:199-239), entryLog
 * (logentry.go:78-84), inMemory (inmemory.go:30-39), Peer.prevState
 * (peer.go:59), node (node.go appliedIndex/confirmedIndex/pushedIndex) and
 * the rsm/KV apply cursor that the fast path reads or writes.  This is
 * the record drb_export_replicas()/drb_import_replicas() move between the
 * device SoA and a CPU raft.Peer on fallback.
 */
typedef struct drb_replica_state {
  uint64_t shard_id;
  uint64_t replica_id;
  uint64_t term;
  uint64_t vote;
  uint64_t leader_id;
  uint64_t applied;                    /* raft.applied */
  uint64_t election_tick;
  uint64_t heartbeat_tick;
  uint64_t randomized_election_timeout;
  uint64_t tick_count;
  uint64_t committed;                  /* entryLog.committed */
  uint64_t processed;                  /* entryLog.processed */
  uint64_t last_index;                 /* entryLog.lastIndex() */
  uint64_t marker_index;               /* inMemory.markerIndex */
  uint64_t saved_to;                   /* inMemory.savedTo */
  uint64_t applied_to_index;           /* inMemory.appliedToIndex */
  uint64_t applied_to_term;            /* inMemory.appliedToTerm */
  uint64_t applied_index;              /* node.appliedIndex */
  uint64_t confirmed_index;            /* node.confirmedIndex */
  uint64_t pushed_index;               /* node.pushedIndex */
  uint64_t prev_term;                  /* Peer.prevState.Term */
  uint64_t prev_vote;                  /* Peer.prevState.Vote */
  uint64_t prev_commit;                /* Peer.prevState.Commit */
  uint64_t sm_index;                   /* StateMachine.index (statemachine.go:716) */
  uint64_t sm_term;                    /* StateMachine.term */
  uint64_t kv_count;                   /* KVTest.Count (kvtest.go:146) */
  /* node.qs, quiesceState (quiesce.go:23-33); all 0 with Quiesce off */
  uint64_t qs_current_tick;
  uint64_t qs_idle_since;
  uint64_t qs_quiesced_since;          /* 0: not quiesced */
  uint64_t qs_exit_quiesce_tick;
  /* the state of raft.rand, the randomized election timeout's source
   * (raft.go:658-661): splitmix64, one draw per reset (elections) */
  uint64_t rng;
  uint32_t role;                       /* drb_role */
  uint32_t flags;                      /* DRB_F_* */
  uint32_t fallback_reason;            /* drb_fallback_reason */
  uint32_t ri_count;                   /* valid entries in ri[] */
  /* a candidate's votes (raft.votes, raft.go:1125-1147): bit s of the low
   * byte = replica slot s answered, of the next byte = it granted */
  uint32_t votes;
  /* a leader's raft.leaderTransferTarget (raft.go:375-381): the replica ID
   * leadership is being handed to, 0 none (elections) */
  uint32_t transfer;
  drb_remote_state remotes[DRB_MAX_REPLICAS];
  drb_read_status ri[DRB_RI_DEPTH];
} drb_replica_state;

/* pb.Entry (raftpb/entry.go:6-16); Cmd bytes live in a caller pool. */
typedef struct drb_entry {
  uint64_t term;
  uint64_t index;
  uint64_t key;
  uint64_t client_id;
  uint64_t series_id;
  uint64_t responded_to;
  uint32_t type;      /* drb_entry_type */
  uint32_t cmd_len;
  uint64_t cmd_off;   /* byte offset of Cmd in the pool */
} drb_entry;

/*
 * pb.Message (raftpb/message.go:6-20) for the fields this path uses; the
 * embedded Snapshot is always empty here.  Entries are
 * ents[entries_off .. entries_off + n_entries).
 */
typedef struct drb_message {
  uint64_t shard_id;
  uint64_t from;
  uint64_t to;
  uint64_t term;
  uint64_t log_term;
  uint64_t log_index;
  uint64_t commit;
  uint64_t hint;
  uint64_t hint_high;
  uint32_t type;      /* drb_message_type */
  uint32_t reject;
  uint64_t n_entries;
  uint64_t entries_off;
} drb_message;

/* pb.ReadyToRead (raftpb/update.go) */
typedef struct drb_ready_to_read {
  uint64_t shard_id;
  uint64_t replica_id;
  uint64_t index;
  uint64_t ctx_low;
  uint64_t ctx_high;
} drb_ready_to_read;

/* Engine sizing.  Raft knobs mirror config.Config (config/config.go:65-200). */
typedef struct drb_config {
  uint64_t num_groups;       /* G groups on this device */
  uint64_t first_shard_id;   /* ShardID of group g = first_shard_id + g */
  uint32_t num_replicas;     /* R, 1..DRB_MAX_REPLICAS; replica IDs 1..R */
  uint32_t window;           /* W resident entries per replica (power of 2) */
  uint32_t cmd_cap;          /* max Cmd bytes per resident entry (mult. of
                              * 16, <= 1040) */
  uint32_t max_props;        /* max proposals per group per round */
  uint32_t prop_slots;       /* staged proposal batches */
  uint32_t ri_slots;         /* staged ReadIndex batches */
  uint32_t mailbox;          /* records per (sender, receiver) per round, 4..24 */
  uint32_t kv_slots;         /* KV open-addressing slots per replica (pow2) */
  uint32_t kv_val_cap;       /* max value bytes per KV slot (<= 124 inline,
                              * else out of line, <= 1024) */
  uint32_t election_rtt;     /* Config.ElectionRTT */
  uint32_t heartbeat_rtt;    /* Config.HeartbeatRTT */
  uint32_t check_quorum;     /* Config.CheckQuorum */
  int32_t device;            /* HIP device ordinal */
  /* bytes per replica for the round's EntriesToSave encoded as an
   * EntryBatch (drb_round_in.encode_saves; multiple of 16, 0: none) */
  uint32_t save_cap;
  /* Placement.  place_world <= 1: co-resident, every replica
   * of group g at lane g.  place_world = N >= 2: replica slot s of global
   * group g lives on rank (g + s) mod N at lane g / N (C4); this engine is
   * rank place_rank, num_groups is its lane count and the round's
   * cross-rank mailbox planes move with drb_exchange_* (RCCL / P2P). */
  uint64_t total_groups;     /* global groups (0: num_groups * N) */
  uint32_t place_world;
  uint32_t place_rank;
  uint32_t entry_mbox;       /* entries per remote (sender, receiver) and
                              * round that travel by value (N >= 2;
                              * 1..255: the plane summary's 8-bit E) */
  /* kv_val_cap > 124 keeps values out of line (C5: 128 B / 1 KB
   * payloads) in a pool of this many value blocks (0: one per KV slot);
   * a replica whose apply finds the pool empty falls back */
  uint32_t kv_pool_blocks;
  /* records of the flagged-replica list (drb_take_flagged; 0: 65536) */
  uint32_t flagged_cap;
  /* Config.Quiesce (config.go:195): node.qs (quiesce.go) enters quiesce
   * after 20 x ElectionRTT idle ticks and stops heartbeating; quiesced
   * replicas without input skip tick rounds (their ticks are applied
   * when they next run) */
  uint32_t quiesce;
  /* 1: the host persists each round's EntriesToSave (a durable ILogDB)
   * before the round's messages may be delivered: drb_step_round of round
   * t+1 and drb_encode_wire of round t require drb_commit_round(t) */
  uint32_t durable_log;
  /* 1: encode_saves writes the batched LogDB's records of EntriesToSave
   * (internal/logdb/batch.go:288-346) instead of one EntryBatch: one
   * EntryBatch record per 48-index batch the round touches (at most
   * DRB_SAVE_RECS), the first merged with that batch's entries saved in
   * earlier rounds (getMergedFirstBatch, from the resident window) and
   * compactBatchFields applied; drb_export_save_records lists them.
   * Needs window >= 64 and save_cap for a full batch. */
  uint32_t save_batched;
  /* 1: encode_saves writes each replica's pb.Update as the record a
   * regular tan LogDB appends to that replica's log (internal/tan/db.go:
   * 97-130, record.go:548-591; drb_export_tan / drb_tan_buffers): the
   * marshalled Update (raftpb/update.go:128-169) in 32 KiB-block chunks
   * with XXH64 checksums, zero padding included, at the log offset the
   * engine tracks per replica (drb_tan_get / drb_tan_set).  Needs
   * save_cap; excludes save_batched. */
  uint32_t save_tan;
  /* 1: elections on the GPU.  The replicas a step round
   * would hand to the CPU for an election timeout, CheckQuorum, a term
   * change, a vote message or the candidate role are stepped by a second
   * launch with the whole raft state machine instead (campaign,
   * RequestVote / RequestVoteResp, becomeFollower / Candidate / Leader,
   * the term gate, raft.go:1052-1217, 1507-1590, 1670-1722, 2235-2253);
   * only capacity and off-path entries still fall back.  With Quiesce a
   * quiesced replica ticks with quiescedTick (raft.go:650-656: no
   * election) until input ends its quiesce (node.go:1296-1345,
   * quiesce.go:56-74); listed rounds allowed.  With placement (place_world
   * > 1) the votes and the new leaders' messages cross ranks in the planes
   * (drb_plane_regions ships the rterm rows of records whose term is not
   * their header's, DRB_PLANE_TOTHER); staged input reaches a group only
   * while its leader is at the stage slot. */
  uint32_t elections;
  /* tan MaxLogFileSize (internal/tan/options.go:29); 0: 64 MiB */
  uint64_t tan_max_log;
  /* with save_tan, 1: the multiplexed tan (CreateLogMultiplexedTan,
   * internal/tan/logdb.go:110-118, db_keeper.go:84-123): each replica slot
   * (one NodeHost) keeps 16 logs, key = ShardID % 16, shared by its
   * replicas; a round's records of one log follow in group order (the
   * step worker's order, engine.go:1316, is a Go map's) and are laid out
   * back to back in that log's staging (drb_export_tan_log).  place_world
   * 1 only. */
  uint32_t tan_multiplexed;
  /* with elections, 1: Config.PreVote (config.go): a timed-out replica
   * first asks for pre-votes at term + 1 without changing its term
   * (preVoteCampaign, raft.go:1149-1174; handleNodeRequestPreVote,
   * :1670-1695; the preVoteCandidate handlers, :2256-2276) */
  uint32_t pre_vote;
  /* > 0: the reads served behind each ReadyToRead (drb_round_in.
   * reads_per_ctx <= this, drb_serve_reads) also leave one result per read
   * -- found, value length, value -- that drb_export_read_results hands to
   * the clients' ReadLocalNode calls; 0: only the per-replica checksum
   * (drb_export_read_sums) */
  uint32_t max_reads_per_ctx;
  /* > 0: the KV grows past kv_slots.  A replica whose table is full puts
   * further keys in overflow buckets of 4 slots, chained per replica and
   * bump-allocated from a pool of this many buckets shared by the engine
   * (KVTest's map grows, kvtest.go:145-162); a lookup that finds a full
   * table walks the chain.  Rounds run the EXT step kernels.  An
   * exhausted pool stops the apply as a full table does; drb_kv_import
   * lays a replica's keys past kv_slots into fresh buckets (its old chain
   * is not reclaimed).  0: a full table stops the replica's apply
   * (DRB_F_APPLY_STOPPED). */
  uint64_t kv_overflow_buckets;
  /* 1: proposals may be made at any replica (drb_round_in.prop_replica),
   * as at any NodeHost: a follower forwards its entry queue to its leader
   * as a Propose message, dropped when it knows no leader
   * (handleFollowerPropose, raft.go:2103-2116), and the leader appends a
   * received Propose's entries (handleLeaderPropose, raft.go:1794-1815).
   * A Propose carries its entries by value in per-(round, sender) rows
   * (max_props entries, at most 15); drb_ingest / drb_ingest_wire accept
   * Propose messages from other NodeHosts into them (one per sender, round
   * and group; a second is dropped as by a full MessageQueue).  Co-resident
   * placement only. */
  uint32_t forward_proposals;
  /* Member kinds of the replica slots (the shards' pb.Membership, the same
   * for every group): bit s of nonvoting_slots makes replica slot s a
   * nonVoting -- replicated, sent heartbeats without a ReadIndex ctx, not
   * counted in commit, CheckQuorum or ReadIndex quorums, never campaigning
   * (raft.go:787-871, 917-924, 395-405, 596-600) -- and bit s of
   * witness_slots a witness -- counted in the quorums, sent metadata-only
   * entries (makeMetadataEntries, raft.go:756-785), applying them as
   * no-ops, never campaigning, ReadIndex from it dropped
   * (raft.go:1848-1849).  The quorum is over the voting members (remotes
   * and witnesses, raft.go:383-389).  drb_init_steady gives those slots
   * their roles; the leader slot must be a voting member. */
  uint32_t nonvoting_slots;
  uint32_t witness_slots;
  /* 1: the engine's large host transfers -- the step worker's download
   * (drb_worker_export) and a pinned one-block proposal upload
   * (drb_stage_proposals_packed*) -- go through hipMemcpyAsync on the
   * engine's copy streams instead of its own SDMA engines (drb_hsa.hpp):
   * the path every engine takes when the HSA copy engines are unavailable,
   * selectable so that it can be tested.  0: SDMA when available. */
  uint32_t host_copies;
  /* 1: listed rounds step every listed replica through the full step
   * kernel; 0: the heartbeat-only rounds of quiet groups go through the
   * lean kernel first (drb_lean.hpp; for A/B measurements) */
  uint32_t no_lean;
} drb_config;

/* One step round (engine.processSteps, engine.go:1304). */
typedef struct drb_round_in {
  uint32_t tick;       /* 1: one LocalTick per hosted replica (nodehost.go:1903) */
  uint32_t prop_slot;  /* staged proposal batch to consume, DRB_NONE for none */
  uint32_t ri_slot;    /* staged ReadIndex batch, DRB_NONE for none */
  /* ReadLocalNode reads served in-round behind every ReadyToRead the round
   * releases, with drb_serve_reads semantics (0: none; then
   * drb_serve_reads can serve them after the round) */
  uint32_t reads_per_ctx;
  uint32_t read_key_space; /* key space of those reads (> 0 if reads) */
  /* 1: encode every replica's pb.Update.EntriesToSave as EntryBatch bytes
   * + CRC32 for the LogDB writer (drb_export_saved; needs save_cap) */
  uint32_t encode_saves;
  /* where the staged ReadIndex batch lands (node.handleReadIndex,
   * node.go:1296-1307): 0 the group's leader; k >= 1 replica ID k, which
   * forwards it to its leader when it is a follower (raft.go:2134-2164).
   * Co-resident placement only. */
  uint32_t ri_replica;
  /* 1: first list the replicas with work this round (input, a tick for a
   * replica not quiesced, anything pending) and step only those, packed
   * into dense waves -- for rounds where most replicas are at rest (C5,
   * Quiesce); the result is the same.  Co-resident placement only. */
  uint32_t listed;
  /* where the staged proposal batch lands (node.handleProposals,
   * node.go:1275-1294): 0 the group's leader; k >= 1 replica ID k, whose
   * NodeHost's entry queue it is -- a follower forwards it to its leader
   * (needs drb_config.forward_proposals). */
  uint32_t prop_replica;
} drb_round_in;

#define DRB_NONE 0xffffffffu

typedef struct drb_round_out {
  uint64_t round;                 /* index of the round just executed */
  uint64_t committed_entries;     /* sum of leader commit advance, app entries */
  uint64_t applied_entries;       /* entries applied over all replicas */
  uint64_t messages;              /* messages sent in this round */
  uint64_t ready_to_reads;        /* ReadyToRead records produced */
  uint64_t dropped_read_indexes;  /* raft.droppedReadIndexes */
  uint64_t fallbacks;             /* replicas newly marked DRB_F_FALLBACK */
  uint64_t errors;                /* replicas newly marked DRB_F_ERROR */
  uint64_t reads_served;          /* ReadLocalNode lookups done (drb_serve_reads) */
  uint64_t reads_deferred;        /* reads whose index is not applied yet */
  uint64_t saved_entries;         /* EntriesToSave encoded (encode_saves) */
  uint64_t saved_bytes;           /* EntryBatch bytes of those */
  uint64_t replicas_stepped;      /* replicas that ran the round; the others
                                   * were at rest with no input (or
                                   * quiesced at rest on a tick round) */
  uint64_t log_records;           /* save_tan: records appended to tan logs */
  uint64_t log_syncs;             /* ... of them with db.write's sync */
  uint64_t log_new;               /* ... of them that started a new log */
  uint64_t elections_stepped;     /* elections: replicas the raft launch
                                   * stepped (term gate, votes, campaign) */
  uint64_t role_changes;          /* elections: replicas whose role changed */
  uint64_t dropped_proposals;     /* entries a leader transferring its
                                   * leadership dropped (raft.go:1796-1800;
                                   * the clients' requests complete Dropped) */
  uint64_t lean_stepped;          /* listed rounds: of replicas_stepped, the
                                   * heartbeat rounds the lean kernel took */
} drb_round_out;

typedef struct drb_engine drb_engine;

/* --- lifecycle --------------------------------------------------------- */

/* Allocates the SoA state in HBM.  Replaces newExecEngine (engine.go:1009)
 * plus per-shard node/raft construction (node.go:136, raft.go:241) for the
 * groups this device hosts. */
int drb_engine_create(const drb_config *cfg, drb_engine **out);
int drb_engine_destroy(drb_engine *e);
/* Bytes of HBM the engine holds. */
uint64_t drb_engine_device_bytes(const drb_engine *e);
/* The hipStream_t every kernel of this engine is launched on. */
void *drb_engine_stream(drb_engine *e);
int drb_engine_sync(drb_engine *e);
uint64_t drb_engine_round(const drb_engine *e);

/* --- state movement (fallback boundary, SURVEY 8b "Fallback") ---------- */

/* st[(g - first_group) * R + slot]. */
int drb_import_replicas(drb_engine *e, uint64_t first_group, uint64_t n_groups,
                        const drb_replica_state *st);
int drb_export_replicas(drb_engine *e, uint64_t first_group, uint64_t n_groups,
                        drb_replica_state *st);
/* Writes entries (contiguous indices) into the resident window of one
 * replica: the inMemory.entries / LogDB content the fast path reads. */
int drb_import_log(drb_engine *e, uint64_t group, uint32_t slot,
                   const drb_entry *ents, size_t n, const uint8_t *pool);
/* Reads indices [lo, hi] of one replica's window.  pool receives Cmd bytes
 * (pool_cap bytes available). */
int drb_export_log(drb_engine *e, uint64_t group, uint32_t slot, uint64_t lo,
                   uint64_t hi, drb_entry *out, uint8_t *pool,
                   size_t pool_cap);

/* Which replicas this engine steps: replica slot `slot` of every group is
 * hosted here (1) or lives on another NodeHost (0), whose messages arrive
 * through drb_ingest / drb_ingest_wire (NodeHost.StartReplica /
 * StopReplica for one replica of every shard, nodehost.go). */
int drb_host_slot(drb_engine *e, uint32_t slot, int hosted);
/* Role census of the hosted replicas that are on the fast path (not
 * FALLBACK / ERROR): counts[slot * 8 + role] for slots 0..R-1, roles
 * drb_role -- how many groups have a leader after a failover, without
 * exporting every replica. */
int drb_role_census(drb_engine *e, uint64_t *counts);

/* Device-side initialisation of every group to the post-election steady
 * state: bootstrap (peer.go:404-428) with R config-change entries at term
 * 1, replica `leader_slot` elected at `term` (raft.go:1176, 1038) and its
 * no-op entry committed and applied everywhere.  Equivalent to running
 * the CPU election path per group; `seed` feeds the randomized election
 * timeout (raft.go:658-661). */
int drb_init_steady(drb_engine *e, uint64_t term, uint32_t leader_slot,
                    uint64_t seed);

/* --- inputs ------------------------------------------------------------- */

/* Stage proposals for one round: counts[g] entries for group g taken from
 * ents[g * max_props ...].  Replaces entryQueue.add (queue.go:60) feeding
 * node.handleProposals (node.go:1275).  Consumed by the group's leader.
 * pool holds pool_len bytes of Cmd data (entries address it by
 * cmd_off / cmd_len).  counts[g] > max_props is DRB_ERANGE (the slot is
 * left as it was); an entry whose Cmd exceeds cmd_cap or the pool is
 * staged as one the leader cannot take, so its group falls back before
 * appending (DRB_FB_CAPACITY).  The arrays are uploaded as-is on a copy
 * stream that overlaps a round still
 * running, and laid out on the device by a kernel ordered on the engine
 * stream ahead of the next round.  Returns once the host arrays have been
 * read: the caller may reuse them.  Pinned host memory makes the upload
 * asynchronous to the running round. */
int drb_stage_proposals(drb_engine *e, uint32_t slot, const uint32_t *counts,
                        const drb_entry *ents, const uint8_t *pool,
                        size_t pool_len);
/* The same for a batch of NoOP-session entries (SeriesID = RespondedTo = 0,
 * every entry of Type `type`: client.go NoOPSession, request.go:1085-1096)
 * in the packed form a host builds its per-round upload in: counts[g]
 * entries for group g (g ascending, counts[g] <= max_props), and per entry
 * -- group by group, in queue order -- its Key, ClientID and Cmd length,
 * the Cmd bytes back to back in pool (pool_len = the sum of the lengths).
 * 1 + n x 18 + pool bytes cross the host link instead of drb_entry rows:
 * 36 B per group at C3 (16 B PBKV writes) against 85 B; client_ids NULL
 * takes each group's registered session client (drb_set_session_clients,
 * DRB_EINVAL without one), 28 B per C3 group.  Offsets are
 * scanned and the entries laid out on the device, ordered and overlapped
 * as drb_stage_proposals; DRB_EINVAL when the counts or lengths do not add
 * up. */
int drb_stage_proposals_packed(drb_engine *e, uint32_t slot, uint32_t type,
                               const uint8_t *counts, uint64_t n_entries,
                               const uint64_t *keys,
                               const uint64_t *client_ids,
                               const uint16_t *cmd_lens, const uint8_t *pool,
                               size_t pool_len);
/* The same, pipelined one call deep for a step worker that stages round
 * t + 1 while round t runs: returns once the previous call's upload is done
 * (that call's arrays are then the caller's again) and this call's upload
 * is queued.  The arrays stay in use until the next call, or
 * drb_stage_wait_upload, returns; pinned host memory required.  Replaces
 * the same entryQueue.add (queue.go:60) as drb_stage_proposals_packed. */
int drb_stage_proposals_packed_async(drb_engine *e, uint32_t slot,
                                     uint32_t type, const uint8_t *counts,
                                     uint64_t n_entries, const uint64_t *keys,
                                     const uint64_t *client_ids,
                                     const uint16_t *cmd_lens,
                                     const uint8_t *pool, size_t pool_len);
/* The ClientID of the host's NoOP session of every group (client.go
 * NewNoOPSession: one per shard, request.go:1085-1096), client_ids[g] for
 * lane g.  A packed batch may then leave client_ids NULL -- each entry
 * carries its group's -- and 8 B per entry stay off the host link; the
 * step-worker export counts a lane's applied entries of that client
 * (drb_worker_bufs).  Synchronous; set again to change them. */
int drb_set_session_clients(drb_engine *e, const uint64_t *client_ids);
/* Until the last staged upload is done (its host arrays free). */
int drb_stage_wait_upload(drb_engine *e);
/* Where a host builds a packed batch of n_entries entries and pool_len Cmd
 * bytes in one pinned block so that either call uploads it in one DMA (of
 * 8 MB and more, on the engine's own upload SDMA engine -- the one its
 * step-worker downloads do not use -- with the call returning once it is
 * up):
 * counts at offset 0, then keys, lengths, the pool and the client ids
 * (256-aligned); offsets[0..3] = keys, client ids, lengths, pool; *bytes =
 * the block's length.  A batch without client ids (drb_set_session_clients)
 * ends at offsets[3] + pool_len, and only that much goes up.  Arrays
 * elsewhere are uploaded one copy each. */
int drb_stage_packed_layout(const drb_engine *e, uint64_t n_entries,
                            size_t pool_len, uint64_t *offsets,
                            size_t *bytes);
/* Device-side synthetic proposal generator (bench / SURVEY 8d inputs):
 * k KVTest PBKV writes per group, NoOP session, EncodedEntry v0. */
int drb_gen_kv_proposals(drb_engine *e, uint32_t slot, uint32_t k,
                         uint32_t key_space, uint32_t val_len, uint64_t seed,
                         uint64_t salt);
/* The same for a seeded Bernoulli subset of the groups (C5: 1 % active
 * per round): group g proposes in batch `salt` iff
 * mix64(seed ^ ACTIVE ^ g * GOLDEN ^ salt << 24) % 1000000 < active_ppm. */
int drb_gen_kv_proposals_active(drb_engine *e, uint32_t slot, uint32_t k,
                                uint32_t key_space, uint32_t val_len,
                                uint64_t seed, uint64_t salt,
                                uint32_t active_ppm);
/* Stage one ReadIndex ctx per group (ctx_low[g] == 0: none).  Replaces
 * pendingReadIndex.read + node.handleReadIndex (request.go:845,
 * node.go:1296). */
int drb_stage_read_index(drb_engine *e, uint32_t slot, const uint64_t *ctx_low,
                         const uint64_t *ctx_high);
/* Device-side synthetic ReadIndex ctx per group (bench / SURVEY 8d):
 * ctx = {mix64(seed ^ RI ^ g * GOLDEN ^ high << 40) | 1, high}
 * (dragonboat_amd/workload.py read_index_ctx with salt = high). */
int drb_gen_read_index(drb_engine *e, uint32_t slot, uint64_t seed,
                       uint64_t high);
/* NodeHost.RequestLeaderTransfer (nodehost.go:1238-1251) at replica slot
 * `slot` (that NodeHost) of every group g with targets[g] != 0, a replica
 * ID <= num_replicas: node.requestLeaderTransfer ->
 * pendingLeaderTransfer.request (node.go:474-482).  The replica's next
 * round takes it after its proposals (node.handleLeaderTransfer,
 * node.go:1198, 1249-1257 -> Peer.RequestLeaderTransfer, peer.go:106-113):
 * a leader starts the transfer (raft.go:1925-1953), a follower forwards it
 * to its leader (raft.go:2145-2153), a candidate ignores it.  The leader
 * then drops proposals (drb_round_out.dropped_proposals) until the target
 * holds its whole log and is sent TimeoutNow, which makes it campaign at
 * once without PreVote (raft.go:1890-1895, 2172-2185); an election timeout
 * without a new leader abandons the transfer (raft.go:622-636).  Needs
 * elections (co-resident placement).  A replica still holding an earlier
 * request, or off the fast path, refuses (ErrSystemBusy): *busy (may be
 * NULL) counts those; unhosted replicas are skipped.  Synchronous. */
int drb_request_leader_transfer(drb_engine *e, uint32_t slot,
                                const uint32_t *targets, uint64_t *busy);

/* Inbound boundary: IMessageHandler.HandleMessageBatch
 * (internal/transport/transport.go:86-91, nodehost.go:2072-2122).  Places
 * messages from replicas NOT hosted by this engine into the inbox of the
 * next round.
 *
 * The reference drops an incoming message only when the receiving node's
 * MessageQueue already holds ReceiveQueueLength = 1024 messages
 * (internal/server/message.go:105-120 MessageQueue.Add, settings/soft.go:202,
 * nodehost.go:2112-2114), and a message for a shard or replica this
 * NodeHost does not host (nodehost.go:2089-2098).  Here, every message is
 * one of:
 *   DRB_ING_PLACED    in the receiver's GPU inbox of the next round;
 *   DRB_ING_DROPPED   the reference drops it too: an unknown shard, a
 *                     receiver this engine does not host (with placement:
 *                     not on this rank), a sender this engine hosts (the
 *                     transport delivers remote senders only);
 *   DRB_ING_DIVERTED  the GPU inbox cannot hold it, or its receiver is off
 *                     the fast path: the message goes to the CPU raft.Peer
 *                     of its receiver, whose MessageQueue.Add applies the
 *                     1024 rule.  A GPU capacity -- a (sender, receiver)
 *                     plane's `mailbox` records, a second Propose of one
 *                     sender in a round or one the forward rows cannot
 *                     hold, a Replicate beyond a remote plane's entry_mbox
 *                     rows, a Cmd longer than cmd_cap -- marks the receiver
 *                     DRB_F_FALLBACK with DRB_FB_CAPACITY (listed by
 *                     drb_take_flagged with the engine's current round),
 *                     and that message and every later one for the
 *                     receiver in the call are diverted.  The receiver's
 *                     CPU inbox is then drb_export_inbox(.., 0, ..) (what
 *                     was placed before, each sender's in order) followed
 *                     by the diverted messages, in call order.
 * With placement (place_world > 1) shard_id names the global group: a
 * message reaches the rank that hosts its receiver ((group + slot) mod N,
 * lane group / N); a sender slot that belongs to another rank is written
 * into the inbound planes, its Replicates' entries into the plane's
 * entry_mbox rows.  Call it after the round's plane exchange.  The same
 * holds for drb_ingest_wire, with one difference of scope: its placement
 * runs one lane per (group, sender, receiver) plane, so a capacity divert
 * diverts that plane's later messages in the call, while other senders'
 * planes to the same receiver keep placing theirs (the receiver is flagged
 * either way, and its CPU inbox -- drb_export_inbox(.., 0, ..) then the
 * diverted messages per sender in stream order -- keeps every sender's
 * order, which is all MessageQueue order promises across senders). */
enum drb_ingest_fate {
  DRB_ING_PLACED = 0,
  DRB_ING_DROPPED = 1,
  DRB_ING_DIVERTED = 2,
  DRB_ING_SNAPSHOT = 3  /* drb_ingest_wire: an InstallSnapshot (CPU path) */
};
/* status (may be NULL): n bytes, each message's drb_ingest_fate */
int drb_ingest_ex(drb_engine *e, const drb_message *msgs, size_t n,
                  const drb_entry *ents, const uint8_t *pool, uint8_t *status,
                  uint64_t *accepted, uint64_t *dropped, uint64_t *diverted);
/* drb_ingest_ex without the per-message status and the diverted count.
 * Deprecated: a caller that cannot see which messages were diverted would
 * lose them, so when any was (a GPU capacity, or a receiver already off the
 * fast path) it returns DRB_EDIVERTED -- the placed ones are in the inbox,
 * the counts are set, and the caller must replay the call's messages for
 * the flagged receivers (drb_take_flagged) through the CPU path or use
 * drb_ingest_ex. */
int drb_ingest(drb_engine *e, const drb_message *msgs, size_t n,
               const drb_entry *ents, const uint8_t *pool, uint64_t *accepted,
               uint64_t *dropped);
/* The messages in replica slot `slot` of `group`'s inbound planes:
 * last_round == 0, the inbox the next round would take (the last round's
 * co-resident sends and what was ingested since); last_round == 1, the one
 * the last round took -- which a replica that round marked DRB_F_FALLBACK
 * left unprocessed (valid until the next round).  Per sender in its send
 * order (Replicates first, as the reference sends them), senders by slot;
 * a Quiesce is a message of its own (node.go:993-1005); Replicate entries
 * and Propose entries with their Cmd bytes in pool.  Hands a replica that
 * leaves the fast path its pending messages for the CPU raft.Peer
 * (node.stepNode's MessageQueue, node.go:1139-1159). */
int drb_export_inbox(drb_engine *e, uint64_t group, uint32_t slot,
                     int last_round, drb_message *out, size_t cap,
                     drb_entry *ents, size_t ent_cap, uint8_t *pool,
                     size_t pool_cap, size_t *n_msgs);

/* --- the step round ---------------------------------------------------- */

/* Replaces engine.processSteps (engine.go:1304) -> node.stepNode
 * (node.go:1139) -> Peer.Handle/GetUpdate/Commit (peer.go:184,198,292)
 * -> StateMachine.Handle (internal/rsm/statemachine.go:599) for every
 * hosted replica, with an in-memory ILogDB.  Stream-ordered; `out` is
 * filled after the round completes (this call synchronises). */
int drb_step_round(drb_engine *e, const drb_round_in *in, drb_round_out *out);
/* Same, without the host synchronisation; counters accumulate on device
 * and are read by drb_read_counters(). */
int drb_step_round_async(drb_engine *e, const drb_round_in *in);
/* k rounds (in[0..k)) at once, chunk by chunk of the groups: each chunk of
 * chunk_groups groups (a multiple of 256) runs all k rounds before the
 * next starts.  Groups are independent -- the reference steps each shard on
 * its own when it is ready (engine.go:1316-1328, workReady :128-226) -- so
 * every group goes through exactly the rounds k drb_step_round_async calls
 * would give it; a chunk's mailbox, state and window rows may stay on-die
 * between its rounds.  No host synchronisation.  Co-resident replicas only,
 * without elections, listed rounds, tan records or durable_log
 * (DRB_EINVAL): those step round by round.  A chunk of every group
 * (chunk_groups >= num_groups) runs the k rounds as k plain rounds from one
 * call: a host loop that steps a small engine round by round (C2) is then
 * bound by the GPU, not by its own per-call cost. */
int drb_step_rounds(drb_engine *e, const drb_round_in *in, uint32_t k,
                    uint64_t chunk_groups);
int drb_read_counters(drb_engine *e, drb_round_out *out, int reset);
/* Timing builds only: per-phase cycle sums of the step kernels' lanes,
 * out[16] = [follower, leader] x {lanes stepped, load + pre-pass, inbox
 * dispatch, tick + proposals, getUpdate, apply, state store, served reads};
 * zeros unless the engine was created with DRB_PHASE=1 in the environment
 * and the step kernels were built with DRB_PHASE_PROF=1. */
int drb_debug_phase(drb_engine *e, uint64_t *out, int reset);

/*
 * The replicas that left the fast path (DRB_F_FALLBACK / DRB_F_ERROR),
 * appended by the step kernels in the round they were marked: the compact
 * list a host walks to hand exactly those groups to the CPU raft.Peer
 * (node.stepNode's error / CPU path, node.go:1139-1159) instead of
 * exporting every replica.  drb_take_flagged copies up to cap records
 * appended since the last reset (in no particular order), reports in
 * *lost how many did not fit the device list (flagged_cap), and with
 * reset != 0 empties it.  Synchronises the engine stream.
 */
typedef struct drb_flagged {
  uint64_t group;      /* lane on this engine */
  uint64_t shard_id;
  uint64_t round;      /* drb_engine_round() of the round that marked it */
  uint32_t slot;       /* replica slot (replica ID - 1) */
  uint32_t reason;     /* drb_fallback_reason */
  uint32_t flags;      /* DRB_F_FALLBACK | DRB_F_ERROR | DRB_F_APPLY_STOPPED */
  uint32_t pad;
} drb_flagged;
int drb_take_flagged(drb_engine *e, drb_flagged *out, size_t cap,
                     size_t *n_out, uint64_t *lost, int reset);

/* --- outputs ----------------------------------------------------------- */

/* Outbound boundary: the messages one replica sent in the last round
 * (node.sendReplicateMessages / sendMessages, node.go:1007-1022 ->
 * Transport.Send, transport.go:346), in send order.  Entries of Replicate
 * messages are copied out with Cmd bytes into pool. */
int drb_export_outbox(drb_engine *e, uint64_t group, uint32_t from_slot,
                      drb_message *out, size_t cap, drb_entry *ents,
                      size_t ent_cap, uint8_t *pool, size_t pool_cap,
                      size_t *n_msgs);
/* pb.Update.ReadyToReads of the last round for one replica. */
int drb_export_ready_to_reads(drb_engine *e, uint64_t group, uint32_t slot,
                              drb_ready_to_read *out, size_t cap,
                              size_t *n_out);

/* pb.Update.ReadyToReads of the last round for replica slot `slot` of
 * groups [first_group, first_group + n_groups), compacted on the device:
 * the records of node.processReadyToRead (node.go:1081 ->
 * pendingReadIndex.addReady, request.go:883) for a whole step worker's
 * groups in one call -- in group order, each replica's in release order.
 * *n_out is the count (DRB_ERANGE with nothing copied if more than cap).
 * Two device-to-host copies (the count, then the records). */
int drb_export_ready_to_reads_batch(drb_engine *e, uint32_t slot,
                                    uint64_t first_group, uint64_t n_groups,
                                    drb_ready_to_read *out, size_t cap,
                                    size_t *n_out);

/*
 * A step worker's round, handed to the host without a host synchronisation
 * (engine.processSteps, engine.go:1304-1364: node.processReadyToRead,
 * node.go:1081 -> pendingReadIndex.addReady, request.go:883; the reads
 * served behind them, pendingReadIndex.applied, request.go:930-953 ->
 * ReadLocalNode, nodehost.go:849; the applied entries,
 * pendingProposals.applied, node.go:243-257).  drb_worker_export enqueues,
 * behind the last round, a compaction of replica slot `slot`'s outputs
 * into device staging (two buffers, by export parity) and their transfer
 * into the caller's host buffers (drb_host_alloc) on the engine's download
 * SDMA engine (no CU time; the staged proposals go up on another one): the
 * transfer overlaps the next rounds.  drb_worker_wait blocks until that
 * export's bytes are in its buffers and fills the counts.
 *
 * The records carry only what the host cannot rebuild from what it staged
 * and what it issued (about 46 B per C3 group-round):
 *   lanes[g]    one word per lane (every lane of the engine, g < num_groups):
 *               bits 0-3 its ReadyToReads this round, bits 4-11 which of
 *               them had their reads served (bit k: the k-th; its
 *               reads_per_ctx results follow in values), bits 12-27 how
 *               many of the host's own proposals it applied -- the entries
 *               carrying the group's session ClientID
 *               (drb_set_session_clients), or, with none registered, every
 *               entry with a ClientID (raft's own empty entries have none,
 *               statemachine.go:939).  They complete the host's pending
 *               proposals in the order it staged them; KVTest's
 *               sm.Result.Value is the length of each one's payload
 *               (kvtest.go:161), known to the host (drb_apply_results has
 *               the per-entry form);
 *   reads       per ReadyToRead, lanes in order, each lane's in release
 *               order: the low 32 bits of its SystemCtx.Low.  The host
 *               issued the ctx (request.go:864-875: Low random, High its
 *               own tick + 30) and a replica releases its requests in the
 *               order they were queued (readindex.go:77-115), so the tag
 *               picks the ctx out of the group's pending ones; a pending
 *               ctx older than a released one was dropped (a host keeps the
 *               low words of a group's pending ctxs distinct);
 *   values      per served read, in ReadyToRead and read order: a word whose
 *               meaning its 2-bit code gives;
 *   value_meta  a 2-bit code per served read (read i: byte i / 4, bits
 *               2 * (i % 4)): DRB_WORKER_MISS the key is not in the KV
 *               (word 0); DRB_WORKER_V4 a 4-byte value, the word; 
 *               DRB_WORKER_SHORT a shorter one, its bytes in the word's low
 *               bytes and its length in bits 24-31; DRB_WORKER_LONG a
 *               longer one, its first 4 bytes (drb_export_read_values has
 *               it whole);
 *   deferred    per ReadyToRead whose reads were not served (reads_per_ctx
 *               0, or its index not yet applied), lanes in order: its
 *               Index, for pendingReadIndex.applied (request.go:930-953).
 */
#define DRB_WORKER_LANE_READS(w) ((w) & 0xfu)
#define DRB_WORKER_LANE_SERVED(w) (((w) >> 4) & 0xffu)
#define DRB_WORKER_LANE_APPLIED(w) (((w) >> 12) & 0xffffu)
#define DRB_WORKER_MISS 0u
#define DRB_WORKER_V4 1u
#define DRB_WORKER_SHORT 2u
#define DRB_WORKER_LONG 3u

typedef struct drb_worker_bufs {
  uint32_t *lanes;             /* host buffers from drb_host_alloc */
  uint64_t lanes_cap;          /* >= num_groups */
  uint32_t *reads;
  uint64_t reads_cap;
  uint32_t *values;
  uint8_t *value_meta;         /* (values_cap + 3) / 4 bytes */
  uint64_t values_cap;
  uint64_t *deferred;
  uint64_t deferred_cap;
  uint64_t n_reads, n_values, n_deferred;  /* set by drb_worker_wait */
} drb_worker_bufs;

/* DRB_EAGAIN: b already has an export in flight (drb_worker_wait it
 * first), or 16 exports are in flight; two drb_worker_bufs alternate in a
 * step worker's loop */
int drb_worker_export(drb_engine *e, uint32_t slot, const drb_worker_bufs *b);
/* The same for one step worker's partition of the shards: the lanes whose
 * ShardID % n_parts == part (engine.go:1036-1049 processSteps over
 * workerID's shards; FixedPartitioner, internal/server/partition.go:28-41),
 * i.e. lanes g0, g0 + n_parts, ... with g0 = (part - first_shard_id) mod
 * n_parts; lanes[i] is lane g0 + i * n_parts's word (lanes_cap >= that
 * partition's lane count) and the other records follow those lanes only.
 * Each worker exports into its own buffer sets, concurrently with the
 * others.  Co-resident placement only (n_parts 1 is drb_worker_export). */
int drb_worker_export_part(drb_engine *e, uint32_t slot, uint32_t n_parts,
                           uint32_t part, const drb_worker_bufs *b);
/* DRB_ERANGE when a count exceeded its cap (the counts are the full ones,
 * the buffers hold the first cap records) */
int drb_worker_wait(drb_engine *e, drb_worker_bufs *b);
/* pinned host memory the engine's device can write (drb_worker_bufs) */
int drb_host_alloc(drb_engine *e, size_t bytes, void **p);
int drb_host_free(drb_engine *e, void *p);

/* One ReadLocalNode result (nodehost.go:849 -> KVTest.Lookup,
 * kvtest.go:164-175) of the reads served behind a ReadyToRead: the read's
 * ctx and position, its key and what the lookup found.  value holds the
 * value's first 4 bytes little-endian (all of it when vlen <= 4, as at
 * C3's 16 B writes); a longer value is read with drb_kv_lookup, valid until
 * the next round. */
typedef struct drb_read_result {
  uint64_t shard_id;
  uint64_t index;       /* the ReadyToRead's index (pendingReadIndex.applied) */
  uint64_t ctx_low;
  uint64_t ctx_high;
  uint64_t key;         /* LE64 key looked up */
  uint32_t replica_id;
  uint32_t read;        /* j: the read's position in its ctx */
  uint32_t found;       /* 1: the key is in the replica's KV */
  uint32_t vlen;
  uint32_t value;
  uint32_t pad;
} drb_read_result;
/* The results of the reads served by replica slot `slot` of groups
 * [first_group, first_group + n_groups) in the last round that served
 * reads (its reads_per_ctx per released ctx; deferred ctx have none), in
 * group order, then ctx order, then read order; compacted on the device.
 * Needs drb_config.max_reads_per_ctx.  *n_out / DRB_ERANGE as above. */
int drb_export_read_results(drb_engine *e, uint32_t slot, uint64_t first_group,
                            uint64_t n_groups, drb_read_result *out,
                            size_t cap, size_t *n_out);
/* The same results with every found value whole (ReadLocalNode returns the
 * value, nodehost.go:849 -> KVTest.Lookup kvtest.go:164-175; C5's 116 B /
 * 1011 B values included): value_off[i] is the byte offset in pool of
 * result i's value (vlen bytes, offsets 16-aligned), gathered on the device
 * from the KV as the round served it and copied in one transfer.
 * *pool_bytes is the pool size the values need; pool_cap below it is
 * DRB_ERANGE (the records are then out already).  Call before the next
 * round. */
int drb_export_read_values(drb_engine *e, uint32_t slot, uint64_t first_group,
                           uint64_t n_groups, drb_read_result *out,
                           uint64_t *value_off, size_t cap, uint8_t *pool,
                           size_t pool_cap, size_t *n_out, size_t *pool_bytes);

/*
 * Serves the linearizable reads behind the ReadyToReads of the last round:
 * pendingReadIndex.applied releases a read once the replica applied its
 * index (request.go:930-953), and the client then calls ReadLocalNode ->
 * IStateMachine.Lookup (nodehost.go:849, kvtest.go:164-175).  Each released
 * ctx carries `reads_per_ctx` reads (the batch of node.go:1296-1305); read j
 * of ctx {low, high} looks up key LE64(mix64(low ^ (j+1)*0x9E3779B97F4A7C15)
 * % key_space).  Results fold into one checksum per replica (see
 * drb_export_read_sums); reads whose index is not yet applied are counted
 * as deferred.  Stream-ordered after drb_step_round*.
 */
int drb_serve_reads(drb_engine *e, uint32_t reads_per_ctx, uint32_t key_space);
/* sums[(g - first_group) * R + slot]: sum over served reads j of
 * mix64(word ^ key ^ (j << 56)), word = found ? vlen << 32 | LE32(value)
 * : ~0; written by the last drb_serve_reads for replicas it served. */
int drb_export_read_sums(drb_engine *e, uint64_t first_group,
                         uint64_t n_groups, uint64_t *sums);

/* Persistence boundary (ILogDB.SaveRaftState, raftio/logdb.go:83, called
 * once per round by engine.processSteps, engine.go:1343): one replica's
 * pb.Update.EntriesToSave of the last round that ran with encode_saves,
 * as EntryBatch bytes (EntryBatch.MarshalTo, raftpb/entrybatch.go:25-58,
 * with Entry.MarshalTo, raftpb/raft_optimized.go:166-300) and their
 * crc32.ChecksumIEEE (the checksum of internal/transport/tcp.go:146).
 * *len = 0 when the replica saved nothing that round. */
int drb_export_saved(drb_engine *e, uint64_t group, uint32_t slot,
                     uint8_t *buf, size_t cap, uint32_t *len, uint32_t *crc);
/* save_batched: the round's LogDB records of one replica, in Put order.
 * Record k is the value of key EntryBatchKey(shard, replica, batch)
 * (batch.go:310-313): bytes [offset, offset + len) of the replica's
 * drb_export_saved buffer, with its CRC32-IEEE.  The merge source of a
 * batch is this engine's own earlier saves of that replica (its LogDB
 * starts empty at drb_engine_create; an imported replica's record stream
 * restarts at its next save). */
#define DRB_SAVE_RECS 4
typedef struct drb_save_record {
  uint64_t batch;   /* index / 48 */
  uint32_t offset;  /* bytes into the replica's save buffer */
  uint32_t len;
  uint32_t crc;
  uint32_t reserved;
} drb_save_record;
int drb_export_save_records(drb_engine *e, uint64_t group, uint32_t slot,
                            drb_save_record *out, size_t cap, size_t *n);
/* save_tan: the record replica (slot, group) appended to its tan log in
 * the last round that ran with encode_saves -- what db.write
 * (internal/tan/db.go:97-130) puts in the log file: the host pwrites `len`
 * bytes at `offset` of log `log` (creating that log first when
 * DRB_TAN_NEW_LOG: createNewLog, open.go:171-198), fsyncs when
 * DRB_TAN_SYNC, and updates its index with {first_index, last_index}
 * (EntriesToSave, 0 when none) and `commit` (the State's, 0 when the
 * Update had none) at position `offset` (db.updateIndex, db.go:139-173). */
#define DRB_TAN_WRITTEN 1u  /* a record was written (else len = 0) */
#define DRB_TAN_SYNC 2u     /* db.write's sync result (db.go:113-114) */
#define DRB_TAN_NEW_LOG 4u  /* makeRoomForWrite switched to a new log */
#define DRB_TAN_OVERFLOW 8u /* save_cap too small (never with the pre-pass) */
typedef struct drb_tan_record {
  uint64_t offset;      /* log offset the bytes start at (d.mu.offset) */
  uint64_t first_index; /* EntriesToSave[0].Index */
  uint64_t last_index;  /* EntriesToSave[n-1].Index */
  uint64_t commit;      /* State.Commit */
  uint32_t len;         /* bytes appended, zero padding and chunk headers
                         * included */
  uint32_t flags;       /* DRB_TAN_* */
  uint32_t log;         /* this replica's log number (0: the first) */
  uint32_t pad;
} drb_tan_record;
int drb_export_tan(drb_engine *e, uint64_t group, uint32_t slot,
                   drb_tan_record *rec, uint8_t *buf, size_t cap);
/* the tan writer position of a replica: the offset in its current log,
 * that log's number, and whether nodeStates holds a non-empty State (the
 * next Update's skip / sync decision, db.go:108-114).  drb_tan_set hands a
 * replica over from a CPU tan db (fallback return, node.go:1139-1159). */
typedef struct drb_tan_state {
  uint64_t offset;
  uint32_t log;
  uint32_t state_stored;
} drb_tan_state;
int drb_tan_get(drb_engine *e, uint64_t group, uint32_t slot,
                drb_tan_state *out);
int drb_tan_set(drb_engine *e, uint64_t group, uint32_t slot,
                const drb_tan_state *in);
/* tan_multiplexed: log (slot, key)'s part of the last encode_saves round
 * -- what concurrentSaveState (internal/tan/logdb.go:265-304) appended to
 * it: `bytes` bytes starting at offset start_offset of log start_log, the
 * records back to back; when DRB_TAN_NEW_LOG a makeRoomForWrite switch
 * happened inside (each record's drb_export_tan says where, the new log
 * starts at offset 0); one fsync of the log when DRB_TAN_SYNC.  buf
 * (cap >= bytes) receives the bytes. */
typedef struct drb_tan_log {
  uint64_t start_offset;
  uint64_t end_offset;  /* the log writer's offset after the round */
  uint64_t bytes;
  uint32_t start_log;
  uint32_t end_log;
  uint32_t flags;       /* DRB_TAN_SYNC | DRB_TAN_NEW_LOG */
  uint32_t pad;
} drb_tan_log;
int drb_export_tan_log(drb_engine *e, uint32_t slot, uint32_t key,
                       drb_tan_log *out, uint8_t *buf, size_t cap);
/* The round's tan records on the device for a bulk writer: replica
 * (slot, g)'s bytes at bytes + (slot * G + g) * save_cap, its record
 * {offset lo, offset hi, len, flags | log << 8} at recs[slot * G + g]. */
int drb_tan_buffers(drb_engine *e, void **bytes, void **recs);

/* The whole round's save output on the device, for a GPU-side writer or
 * one D2H copy: replica (slot, g) owns bytes[(slot * G + g) * save_cap ..]
 * with lens[slot * G + g] and crcs[slot * G + g]. */
int drb_saved_buffers(drb_engine *e, void **bytes, uint32_t **lens,
                      uint32_t **crcs);

/* --- cross-rank mailbox exchange (place_world >= 2) ------
 * The round's messages to replicas on other ranks stay in this engine's
 * outbox planes; plane (from, to) moves whole to rank
 * (place_rank + to - from) mod N, whose next round reads it as its inbox
 * plane (from, to).  This replaces the reference transport
 * (Transport.Send, transport.go:346 -> handleRequest, :305) for
 * GPU-resident replicas: per round, drb_plane_counts, exchange the count
 * words with the peers, then move drb_plane_regions (RCCL send/recv, or
 * drb_exchange_local in one process). */
typedef struct drb_region {
  void *ptr;       /* device address */
  uint64_t bytes;
} drb_region;

#define DRB_PLANE_REGIONS 10
/* per lane (max): Replicate records (positions 0..), other records
 * (positions mailbox-1 downwards), entry rows; a record's 2nd chunk */
#define DRB_PLANE_KREP(w) ((w) & 0x1fu)
#define DRB_PLANE_KOTH(w) (((w) >> 5) & 0x1fu)
#define DRB_PLANE_E(w) (((w) >> 10) & 0xffu)
#define DRB_PLANE_C1 (1u << 18)
#define DRB_PLANE_HDR (1u << 19)  /* a header without records (Quiesce) */
/* records with a term of their own (elections: the raft launch's
 * MF_TERM_OTHER records): their rterm rows travel with the plane */
#define DRB_PLANE_TOTHER (1u << 20)

/* words[from * R + to] for this rank's remote planes of the last round
 * (0 for local or empty ones).  Synchronises the engine stream. */
int drb_plane_counts(drb_engine *e, uint32_t *words);
/* The rank a plane goes to (dir 0) or comes from (dir 1); -1 if local. */
int drb_plane_peer(const drb_engine *e, uint32_t from, uint32_t to, int dir);
/* The same routing as a pure function of the placement (no device). */
int drb_place_peer(uint32_t world, uint32_t rank, uint32_t from, uint32_t to,
                   int dir);
/* The engine's role map, kept on the host (without elections roles change
 * only by init and import; a replica whose role would change in a round
 * falls back): bit s of *leader_slots when a hosted replica at slot s is a
 * leader, of *follower_slots when one is not.  No device work.  With
 * fixed-capacity exchange, plane (from, to) can carry fast-path messages
 * only when `from` or `to` is a leader slot on some rank (followers send
 * only to leaders).  With drb_config.elections roles change on the device
 * (the raft launch), so a fixed exchange moves every remote plane, with
 * DRB_PLANE_TOTHER (dragonboat_amd/exchange.py fixed_words). */
int drb_role_slots(const drb_engine *e, uint32_t *leader_slots,
                   uint32_t *follower_slots);
/* The device regions of plane (from, to) for the last round, sized by the
 * SENDER's word: dir 0 in this engine's outbox planes, dir 1 in its inbox
 * planes.  Sender and receiver list identical sizes in the same order.
 * Returns the region count (<= DRB_PLANE_REGIONS) or < 0. */
int drb_plane_regions(drb_engine *e, uint32_t from, uint32_t to,
                      uint32_t word, int dir, drb_region *out);
/* The whole exchange among engines[rank] of one process, every engine at
 * the same round (NodeHost is one process per machine driving every GPU;
 * Transport.Send -> handleRequest, transport.go:346, :305).  No host
 * synchronisation either way: the work is enqueued on the receivers'
 * streams behind the senders' rounds (cross-stream events), and each
 * sender's next round waits for the work that read its outbox.
 *  - Every engine on one device (n <= 16): a pull kernel per receiver reads
 *    each sender plane's header on the device and copies, lane by lane,
 *    only what it counts (records, rterm rows, max-append word, entry rows
 *    up to the last entry sent) -- a counted exchange without host reads.
 *  - Otherwise: every plane that can carry fast-path messages -- one with a
 *    leader slot at either end (drb_role_slots, OR over the engines), or
 *    every plane with drb_config.elections -- moves at its full capacity
 *    (all mailbox positions, both chunks, the header, the max-append word,
 *    the entry-row base and entry_mbox entry rows: what the pre-pass
 *    bounds) by peer copies, so no counts are read.
 * The receivers read only what the plane headers count.
 *  - Engines bound by drb_exchange_local_bind: nothing moves; only the
 *    rounds' order is enqueued (each engine's next round waits for every
 *    engine's last one). */
int drb_exchange_local(drb_engine *const *engines, uint32_t n);
/* Binds the n engines of one process on one device (engines[r] rank r of
 * the placement, n >= 2, every engine at the same round) for the zero-copy
 * exchange: their step kernels read each remote plane straight from the
 * sender rank's outbox -- every lane of an inbound plane (from, to) comes
 * from one rank, at the same lane (drb_place_peer) -- so drb_exchange_local
 * copies nothing.  For the rest of their lives the bound engines take no
 * other exchange and no delivered messages (drb_ingest_ex, drb_ingest_wire,
 * drb_exchange_rccl*, drb_exchange_local_counted, drb_plane_regions dir 1:
 * DRB_EINVAL); they are destroyed together (a peer's destroy waits for the
 * others' queued work and fails their later rounds). */
int drb_exchange_local_bind(drb_engine *const *engines, uint32_t n);
/* The fixed-capacity exchange step of a process-per-GPU host as a list of
 * point-to-point transfers: every remote plane that can carry fast-path
 * messages -- a leader slot at either end on some rank (leader_mask: the
 * OR over the ranks of drb_role_slots' leader_slots; every plane with
 * drb_config.elections) -- at its full capacity (what the step pre-pass
 * bounds), its drb_plane_regions sent to the rank the plane goes to and
 * received from the rank it comes from.  Every rank lists its transfers in
 * the same (from, to, region) order, so each pair of ranks posts matching
 * sends and receives (dragonboat_amd/exchange.py plan(), fixed mode).
 * *n_xfers = the count; DRB_ERANGE when it exceeds cap (xfers may be NULL
 * with cap 0 to size the list).  Empty before the first round and with
 * place_world < 2. */
typedef struct drb_xfer {
  uint32_t peer;  /* the other rank */
  uint32_t recv;  /* 0: send this region, 1: receive into it */
  void *ptr;      /* device address */
  uint64_t bytes;
} drb_xfer;
int drb_exchange_plan(drb_engine *e, uint32_t leader_mask, drb_xfer *xfers,
                      size_t cap, size_t *n_xfers);
/* The same step over RCCL (xGMI between the GPUs of a node): the transfers
 * as ncclSend / ncclRecv in one ncclGroupStart .. ncclGroupEnd on the
 * engine stream -- behind the round that wrote the outbox planes, ahead of
 * the next one, no host synchronisation -- then drb_exchange_mark.  comm is
 * the rank's ncclComm_t over the placement's ranks (rank place_rank of
 * place_world; DRB_EINVAL otherwise); RCCL errors are DRB_EDEVICE.
 * Replaces Transport.Send -> handleRequest (transport.go:346, :305) for
 * GPU-resident replicas, with no Python in the host process. */
int drb_exchange_rccl(drb_engine *e, void *comm, uint32_t leader_mask);
/* The transfer list of an exchange step from every rank's plane words:
 * words[q * R * R + from * R + to] is rank q's summary word of plane
 * (from, to) -- drb_plane_counts' on each rank for the counted step, the
 * full-capacity row for the fixed one (drb_exchange_plan) -- this rank
 * sending each plane at its own word and receiving it at its sender's, in
 * the same order on every rank (dragonboat_amd/exchange.py plan()). */
int drb_exchange_plan_words(drb_engine *e, const uint32_t *words,
                            drb_xfer *xfers, size_t cap, size_t *n_xfers);
/* The counted step over RCCL: drb_plane_counts (a synchronisation of the
 * engine stream), an ncclAllGather of every rank's words, then the planes
 * at those sizes as ncclSend / ncclRecv in one group on the engine stream
 * and drb_exchange_mark.  At C4's steady state about half the fixed step's
 * bytes, for one host round trip per round.
 * Collective: every rank calls it after the same round. */
int drb_exchange_rccl_counted(drb_engine *e, void *comm);
/* leader_mask for drb_exchange_rccl / drb_exchange_plan: the OR over comm's
 * ranks of each engine's leader slots (an ncclAllReduce; synchronises the
 * engine stream).  Collective: every rank calls it after its imports. */
int drb_exchange_rccl_roles(drb_engine *e, void *comm, uint32_t *leader_mask);
/* Inbound plane bytes the exchanges moved into this engine since the last
 * reset (the device pull's own count plus region copies); synchronises the
 * engine stream. */
int drb_exchange_bytes(drb_engine *e, uint64_t *bytes, int reset);
/* The same exchange at the planes' counted sizes (drb_plane_counts per
 * engine, i.e. one stream synchronisation each, then the copies and a
 * synchronisation of every stream): fewer bytes, host round trips. */
int drb_exchange_local_counted(drb_engine *const *engines, uint32_t n);
/* A process-per-GPU host (RCCL send/recv of drb_plane_regions) tells the
 * engine its exchange of the last round is enqueued.  With replicas spread
 * over ranks, drb_ingest / drb_ingest_wire return DRB_EAGAIN between a
 * round's launch and its exchange: a message for a remote plane written
 * then would be overwritten by the exchange's copy of that plane (the
 * receiver's inbound header), so the transport retries after the exchange.
 * Ordering contract: the exchange's receives must be enqueued on the
 * engine stream (drb_engine_stream; ncclGroupStart ... ncclGroupEnd on it,
 * as dragonboat_amd/exchange.py does) or have completed before this call
 * -- drb_ingest's placement is ordered behind them only on that stream.  A
 * host whose collectives run on a stream of its own makes the engine
 * stream wait on an event recorded after them (hipStreamWaitEvent), or
 * synchronises that stream, before drb_exchange_mark.
 * drb_exchange_local marks it itself. */
int drb_exchange_mark(drb_engine *e);

/*
 * The entries one replica slot applied in the last round, for
 * node.ApplyUpdate -> pendingProposals.applied (node.go:243-257,
 * request.go:1041-1045; rsm handleEntry statemachine.go:935-969): per
 * entry its Key / ClientID / SeriesID and sm.Result.Value, which KVTest
 * sets to the length of the update's Cmd payload (kvtest.go:161).  Groups
 * [first_group, first_group + n_groups), sorted by (group, index); *n_out
 * is the count (DRB_ERANGE if more than cap).  Replicas handed to the CPU
 * path report nothing, except those whose apply stopped
 * (DRB_F_APPLY_STOPPED): their entries applied before the stop.
 */
typedef struct drb_apply_result {
  uint64_t group;      /* lane */
  uint64_t index;
  uint64_t key;        /* pb.Entry.Key: the proposal's RequestState key */
  uint64_t client_id;
  uint64_t series_id;
  uint64_t value;      /* sm.Result.Value */
  uint32_t slot;
  uint32_t ignored;    /* 1: an empty no-op entry (statemachine.go:939-942) */
} drb_apply_result;
int drb_apply_results(drb_engine *e, uint32_t slot, uint64_t first_group,
                      uint64_t n_groups, drb_apply_result *out, size_t cap,
                      size_t *n_out);

/* Peer.Commit's ordering for a durable LogDB (engine.go:1343-1359,
 * raftpb/update.go:60-69): the host calls this once round `round`'s
 * EntriesToSave (drb_saved_buffers / drb_export_saved) are persisted; with
 * drb_config.durable_log the round's non-Replicate messages (ReplicateResp
 * and the rest, sent after SaveRaftState, node.go:1104-1108) are not
 * delivered -- no later round runs, no wire stream is encoded -- before. */
int drb_commit_round(drb_engine *e, uint64_t round);
/* The last round committed so far (durable_log). */
uint64_t drb_committed_round(const drb_engine *e);

/* IStateMachine.Lookup used by NodeHost.ReadLocalNode (nodehost.go:849). */
int drb_kv_lookup(drb_engine *e, uint64_t group, uint32_t slot,
                  const uint8_t *key, uint32_t key_len, uint8_t *val,
                  uint32_t val_cap, uint32_t *val_len);
/* Replaces one replica's KV state machine with n pairs: the state machine
 * a CPU StateMachine hands back with its group after a fallback, next to
 * drb_import_replicas (IStateMachine.RecoverFromSnapshot,
 * statemachine/rsm.go:189; KVTest.RecoverFromSnapshot,
 * internal/tests/kvtest.go:200-239).  keys[i*8..] (key_lens[i] <= 8,
 * distinct), vals[i*val_stride..] (val_lens[i] <= kv_val_cap).  Out-of-line
 * values take fresh blocks from the value pool (the replica's old blocks
 * are not reused).  DRB_ERANGE when the pairs do not fit. */
int drb_kv_import(drb_engine *e, uint64_t group, uint32_t slot,
                  const uint8_t *keys, const uint32_t *key_lens,
                  const uint8_t *vals, const uint32_t *val_lens,
                  size_t val_stride, size_t n);
/* Dumps every KV pair of one replica: keys[i*8..], key_lens[i],
 * vals[i*kv_val_cap..], val_lens[i]; returns the count in *n_out (the
 * table's slots, then the overflow chain's); DRB_ERANGE, with the full
 * count in *n_out, when it exceeds cap. */
int drb_kv_export(drb_engine *e, uint64_t group, uint32_t slot, uint8_t *keys,
                  uint32_t *key_lens, uint8_t *vals, uint32_t *val_lens,
                  size_t cap, size_t *n_out);

/* --- codecs (raftpb EntryBatch encode / CRC path) ---------------------- */

/* crc32.ChecksumIEEE (Go hash/crc32) over n independent buffers on the
 * device: crc[i] = CRC32-IEEE(data[off[i] .. off[i]+len[i])).  The framing
 * CRC of internal/transport/tcp.go:146,232.  Host pointers; the engine
 * stages them through HBM. */
int drb_crc32_ieee_batch(drb_engine *e, const uint8_t *data, size_t data_len,
                         const uint64_t *off, const uint32_t *len, size_t n,
                         uint32_t *crc);

/* --- wire path to replicas on other machines (raftpb MessageBatch) ---- */

/* MessageBatch fields Transport.processMessages sets
 * (internal/transport/transport.go:447-458) and the batch cut it applies. */
typedef struct drb_wire_cfg {
  uint64_t deployment_id;      /* NodeHostConfig.GetDeploymentID() */
  const char *source_address;  /* Transport.sourceID (RaftAddress) */
  uint32_t source_len;         /* <= 256 */
  uint32_t bin_ver;            /* raftio.TransportBinVersion = 210 */
  uint64_t max_batch_bytes;    /* settings.MaxMessageBatchSize; 0 = 64 MiB */
} drb_wire_cfg;

typedef struct drb_wire_out {
  uint64_t n_msgs;    /* pb.Messages encoded */
  uint64_t n_frames;  /* MessageBatches (TCP frames) */
  uint64_t n_bytes;   /* stream length */
} drb_wire_out;

/* Replaces, for every group, Transport.Send (transport.go:346) of the
 * messages replica slot from_slot sent to replica slot to_slot in the last
 * round, through processMessages -> sendMessageBatch -> writeMessage
 * (transport.go:443-508, tcp.go:142-178): encodes them on the device as
 * the byte stream of the TCP connection to the NodeHost hosting slot
 * to_slot -- per batch magic 0xAE7D, the 18-byte requestHeader (method
 * 100, size, header CRC32, payload CRC32) and the MessageBatch payload
 * (messagebatch.go:23-51, message.go:32-90, colfer Entries
 * raft_optimized.go:166-300).  Messages are taken group by group in shard
 * order, in send order within a group; a batch is cut where the sum of
 * Message.SizeUpperLimit (raft_optimized.go:1210) reaches max_batch_bytes,
 * the crossing message travelling alone (transport.go:481-500).  The
 * stream stays in an engine-owned device buffer until the next call. */
int drb_encode_wire(drb_engine *e, uint32_t from_slot, uint32_t to_slot,
                    const drb_wire_cfg *cfg, drb_wire_out *out);
/* Device pointer and length of the last drb_encode_wire stream. */
int drb_wire_buffer(drb_engine *e, const uint8_t **dev, uint64_t *len);
/* Copies that stream to host memory (synchronises the engine stream). */
int drb_export_wire(drb_engine *e, uint8_t *out, size_t cap, size_t *len);

typedef struct drb_wire_in {
  uint64_t frames;     /* frames read */
  uint64_t messages;   /* pb.Messages decoded and handed to drb_ingest */
  uint64_t accepted;   /* placed into the next round's inbox */
  uint64_t dropped;    /* DeploymentId / BinVer mismatch or drb_ingest drop */
  uint64_t snapshots;  /* snapshot chunks / InstallSnapshot (CPU path) */
  uint64_t consumed;   /* stream bytes consumed */
  uint64_t bad;        /* 1: stopped at a bad frame (ErrBadMessage) */
  uint64_t diverted;   /* DRB_ING_DIVERTED (drb_ingest_ex) */
} drb_wire_in;

/* A message of the last drb_ingest_wire stream that goes to the CPU path:
 * its Requests element (a marshalled pb.Message) at stream[offset, offset +
 * length), for pb.Message.Unmarshal and the receiver's raft.Peer. */
typedef struct drb_wire_cpu {
  uint64_t offset;
  uint32_t length;
  uint32_t fate;  /* DRB_ING_DIVERTED or DRB_ING_SNAPSHOT */
} drb_wire_cpu;

/* The receiving end of that connection, for replicas hosted here whose
 * peers are elsewhere: readMessage (tcp.go:180-237: header and payload
 * CRC32), MessageBatch / Message / colfer Entry Unmarshal
 * (raft_optimized.go:308-656, 659-983, 1056-1207), the DeploymentId /
 * BinVer filter of Transport.handleRequest (transport.go:305-316), then
 * drb_ingest's placement.  Frames are consumed in order; a bad frame stops
 * the stream as ErrBadMessage closes the connection.  A stream that ends
 * inside a frame whose bytes so far are sound is not bad: `consumed` stops
 * before that frame, and the transport passes its bytes again with the
 * ones that follow (readMessage's io.ReadFull would still be waiting).  The stream is
 * uploaded once: payload CRCs, message decode and placement run on the
 * GPU (drb_ingest.hpp); the host reads the 20 B frame headers and walks
 * each batch's top-level fields.  Messages are placed, dropped or diverted
 * as by drb_ingest_ex (a delivered entry's Cmd longer than cmd_cap is a
 * capacity divert); the diverted ones and the InstallSnapshot messages are
 * listed, in stream order, by drb_ingest_wire_cpu. */
int drb_ingest_wire(drb_engine *e, const uint8_t *stream, size_t len,
                    uint64_t deployment_id, drb_wire_in *out);
/* The CPU path's messages of the last drb_ingest_wire call (valid until
 * the next one): *n_out is the count, DRB_ERANGE when it exceeds cap. */
int drb_ingest_wire_cpu(drb_engine *e, drb_wire_cpu *out, size_t cap,
                        size_t *n_out);
/* A receive buffer of at least `cap` bytes in pinned (page-locked) host
 * memory, owned by the engine (grow-only; valid until the next call or
 * drb_engine_destroy).  A transport that reads its connection into it
 * (conn.Read in tcp.go:180-237's readMessage) and passes it to
 * drb_ingest_wire has the stream uploaded by DMA at the link's rate
 * instead of through the driver's pageable staging. */
int drb_ingest_buffer(drb_engine *e, size_t cap, uint8_t **buf);
/* drb_ingest_buffer is the engine's one buffer, for a single transport
 * thread (a later call with a larger cap replaces it).  Several transport
 * threads each take a buffer of their own, pinned, and free it when their
 * connection closes; drb_ingest_wire waits for its upload before
 * returning, so a buffer may be refilled as soon as the call returns. */
int drb_ingest_buffer_alloc(drb_engine *e, size_t cap, uint8_t **buf);
int drb_ingest_buffer_free(drb_engine *e, uint8_t *buf);

#ifdef __cplusplus
}
#endif

#endif /* DRB_ENGINE_H */
