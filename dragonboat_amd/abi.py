"""ctypes mirror of include/drb_engine.h (the C-ABI boundary).

Plain data only: these Structures describe the records that cross the
boundary (pb.Entry, pb.Message, per-replica raft state, round I/O).
"""
import ctypes as C

DRB_MAX_REPLICAS = 8
DRB_RI_DEPTH = 4
DRB_NONE = 0xFFFFFFFF

# status codes
DRB_OK = 0
DRB_EINVAL = -1
DRB_EDEVICE = -2
DRB_ENOMEM = -3
DRB_ENOSYS = -4
DRB_ERANGE = -5
DRB_EAGAIN = -6  # retry: ingest between a round and its exchange
DRB_EDIVERTED = -7  # drb_ingest: some messages went to the CPU path

# raftpb.MessageType (raftpb/types.go:8-37)
MSG = dict(
    LocalTick=0, Election=1, LeaderHeartbeat=2, ConfigChangeEvent=3, NoOP=4,
    Ping=5, Pong=6, Propose=7, SnapshotStatus=8, Unreachable=9,
    CheckQuorum=10, BatchedReadIndex=11, Replicate=12, ReplicateResp=13,
    RequestVote=14, RequestVoteResp=15, InstallSnapshot=16, Heartbeat=17,
    HeartbeatResp=18, ReadIndex=19, ReadIndexResp=20, Quiesce=21,
    SnapshotReceived=22, LeaderTransfer=23, TimeoutNow=24, RateLimit=25,
    RequestPreVote=26, RequestPreVoteResp=27, LogQuery=28)
MSG_NAME = {v: k for k, v in MSG.items()}

# raftpb.EntryType
ENTRY_APPLICATION = 0
ENTRY_CONFIG_CHANGE = 1
ENTRY_ENCODED = 2
ENTRY_METADATA = 3

# raft.State (internal/raft/raft.go:63-71)
FOLLOWER, CANDIDATE, PREVOTE_CANDIDATE, LEADER, NONVOTING, WITNESS = range(6)

# remoteStateType (internal/raft/remote.go:54-59)
REMOTE_RETRY, REMOTE_WAIT, REMOTE_REPLICATE, REMOTE_SNAPSHOT = range(4)

F_HOSTED = 1
F_FALLBACK = 2
F_ERROR = 4
F_APPLY_STOPPED = 8

FB = dict(NONE=0, TERM_MISMATCH=1, MESSAGE_TYPE=2, ELECTION=3,
          CHECK_QUORUM=4, ENTRY_TYPE=5, CAPACITY=6, ROLE=7, SNAPSHOT=9,
          ERR_LOG_RANGE=100, ERR_COMMIT=101, ERR_APPEND=103, ERR_APPLY=104,
          ERR_READINDEX=105, ERR_TRANSFER=106, ERR_PROPOSE=107)
FB_NAME = {v: k for k, v in FB.items()}


class RemoteState(C.Structure):
    _fields_ = [("match", C.c_uint64), ("next", C.c_uint64),
                ("state", C.c_uint32), ("active", C.c_uint32)]


class ReadStatus(C.Structure):
    _fields_ = [("ctx_low", C.c_uint64), ("ctx_high", C.c_uint64),
                ("index", C.c_uint64), ("from_", C.c_uint64),
                ("confirmed", C.c_uint32), ("pad", C.c_uint32)]


_REPLICA_U64 = [
    "shard_id", "replica_id", "term", "vote", "leader_id", "applied",
    "election_tick", "heartbeat_tick", "randomized_election_timeout",
    "tick_count", "committed", "processed", "last_index", "marker_index",
    "saved_to", "applied_to_index", "applied_to_term", "applied_index",
    "confirmed_index", "pushed_index", "prev_term", "prev_vote",
    "prev_commit", "sm_index", "sm_term", "kv_count", "qs_current_tick",
    "qs_idle_since", "qs_quiesced_since", "qs_exit_quiesce_tick", "rng"]


class ReplicaState(C.Structure):
    _fields_ = ([(n, C.c_uint64) for n in _REPLICA_U64] +
                [("role", C.c_uint32), ("flags", C.c_uint32),
                 ("fallback_reason", C.c_uint32), ("ri_count", C.c_uint32),
                 ("votes", C.c_uint32), ("transfer", C.c_uint32),
                 ("remotes", RemoteState * DRB_MAX_REPLICAS),
                 ("ri", ReadStatus * DRB_RI_DEPTH)])

    def to_dict(self, num_replicas=None):
        d = {n: getattr(self, n) for n in _REPLICA_U64}
        for n in ("role", "flags", "fallback_reason", "ri_count", "votes",
                  "transfer"):
            d[n] = getattr(self, n)
        nr = num_replicas or DRB_MAX_REPLICAS
        d["remotes"] = [(r.match, r.next, r.state, r.active)
                        for r in list(self.remotes)[:nr]]
        d["ri"] = [(x.ctx_low, x.ctx_high, x.index, x.from_, x.confirmed)
                   for x in list(self.ri)[:self.ri_count]]
        return d


class Entry(C.Structure):
    _fields_ = [("term", C.c_uint64), ("index", C.c_uint64),
                ("key", C.c_uint64), ("client_id", C.c_uint64),
                ("series_id", C.c_uint64), ("responded_to", C.c_uint64),
                ("type", C.c_uint32), ("cmd_len", C.c_uint32),
                ("cmd_off", C.c_uint64)]


class Message(C.Structure):
    _fields_ = [("shard_id", C.c_uint64), ("from_", C.c_uint64),
                ("to", C.c_uint64), ("term", C.c_uint64),
                ("log_term", C.c_uint64), ("log_index", C.c_uint64),
                ("commit", C.c_uint64), ("hint", C.c_uint64),
                ("hint_high", C.c_uint64), ("type", C.c_uint32),
                ("reject", C.c_uint32), ("n_entries", C.c_uint64),
                ("entries_off", C.c_uint64)]


class ReadyToRead(C.Structure):
    _fields_ = [("shard_id", C.c_uint64), ("replica_id", C.c_uint64),
                ("index", C.c_uint64), ("ctx_low", C.c_uint64),
                ("ctx_high", C.c_uint64)]


class Config(C.Structure):
    _fields_ = [("num_groups", C.c_uint64), ("first_shard_id", C.c_uint64),
                ("num_replicas", C.c_uint32), ("window", C.c_uint32),
                ("cmd_cap", C.c_uint32), ("max_props", C.c_uint32),
                ("prop_slots", C.c_uint32), ("ri_slots", C.c_uint32),
                ("mailbox", C.c_uint32), ("kv_slots", C.c_uint32),
                ("kv_val_cap", C.c_uint32), ("election_rtt", C.c_uint32),
                ("heartbeat_rtt", C.c_uint32), ("check_quorum", C.c_uint32),
                ("device", C.c_int32), ("save_cap", C.c_uint32),
                ("total_groups", C.c_uint64), ("place_world", C.c_uint32),
                ("place_rank", C.c_uint32), ("entry_mbox", C.c_uint32),
                ("kv_pool_blocks", C.c_uint32), ("flagged_cap", C.c_uint32),
                ("quiesce", C.c_uint32), ("durable_log", C.c_uint32),
                ("save_batched", C.c_uint32), ("save_tan", C.c_uint32),
                ("elections", C.c_uint32), ("tan_max_log", C.c_uint64),
                ("tan_multiplexed", C.c_uint32), ("pre_vote", C.c_uint32),
                ("max_reads_per_ctx", C.c_uint32),
                ("kv_overflow_buckets", C.c_uint64),
                ("forward_proposals", C.c_uint32),
                ("nonvoting_slots", C.c_uint32),
                ("witness_slots", C.c_uint32),
                ("host_copies", C.c_uint32), ("no_lean", C.c_uint32)]


class ReadResult(C.Structure):
    """drb_read_result: one served ReadLocalNode read of the last round."""
    _fields_ = [("shard_id", C.c_uint64), ("index", C.c_uint64),
                ("ctx_low", C.c_uint64), ("ctx_high", C.c_uint64),
                ("key", C.c_uint64), ("replica_id", C.c_uint32),
                ("read", C.c_uint32), ("found", C.c_uint32),
                ("vlen", C.c_uint32), ("value", C.c_uint32),
                ("pad", C.c_uint32)]


class ApplyResult(C.Structure):
    """drb_apply_result: one entry applied in the last round."""
    _fields_ = [("group", C.c_uint64), ("index", C.c_uint64),
                ("key", C.c_uint64), ("client_id", C.c_uint64),
                ("series_id", C.c_uint64), ("value", C.c_uint64),
                ("slot", C.c_uint32), ("ignored", C.c_uint32)]


# drb_worker_bufs value_meta codes (include/drb_engine.h)
WORKER_MISS, WORKER_V4, WORKER_SHORT, WORKER_LONG = 0, 1, 2, 3


def worker_lane(w):
    """(ReadyToReads, served mask, applied own proposals) of a lanes[]
    word."""
    return w & 0xF, (w >> 4) & 0xFF, (w >> 12) & 0xFFFF


def worker_value(code, word):
    """A served read's result from its 2-bit code and value word: None (not
    found), the value bytes, or (first 4 bytes, True) for a longer one."""
    if code == WORKER_MISS:
        return None
    if code == WORKER_V4:
        return word.to_bytes(4, "little")
    if code == WORKER_SHORT:
        return (word & 0xFFFFFF).to_bytes(3, "little")[:word >> 24]
    return (word.to_bytes(4, "little"), True)


class WorkerBufs(C.Structure):
    """drb_worker_bufs: pinned host buffers of one step-worker export."""
    _fields_ = [("lanes", C.POINTER(C.c_uint32)), ("lanes_cap", C.c_uint64),
                ("reads", C.POINTER(C.c_uint32)), ("reads_cap", C.c_uint64),
                ("values", C.POINTER(C.c_uint32)),
                ("value_meta", C.POINTER(C.c_uint8)),
                ("values_cap", C.c_uint64),
                ("deferred", C.POINTER(C.c_uint64)),
                ("deferred_cap", C.c_uint64),
                ("n_reads", C.c_uint64), ("n_values", C.c_uint64),
                ("n_deferred", C.c_uint64)]


class SaveRecord(C.Structure):
    """drb_save_record: one batched LogDB record of the last round."""
    _fields_ = [("batch", C.c_uint64), ("offset", C.c_uint32),
                ("len", C.c_uint32), ("crc", C.c_uint32),
                ("reserved", C.c_uint32)]


class Flagged(C.Structure):
    """drb_flagged: a replica that left the fast path (drb_take_flagged)."""
    _fields_ = [("group", C.c_uint64), ("shard_id", C.c_uint64),
                ("round", C.c_uint64), ("slot", C.c_uint32),
                ("reason", C.c_uint32), ("flags", C.c_uint32),
                ("pad", C.c_uint32)]


TAN_WRITTEN, TAN_SYNC, TAN_NEW_LOG, TAN_OVERFLOW = 1, 2, 4, 8


class TanRecord(C.Structure):
    """drb_tan_record: what one replica's tan log grew by last round."""
    _fields_ = [("offset", C.c_uint64), ("first_index", C.c_uint64),
                ("last_index", C.c_uint64), ("commit", C.c_uint64),
                ("len", C.c_uint32), ("flags", C.c_uint32),
                ("log", C.c_uint32), ("pad", C.c_uint32)]


class TanState(C.Structure):
    """drb_tan_state: a replica's tan writer position."""
    _fields_ = [("offset", C.c_uint64), ("log", C.c_uint32),
                ("state_stored", C.c_uint32)]


class TanLog(C.Structure):
    """drb_tan_log: a multiplexed tan log's part of the last round."""
    _fields_ = [("start_offset", C.c_uint64), ("end_offset", C.c_uint64),
                ("bytes", C.c_uint64), ("start_log", C.c_uint32),
                ("end_log", C.c_uint32), ("flags", C.c_uint32),
                ("pad", C.c_uint32)]


class Region(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("bytes", C.c_uint64)]


class Xfer(C.Structure):
    """drb_xfer: one transfer of the fixed exchange (drb_exchange_plan)."""
    _fields_ = [("peer", C.c_uint32), ("recv", C.c_uint32),
                ("ptr", C.c_void_p), ("bytes", C.c_uint64)]


PLANE_REGIONS = 10
PLANE_C1 = 1 << 18


def plane_krep(w):
    return w & 0x1f


def plane_koth(w):
    return (w >> 5) & 0x1f


def plane_e(w):
    return (w >> 10) & 0xff


class WireCfg(C.Structure):
    _fields_ = [("deployment_id", C.c_uint64),
                ("source_address", C.c_char_p), ("source_len", C.c_uint32),
                ("bin_ver", C.c_uint32), ("max_batch_bytes", C.c_uint64)]


class WireOut(C.Structure):
    _fields_ = [("n_msgs", C.c_uint64), ("n_frames", C.c_uint64),
                ("n_bytes", C.c_uint64)]


class WireIn(C.Structure):
    _fields_ = [("frames", C.c_uint64), ("messages", C.c_uint64),
                ("accepted", C.c_uint64), ("dropped", C.c_uint64),
                ("snapshots", C.c_uint64), ("consumed", C.c_uint64),
                ("bad", C.c_uint64), ("diverted", C.c_uint64)]


class WireCpu(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("length", C.c_uint32),
                ("fate", C.c_uint32)]


# drb_ingest_fate
ING_PLACED, ING_DROPPED, ING_DIVERTED, ING_SNAPSHOT = range(4)


class RoundIn(C.Structure):
    _fields_ = [("tick", C.c_uint32), ("prop_slot", C.c_uint32),
                ("ri_slot", C.c_uint32), ("reads_per_ctx", C.c_uint32),
                ("read_key_space", C.c_uint32),
                ("encode_saves", C.c_uint32), ("ri_replica", C.c_uint32),
                ("listed", C.c_uint32), ("prop_replica", C.c_uint32)]


class RoundOut(C.Structure):
    _fields_ = [("round", C.c_uint64), ("committed_entries", C.c_uint64),
                ("applied_entries", C.c_uint64), ("messages", C.c_uint64),
                ("ready_to_reads", C.c_uint64),
                ("dropped_read_indexes", C.c_uint64),
                ("fallbacks", C.c_uint64), ("errors", C.c_uint64),
                ("reads_served", C.c_uint64), ("reads_deferred", C.c_uint64),
                ("saved_entries", C.c_uint64), ("saved_bytes", C.c_uint64),
                ("replicas_stepped", C.c_uint64),
                ("log_records", C.c_uint64), ("log_syncs", C.c_uint64),
                ("log_new", C.c_uint64),
                ("elections_stepped", C.c_uint64),
                ("role_changes", C.c_uint64),
                ("dropped_proposals", C.c_uint64),
                ("lean_stepped", C.c_uint64)]

    def to_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


def message_to_tuple(m, ents, pool):
    """Canonical comparable form of a pb.Message (+ its entries)."""
    es = []
    for i in range(m.n_entries):
        e = ents[m.entries_off + i]
        es.append(entry_to_tuple(e, pool))
    return (m.shard_id, m.from_, m.to, m.type, m.term, m.log_term,
            m.log_index, m.commit, m.reject, m.hint, m.hint_high, tuple(es))


def entry_to_tuple(e, pool):
    cmd = bytes(pool[e.cmd_off:e.cmd_off + e.cmd_len]) if e.cmd_len else b""
    return (e.term, e.index, e.type, e.key, e.client_id, e.series_id,
            e.responded_to, cmd)
