"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the dragonboat_amd product path.
"""
import ctypes as C
import os
import subprocess

from dragonboat_amd.abi import (Entry, Message, ReadyToRead, ReplicaState,
                                RoundOut, entry_to_tuple, message_to_tuple)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


class Remote(C.Structure):
    """remote (internal/raft/remote.go:72-80)."""
    _fields_ = [("match", C.c_uint64), ("next", C.c_uint64),
                ("snapshot_index", C.c_uint64), ("state", C.c_uint32),
                ("active", C.c_int)]


class ClusterCfg(C.Structure):
    _fields_ = [("num_groups", C.c_uint64), ("first_shard_id", C.c_uint64),
                ("num_replicas", C.c_uint32), ("election_rtt", C.c_uint32),
                ("heartbeat_rtt", C.c_uint32), ("check_quorum", C.c_uint32),
                ("seed", C.c_uint64), ("logdb_keep", C.c_uint64),
                ("quiesce", C.c_uint32), ("pre_vote", C.c_uint32),
                ("gids", C.POINTER(C.c_uint64))]


P = C.c_void_p
U64 = C.c_uint64
U32 = C.c_uint32
PU64 = C.POINTER(C.c_uint64)
PU32 = C.POINTER(C.c_uint32)
PU8 = C.POINTER(C.c_uint8)
PE = C.POINTER(Entry)
PM = C.POINTER(Message)
PR = C.POINTER(Remote)


def _declare(L):
    sig = {
        "orc_last_error": (C.c_char_p, []),
        "orc_remote_become_retry": (None, [PR]),
        "orc_remote_retry_to_wait": (None, [PR]),
        "orc_remote_wait_to_retry": (None, [PR]),
        "orc_remote_become_wait": (None, [PR]),
        "orc_remote_become_replicate": (None, [PR]),
        "orc_remote_become_snapshot": (None, [PR, U64]),
        "orc_remote_try_update": (C.c_int, [PR, U64]),
        "orc_remote_progress": (C.c_int, [PR, U64]),
        "orc_remote_responded_to": (None, [PR]),
        "orc_remote_decrease_to": (C.c_int, [PR, U64, U64]),
        "orc_remote_is_paused": (C.c_int, [PR]),
        "orc_readindex_new": (P, []),
        "orc_readindex_free": (None, [P]),
        "orc_readindex_add_request": (C.c_int, [P, U64, U64, U64, U64]),
        "orc_readindex_len": (C.c_size_t, [P]),
        "orc_readindex_get": (C.c_int, [P, C.c_size_t, PU64, PU64, PU64, PU64]),
        "orc_readindex_confirm": (C.c_int, [P, U64, U64, U64, C.c_int, PU64,
                                            PU64, PU64, PU64, C.c_int]),
        "orc_readindex_push_raw_queue": (C.c_int, [P, U64, U64, C.c_int]),
        "orc_sort_match_values": (None, [PU64, C.c_int]),
        "orc_logdb_new": (P, []),
        "orc_logdb_free": (None, [P]),
        "orc_logdb_append": (C.c_int, [P, PE, C.c_size_t, PU8]),
        "orc_logdb_compact": (C.c_int, [P, U64]),
        "orc_logdb_set_state": (None, [P, U64, U64, U64]),
        "orc_raft_new_test": (P, [U64, PU64, C.c_int, U64, U64, P]),
        "orc_raft_new_test_kind": (P, [U64, PU64, C.c_int, PU64, C.c_int,
                                       C.c_int, U64, U64, P]),
        "orc_raft_add_member": (C.c_int, [P, U64, C.c_int]),
        "orc_raft_remote_kind": (C.c_int, [P, U64]),
        "orc_raft_free": (None, [P]),
        "orc_raft_handle": (C.c_int, [P, PM, PE, PU8]),
        "orc_raft_peer_handle": (C.c_int, [P, PM, PE, PU8]),
        "orc_raft_become_follower": (C.c_int, [P, U64, U64]),
        "orc_raft_become_candidate": (C.c_int, [P]),
        "orc_raft_become_leader": (C.c_int, [P]),
        "orc_raft_load_state": (C.c_int, [P, U64, U64, U64]),
        "orc_raft_broadcast_replicate": (C.c_int, [P]),
        "orc_raft_broadcast_heartbeat": (C.c_int, [P]),
        "orc_raft_try_commit": (C.c_int, [P]),
        "orc_raft_tick": (C.c_int, [P]),
        "orc_raft_campaign": (C.c_int, [P]),
        "orc_raft_set_randomized_election_timeout": (None, [P, U64]),
        "orc_raft_set_check_quorum": (None, [P, C.c_int]),
        "orc_raft_set_pre_vote": (None, [P, C.c_int]),
        "orc_raft_network_reset": (C.c_int, [P, U64, PU64, C.c_int]),
        "orc_raft_poke": (C.c_int, [P, C.c_int, U64]),
        "orc_raft_peek": (U64, [P, C.c_int]),
        "orc_raft_reset": (C.c_int, [P, U64]),
        "orc_raft_become_pre_vote_candidate": (C.c_int, [P]),
        "orc_raft_draw_timeout_time_for_election": (C.c_int, [P]),
        "orc_raft_term_not_matched": (C.c_int, [P, PM, PE, PU8]),
        "orc_raft_read_messages": (C.c_long, [P, PM, C.c_size_t, PE,
                                              C.c_size_t, PU8, C.c_size_t]),
        "orc_raft_log_entries": (C.c_long, [P, C.c_int, PE, C.c_size_t, PU8,
                                            C.c_size_t]),
        "orc_raft_log_term": (C.c_int, [P, U64, PU64]),
        "orc_raft_info": (None, [P, C.POINTER(ReplicaState)]),
        "orc_raft_remote": (C.c_int, [P, U64, PR]),
        "orc_raft_set_remote": (C.c_int, [P, U64, PR]),
        "orc_raft_ready_to_read": (C.c_size_t, [P, PU64, PU64, PU64,
                                                C.c_size_t]),
        "orc_raft_dropped_read_indexes": (C.c_size_t, [P]),
        "orc_log_commit_to": (C.c_int, [P, U64]),
        "orc_log_try_commit": (C.c_int, [P, U64, U64]),
        "orc_log_match_term": (C.c_int, [P, U64, U64]),
        "orc_log_up_to_date": (C.c_int, [P, U64, U64]),
        "orc_log_conflict_index": (C.c_long, [P, PE, C.c_size_t]),
        "orc_log_try_append": (C.c_int, [P, U64, PE, C.c_size_t, PU8]),
        "orc_log_append": (C.c_int, [P, PE, C.c_size_t, PU8]),
        "orc_log_commit_update": (C.c_int, [P, U64, U64, U64, U64]),
        "orc_raft_make_replicate": (C.c_long, [P, U64, U64, U64, PM, PE,
                                               C.c_size_t, PU8, C.c_size_t]),
        "orc_raft_append_entries": (C.c_int, [P, PE, C.c_size_t, PU8]),
        "orc_raft_has_committed_entry_at_current_term": (C.c_int, [P]),
        "orc_raft_broadcast_heartbeat_hint": (C.c_int, [P, U64, U64]),
        "orc_raft_read_index_len": (C.c_size_t, [P]),
        "orc_inmem_new": (P, [U64, PE, C.c_size_t, U64, C.c_int]),
        "orc_inmem_free": (None, [P]),
        "orc_inmem_merge": (C.c_int, [P, PE, C.c_size_t]),
        "orc_inmem_saved_log_to": (C.c_int, [P, U64, U64]),
        "orc_inmem_applied_log_to": (C.c_int, [P, U64]),
        "orc_inmem_restore": (None, [P, U64, U64]),
        "orc_inmem_entries_to_save": (C.c_long, [P, PU64]),
        "orc_inmem_last_index": (C.c_int, [P, PU64]),
        "orc_inmem_get_term": (C.c_int, [P, U64, PU64]),
        "orc_inmem_info": (None, [P, PU64]),
        "orc_get_payload": (C.c_long, [U32, PU8, C.c_size_t, PU8,
                                       C.c_size_t]),
        "orc_batchdb_new": (P, []),
        "orc_batchdb_free": (None, [P]),
        "orc_batchdb_record": (C.c_long, [P, U64, U64, PE, C.c_size_t, PU8]),
        "orc_batchdb_out": (C.c_long, [P, C.c_size_t, PU64, PU8,
                                       C.c_size_t]),
        "orc_batch_id_range": (None, [U64, U64, PU64, PU64]),
        "orc_batch_compact": (C.c_int, [PE, C.c_size_t, C.c_int]),
        "orc_batch_merged_first": (C.c_long, [PE, C.c_size_t, PE, C.c_size_t,
                                              PE]),
        "orc_xxh64": (U64, [PU8, C.c_size_t]),
        "orc_tanw_new": (P, []),
        "orc_tanw_free": (None, [P]),
        "orc_tanw_write_record": (C.c_int64, [P, PU8, C.c_size_t]),
        "orc_tanw_flush": (C.c_int, [P, C.c_int]),
        "orc_tanw_size": (C.c_int64, [P]),
        "orc_tanw_last_record_offset": (C.c_int64, [P]),
        "orc_tanw_bytes": (C.c_long, [P, PU8, C.c_size_t]),
        "orc_tan_read": (C.c_long, [PU8, C.c_size_t, C.POINTER(C.c_int64),
                                    C.POINTER(C.c_size_t), C.c_size_t, PU8,
                                    C.c_size_t]),
        "orc_update_size_bound": (C.c_size_t, [PE, C.c_size_t]),
        "orc_update_marshal": (C.c_size_t, [U64, U64, U64, U64, U64, PE,
                                            C.c_size_t, PU8, PU8]),
        "orc_tandb_new": (P, [C.c_int64]),
        "orc_tandb_free": (None, [P]),
        "orc_tandb_write": (C.c_int, [P, U64, U64, U64, U64, U64, PE,
                                      C.c_size_t, PU8, C.POINTER(C.c_int)]),
        "orc_tandb_last": (None, [P, C.POINTER(C.c_int64)]),
        "orc_tandb_file": (C.c_long, [P, C.c_size_t, PU8, C.c_size_t]),
        "orc_cluster_tan_write": (C.c_int, [P, U64, U32, P,
                                            C.POINTER(C.c_int)]),
        "orc_sm_new": (P, [U64, U64]),
        "orc_sm_free": (None, [P]),
        "orc_sm_handle": (C.c_long, [P, PE, C.c_size_t, PU8]),
        "orc_sm_last_applied": (U64, [P]),
        "orc_sm_count": (U64, [P]),
        "orc_sm_lookup": (C.c_int, [P, PU8, U32, PU8, U32, PU32]),
        "orc_cluster_new": (P, [C.POINTER(ClusterCfg)]),
        "orc_cluster_free": (None, [P]),
        "orc_cluster_setup_steady": (C.c_int, [P, U32]),
        "orc_cluster_stage_proposals": (C.c_int, [P, PU32, U32, PE, PU8]),
        "orc_cluster_set_member_kinds": (C.c_int, [P, U32, U32]),
        "orc_cluster_stage_proposals_at": (C.c_int, [P, PU32, U32, PE, PU8,
                                                     U32]),
        "orc_cluster_stage_read_index": (C.c_int, [P, PU64, PU64]),
        "orc_cluster_stage_read_index_at": (C.c_int, [P, PU64, PU64, U32]),
        "orc_cluster_request_leader_transfer": (C.c_int64, [P, U32, PU32]),
        "orc_cluster_ingest": (C.c_int, [P, PM, C.c_size_t, PE, PU8]),
        "orc_cluster_round": (C.c_int, [P, C.c_int, C.POINTER(RoundOut)]),
        "orc_cluster_round_range": (C.c_int, [P, C.c_int, U64, U64,
                                              C.POINTER(RoundOut)]),
        "orc_cluster_end_round": (C.c_int, [P]),
        "orc_cluster_export": (C.c_int, [P, U64, U32,
                                         C.POINTER(ReplicaState)]),
        "orc_cluster_import": (C.c_int, [P, U64, U32,
                                         C.POINTER(ReplicaState), PE,
                                         C.c_size_t, PU8]),
        "orc_cluster_export_log": (C.c_long, [P, U64, U32, U64, U64, PE, PU8,
                                              C.c_size_t]),
        "orc_cluster_export_outbox": (C.c_long, [P, U64, U32, PM, C.c_size_t,
                                                 PE, C.c_size_t, PU8,
                                                 C.c_size_t]),
        "orc_cluster_export_kv": (C.c_long, [P, U64, U32, PU8, PU32, PU8, PU32,
                                             C.c_size_t, C.c_size_t,
                                             C.c_size_t]),
        "orc_cluster_export_ready": (C.c_long, [P, U64, U32,
                                                C.POINTER(ReadyToRead),
                                                C.c_size_t]),
        "orc_cluster_set_hosted": (C.c_int, [P, U64, U32, C.c_int]),
        "orc_cluster_set_pre_vote": (None, [P, C.c_int]),
        "orc_cluster_export_saved": (C.c_long, [P, U64, U32, PU8,
                                                C.c_size_t, PU32]),
        "orc_cluster_kv_lookup": (C.c_int, [P, U64, U32, PU8, U32, PU8, U32,
                                            PU32]),
        "orc_cluster_serve_reads": (C.c_int, [P, U32, U32, U64, U64,
                                              C.POINTER(C.c_uint64),
                                              C.POINTER(C.c_uint64),
                                              C.POINTER(C.c_uint64)]),
        "orc_entry_size": (C.c_size_t, [PE]),
        "orc_entry_marshal": (C.c_size_t, [PE, PU8, PU8]),
        "orc_entry_unmarshal": (C.c_long, [PU8, C.c_size_t, PE, PU8,
                                           C.c_size_t, C.POINTER(C.c_size_t)]),
        "orc_entrybatch_size": (C.c_size_t, [PE, C.c_size_t]),
        "orc_entrybatch_marshal": (C.c_size_t, [PE, C.c_size_t, PU8, PU8]),
        "orc_entrybatch_unmarshal": (C.c_long, [PU8, C.c_size_t, PE,
                                                C.c_size_t, PU8, C.c_size_t]),
        "orc_crc32_ieee": (C.c_uint32, [PU8, C.c_size_t]),
        "orc_pbkv_marshal": (C.c_size_t, [PU8, U32, PU8, U32, PU8]),
        "orc_message_size": (C.c_size_t, [PM, PE]),
        "orc_message_marshal": (C.c_size_t, [PM, PE, PU8, PU8]),
        "orc_message_unmarshal": (C.c_long, [PU8, C.c_size_t, PM, PE,
                                             C.c_size_t,
                                             C.POINTER(C.c_size_t), PU8,
                                             C.c_size_t,
                                             C.POINTER(C.c_size_t)]),
        "orc_messagebatch_marshal": (C.c_size_t, [PM, C.c_size_t, PE, PU8,
                                                  U64, C.c_char_p,
                                                  C.c_size_t, U32, PU8]),
        "orc_messagebatch_unmarshal": (C.c_long, [PU8, C.c_size_t, PM,
                                                  C.c_size_t, PE, C.c_size_t,
                                                  PU8, C.c_size_t,
                                                  C.POINTER(U64), PU32,
                                                  C.c_char_p, C.c_size_t,
                                                  C.POINTER(C.c_size_t)]),
        "orc_request_header_encode": (None, [C.c_uint16, U64, U32, PU8]),
        "orc_request_header_decode": (C.c_int, [PU8,
                                                C.POINTER(C.c_uint16),
                                                C.POINTER(U64), PU32]),
        "orc_wire_frame": (C.c_size_t, [PU8, C.c_size_t, PU8]),
        "orc_pbkv_unmarshal": (C.c_int, [PU8, C.c_size_t,
                                         C.POINTER(PU8), PU32,
                                         C.POINTER(PU8), PU32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


class OracleError(RuntimeError):
    """The reference would have panicked (plog.Panicf / panic)."""


def _check(rc):
    if rc == -1:
        raise OracleError(lib().orc_last_error().decode())
    return rc


def _u8(buf):
    return (C.c_uint8 * max(1, len(buf))).from_buffer_copy(buf or b"\0")


# ---------------------------------------------------------------- entries
class EntryPool:
    """Builds drb_entry arrays + a Cmd byte pool from python tuples/dicts."""

    def __init__(self, entries=()):
        self.items = []
        self.pool = bytearray()
        for e in entries:
            self.add(**e) if isinstance(e, dict) else self.add(*e)

    def add(self, term=0, index=0, type=0, key=0, client_id=0, series_id=0,
            responded_to=0, cmd=b""):
        self.items.append(Entry(term, index, key, client_id, series_id,
                                responded_to, type, len(cmd), len(self.pool)))
        self.pool += bytes(cmd)

    def arrays(self):
        n = len(self.items)
        arr = (Entry * max(1, n))(*self.items)
        return arr, _u8(bytes(self.pool)), n


def ent(term=0, index=0, type=0, key=0, client_id=0, series_id=0,
        responded_to=0, cmd=b""):
    return dict(term=term, index=index, type=type, key=key,
                client_id=client_id, series_id=series_id,
                responded_to=responded_to, cmd=cmd)


def msg(type, from_=0, to=0, term=0, log_term=0, log_index=0, commit=0,
        reject=False, hint=0, hint_high=0, entries=(), shard_id=0):
    return dict(type=type, from_=from_, to=to, term=term, log_term=log_term,
                log_index=log_index, commit=commit, reject=int(bool(reject)),
                hint=hint, hint_high=hint_high, entries=list(entries),
                shard_id=shard_id)


def build_messages(msgs):
    ep = EntryPool()
    out = []
    for m in msgs:
        off = len(ep.items)
        for e in m["entries"]:
            ep.add(**e)
        out.append(Message(m["shard_id"], m["from_"], m["to"], m["term"],
                           m["log_term"], m["log_index"], m["commit"],
                           m["hint"], m["hint_high"], m["type"], m["reject"],
                           len(m["entries"]), off))
    marr = (Message * max(1, len(out)))(*out)
    earr, pool, _ = ep.arrays()
    return marr, len(out), earr, pool


def msg_tuple(m):
    """The canonical tuple (abi.message_to_tuple) of a msg() dict."""
    marr, n, earr, pool = build_messages([m])
    return message_to_tuple(marr[0], earr, pool)


def _unpack_messages(marr, n, earr, pool):
    res = []
    for i in range(n):
        m = marr[i]
        t = message_to_tuple(m, earr, pool)
        res.append(dict(shard_id=t[0], from_=t[1], to=t[2], type=t[3],
                        term=t[4], log_term=t[5], log_index=t[6], commit=t[7],
                        reject=bool(t[8]), hint=t[9], hint_high=t[10],
                        entries=[_etuple_to_dict(x) for x in t[11]]))
    return res


def _etuple_to_dict(t):
    return dict(term=t[0], index=t[1], type=t[2], key=t[3], client_id=t[4],
                series_id=t[5], responded_to=t[6], cmd=t[7])


# ---------------------------------------------------------------- remote
def new_remote(match=0, next=0, state=0, snapshot_index=0, active=0):
    return Remote(match, next, snapshot_index, state, active)


# ---------------------------------------------------------------- readIndex
class ReadIndexQ:
    def __init__(self):
        self.p = lib().orc_readindex_new()

    def __del__(self):
        if getattr(self, "p", None):
            lib().orc_readindex_free(self.p)

    def add_request(self, index, ctx, from_):
        _check(lib().orc_readindex_add_request(self.p, index, ctx[0], ctx[1],
                                               from_))

    def __len__(self):
        return lib().orc_readindex_len(self.p)

    def items(self):
        out = []
        for i in range(len(self)):
            a, b, c, d = U64(), U64(), U64(), U64()
            lib().orc_readindex_get(self.p, i, a, b, c, d)
            out.append(((a.value, b.value), c.value, d.value))
        return out

    def confirm(self, ctx, from_, quorum):
        cap = 64
        lo, hi, ix, fr = [(U64 * cap)() for _ in range(4)]
        n = _check(lib().orc_readindex_confirm(self.p, ctx[0], ctx[1], from_,
                                               quorum, lo, hi, ix, fr, cap))
        return [((lo[i], hi[i]), ix[i], fr[i]) for i in range(n)]

    def push_raw(self, ctx, front=False):
        lib().orc_readindex_push_raw_queue(self.p, ctx[0], ctx[1], int(front))


def sort_match_values(vals):
    arr = (U64 * len(vals))(*vals)
    lib().orc_sort_match_values(arr, len(vals))
    return list(arr)


# ---------------------------------------------------------------- raft
class LogDB:
    """TestLogDB (internal/raft/logdb_test.go:24-170)."""

    def __init__(self, entries=()):
        self.p = lib().orc_logdb_new()
        if entries:
            self.append(entries)

    def append(self, entries):
        arr, pool, n = EntryPool(entries).arrays()
        _check(lib().orc_logdb_append(self.p, arr, n, pool))

    def compact(self, index):
        return lib().orc_logdb_compact(self.p, index)

    def set_state(self, term=0, vote=0, commit=0):
        lib().orc_logdb_set_state(self.p, term, vote, commit)

    def __del__(self):
        if getattr(self, "p", None):
            lib().orc_logdb_free(self.p)


class TestRaft:
    """newTestRaft (internal/raft/raft_etcd_test.go:3071)."""

    __test__ = False  # not a pytest class

    def __init__(self, id, peers, election, heartbeat, logdb=None):
        self.logdb = logdb or LogDB()
        ps = (U64 * max(1, len(peers)))(*peers)
        self.p = lib().orc_raft_new_test(id, ps, len(peers), election,
                                         heartbeat, self.logdb.p)
        if not self.p:
            raise OracleError(lib().orc_last_error().decode())
        self.id = id

    def __del__(self):
        if getattr(self, "p", None):
            lib().orc_raft_free(self.p)

    def handle(self, m):
        marr, n, earr, pool = build_messages([m])
        _check(lib().orc_raft_handle(self.p, marr, earr, pool))

    def peer_handle(self, m):
        marr, n, earr, pool = build_messages([m])
        _check(lib().orc_raft_peer_handle(self.p, marr, earr, pool))

    def become_follower(self, term, leader):
        _check(lib().orc_raft_become_follower(self.p, term, leader))

    def become_candidate(self):
        _check(lib().orc_raft_become_candidate(self.p))

    def become_leader(self):
        _check(lib().orc_raft_become_leader(self.p))

    def load_state(self, term=0, vote=0, commit=0):
        _check(lib().orc_raft_load_state(self.p, term, vote, commit))

    def broadcast_replicate(self):
        _check(lib().orc_raft_broadcast_replicate(self.p))

    def broadcast_heartbeat(self):
        _check(lib().orc_raft_broadcast_heartbeat(self.p))

    def try_commit(self):
        return bool(_check(lib().orc_raft_try_commit(self.p)))

    def tick(self):
        _check(lib().orc_raft_tick(self.p))

    def campaign(self):
        _check(lib().orc_raft_campaign(self.p))

    def set_check_quorum(self, on):
        lib().orc_raft_set_check_quorum(self.p, int(bool(on)))

    def set_pre_vote(self, on):
        lib().orc_raft_set_pre_vote(self.p, int(bool(on)))

    def set_randomized_election_timeout(self, v):
        lib().orc_raft_set_randomized_election_timeout(self.p, v)

    # fields the reference's tests assign directly (orc_raft_poke)
    POKE = dict(state=0, term=1, vote=2, election_tick=3,
                election_timeout=4, committed=5, applied=6,
                config_change_hook=7, leader_transfer_target=8,
                is_leader_transfer_target=9)

    def poke(self, **kw):
        for k, v in kw.items():
            if lib().orc_raft_poke(self.p, self.POKE[k], int(v)):
                raise KeyError(k)

    def peek(self, field):
        return lib().orc_raft_peek(self.p, self.POKE[field])

    def reset(self, term):
        """reset(term, true) (raft.go:1052-1073)."""
        _check(lib().orc_raft_reset(self.p, term))

    def become_pre_vote_candidate(self):
        _check(lib().orc_raft_become_pre_vote_candidate(self.p))

    def draw_timeout_time_for_election(self):
        """setRandomizedElectionTimeout(); timeForElection()."""
        return bool(lib().orc_raft_draw_timeout_time_for_election(self.p))

    def term_not_matched(self, m):
        """onMessageTermNotMatched (raft.go:1540-1590): True = dropped."""
        marr, n, earr, pool = build_messages([m])
        return bool(_check(lib().orc_raft_term_not_matched(self.p, marr, earr,
                                                           pool)))

    # member kinds (oracle.h ORC_VOTING / ORC_NONVOTING / ORC_WITNESS)
    VOTING, NONVOTING, WITNESS = 0, 1, 2

    @classmethod
    def with_kind(cls, id, peers, others, kind, election, heartbeat,
                  logdb=None):
        """newTestNonVoting / newTestWitness (raft_etcd_test.go:3099-3140):
        others are the nonVotings (kind NONVOTING) or witnesses (WITNESS),
        this replica among them."""
        self = cls.__new__(cls)
        self.logdb = logdb or LogDB()
        ps = (U64 * max(1, len(peers)))(*peers)
        os_ = (U64 * max(1, len(others)))(*others)
        self.p = lib().orc_raft_new_test_kind(id, ps, len(peers), os_,
                                              len(others), kind, election,
                                              heartbeat, self.logdb.p)
        if not self.p:
            raise OracleError(lib().orc_last_error().decode())
        self.id = id
        return self

    def add_node(self, id):
        _check(lib().orc_raft_add_member(self.p, id, self.VOTING))

    def add_nonvoting(self, id):
        _check(lib().orc_raft_add_member(self.p, id, self.NONVOTING))

    def add_witness(self, id):
        _check(lib().orc_raft_add_member(self.p, id, self.WITNESS))

    def remote_kind(self, id):
        return lib().orc_raft_remote_kind(self.p, id)

    def network_reset(self, id, ids):
        arr = (U64 * len(ids))(*ids)
        _check(lib().orc_raft_network_reset(self.p, id, arr, len(ids)))
        self.id = id

    def read_messages(self):
        cap, ecap, pcap = 256, 4096, 1 << 20
        marr = (Message * cap)()
        earr = (Entry * ecap)()
        pool = (C.c_uint8 * pcap)()
        n = lib().orc_raft_read_messages(self.p, marr, cap, earr, ecap, pool,
                                         pcap)
        if n < 0 or n > cap:
            raise OracleError("read_messages failed %d" % n)
        return _unpack_messages(marr, n, earr, pool)

    def _entries(self, which):
        cap, pcap = 4096, 1 << 20
        arr = (Entry * cap)()
        pool = (C.c_uint8 * pcap)()
        n = lib().orc_raft_log_entries(self.p, which, arr, cap, pool, pcap)
        if n == -1:
            raise OracleError(lib().orc_last_error().decode())
        if n < 0:
            raise OracleError("log entries failed %d" % n)
        return [_etuple_to_dict(entry_to_tuple(arr[i], pool))
                for i in range(n)]

    def entries_to_apply(self):
        return self._entries(0)

    def entries_to_save(self):
        return self._entries(1)

    def all_entries(self):
        return self._entries(2)

    def term(self, index):
        t = U64()
        rc = _check(lib().orc_raft_log_term(self.p, index, t))
        return rc, t.value

    def info(self):
        st = ReplicaState()
        lib().orc_raft_info(self.p, st)
        return st

    def remote(self, id):
        r = Remote()
        if lib().orc_raft_remote(self.p, id, r):
            raise KeyError(id)
        return r

    def set_remote(self, id, r):
        lib().orc_raft_set_remote(self.p, id, r)

    def ready_to_read(self):
        cap = 64
        a, b, c = (U64 * cap)(), (U64 * cap)(), (U64 * cap)()
        n = lib().orc_raft_ready_to_read(self.p, a, b, c, cap)
        return [(a[i], (b[i], c[i])) for i in range(min(n, cap))]

    def dropped_read_indexes(self):
        return lib().orc_raft_dropped_read_indexes(self.p)

    # entryLog hooks
    def commit_to(self, index):
        _check(lib().orc_log_commit_to(self.p, index))

    def log_try_commit(self, index, term):
        return bool(_check(lib().orc_log_try_commit(self.p, index, term)))

    def match_term(self, index, term):
        return bool(_check(lib().orc_log_match_term(self.p, index, term)))

    def up_to_date(self, index, term):
        return bool(_check(lib().orc_log_up_to_date(self.p, index, term)))

    def conflict_index(self, entries):
        arr, pool, n = EntryPool(entries).arrays()
        return _check(lib().orc_log_conflict_index(self.p, arr, n))

    def try_append(self, index, entries):
        arr, pool, n = EntryPool(entries).arrays()
        return bool(_check(lib().orc_log_try_append(self.p, index, arr, n,
                                                    pool)))

    def append(self, entries):
        arr, pool, n = EntryPool(entries).arrays()
        _check(lib().orc_log_append(self.p, arr, n, pool))

    def commit_update(self, stable_log_to=0, stable_log_term=0, processed=0,
                      last_applied=0):
        _check(lib().orc_log_commit_update(self.p, stable_log_to,
                                           stable_log_term, processed,
                                           last_applied))

    # raft KAT hooks (raft_test.go:1578-1611, 2952-3037)
    def make_replicate(self, to, next, max_size):
        """makeReplicateMessage(to, next, maxSize) (raft.go:738-769)."""
        marr, earr = (Message * 1)(), (Entry * 4096)()
        pool = (C.c_uint8 * (1 << 20))()
        n = _check(lib().orc_raft_make_replicate(self.p, to, next, max_size,
                                                 marr, earr, 4096, pool,
                                                 1 << 20))
        if n < 0:
            raise OracleError("makeReplicateMessage failed %d" % n)
        return _unpack_messages(marr, 1, earr, pool)[0]

    def append_entries(self, entries):
        """raft.appendEntries (raft.go:944-955)."""
        arr, pool, n = EntryPool(entries).arrays()
        _check(lib().orc_raft_append_entries(self.p, arr, n, pool))

    def broadcast_heartbeat_hint(self, ctx):
        _check(lib().orc_raft_broadcast_heartbeat_hint(self.p, ctx[0], ctx[1]))

    def has_committed_entry_at_current_term(self):
        return bool(_check(
            lib().orc_raft_has_committed_entry_at_current_term(self.p)))

    def read_index_len(self):
        return lib().orc_raft_read_index_len(self.p)

    @property
    def committed(self):
        return self.info().committed

    @property
    def last_index(self):
        return self.info().last_index


class BlackHole:
    """blackHole / nopStepper (raft_etcd_test.go:3036-3041)."""

    def handle(self, m):
        pass

    def read_messages(self):
        return []


class Network:
    """network (raft_etcd_test.go:2896-3030): synchronous delivery, with the
    drop / cut / isolate / ignore / recover filters (:2980-3026; drop rates
    are 0 or 1 in every test restated here, so the filter is exact)."""

    def __init__(self, *peers, pre_vote=False, check_quorum=False):
        ids = list(range(1, len(peers) + 1))
        self.peers = {}
        for i, p in zip(ids, peers):
            if p is None:
                p = TestRaft(i, ids, 10, 1)
                if pre_vote:
                    p.set_pre_vote(True)
                if check_quorum:
                    p.set_check_quorum(True)
            elif isinstance(p, TestRaft):
                p.network_reset(i, ids)
            self.peers[i] = p
        self.dropm = {}
        self.ignorem = set()

    def send(self, *msgs):
        q = list(msgs)
        while q:
            m = q.pop(0)
            p = self.peers[m["to"]]
            p.handle(m)
            q.extend(self.filter(p.read_messages()))

    def drop(self, frm, to, perc):
        self.dropm[(frm, to)] = perc

    def cut(self, one, other):
        self.drop(one, other, 1.0)
        self.drop(other, one, 1.0)

    def isolate(self, id):
        for nid in self.peers:
            if nid != id:
                self.drop(id, nid, 1.0)
                self.drop(nid, id, 1.0)

    def ignore(self, t):
        self.ignorem.add(t)

    def recover(self):
        self.dropm = {}
        self.ignorem = set()

    def filter(self, msgs):
        out = []
        for m in msgs:
            if m["type"] in self.ignorem:
                continue
            if m["type"] == MSG_ELECTION:
                raise OracleError("unexpected msgHup")
            if self.dropm.get((m["from_"], m["to"]), 0.0) >= 1.0:
                continue
            out.append(m)
        return out


MSG_ELECTION = 1


def ents_with_config(*terms, pre_vote=False):
    """entsWithConfig (raft_etcd_test.go:2865-2878): a raft (election 5)
    whose LogDB holds one entry per term given, reset to the last term."""
    db = LogDB([ent(term=t, index=i + 1) for i, t in enumerate(terms)])
    r = TestRaft(1, [], 5, 1, db)
    r.poke(config_change_hook=0)  # newRaft, not newTestRaft
    if pre_vote:
        r.set_pre_vote(True)
    r.reset(terms[-1])
    return r


def voted_with_config(vote, term, pre_vote=False):
    """votedWithConfig (raft_etcd_test.go:2880-2893): Vote and Term set in
    the LogDB's state, no entries."""
    db = LogDB()
    db.set_state(term=term, vote=vote)
    r = TestRaft(1, [], 5, 1, db)
    r.poke(config_change_hook=0)  # newRaft, not newTestRaft
    if pre_vote:
        r.set_pre_vote(True)
    r.reset(term)
    return r


# ---------------------------------------------------------------- cluster
class Cluster:
    """The node_test.go step() loop over G groups x R replicas."""

    def __init__(self, num_groups, num_replicas=3, election_rtt=10,
                 heartbeat_rtt=1, check_quorum=1, seed=0x5EEDD8B0,
                 first_shard_id=1, logdb_keep=0, quiesce=0, gids=None,
                 pre_vote=0):
        """gids: simulate only these global group ids (group i of the
        cluster is global group gids[i]; None: 0..num_groups-1)."""
        self.gids = None if gids is None else \
            (C.c_uint64 * len(gids))(*gids)
        if gids is not None:
            num_groups = len(gids)
        cfg = ClusterCfg(num_groups, first_shard_id, num_replicas,
                         election_rtt, heartbeat_rtt, check_quorum, seed,
                         logdb_keep, int(bool(quiesce)), int(bool(pre_vote)),
                         self.gids)
        self.cfg = cfg
        self.G = num_groups
        self.R = num_replicas
        self.p = lib().orc_cluster_new(cfg)
        if not self.p:
            raise OracleError(lib().orc_last_error().decode())

    def __del__(self):
        if getattr(self, "p", None):
            lib().orc_cluster_free(self.p)

    def setup_steady(self, leader_slot=0):
        _check(lib().orc_cluster_setup_steady(self.p, leader_slot))

    def set_member_kinds(self, nonvoting_mask=0, witness_mask=0):
        """Replica slots that are nonVotings / witnesses in every group."""
        _check(lib().orc_cluster_set_member_kinds(self.p, nonvoting_mask,
                                                  witness_mask))

    def stage_proposals(self, counts, max_per_group, ents, pool, replica=0):
        """counts: uint32[G] array; ents: Entry[G*max] array; pool: uint8.
        At each group's leader, or at replica ID `replica` (a follower
        forwards them to its leader, raft.go:2103-2116)."""
        _check(lib().orc_cluster_stage_proposals_at(self.p, counts,
                                                    max_per_group, ents, pool,
                                                    replica))

    def stage_read_index(self, low, high, replica=0):
        """One ReadIndex ctx per group at its leader, or at replica ID
        `replica` (which forwards it when it is a follower)."""
        _check(lib().orc_cluster_stage_read_index_at(self.p, low, high,
                                                     replica))

    def request_leader_transfer(self, slot, targets):
        """NodeHost.RequestLeaderTransfer at replica slot `slot` of every
        group g with targets[g] (a replica ID) != 0, taken by that node's
        next round (node.handleLeaderTransfer, node.go:1249).  Returns the
        number refused as busy (a request still pending)."""
        arr = (C.c_uint32 * self.G)(*targets)
        n = lib().orc_cluster_request_leader_transfer(self.p, slot, arr)
        if n < 0:
            raise OracleError("request_leader_transfer: bad slot")
        return n

    def ingest(self, msgs):
        marr, n, earr, pool = build_messages(msgs)
        _check(lib().orc_cluster_ingest(self.p, marr, n, earr, pool))

    def round(self, tick=False):
        out = RoundOut()
        _check(lib().orc_cluster_round(self.p, int(bool(tick)), out))
        return out

    def export(self, g, slot):
        st = ReplicaState()
        if lib().orc_cluster_export(self.p, g, slot, st):
            raise IndexError((g, slot))
        return st

    def import_replica(self, g, slot, st, entries):
        """Replica (g, slot) takes state `st` (a ReplicaState) and the log
        `entries` (entry dicts, indices from 1 up to st.last_index);
        drb_import_replicas + drb_import_log on the engine side."""
        arr, pool, n = EntryPool(entries).arrays()
        for i in range(n):
            arr[i].index = i + 1
        _check(lib().orc_cluster_import(self.p, g, slot, C.byref(st), arr, n,
                                        pool))

    def export_log(self, g, slot, lo, hi):
        cap = hi - lo + 1
        if cap <= 0:
            return []
        arr = (Entry * cap)()
        pcap = 1 << 20
        pool = (C.c_uint8 * pcap)()
        n = lib().orc_cluster_export_log(self.p, g, slot, lo, hi, arr, pool,
                                         pcap)
        if n < 0:
            raise OracleError("export_log %d" % n)
        return [entry_to_tuple(arr[i], pool) for i in range(n)]

    def export_outbox(self, g, slot):
        cap, ecap, pcap = 256, 8192, 1 << 20
        marr = (Message * cap)()
        earr = (Entry * ecap)()
        pool = (C.c_uint8 * pcap)()
        n = lib().orc_cluster_export_outbox(self.p, g, slot, marr, cap, earr,
                                            ecap, pool, pcap)
        if n < 0 or n > cap:
            raise OracleError("export_outbox %d" % n)
        return [message_to_tuple(marr[i], earr, pool) for i in range(n)]

    def export_kv(self, g, slot, key_cap=64, val_cap=2048, cap=4096):
        keys = (C.c_uint8 * (cap * key_cap))()
        vals = (C.c_uint8 * (cap * val_cap))()
        kl, vl = (U32 * cap)(), (U32 * cap)()
        n = lib().orc_cluster_export_kv(self.p, g, slot, keys, kl, vals, vl,
                                        cap, key_cap, val_cap)
        if n < 0 or n > cap:
            raise OracleError("export_kv %d" % n)
        kb, vb = bytes(keys), bytes(vals)
        return {kb[i * key_cap:i * key_cap + kl[i]]:
                vb[i * val_cap:i * val_cap + vl[i]] for i in range(n)}

    def export_ready(self, g, slot):
        cap = 64
        arr = (ReadyToRead * cap)()
        n = lib().orc_cluster_export_ready(self.p, g, slot, arr, cap)
        return [(arr[i].index, arr[i].ctx_low, arr[i].ctx_high)
                for i in range(min(n, cap))]

    def export_saved(self, g, slot, cap=1 << 16):
        """(EntryBatch bytes, crc32) of one replica's last EntriesToSave."""
        buf = (C.c_uint8 * cap)()
        crc = C.c_uint32()
        n = lib().orc_cluster_export_saved(self.p, g, slot, buf, cap,
                                           C.byref(crc))
        if n < 0:
            raise RuntimeError("export_saved: buffer too small")
        return bytes(buf[:n]), crc.value

    def tan_write(self, g, slot, db):
        """SaveRaftState of replica (g, slot)'s last pb.Update into a
        TanDB: None when there was nothing to write, else the write's
        TanDB.last() record."""
        sync = C.c_int()
        rc = _check(lib().orc_cluster_tan_write(self.p, g, slot, db.p,
                                                C.byref(sync)))
        return db.last() if rc == 1 else None

    def serve_reads(self, reads_per_ctx=9, key_space=256):
        """Returns (sums[G*R] -- None where nothing was served, served,
        deferred)."""
        n = self.G * self.R
        marker = (1 << 64) - 1
        sums = (C.c_uint64 * n)(*([marker] * n))
        sv, df = C.c_uint64(), C.c_uint64()
        _check(lib().orc_cluster_serve_reads(self.p, reads_per_ctx, key_space,
                                             0, self.G, sums, C.byref(sv),
                                             C.byref(df)))
        return ([None if x == marker else x for x in sums], sv.value,
                df.value)

    def set_hosted(self, g, slot, hosted):
        lib().orc_cluster_set_hosted(self.p, g, slot, int(bool(hosted)))

    def set_pre_vote(self, on):
        lib().orc_cluster_set_pre_vote(self.p, int(bool(on)))


# ---------------------------------------------------------------- codecs
def entry_size(e):
    arr, pool, _ = EntryPool([e]).arrays()
    return lib().orc_entry_size(arr)


def entry_marshal(e):
    arr, pool, _ = EntryPool([e]).arrays()
    buf = (C.c_uint8 * (lib().orc_entry_size(arr) + 16))()
    n = lib().orc_entry_marshal(arr, pool, buf)
    return bytes(buf[:n])


def entry_unmarshal(data):
    e = Entry()
    pool = (C.c_uint8 * max(1, len(data)))()
    used = C.c_size_t(0)
    n = lib().orc_entry_unmarshal(_u8(data), len(data), e, pool, len(data),
                                  C.byref(used))
    if n < 0:
        raise ValueError("entry unmarshal failed")
    return _etuple_to_dict(entry_to_tuple(e, pool)), n


def entrybatch_marshal(entries):
    arr, pool, n = EntryPool(entries).arrays()
    size = lib().orc_entrybatch_size(arr, n)
    buf = (C.c_uint8 * max(1, size))()
    w = lib().orc_entrybatch_marshal(arr, n, pool, buf)
    assert w == size
    return bytes(buf[:w])


def entrybatch_unmarshal(data, cap=4096):
    arr = (Entry * cap)()
    pool = (C.c_uint8 * max(1, len(data)))()
    n = lib().orc_entrybatch_unmarshal(_u8(data), len(data), arr, cap, pool,
                                       len(data))
    if n < 0:
        raise ValueError("entrybatch unmarshal failed")
    return [_etuple_to_dict(entry_to_tuple(arr[i], pool)) for i in range(n)]


def crc32_ieee(data):
    return lib().orc_crc32_ieee(_u8(data), len(data))


def pbkv_marshal(key, val):
    buf = (C.c_uint8 * (len(key) + len(val) + 24))()
    n = lib().orc_pbkv_marshal(_u8(key), len(key), _u8(val), len(val), buf)
    return bytes(buf[:n])


def pbkv_unmarshal(data):
    kp, vp = PU8(), PU8()
    kl, vl = U32(), U32()
    src = _u8(data)
    rc = lib().orc_pbkv_unmarshal(src, len(data), C.byref(kp), kl,
                                  C.byref(vp), vl)
    if rc:
        raise ValueError("pbkv unmarshal failed")
    return bytes(kp[:kl.value]), bytes(vp[:vl.value])


# pb.Message / pb.MessageBatch (raftpb/message.go, messagebatch.go,
# raft_optimized.go:659-1207) and the TCP frame (internal/transport/tcp.go)
TRANSPORT_BIN_VERSION = 210  # raftio/binversion.go:30


def _msg_cmd_bytes(msgs):
    return sum(len(e["cmd"]) for m in msgs for e in m["entries"])


def message_marshal(m):
    marr, n, earr, pool = build_messages([m])
    size = lib().orc_message_size(marr, earr)
    buf = (C.c_uint8 * max(1, size))()
    w = lib().orc_message_marshal(marr, earr, pool, buf)
    assert w == size
    return bytes(buf[:w])


def messagebatch_marshal(msgs, deployment_id=0, source=b"",
                         bin_ver=TRANSPORT_BIN_VERSION):
    marr, n, earr, pool = build_messages(msgs)
    cap = 64 + len(source) + sum(
        32 + 12 * 11 + 26 + sum(64 + len(e["cmd"]) for e in m["entries"])
        for m in msgs)
    buf = (C.c_uint8 * cap)()
    w = lib().orc_messagebatch_marshal(marr, n, earr, pool, deployment_id,
                                       source, len(source), bin_ver, buf)
    assert w <= cap
    return bytes(buf[:w])


def messagebatch_unmarshal(data, cap=4096):
    """-> (messages, deployment_id, source, bin_ver); ValueError when
    malformed, NotImplementedError for a non-empty Snapshot."""
    marr = (Message * cap)()
    earr = (Entry * cap)()
    pool = (C.c_uint8 * max(1, len(data)))()
    did, bv, sl = U64(), U32(), C.c_size_t()
    src = C.create_string_buffer(max(1, len(data)))
    n = lib().orc_messagebatch_unmarshal(_u8(data), len(data), marr, cap,
                                         earr, cap, pool, len(data),
                                         C.byref(did), bv, src, len(data),
                                         C.byref(sl))
    if n == -2:
        raise NotImplementedError("non-empty snapshot")
    if n < 0:
        raise ValueError("messagebatch unmarshal failed")
    return (_unpack_messages(marr, n, earr, pool), did.value,
            src.raw[:sl.value], bv.value)


def request_header_encode(method, size, crc):
    b = (C.c_uint8 * 18)()
    lib().orc_request_header_encode(method, size, crc, b)
    return bytes(b)


def request_header_decode(b):
    me, sz, crc = C.c_uint16(), U64(), U32()
    if lib().orc_request_header_decode(_u8(b), C.byref(me), C.byref(sz),
                                       crc):
        return None
    return me.value, sz.value, crc.value


def wire_frame(payload):
    out = (C.c_uint8 * (len(payload) + 20))()
    n = lib().orc_wire_frame(_u8(payload), len(payload), out)
    return bytes(out[:n])


# ---------------------------------------------------------------- inMemory
class InMem:
    """inMemory (internal/raft/inmemory.go) built the way the reference's
    tests build it: markerIndex, entries, savedTo, shrunk."""

    def __init__(self, marker_index, entries=(), saved_to=0, shrunk=False):
        arr, _, n = EntryPool(entries).arrays()
        self.p = lib().orc_inmem_new(marker_index, arr, n, saved_to,
                                     int(shrunk))

    def __del__(self):
        if getattr(self, "p", None):
            lib().orc_inmem_free(self.p)

    def merge(self, entries):
        arr, _, n = EntryPool(entries).arrays()
        _check(lib().orc_inmem_merge(self.p, arr, n))

    def saved_log_to(self, index, term):
        _check(lib().orc_inmem_saved_log_to(self.p, index, term))

    def applied_log_to(self, index):
        _check(lib().orc_inmem_applied_log_to(self.p, index))

    def restore(self, index, term):
        lib().orc_inmem_restore(self.p, index, term)

    def entries_to_save(self):
        """(count, first index)"""
        f = U64()
        n = lib().orc_inmem_entries_to_save(self.p, f)
        return n, f.value

    def last_index(self):
        v = U64()
        ok = lib().orc_inmem_last_index(self.p, v)
        return v.value, bool(ok)

    def term(self, index):
        v = U64()
        ok = _check(lib().orc_inmem_get_term(self.p, index, v))
        return v.value, bool(ok)

    def info(self):
        o = (U64 * 5)()
        lib().orc_inmem_info(self.p, o)
        return dict(marker_index=o[0], saved_to=o[1], shrunk=bool(o[2]),
                    n=o[3], first=o[4])


# ---------------------------------------------------------------- rsm
def get_payload(type, cmd):
    """GetPayload (internal/rsm/encoded.go:55-66)."""
    out = (C.c_uint8 * (len(cmd) * 64 + 1024))()
    n = _check(lib().orc_get_payload(type, _u8(cmd), len(cmd), out,
                                     len(out)))
    if n < 0:
        raise OracleError("GetPayload failed %d" % n)
    return bytes(out[:n])


class StateMachine:
    """StateMachine over KVTest with sm.lastApplied.index = sm.index =
    applied (internal/rsm/statemachine_test.go:348-349)."""

    def __init__(self, applied_index=0, applied_term=0):
        self.p = lib().orc_sm_new(applied_index, applied_term)

    def __del__(self):
        if getattr(self, "p", None):
            lib().orc_sm_free(self.p)

    def handle(self, entries):
        """taskQ.Add(Task{Entries}) + Handle; returns the number of entries
        that reached the user state machine's Update."""
        arr, pool, n = EntryPool(entries).arrays()
        return _check(lib().orc_sm_handle(self.p, arr, n, pool))

    @property
    def last_applied(self):
        return lib().orc_sm_last_applied(self.p)

    @property
    def count(self):
        return lib().orc_sm_count(self.p)

    def lookup(self, key):
        buf = (C.c_uint8 * 4096)()
        vl = U32()
        rc = lib().orc_sm_lookup(self.p, _u8(key), len(key), buf, 4096, vl)
        return None if rc else bytes(buf[:vl.value])


# ---------------------------------------------------------------- LogDB
class BatchDB:
    """batchedEntries (internal/logdb/batch.go) over an in-memory store."""

    def __init__(self):
        self.p = lib().orc_batchdb_new()

    def __del__(self):
        if getattr(self, "p", None):
            lib().orc_batchdb_free(self.p)

    def record(self, shard, replica, entries):
        """SaveRaftState of one Update: [(batch id, record value)]."""
        arr, pool, n = EntryPool(entries).arrays()
        k = _check(lib().orc_batchdb_record(self.p, shard, replica, arr, n,
                                            pool))
        out = []
        for i in range(k):
            b = U64()
            buf = (C.c_uint8 * (1 << 20))()
            ln = lib().orc_batchdb_out(self.p, i, b, buf, len(buf))
            assert ln >= 0
            out.append((b.value, bytes(buf[:ln])))
        return out


def batch_id_range(low, high):
    a, b = U64(), U64()
    lib().orc_batch_id_range(low, high, a, b)
    return a.value, b.value


def _term_index(entries):
    arr = (Entry * max(1, len(entries)))()
    for i, (t, x) in enumerate(entries):
        arr[i].term, arr[i].index = t, x
    return arr


def batch_compact(entries, restore=False):
    """compactBatchFields / restoreBatchFields on [(term, index)]."""
    arr = _term_index(entries)
    _check(lib().orc_batch_compact(arr, len(entries), int(restore)))
    return [(arr[i].term, arr[i].index) for i in range(len(entries))]


def batch_merged_first(eb, lb):
    """getMergedFirstBatch on [(term, index)] lists."""
    a, b = _term_index(eb), _term_index(lb)
    out = (Entry * max(1, len(eb) + len(lb)))()
    n = _check(lib().orc_batch_merged_first(a, len(eb), b, len(lb), out))
    return [(out[i].term, out[i].index) for i in range(n)]


# ---------------------------------------------------------------- tan
ORC_TAN_ERRORS = {-2: "zeroed chunk", -3: "invalid chunk", -4: "crc mismatch",
                  -5: "unexpected EOF"}


def xxh64(data):
    """xxhash.Sum64 (cespare/xxhash/v2); tan getCRC is its low 32 bits."""
    return lib().orc_xxh64(_u8(data), len(data))


class TanWriter:
    """The tan record writer (internal/tan/record.go:414-653) over an
    in-memory io.Writer."""

    def __init__(self):
        self.p = lib().orc_tanw_new()

    def __del__(self):
        if getattr(self, "p", None):
            lib().orc_tanw_free(self.p)

    def write_record(self, data):
        return _check(lib().orc_tanw_write_record(self.p, _u8(data),
                                                  len(data)))

    def flush(self):
        return _check(lib().orc_tanw_flush(self.p, 0))

    def close(self):
        return _check(lib().orc_tanw_flush(self.p, 1))

    def size(self):
        return lib().orc_tanw_size(self.p)

    def last_record_offset(self):
        return lib().orc_tanw_last_record_offset(self.p)

    def bytes(self):
        n = lib().orc_tanw_bytes(self.p, None, 0)
        buf = (C.c_uint8 * max(1, n))()
        lib().orc_tanw_bytes(self.p, buf, n)
        return bytes(buf[:n])


def tan_read(data, max_recs=1 << 20):
    """The records of a tan log (record.go reader): [(offset, payload)];
    raises on a format error."""
    offs = (C.c_int64 * max_recs)()
    lens = (C.c_size_t * max_recs)()
    cap = max(1, len(data))
    out = (C.c_uint8 * cap)()
    n = lib().orc_tan_read(_u8(data), len(data), offs, lens, max_recs, out,
                           cap)
    if n < 0:
        raise OracleError("tan read: " + ORC_TAN_ERRORS.get(n, str(n)))
    recs, pos = [], 0
    for i in range(n):
        recs.append((offs[i], bytes(out[pos:pos + lens[i]])))
        pos += lens[i]
    return recs


def update_marshal(shard, replica, state, entries):
    """Update.MarshalTo (raftpb/update.go:128-169); state (term, vote,
    commit) or None."""
    arr, pool, n = EntryPool(entries).arrays()
    buf = (C.c_uint8 * lib().orc_update_size_bound(arr, n))()
    t, v, c = state or (0, 0, 0)
    k = lib().orc_update_marshal(shard, replica, t, v, c, arr, n, pool, buf)
    return bytes(buf[:k])


class TanDB:
    """One replica's regular tan db (internal/tan/db.go:97-130)."""

    def __init__(self, max_log_size=0):
        self.p = lib().orc_tandb_new(max_log_size)

    def __del__(self):
        if getattr(self, "p", None):
            lib().orc_tandb_free(self.p)

    def write(self, shard, replica, state, entries):
        """db.write: None when nothing is written, else last()."""
        arr, pool, n = EntryPool(entries).arrays()
        t, v, c = state or (0, 0, 0)
        sync = C.c_int()
        rc = _check(lib().orc_tandb_write(self.p, shard, replica, t, v, c,
                                          arr, n, pool, C.byref(sync)))
        return self.last() if rc == 1 else None

    def last(self):
        """{off, len, sync, new_log, log, offset} of the last write."""
        o = (C.c_int64 * 6)()
        lib().orc_tandb_last(self.p, o)
        return dict(off=o[0], len=o[1], sync=bool(o[2]), new_log=bool(o[3]),
                    log=o[4], offset=o[5])

    def file(self, log):
        n = _check(lib().orc_tandb_file(self.p, log, None, 0))
        buf = (C.c_uint8 * max(1, n))()
        lib().orc_tandb_file(self.p, log, buf, n)
        return bytes(buf[:n])
