"""Python binding of the C ABI (include/drb_engine.h).

This is plumbing for tests and bench.py: every call goes straight to the
HIP engine in dragonboat_amd/_lib/libdrb_engine.so.  There is no CPU
fallback -- if the library or the GPU is missing, Engine() raises.
"""
import ctypes as C
import os

from . import abi
from .abi import (ApplyResult, Config, Entry, Flagged, Message, ReadyToRead, Region, ReplicaState,
                  RoundIn, RoundOut, WireCfg, WireCpu, WireIn, WireOut,
                  entry_to_tuple,
                  message_to_tuple)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DRB_ENGINE_LIB") or \
    os.path.join(HERE, "_lib", "libdrb_engine.so")

_lib = None

P = C.c_void_p
U64 = C.c_uint64
U32 = C.c_uint32
PU64 = C.POINTER(C.c_uint64)
PU32 = C.POINTER(C.c_uint32)
PU8 = C.POINTER(C.c_uint8)
SZ = C.c_size_t

# every symbol include/drb_engine.h declares, with its signature
SIGNATURES = {
    "drb_engine_create": (C.c_int, [C.POINTER(Config), C.POINTER(P)]),
    "drb_engine_destroy": (C.c_int, [P]),
    "drb_engine_device_bytes": (U64, [P]),
    "drb_engine_stream": (P, [P]),
    "drb_engine_sync": (C.c_int, [P]),
    "drb_engine_round": (U64, [P]),
    "drb_import_replicas": (C.c_int, [P, U64, U64,
                                      C.POINTER(ReplicaState)]),
    "drb_export_replicas": (C.c_int, [P, U64, U64,
                                      C.POINTER(ReplicaState)]),
    "drb_import_log": (C.c_int, [P, U64, U32, C.POINTER(Entry), SZ, PU8]),
    "drb_export_log": (C.c_int, [P, U64, U32, U64, U64, C.POINTER(Entry),
                                 PU8, SZ]),
    "drb_init_steady": (C.c_int, [P, U64, U32, U64]),
    "drb_host_slot": (C.c_int, [P, U32, C.c_int]),
    "drb_role_census": (C.c_int, [P, PU64]),
    "drb_export_save_records": (C.c_int, [P, U64, U32,
                                          C.POINTER(abi.SaveRecord), SZ,
                                          C.POINTER(SZ)]),
    "drb_role_slots": (C.c_int, [P, PU32, PU32]),
    "drb_stage_proposals": (C.c_int, [P, U32, PU32, C.POINTER(Entry), PU8,
                                      SZ]),
    "drb_stage_proposals_packed": (C.c_int, [P, U32, U32, PU8, U64, PU64,
                                             PU64, C.POINTER(C.c_uint16),
                                             PU8, SZ]),
    "drb_stage_proposals_packed_async": (C.c_int, [P, U32, U32, PU8, U64, PU64,
                                             PU64, C.POINTER(C.c_uint16),
                                             PU8, SZ]),
    "drb_stage_wait_upload": (C.c_int, [P]),
    "drb_set_session_clients": (C.c_int, [P, PU64]),
    "drb_stage_packed_layout": (C.c_int, [P, U64, SZ, PU64, C.POINTER(SZ)]),
    "drb_gen_kv_proposals": (C.c_int, [P, U32, U32, U32, U32, U64, U64]),
    "drb_gen_kv_proposals_active": (C.c_int, [P, U32, U32, U32, U32, U64,
                                              U64, U32]),
    "drb_stage_read_index": (C.c_int, [P, U32, PU64, PU64]),
    "drb_gen_read_index": (C.c_int, [P, U32, U64, U64]),
    "drb_request_leader_transfer": (C.c_int, [P, U32, PU32, PU64]),
    "drb_ingest": (C.c_int, [P, C.POINTER(Message), SZ, C.POINTER(Entry),
                             PU8, PU64, PU64]),
    "drb_ingest_ex": (C.c_int, [P, C.POINTER(Message), SZ, C.POINTER(Entry),
                                PU8, PU8, PU64, PU64, PU64]),
    "drb_export_inbox": (C.c_int, [P, U64, U32, C.c_int, C.POINTER(Message),
                                   SZ, C.POINTER(Entry), SZ, PU8, SZ,
                                   C.POINTER(SZ)]),
    "drb_ingest_wire_cpu": (C.c_int, [P, C.POINTER(WireCpu), SZ,
                                      C.POINTER(SZ)]),
    "drb_step_round": (C.c_int, [P, C.POINTER(RoundIn),
                                 C.POINTER(RoundOut)]),
    "drb_step_round_async": (C.c_int, [P, C.POINTER(RoundIn)]),
    "drb_step_rounds": (C.c_int, [P, C.POINTER(RoundIn), U32, U64]),
    "drb_read_counters": (C.c_int, [P, C.POINTER(RoundOut), C.c_int]),
    "drb_debug_phase": (C.c_int, [P, C.POINTER(U64), C.c_int]),
    "drb_take_flagged": (C.c_int, [P, C.POINTER(Flagged), SZ, C.POINTER(SZ),
                                   PU64, C.c_int]),
    "drb_apply_results": (C.c_int, [P, U32, U64, U64, C.POINTER(ApplyResult),
                                    SZ, C.POINTER(SZ)]),
    "drb_commit_round": (C.c_int, [P, U64]),
    "drb_committed_round": (U64, [P]),
    "drb_export_outbox": (C.c_int, [P, U64, U32, C.POINTER(Message), SZ,
                                    C.POINTER(Entry), SZ, PU8, SZ,
                                    C.POINTER(SZ)]),
    "drb_export_ready_to_reads": (C.c_int, [P, U64, U32,
                                            C.POINTER(ReadyToRead), SZ,
                                            C.POINTER(SZ)]),
    "drb_export_ready_to_reads_batch": (C.c_int, [P, U32, U64, U64,
                                                  C.POINTER(ReadyToRead), SZ,
                                                  C.POINTER(SZ)]),
    "drb_export_read_results": (C.c_int, [P, U32, U64, U64,
                                          C.POINTER(abi.ReadResult), SZ,
                                          C.POINTER(SZ)]),
    "drb_export_read_values": (C.c_int, [P, U32, U64, U64,
                                         C.POINTER(abi.ReadResult), PU64, SZ,
                                         PU8, SZ, C.POINTER(SZ),
                                         C.POINTER(SZ)]),
    "drb_serve_reads": (C.c_int, [P, U32, U32]),
    "drb_export_read_sums": (C.c_int, [P, U64, U64, PU64]),
    "drb_kv_lookup": (C.c_int, [P, U64, U32, PU8, U32, PU8, U32, PU32]),
    "drb_kv_export": (C.c_int, [P, U64, U32, PU8, PU32, PU8, PU32, SZ,
                                C.POINTER(SZ)]),
    "drb_kv_import": (C.c_int, [P, U64, U32, PU8, PU32, PU8, PU32, SZ, SZ]),
    "drb_crc32_ieee_batch": (C.c_int, [P, PU8, SZ, PU64, PU32, SZ, PU32]),
    "drb_export_saved": (C.c_int, [P, U64, U32, PU8, SZ, PU32, PU32]),
    "drb_saved_buffers": (C.c_int, [P, C.POINTER(P), C.POINTER(PU32),
                                    C.POINTER(PU32)]),
    "drb_export_tan": (C.c_int, [P, U64, U32, C.POINTER(abi.TanRecord), PU8,
                                 SZ]),
    "drb_tan_get": (C.c_int, [P, U64, U32, C.POINTER(abi.TanState)]),
    "drb_export_tan_log": (C.c_int, [P, U32, U32, C.POINTER(abi.TanLog), PU8,
                                     C.c_size_t]),
    "drb_tan_set": (C.c_int, [P, U64, U32, C.POINTER(abi.TanState)]),
    "drb_tan_buffers": (C.c_int, [P, C.POINTER(P), C.POINTER(P)]),
    "drb_plane_counts": (C.c_int, [P, PU32]),
    "drb_plane_peer": (C.c_int, [P, U32, U32, C.c_int]),
    "drb_place_peer": (C.c_int, [U32, U32, U32, U32, C.c_int]),
    "drb_plane_regions": (C.c_int, [P, U32, U32, U32, C.c_int,
                                    C.POINTER(Region)]),
    "drb_exchange_local": (C.c_int, [C.POINTER(P), U32]),
    "drb_exchange_local_counted": (C.c_int, [C.POINTER(P), U32]),
    "drb_exchange_local_bind": (C.c_int, [C.POINTER(P), U32]),
    "drb_exchange_mark": (C.c_int, [P]),
    "drb_exchange_plan": (C.c_int, [P, U32, C.POINTER(abi.Xfer), SZ,
                                    C.POINTER(SZ)]),
    "drb_exchange_rccl": (C.c_int, [P, P, U32]),
    "drb_exchange_plan_words": (C.c_int, [P, PU32, C.POINTER(abi.Xfer), SZ,
                                          C.POINTER(SZ)]),
    "drb_exchange_rccl_counted": (C.c_int, [P, P]),
    "drb_exchange_rccl_roles": (C.c_int, [P, P, PU32]),
    "drb_exchange_bytes": (C.c_int, [P, C.POINTER(U64), C.c_int]),
    "drb_encode_wire": (C.c_int, [P, U32, U32, C.POINTER(WireCfg),
                                  C.POINTER(WireOut)]),
    "drb_wire_buffer": (C.c_int, [P, C.POINTER(P), PU64]),
    "drb_export_wire": (C.c_int, [P, PU8, SZ, C.POINTER(SZ)]),
    "drb_ingest_wire": (C.c_int, [P, PU8, SZ, U64, C.POINTER(WireIn)]),
    "drb_ingest_buffer": (C.c_int, [P, SZ, C.POINTER(PU8)]),
    "drb_ingest_buffer_alloc": (C.c_int, [P, SZ, C.POINTER(PU8)]),
    "drb_ingest_buffer_free": (C.c_int, [P, PU8]),
    "drb_worker_export": (C.c_int, [P, U32, C.POINTER(abi.WorkerBufs)]),
    "drb_worker_export_part": (C.c_int, [P, U32, U32, U32,
                                         C.POINTER(abi.WorkerBufs)]),
    "drb_worker_wait": (C.c_int, [P, C.POINTER(abi.WorkerBufs)]),
    "drb_host_alloc": (C.c_int, [P, SZ, C.POINTER(P)]),
    "drb_host_free": (C.c_int, [P, P]),
}


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "dragonboat_amd: %s is missing; run "
                "python -c 'import __graft_entry__; __graft_entry__.build()'"
                % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        variant = bool(os.environ.get("DRB_ENGINE_LIB"))
        for name, (res, args) in SIGNATURES.items():
            if variant and not hasattr(L, name):
                continue  # an older timing variant (tools/variants.sh)
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class DrbError(RuntimeError):
    pass


def _ck(rc, what):
    if rc < 0:
        raise DrbError("%s failed with status %d" % (what, rc))
    return rc


def _u8(b):
    return (C.c_uint8 * max(1, len(b))).from_buffer_copy(bytes(b) or b"\0")


DEFAULTS = dict(num_groups=1, first_shard_id=1, num_replicas=3, window=32,
                cmd_cap=32, max_props=4, prop_slots=2, ri_slots=2,
                mailbox=16, kv_slots=512, kv_val_cap=4, election_rtt=10,
                heartbeat_rtt=1, check_quorum=1, device=0, save_cap=0,
                total_groups=0, place_world=1, place_rank=0, entry_mbox=0,
                kv_pool_blocks=0, flagged_cap=0, quiesce=0, durable_log=0,
                save_batched=0, save_tan=0, tan_max_log=0, elections=0,
                tan_multiplexed=0, pre_vote=0, max_reads_per_ctx=0,
                kv_overflow_buckets=0, forward_proposals=0,
                nonvoting_slots=0, witness_slots=0, host_copies=0,
                no_lean=0)


class Engine:
    """One MI355X-resident set of G groups x R replica slots."""

    def __init__(self, **kw):
        cfg = dict(DEFAULTS)
        cfg.update(kw)
        self.cfg = cfg
        c = Config(cfg["num_groups"], cfg["first_shard_id"],
                   cfg["num_replicas"], cfg["window"], cfg["cmd_cap"],
                   cfg["max_props"], cfg["prop_slots"], cfg["ri_slots"],
                   cfg["mailbox"], cfg["kv_slots"], cfg["kv_val_cap"],
                   cfg["election_rtt"], cfg["heartbeat_rtt"],
                   cfg["check_quorum"], cfg["device"], cfg["save_cap"],
                   cfg["total_groups"], cfg["place_world"], cfg["place_rank"],
                   cfg["entry_mbox"], cfg["kv_pool_blocks"],
                   cfg["flagged_cap"], cfg["quiesce"],
                   cfg["durable_log"], cfg["save_batched"],
                   cfg["save_tan"], cfg["elections"], cfg["tan_max_log"],
                   cfg["tan_multiplexed"], cfg["pre_vote"],
                   cfg["max_reads_per_ctx"], cfg["kv_overflow_buckets"],
                   cfg["forward_proposals"], cfg["nonvoting_slots"],
                   cfg["witness_slots"], cfg["host_copies"],
                   cfg["no_lean"])
        h = P()
        _ck(lib().drb_engine_create(C.byref(c), C.byref(h)),
            "drb_engine_create")
        self.h = h
        self.G = cfg["num_groups"]
        self.R = cfg["num_replicas"]

    def close(self):
        if getattr(self, "h", None):
            lib().drb_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # ---------------------------------------------------------- state
    @property
    def device_bytes(self):
        return lib().drb_engine_device_bytes(self.h)

    @property
    def round(self):
        return lib().drb_engine_round(self.h)

    @property
    def stream(self):
        return lib().drb_engine_stream(self.h)

    def sync(self):
        _ck(lib().drb_engine_sync(self.h), "drb_engine_sync")

    def import_replicas(self, first_group, states):
        n = len(states) // self.R
        arr = (ReplicaState * len(states))(*states)
        _ck(lib().drb_import_replicas(self.h, first_group, n, arr),
            "drb_import_replicas")

    def export_replicas(self, first_group, n_groups):
        arr = (ReplicaState * (n_groups * self.R))()
        _ck(lib().drb_export_replicas(self.h, first_group, n_groups, arr),
            "drb_export_replicas")
        return list(arr)

    def export(self, g, slot):
        return self.export_replicas(g, 1)[slot]

    def import_log(self, g, slot, entries, pool):
        """entries: Entry array (indices set), pool: uint8 array."""
        _ck(lib().drb_import_log(self.h, g, slot, entries, len(entries), pool),
            "drb_import_log")

    def export_log(self, g, slot, lo, hi):
        n = hi - lo + 1
        if n <= 0:
            return []
        arr = (Entry * n)()
        pcap = n * self.cfg["cmd_cap"] + 16
        pool = (C.c_uint8 * pcap)()
        _ck(lib().drb_export_log(self.h, g, slot, lo, hi, arr, pool, pcap),
            "drb_export_log")
        return [entry_to_tuple(arr[i], pool) for i in range(n)]

    def role_slots(self):
        """(leader slot mask, follower slot mask) of the hosted replicas."""
        a, b = U32(), U32()
        _ck(lib().drb_role_slots(self.h, C.byref(a), C.byref(b)),
            "drb_role_slots")
        return a.value, b.value

    def host_slot(self, slot, hosted):
        _ck(lib().drb_host_slot(self.h, slot, int(bool(hosted))),
            "drb_host_slot")

    def init_steady(self, term=2, leader_slot=0, seed=0x5EEDD8B0):
        _ck(lib().drb_init_steady(self.h, term, leader_slot, seed),
            "drb_init_steady")

    # ---------------------------------------------------------- inputs
    def stage_proposals(self, slot, counts, ents, pool, pool_len=None):
        """pool: a ctypes byte array (its size is the pool length) or a
        pointer with pool_len."""
        if pool_len is None:
            pool_len = C.sizeof(pool)
        _ck(lib().drb_stage_proposals(self.h, slot, counts, ents, pool,
                                      pool_len), "drb_stage_proposals")

    def stage_proposals_packed(self, slot, type, counts, n, keys, clients,
                               lens, pool, pool_len):
        """drb_stage_proposals_packed; the arrays are ctypes pointers (or
        arrays): counts u8[G], keys / clients u64[n], lens u16[n]."""
        _ck(lib().drb_stage_proposals_packed(self.h, slot, type, counts, n,
                                             keys, clients, lens, pool,
                                             pool_len),
            "drb_stage_proposals_packed")

    def stage_proposals_packed_async(self, slot, type, counts, n, keys,
                                     clients, lens, pool, pool_len):
        """drb_stage_proposals_packed_async: the arrays stay in use until
        the next call (or stage_wait_upload) returns."""
        _ck(lib().drb_stage_proposals_packed_async(
            self.h, slot, type, counts, n, keys, clients, lens, pool,
            pool_len), "drb_stage_proposals_packed_async")

    def stage_packed_layout(self, n_entries, pool_len):
        """drb_stage_packed_layout: ([keys, client ids, lengths, pool]
        offsets, block bytes) of a one-block packed batch."""
        off = (U64 * 4)()
        nb = SZ()
        _ck(lib().drb_stage_packed_layout(self.h, n_entries, pool_len, off,
                                          C.byref(nb)),
            "drb_stage_packed_layout")
        return list(off), nb.value

    def set_session_clients(self, client_ids):
        """drb_set_session_clients: the ClientID of the host's NoOP session
        of every lane's group (a sequence of G ints or a u64 array)."""
        if hasattr(client_ids, "ctypes"):  # a numpy array
            import numpy as np
            arr = np.ascontiguousarray(client_ids, dtype=np.uint64)
            assert arr.size >= self.G
            ptr = arr.ctypes.data_as(PU64)
        else:
            arr = (U64 * self.G)(*client_ids)
            ptr = C.cast(arr, PU64)
        _ck(lib().drb_set_session_clients(self.h, ptr),
            "drb_set_session_clients")

    def stage_wait_upload(self):
        _ck(lib().drb_stage_wait_upload(self.h), "drb_stage_wait_upload")

    def gen_kv_proposals(self, slot, k, key_space, val_len, seed, salt,
                         active_ppm=1000000):
        _ck(lib().drb_gen_kv_proposals_active(self.h, slot, k, key_space,
                                              val_len, seed, salt,
                                              active_ppm),
            "drb_gen_kv_proposals_active")

    def stage_read_index(self, slot, low, high):
        _ck(lib().drb_stage_read_index(self.h, slot, low, high),
            "drb_stage_read_index")

    def gen_read_index(self, slot, seed, high):
        _ck(lib().drb_gen_read_index(self.h, slot, seed, high),
            "drb_gen_read_index")

    def request_leader_transfer(self, slot, targets):
        """NodeHost.RequestLeaderTransfer at replica slot `slot` of every
        group g with targets[g] (a replica ID) != 0; returns how many were
        refused as busy (drb_request_leader_transfer)."""
        arr = (C.c_uint32 * self.G)(*targets)
        busy = U64()
        _ck(lib().drb_request_leader_transfer(self.h, slot, arr,
                                              C.byref(busy)),
            "drb_request_leader_transfer")
        return busy.value

    def ingest(self, marr, n, earr, pool):
        """drb_ingest: (accepted, dropped); raises DrbError (DRB_EDIVERTED)
        when a message had to go to the CPU path -- use ingest_ex there."""
        acc, drop = U64(), U64()
        _ck(lib().drb_ingest(self.h, marr, n, earr, pool, C.byref(acc),
                             C.byref(drop)), "drb_ingest")
        return acc.value, drop.value

    def ingest_ex(self, marr, n, earr, pool):
        """drb_ingest_ex: counts and each message's fate (abi.ING_*)."""
        acc, drop, div = U64(), U64(), U64()
        st = (C.c_uint8 * max(1, n))()
        _ck(lib().drb_ingest_ex(self.h, marr, n, earr, pool, st,
                                C.byref(acc), C.byref(drop), C.byref(div)),
            "drb_ingest_ex")
        return {"accepted": acc.value, "dropped": drop.value,
                "diverted": div.value, "status": list(st[:n])}

    # ---------------------------------------------------------- round
    def step(self, tick=False, prop_slot=abi.DRB_NONE, ri_slot=abi.DRB_NONE,
             reads_per_ctx=0, key_space=0, encode_saves=False, ri_replica=0,
             listed=False, prop_replica=0):
        rin = RoundIn(int(bool(tick)), prop_slot, ri_slot, reads_per_ctx,
                      key_space, int(bool(encode_saves)), ri_replica,
                      int(bool(listed)), prop_replica)
        out = RoundOut()
        _ck(lib().drb_step_round(self.h, C.byref(rin), C.byref(out)),
            "drb_step_round")
        return out

    def step_async(self, tick=False, prop_slot=abi.DRB_NONE,
                   ri_slot=abi.DRB_NONE, reads_per_ctx=0, key_space=0,
                   encode_saves=False, ri_replica=0, listed=False,
                   prop_replica=0):
        """One round, stream-ordered; reads_per_ctx > 0 also serves the
        reads behind the round's ReadyToReads, encode_saves encodes the
        EntriesToSave (drb_round_in)."""
        rin = RoundIn(int(bool(tick)), prop_slot, ri_slot, reads_per_ctx,
                      key_space, int(bool(encode_saves)), ri_replica,
                      int(bool(listed)), prop_replica)
        _ck(lib().drb_step_round_async(self.h, C.byref(rin)),
            "drb_step_round_async")

    @staticmethod
    def round_array(rounds):
        """The drb_round_in array of rounds ([dict(tick=, prop_slot=,
        ri_slot=, reads_per_ctx=, key_space=, encode_saves=)]), for
        step_rounds (built once, stepped many times)."""
        arr = (RoundIn * len(rounds))()
        for i, r in enumerate(rounds):
            arr[i] = RoundIn(int(bool(r.get("tick"))),
                             r.get("prop_slot", abi.DRB_NONE),
                             r.get("ri_slot", abi.DRB_NONE),
                             r.get("reads_per_ctx", 0), r.get("key_space", 0),
                             int(bool(r.get("encode_saves"))),
                             r.get("ri_replica", 0), 0,
                             r.get("prop_replica", 0))
        return arr

    def step_rounds(self, rounds, chunk_groups):
        """drb_step_rounds: the rounds chunk by chunk of the groups (a
        chunk of every group: plain rounds, one C call); rounds: a list of
        dicts or a round_array."""
        arr = rounds if isinstance(rounds, C.Array) else \
            self.round_array(rounds)
        _ck(lib().drb_step_rounds(self.h, arr, len(arr), chunk_groups),
            "drb_step_rounds")

    def read_counters(self, reset=True):
        out = RoundOut()
        _ck(lib().drb_read_counters(self.h, C.byref(out), int(reset)),
            "drb_read_counters")
        return out

    def debug_phase(self, reset=True):
        """drb_debug_phase: {role: [lanes, cycles of each round phase]}
        (timing builds only; zeros otherwise)."""
        out = (U64 * 16)()
        _ck(lib().drb_debug_phase(self.h, out, int(reset)), "drb_debug_phase")
        return {"follower": list(out[:8]), "leader": list(out[8:])}

    def take_flagged(self, cap=65536, reset=True):
        """[(group, slot, reason, flags, round, shard_id)] of the replicas
        marked FALLBACK / ERROR since the last reset, and the count lost."""
        arr = (Flagged * max(1, cap))()
        n, lost = SZ(), U64()
        _ck(lib().drb_take_flagged(self.h, arr, cap, C.byref(n),
                                   C.byref(lost), int(reset)),
            "drb_take_flagged")
        return ([(arr[i].group, arr[i].slot, arr[i].reason, arr[i].flags,
                  arr[i].round, arr[i].shard_id) for i in range(n.value)],
                lost.value)

    def apply_results(self, slot, first_group=0, n_groups=None, cap=None):
        """[(group, index, key, client_id, series_id, value, ignored)] of
        the entries replica slot applied in the last round."""
        n_groups = self.G - first_group if n_groups is None else n_groups
        cap = cap or n_groups * self.cfg["max_props"] * 4 + 16
        arr = (ApplyResult * cap)()
        n = SZ()
        _ck(lib().drb_apply_results(self.h, slot, first_group, n_groups, arr,
                                    cap, C.byref(n)), "drb_apply_results")
        return [(a.group, a.index, a.key, a.client_id, a.series_id, a.value,
                 a.ignored) for a in arr[:n.value]]

    def commit_round(self, rnd):
        _ck(lib().drb_commit_round(self.h, rnd), "drb_commit_round")

    @property
    def committed_round(self):
        return lib().drb_committed_round(self.h)

    # ---------------------------------------------------------- outputs
    def export_outbox(self, g, slot):
        cap, ecap = 16 * self.R, 16 * self.R * self.cfg["window"]
        pcap = ecap * self.cfg["cmd_cap"] + 16
        marr = (Message * cap)()
        earr = (Entry * ecap)()
        pool = (C.c_uint8 * pcap)()
        n = SZ()
        _ck(lib().drb_export_outbox(self.h, g, slot, marr, cap, earr, ecap,
                                    pool, pcap, C.byref(n)),
            "drb_export_outbox")
        return [message_to_tuple(marr[i], earr, pool) for i in range(n.value)]

    def export_inbox(self, g, slot, last_round=False):
        """drb_export_inbox: the messages in (g, slot)'s inbound planes."""
        cap, ecap = 32 * self.R, 32 * self.R * self.cfg["window"]
        pcap = ecap * self.cfg["cmd_cap"] + 16
        marr = (Message * cap)()
        earr = (Entry * ecap)()
        pool = (C.c_uint8 * pcap)()
        n = SZ()
        _ck(lib().drb_export_inbox(self.h, g, slot, int(bool(last_round)),
                                   marr, cap, earr, ecap, pool, pcap,
                                   C.byref(n)), "drb_export_inbox")
        return [message_to_tuple(marr[i], earr, pool) for i in range(n.value)]

    def export_ready(self, g, slot):
        cap = 16
        arr = (ReadyToRead * cap)()
        n = SZ()
        _ck(lib().drb_export_ready_to_reads(self.h, g, slot, arr, cap,
                                            C.byref(n)),
            "drb_export_ready_to_reads")
        return [(arr[i].index, arr[i].ctx_low, arr[i].ctx_high)
                for i in range(min(n.value, cap))]

    def _batch(self, fn, typ, slot, first_group, n_groups, cap):
        n_groups = self.G - first_group if n_groups is None else n_groups
        n = SZ()
        arr = (typ * max(1, cap))()
        rc = fn(self.h, slot, first_group, n_groups, arr, cap, C.byref(n))
        if rc == abi.DRB_ERANGE and n.value > cap:  # sized by the count
            arr = (typ * n.value)()
            rc = fn(self.h, slot, first_group, n_groups, arr, n.value,
                    C.byref(n))
        _ck(rc, fn.__name__)
        return arr, n.value

    def export_ready_batch(self, slot, first_group=0, n_groups=None,
                           cap=1 << 16):
        """{group: [(index, ctx_low, ctx_high)]} of replica slot's
        ReadyToReads of the last round (drb_export_ready_to_reads_batch)."""
        arr, n = self._batch(lib().drb_export_ready_to_reads_batch,
                             ReadyToRead, slot, first_group, n_groups, cap)
        out = {}
        base = self.cfg["first_shard_id"]
        for i in range(n):
            r = arr[i]
            out.setdefault(r.shard_id - base, []).append(
                (r.index, r.ctx_low, r.ctx_high))
        return out

    def export_read_results(self, slot, first_group=0, n_groups=None,
                            cap=1 << 16):
        """[(group, index, ctx_low, read j, key, found, vlen, value)] of the
        reads replica slot served in the last round (drb_export_read_
        results)."""
        arr, n = self._batch(lib().drb_export_read_results, abi.ReadResult,
                             slot, first_group, n_groups, cap)
        base = self.cfg["first_shard_id"]
        return [(r.shard_id - base, r.index, r.ctx_low, r.read, r.key,
                 r.found, r.vlen, r.value) for r in arr[:n]]

    def export_read_values(self, slot, first_group=0, n_groups=None,
                           cap=1 << 16, pool_cap=1 << 20):
        """[(group, index, ctx_low, read j, key, found, value bytes or None)]
        of the reads replica slot served in the last round, values whole
        (drb_export_read_values)."""
        n_groups = self.G - first_group if n_groups is None else n_groups
        while True:
            arr = (abi.ReadResult * max(1, cap))()
            off = (U64 * max(1, cap))()
            pool = (C.c_uint8 * max(16, pool_cap))()
            n, pb = SZ(), SZ()
            rc = lib().drb_export_read_values(
                self.h, slot, first_group, n_groups, arr, off, cap, pool,
                pool_cap, C.byref(n), C.byref(pb))
            if rc == abi.DRB_ERANGE and (n.value > cap or pb.value > pool_cap):
                cap, pool_cap = max(cap, n.value), max(pool_cap, pb.value)
                continue
            _ck(rc, "drb_export_read_values")
            break
        base = self.cfg["first_shard_id"]
        out = []
        for i in range(n.value):
            r = arr[i]
            val = bytes(pool[off[i]:off[i] + r.vlen]) if r.found else None
            out.append((r.shard_id - base, r.index, r.ctx_low, r.read, r.key,
                        r.found, val))
        return out

    def kv_export(self, g, slot):
        cap = self.cfg["kv_slots"]
        vcap = self.cfg["kv_val_cap"]
        while True:  # (a KV with overflow buckets may hold more)
            keys = (C.c_uint8 * (8 * cap))()
            vals = (C.c_uint8 * (vcap * cap))()
            kl, vl = (U32 * cap)(), (U32 * cap)()
            n = SZ()
            rc = lib().drb_kv_export(self.h, g, slot, keys, kl, vals, vl, cap,
                                     C.byref(n))
            if rc == -5 and n.value > cap:  # DRB_ERANGE: the full count
                cap = n.value
                continue
            _ck(rc, "drb_kv_export")
            break
        kb, vb = bytes(keys), bytes(vals)
        return {kb[i * 8:i * 8 + kl[i]]: vb[i * vcap:i * vcap + vl[i]]
                for i in range(n.value)}

    def kv_import(self, g, slot, kv):
        """Replaces replica (g, slot)'s KV with the {key: value} dict
        (drb_kv_import, the state machine handed back after a fallback)."""
        n = len(kv)
        stride = max([len(x) for x in kv.values()] + [1])
        keys = (C.c_uint8 * max(1, 8 * n))()
        vals = (C.c_uint8 * max(1, stride * n))()
        kl, vl = (U32 * max(1, n))(), (U32 * max(1, n))()
        for i, (k, x) in enumerate(kv.items()):
            C.memmove(C.addressof(keys) + 8 * i, bytes(k), len(k))
            C.memmove(C.addressof(vals) + stride * i, bytes(x), len(x))
            kl[i], vl[i] = len(k), len(x)
        _ck(lib().drb_kv_import(self.h, g, slot, keys, kl, vals, vl, stride,
                                n), "drb_kv_import")

    def export_saved(self, g, slot):
        """(EntryBatch bytes, crc32) of one replica's last EntriesToSave."""
        cap = self.cfg["save_cap"]
        buf = (C.c_uint8 * max(1, cap))()
        ln, crc = U32(), U32()
        _ck(lib().drb_export_saved(self.h, g, slot, buf, cap, C.byref(ln),
                                   C.byref(crc)), "drb_export_saved")
        return bytes(buf[:ln.value]), crc.value

    def role_census(self):
        """[slot][role] counts of the hosted fast-path replicas."""
        c = (C.c_uint64 * (8 * self.R))()
        _ck(lib().drb_role_census(self.h, c), "drb_role_census")
        return [[c[s * 8 + k] for k in range(8)] for s in range(self.R)]

    def export_tan(self, g, slot):
        """save_tan: (drb_tan_record as a dict, the bytes appended) of one
        replica's last round."""
        rec = abi.TanRecord()
        cap = self.cfg["save_cap"]
        buf = (C.c_uint8 * max(1, cap))()
        _ck(lib().drb_export_tan(self.h, g, slot, C.byref(rec), buf, cap),
            "drb_export_tan")
        d = {f: getattr(rec, f) for f, _ in rec._fields_ if f != "pad"}
        return d, bytes(buf[:rec.len])

    def export_tan_log(self, slot, key):
        """tan_multiplexed: (drb_tan_log as a dict, the round's bytes) of
        log (slot, key)."""
        lg = abi.TanLog()
        _ck(lib().drb_export_tan_log(self.h, slot, key, C.byref(lg), None, 0),
            "drb_export_tan_log")
        buf = (C.c_uint8 * max(1, lg.bytes))()
        _ck(lib().drb_export_tan_log(self.h, slot, key, C.byref(lg), buf,
                                     lg.bytes), "drb_export_tan_log")
        d = {f: getattr(lg, f) for f, _ in lg._fields_ if f != "pad"}
        return d, bytes(buf[:lg.bytes])

    def tan_get(self, g, slot):
        st = abi.TanState()
        _ck(lib().drb_tan_get(self.h, g, slot, C.byref(st)), "drb_tan_get")
        return st.offset, st.log, st.state_stored

    def tan_set(self, g, slot, offset, log, state_stored):
        st = abi.TanState(offset, log, int(bool(state_stored)))
        _ck(lib().drb_tan_set(self.h, g, slot, C.byref(st)), "drb_tan_set")

    def export_save_records(self, g, slot):
        """save_batched: [(batch id, record value, crc32)] of one replica's
        last round, in Put order."""
        recs = (abi.SaveRecord * 4)()
        n = SZ()
        _ck(lib().drb_export_save_records(self.h, g, slot, recs, 4,
                                          C.byref(n)),
            "drb_export_save_records")
        if not n.value:
            return []
        data, _ = self.export_saved(g, slot)
        return [(recs[i].batch, data[recs[i].offset:recs[i].offset +
                                     recs[i].len], recs[i].crc)
                for i in range(n.value)]

    # ---------------------------------------------------------- exchange
    def plane_counts(self):
        """Summary words [from * R + to] of the last round's remote planes."""
        w = (C.c_uint32 * (self.R * self.R))()
        _ck(lib().drb_plane_counts(self.h, w), "drb_plane_counts")
        return list(w)

    def plane_peer(self, a, b, direction):
        return lib().drb_plane_peer(self.h, a, b, direction)

    def plane_regions(self, a, b, word, direction):
        """[(device address, bytes)] of plane (a, b) for the last round."""
        arr = (Region * abi.PLANE_REGIONS)()
        n = _ck(lib().drb_plane_regions(self.h, a, b, word, direction, arr),
                "drb_plane_regions")
        return [(arr[i].ptr, arr[i].bytes) for i in range(n)]

    @staticmethod
    def exchange_local(engines, counted=False):
        """One process holding every rank's engine: move the planes
        (full-capacity planes behind cross-stream events, or at the counted
        sizes with host synchronisation)."""
        arr = (P * len(engines))(*[e.h for e in engines])
        fn = lib().drb_exchange_local_counted if counted else \
            lib().drb_exchange_local
        _ck(fn(arr, len(engines)), "drb_exchange_local")

    @staticmethod
    def exchange_local_bind(engines):
        """Bind one process's engines on one GPU (rank order) for the
        zero-copy exchange (drb_exchange_local_bind): their rounds read
        remote planes from the senders' outboxes, exchange_local then only
        orders the rounds.  For good: destroy them together."""
        arr = (P * len(engines))(*[e.h for e in engines])
        _ck(lib().drb_exchange_local_bind(arr, len(engines)),
            "drb_exchange_local_bind")

    def exchange_bytes(self, reset=False):
        """Inbound plane bytes moved into this engine by the exchanges
        (drb_exchange_bytes)."""
        b = U64()
        _ck(lib().drb_exchange_bytes(self.h, C.byref(b), int(bool(reset))),
            "drb_exchange_bytes")
        return b.value

    def exchange_plan(self, leader_mask):
        """drb_exchange_plan: [(peer, recv, device address, bytes)] of this
        rank's fixed-capacity exchange step, in posting order."""
        n = SZ()
        _ck(lib().drb_exchange_plan(self.h, leader_mask, None, 0,
                                    C.byref(n)), "drb_exchange_plan")
        arr = (abi.Xfer * max(1, n.value))()
        _ck(lib().drb_exchange_plan(self.h, leader_mask, arr, n.value,
                                    C.byref(n)), "drb_exchange_plan")
        return [(arr[i].peer, arr[i].recv, arr[i].ptr, arr[i].bytes)
                for i in range(n.value)]

    def exchange_plan_words(self, words):
        """drb_exchange_plan_words: the transfer list from every rank's
        plane words (a list of world rows of R * R words)."""
        flat = [w for row in words for w in row]
        arr = (U32 * max(1, len(flat)))(*flat)
        n = SZ()
        _ck(lib().drb_exchange_plan_words(self.h, arr, None, 0, C.byref(n)),
            "drb_exchange_plan_words")
        ops = (abi.Xfer * max(1, n.value))()
        _ck(lib().drb_exchange_plan_words(self.h, arr, ops, n.value,
                                          C.byref(n)),
            "drb_exchange_plan_words")
        return [(ops[i].peer, ops[i].recv, ops[i].ptr, ops[i].bytes)
                for i in range(n.value)]

    def exchange_rccl_counted(self, comm):
        """drb_exchange_rccl_counted over an ncclComm_t (an address)."""
        _ck(lib().drb_exchange_rccl_counted(self.h, comm),
            "drb_exchange_rccl_counted")

    def exchange_rccl(self, comm, leader_mask):
        """drb_exchange_rccl over an ncclComm_t (an address)."""
        _ck(lib().drb_exchange_rccl(self.h, comm, leader_mask),
            "drb_exchange_rccl")

    def exchange_rccl_roles(self, comm):
        m = U32()
        _ck(lib().drb_exchange_rccl_roles(self.h, comm, C.byref(m)),
            "drb_exchange_rccl_roles")
        return m.value

    def exchange_mark(self):
        """This rank's own exchange of the last round is enqueued (RCCL):
        ingest may write the remote planes again (drb_exchange_mark)."""
        _ck(lib().drb_exchange_mark(self.h), "drb_exchange_mark")

    def serve_reads(self, reads_per_ctx=9, key_space=256):
        _ck(lib().drb_serve_reads(self.h, reads_per_ctx, key_space),
            "drb_serve_reads")

    def export_read_sums(self, first_group, n_groups):
        arr = (U64 * (n_groups * self.R))()
        _ck(lib().drb_export_read_sums(self.h, first_group, n_groups, arr),
            "drb_export_read_sums")
        return list(arr)

    def kv_lookup(self, g, slot, key):
        vcap = self.cfg["kv_val_cap"]
        val = (C.c_uint8 * vcap)()
        vl = U32()
        rc = _ck(lib().drb_kv_lookup(self.h, g, slot, _u8(key), len(key),
                                     val, vcap, C.byref(vl)), "drb_kv_lookup")
        return None if rc == 1 else bytes(val[:vl.value])

    def encode_wire(self, from_slot, to_slot, deployment_id=0,
                    source=b"", bin_ver=210, max_batch=0, fetch=True):
        """drb_encode_wire: the TCP byte stream (framed MessageBatches) of
        the messages slot from_slot sent to slot to_slot last round.
        Returns (WireOut dict, bytes or None)."""
        cfg = WireCfg(deployment_id, source, len(source), bin_ver, max_batch)
        out = WireOut()
        _ck(lib().drb_encode_wire(self.h, from_slot, to_slot, C.byref(cfg),
                                  C.byref(out)), "drb_encode_wire")
        res = {f: getattr(out, f) for f, _ in WireOut._fields_}
        if not fetch:
            return res, None
        buf = (C.c_uint8 * max(1, out.n_bytes))()
        n = SZ()
        _ck(lib().drb_export_wire(self.h, buf, out.n_bytes, C.byref(n)),
            "drb_export_wire")
        return res, bytes(buf[:n.value])

    def ingest_wire(self, data, deployment_id=0):
        """drb_ingest_wire: a TCP byte stream of framed MessageBatches."""
        res = WireIn()
        # the bytes object's own buffer (no copy: a C3 plane is ~400 MB)
        buf = C.cast(C.c_char_p(bytes(data)), PU8) if data else _u8(b"")
        _ck(lib().drb_ingest_wire(self.h, buf, len(data), deployment_id,
                                  C.byref(res)), "drb_ingest_wire")
        return {f: getattr(res, f) for f, _ in WireIn._fields_}

    def ingest_wire_cpu(self):
        """drb_ingest_wire_cpu: [(offset, length, fate)] of the last
        drb_ingest_wire stream's CPU-path messages, in stream order."""
        n = SZ()
        rc = lib().drb_ingest_wire_cpu(self.h, None, 0, C.byref(n))
        if rc not in (abi.DRB_OK, abi.DRB_ERANGE):
            _ck(rc, "drb_ingest_wire_cpu")
        arr = (WireCpu * max(1, n.value))()
        _ck(lib().drb_ingest_wire_cpu(self.h, arr, n.value, C.byref(n)),
            "drb_ingest_wire_cpu")
        return [(arr[i].offset, arr[i].length, arr[i].fate)
                for i in range(n.value)]

    def ingest_buffer(self, data):
        """Copies data into the engine's pinned receive buffer
        (drb_ingest_buffer), as a transport reading its connection into it
        would; returns the buffer pointer for ingest_wire_pinned."""
        ptr = PU8()
        _ck(lib().drb_ingest_buffer(self.h, max(1, len(data)), C.byref(ptr)),
            "drb_ingest_buffer")
        C.memmove(ptr, bytes(data), len(data))
        return ptr

    def ingest_buffer_alloc(self, cap):
        """A pinned receive buffer of this caller's own
        (drb_ingest_buffer_alloc); free it with ingest_buffer_free."""
        ptr = PU8()
        _ck(lib().drb_ingest_buffer_alloc(self.h, max(1, cap), C.byref(ptr)),
            "drb_ingest_buffer_alloc")
        return ptr

    def ingest_buffer_free(self, ptr):
        _ck(lib().drb_ingest_buffer_free(self.h, ptr),
            "drb_ingest_buffer_free")

    def ingest_wire_pinned(self, ptr, n, deployment_id=0):
        """drb_ingest_wire of n bytes already in the pinned buffer."""
        res = WireIn()
        _ck(lib().drb_ingest_wire(self.h, ptr, n, deployment_id,
                                  C.byref(res)), "drb_ingest_wire")
        return {f: getattr(res, f) for f, _ in WireIn._fields_}

    # ---------------------------------------------------------- step worker
    def worker_bufs(self, reads_cap, values_cap, deferred_cap, lanes=None):
        """A drb_worker_bufs over fresh pinned host buffers (drb_host_alloc);
        free them with free_worker_bufs.  lanes: the lanes word capacity
        (default: every lane)."""
        b = abi.WorkerBufs()
        nl = self.G if lanes is None else lanes
        for name, typ, n, cap in (
                ("lanes", C.c_uint32, nl, nl),
                ("reads", C.c_uint32, reads_cap, reads_cap),
                ("values", C.c_uint32, values_cap, values_cap),
                ("value_meta", C.c_uint8, (values_cap + 3) // 4, None),
                ("deferred", C.c_uint64, deferred_cap, deferred_cap)):
            p = P()
            _ck(lib().drb_host_alloc(self.h, max(1, n) * C.sizeof(typ),
                                     C.byref(p)), "drb_host_alloc")
            setattr(b, name, C.cast(p, C.POINTER(typ)))
            if cap is not None:
                setattr(b, name + "_cap", cap)
        return b

    def free_worker_bufs(self, b):
        for name in ("lanes", "reads", "values", "value_meta", "deferred"):
            _ck(lib().drb_host_free(self.h, C.cast(getattr(b, name), P)),
                "drb_host_free")

    def worker_export(self, slot, b, n_parts=1, part=0):
        """drb_worker_export(_part): enqueue the last round's outputs of
        replica slot `slot` (of one step worker's partition of the shards)
        into b (returns at once)."""
        if n_parts == 1:
            _ck(lib().drb_worker_export(self.h, slot, C.byref(b)),
                "drb_worker_export")
        else:
            _ck(lib().drb_worker_export_part(self.h, slot, n_parts, part,
                                             C.byref(b)),
                "drb_worker_export_part")

    def worker_wait(self, b):
        """drb_worker_wait: (n_reads, n_values, n_deferred); raises when a
        count exceeded its buffer."""
        _ck(lib().drb_worker_wait(self.h, C.byref(b)), "drb_worker_wait")
        return b.n_reads, b.n_values, b.n_deferred

    def crc32_batch(self, buffers):
        data = b"".join(buffers)
        offs, lens, o = [], [], 0
        for b in buffers:
            offs.append(o)
            lens.append(len(b))
            o += len(b)
        n = len(buffers)
        crc = (U32 * max(1, n))()
        _ck(lib().drb_crc32_ieee_batch(self.h, _u8(data), len(data),
                                       (U64 * max(1, n))(*offs),
                                       (U32 * max(1, n))(*lens), n, crc),
            "drb_crc32_ieee_batch")
        return list(crc[:n])
