"""Shared harness for the GPU parity tests: drive the HIP engine and the CPU
oracle with the same inputs and compare everything the round produces.

Parity bar (bit-exact, integer state): every field of drb_replica_state,
the resident log window, the KV contents, the messages each replica sent
(compared per destination, in send order -- the reference's cross-
destination order depends on Go map iteration, raft.go:828) and the
ReadyToRead records.
"""
import ctypes as C

from dragonboat_amd import abi, workload
from dragonboat_amd.engine import Engine
from oracle import pyoracle as po

STATE_FIELDS = [
    "term", "vote", "leader_id", "applied", "election_tick",
    "heartbeat_tick", "randomized_election_timeout", "tick_count",
    "committed", "processed", "last_index", "marker_index", "saved_to",
    "applied_to_index", "applied_to_term", "applied_index",
    "confirmed_index", "pushed_index", "prev_term", "prev_vote",
    "prev_commit", "sm_index", "sm_term", "kv_count", "qs_current_tick",
    "qs_idle_since", "qs_quiesced_since", "qs_exit_quiesce_tick", "rng",
    "role"]


def state_diff(a, b, R):
    d = {}
    for f in STATE_FIELDS:
        if getattr(a, f) != getattr(b, f):
            d[f] = (getattr(a, f), getattr(b, f))
    if a.role == abi.LEADER:
        for s in range(R):
            x, y = a.remotes[s], b.remotes[s]
            if (x.match, x.next, x.state, x.active) != \
                    (y.match, y.next, y.state, y.active):
                d["remote%d" % s] = ((x.match, x.next, x.state, x.active),
                                     (y.match, y.next, y.state, y.active))
    if a.votes != b.votes:
        d["votes"] = (a.votes, b.votes)
    if a.transfer != b.transfer:
        d["transfer"] = (a.transfer, b.transfer)
    if a.ri_count != b.ri_count:
        d["ri_count"] = (a.ri_count, b.ri_count)
    else:
        for i in range(a.ri_count):
            x, y = a.ri[i], b.ri[i]
            tx = (x.ctx_low, x.ctx_high, x.index, x.from_, x.confirmed)
            ty = (y.ctx_low, y.ctx_high, y.index, y.from_, y.confirmed)
            if tx != ty:
                d["ri%d" % i] = (tx, ty)
    return d


def by_dest(msgs):
    out = {}
    for m in msgs:
        out.setdefault(m[2], []).append(m)
    return out


class Pair:
    """An engine and an oracle cluster stepped in lock-step."""

    def __init__(self, G, R=3, seed=0x5EEDD8B0, window=32, leader_slot=0,
                 election_rtt=10, quiesce=False, **engine_kw):
        self.G, self.R, self.seed = G, R, seed
        self.eng = Engine(num_groups=G, num_replicas=R, window=window,
                          election_rtt=election_rtt, quiesce=int(quiesce),
                          **engine_kw)
        self.orc = po.Cluster(G, R, seed=seed, election_rtt=election_rtt,
                              quiesce=quiesce)
        self.orc.setup_steady(leader_slot)
        nv, wt = (engine_kw.get("nonvoting_slots", 0),
                  engine_kw.get("witness_slots", 0))
        if nv or wt:  # member kinds (drb_config.nonvoting_slots, ...)
            self.orc.set_member_kinds(nv, wt)
        if engine_kw.get("pre_vote"):
            self.orc.set_pre_vote(True)
        self.eng.init_steady(term=2, leader_slot=leader_slot, seed=seed)
        self.rounds = 0
        self.cpu = set()  # groups handed to the CPU path (the oracle)

    def stage(self, k=1, salt=None, read_index=False, groups=None,
              key_space=256, val_len=4, prop_slot=0, ri_slot=0,
              ri_replica=0, prop_replica=0):
        salt = self.rounds if salt is None else salt
        pin = ri_in = abi.DRB_NONE
        if self.cpu:  # no client input for groups on the CPU path
            groups = [g for g in (range(self.G) if groups is None else groups)
                      if g not in self.cpu]
        if k:
            counts, ents, pool = workload.build_batch(
                self.G, k, self.seed, salt, key_space, val_len, groups)
            self.orc.stage_proposals(counts, k, ents, pool, prop_replica)
            # the engine's staging layout is [g][max_props]
            mp = self.eng.cfg["max_props"]
            eents = (abi.Entry * (self.G * mp))()
            for g in range(self.G):
                for j in range(counts[g]):
                    eents[g * mp + j] = ents[g * k + j]
            self.eng.stage_proposals(prop_slot, counts, eents, pool)
            pin = prop_slot
        if read_index:
            lo, hi = workload.build_read_index(self.G, self.seed, salt,
                                               salt + 30, groups)
            self.orc.stage_read_index(lo, hi, ri_replica)
            self.eng.stage_read_index(ri_slot, lo, hi)
            ri_in = ri_slot
        return pin, ri_in

    def round(self, k=1, tick=False, read_index=False, groups=None,
              reads=0, read_key_space=256, encode_saves=False, ri_replica=0,
              listed=False, prop_replica=0, **kw):
        pin, ri_in = self.stage(k, read_index=read_index, groups=groups,
                                ri_replica=ri_replica,
                                prop_replica=prop_replica, **kw)
        o = self.orc.round(tick=tick)
        e = self.eng.step(tick=tick, prop_slot=pin, ri_slot=ri_in,
                          reads_per_ctx=reads, key_space=read_key_space,
                          encode_saves=encode_saves, ri_replica=ri_replica,
                          listed=listed, prop_replica=prop_replica)
        self.rounds += 1
        return o, e

    def why(self, n=3):
        """The replicas flagged since the last call, by reason, with the
        first few states (for assertion messages)."""
        recs, lost = self.eng.take_flagged()
        out = {}
        for (g, s, reason, flags, rnd, _) in recs:
            out.setdefault(abi.FB_NAME.get(reason, reason), []).append(
                (g, s, flags, rnd))
        first = [(g, s, self.eng.export_replicas(g, 1)[s].to_dict(self.R))
                 for (g, s, *_r) in recs[:n]]
        return out, lost, first

    def check_saves(self, groups=None):
        """EntriesToSave of the last round: EntryBatch bytes and CRC32."""
        errs = []
        for g in (range(self.G) if groups is None else groups):
            for s in range(self.R):
                eb = self.eng.export_saved(g, s)
                ob = self.orc.export_saved(g, s)
                if eb != ob:
                    errs.append((g, s, "saved", eb, ob))
        return errs

    # ---------------------------------------------- fallback round trip
    # SURVEY 8b "Fallback": a replica the engine flags hands its group to
    # the CPU raft.Peer -- here the oracle, which is the reference step
    # loop -- until the event is over; then the group's state and window
    # are imported back (node.go:1139-1159, peer.go:64).
    def snapshot(self):
        """Oracle states before a round, {(g, s): ReplicaState}."""
        return {(g, s): self.orc.export(g, s)
                for g in range(self.G) for s in range(self.R)}

    def to_cpu(self, g):
        """Every replica of group g leaves the engine (marked FALLBACK)."""
        sts = self.eng.export_replicas(g, 1)
        for st in sts:
            st.flags |= abi.F_FALLBACK
        self.eng.import_replicas(g, sts)
        self.cpu.add(g)

    def settled(self, g):
        """The CPU group has a leader, its log committed and applied
        everywhere, nothing in flight and no readIndex work pending."""
        lead = 0
        for s in range(self.R):
            st = self.orc.export(g, s)
            if not st.flags & abi.F_HOSTED:
                continue
            if st.role == abi.LEADER:
                lead += 1
            elif st.role not in (abi.FOLLOWER, abi.NONVOTING, abi.WITNESS):
                return False
            if self.orc.export_outbox(g, s) or st.ri_count:
                return False
            if not (st.committed == st.last_index == st.processed ==
                    st.sm_index):
                return False
        return lead == 1

    def from_cpu(self, g):
        """Imports group g back from the oracle: states and the resident
        window (the last W entries)."""
        W = self.eng.cfg["window"]
        sts = []
        for s in range(self.R):
            st = self.orc.export(g, s)
            lo = max(1, st.last_index - W + 1)
            ents = self.orc.export_log(g, s, lo, st.last_index)
            ep = po.EntryPool([po._etuple_to_dict(t) for t in ents])
            arr, pool, n = ep.arrays()
            self.eng.import_log(g, s, arr, pool)
            # the state machine comes back with the group (its CPU
            # StateMachine applied what committed meanwhile)
            self.eng.kv_import(g, s, self.orc.export_kv(g, s))
            st.flags &= abi.F_HOSTED
            st.fallback_reason = 0
            sts.append(st)
        self.eng.import_replicas(g, sts)
        self.cpu.discard(g)

    def import_group(self, g, reps):
        """Every replica of group g takes reps[slot] = (ReplicaState, log
        entry dicts from index 1) on both sides: orc_cluster_import and
        drb_import_log + drb_kv_import (empty) + drb_import_replicas."""
        sts = []
        for s, (st, log) in enumerate(reps):
            self.orc.import_replica(g, s, st, log)
            if log:
                ep = po.EntryPool(log)
                arr, pool, n = ep.arrays()
                for i in range(n):
                    arr[i].index = i + 1
                self.eng.import_log(g, s, arr, pool)
            self.eng.kv_import(g, s, {})
            sts.append(st)
        self.eng.import_replicas(g, sts)

    def ingest(self, msgs):
        """The same messages from unhosted senders into both sides
        (drb_ingest / orc_cluster_ingest)."""
        self.orc.ingest(msgs)
        marr, n, earr, pool = po.build_messages(msgs)
        return self.eng.ingest(marr, n, earr, pool)

    def live_groups(self):
        return [g for g in range(self.G) if g not in self.cpu]

    def check(self, groups=None, logs=True, kv=True, msgs=True,
              ready=True):
        errs = []
        gs = self.live_groups() if groups is None else groups
        for g in gs:
            est = self.eng.export_replicas(g, 1)
            for s in range(self.R):
                a, b = est[s], self.orc.export(g, s)
                if a.flags & (abi.F_FALLBACK | abi.F_ERROR):
                    errs.append((g, s, "flags", a.flags, a.fallback_reason))
                    continue
                d = state_diff(a, b, self.R)
                if d:
                    errs.append((g, s, "state", d))
                    continue
                if logs:
                    lo = max(1, b.last_index - self.eng.cfg["window"] + 1)
                    lo = max(lo, b.last_index - 8)
                    el = self.eng.export_log(g, s, lo, b.last_index)
                    ol = self.orc.export_log(g, s, lo, b.last_index)
                    if el != ol:
                        errs.append((g, s, "log", el, ol))
                if kv:
                    ek = self.eng.kv_export(g, s)
                    ok = self.orc.export_kv(g, s)
                    if ek != ok:
                        errs.append((g, s, "kv", len(ek), len(ok)))
                if msgs:
                    em = by_dest(self.eng.export_outbox(g, s))
                    om = by_dest(self.orc.export_outbox(g, s))
                    if em != om:
                        errs.append((g, s, "msgs", em, om))
                if ready:
                    er = self.eng.export_ready(g, s)
                    orr = self.orc.export_ready(g, s)
                    if er != orr:
                        errs.append((g, s, "ready", er, orr))
        return errs


class DistPair:
    """C4 placement on one GPU: N engines (one per rank) hold replica slot s
    of global group g at rank (g + s) mod N, lane g // N (drb_config
    place_world); the mailbox planes move between them after every round
    with drb_exchange_local -- the same regions RCCL moves between GPUs.
    Stepped in lock-step with one oracle cluster of all G groups."""

    def __init__(self, G, R=5, N=8, seed=0x5EEDD8B0, window=32, E=4,
                 counted=False, bound=False, **engine_kw):
        self.G, self.R, self.N, self.seed = G, R, N, seed
        self.counted = counted  # drb_exchange_local_counted
        self.bound = bound  # drb_exchange_local_bind: zero-copy planes
        self.lanes = (G + N - 1) // N
        self.engs = [Engine(num_groups=self.lanes, num_replicas=R,
                            window=window, total_groups=G, place_world=N,
                            place_rank=r, entry_mbox=E, **engine_kw)
                     for r in range(N)]
        self.orc = po.Cluster(G, R, seed=seed)
        self.orc.setup_steady(0)
        nv, wt = (engine_kw.get("nonvoting_slots", 0),
                  engine_kw.get("witness_slots", 0))
        if nv or wt:  # member kinds (drb_config.nonvoting_slots, ...)
            self.orc.set_member_kinds(nv, wt)
        if engine_kw.get("pre_vote"):
            self.orc.set_pre_vote(True)
        for e in self.engs:
            e.init_steady(term=2, leader_slot=0, seed=seed)
        if bound:
            Engine.exchange_local_bind(self.engs)
        self.rounds = 0
        self.cpu = set()  # groups handed to the CPU path (the oracle)

    def set_hosted(self, g, s, hosted):
        """Replica slot s of group g stops (or returns) on both sides."""
        self.orc.set_hosted(g, s, hosted)
        r, j = self.where(g, s)
        sts = self.engs[r].export_replicas(j, 1)
        if hosted:
            sts[s].flags |= abi.F_HOSTED
        else:
            sts[s].flags &= ~abi.F_HOSTED
        self.engs[r].import_replicas(j, sts)

    def why(self):
        """The replicas flagged since the last call on every rank:
        (global group, slot, reason, flags, round)."""
        out = []
        for r, e in enumerate(self.engs):
            recs, _ = e.take_flagged()
            for (j, s, reason, flags, rnd, _) in recs:
                out.append((self.lane_group(r, s, j), s,
                            abi.FB_NAME.get(reason, reason), flags, rnd))
        return out

    def replica(self, g, s):
        r, j = self.where(g, s)
        return self.engs[r].export_replicas(j, 1)[s]

    def where(self, g, s):
        """(rank, lane) of replica slot s of group g."""
        return (g + s) % self.N, g // self.N

    def lane_group(self, r, s, j):
        return self.N * j + (r - s) % self.N

    # ---------------------------------------------- fallback round trip
    # (Pair.to_cpu / settled / from_cpu over the ranks that hold a group)
    def to_cpu(self, g):
        for s in range(self.R):
            r, j = self.where(g, s)
            sts = self.engs[r].export_replicas(j, 1)
            sts[s].flags |= abi.F_FALLBACK
            self.engs[r].import_replicas(j, sts)
        self.cpu.add(g)

    def settled(self, g):
        lead = 0
        for s in range(self.R):
            st = self.orc.export(g, s)
            if not st.flags & abi.F_HOSTED:
                continue
            if st.role == abi.LEADER:
                lead += 1
            elif st.role not in (abi.FOLLOWER, abi.NONVOTING, abi.WITNESS):
                return False
            if self.orc.export_outbox(g, s) or st.ri_count:
                return False
            if not (st.committed == st.last_index == st.processed ==
                    st.sm_index):
                return False
        return lead == 1

    def from_cpu(self, g, W=32):
        """Group g back from the oracle into the replicas the engines host
        (a slot on a CPU NodeHost stays unhosted)."""
        for s in range(self.R):
            r, j = self.where(g, s)
            e = self.engs[r]
            sts = e.export_replicas(j, 1)
            hosted = sts[s].flags & abi.F_HOSTED
            st = self.orc.export(g, s)
            if hosted:
                lo = max(1, st.last_index - W + 1)
                ents = self.orc.export_log(g, s, lo, st.last_index)
                ep = po.EntryPool([po._etuple_to_dict(t) for t in ents])
                arr, pool, n = ep.arrays()
                e.import_log(j, s, arr, pool)
                e.kv_import(j, s, self.orc.export_kv(g, s))
            st.flags = hosted
            st.fallback_reason = 0
            sts[s] = st
            e.import_replicas(j, sts)
        self.cpu.discard(g)

    def exchange(self):
        Engine.exchange_local(self.engs, counted=self.counted)

    def round(self, k=1, tick=False, read_index=False, groups=None,
              exchange=True):
        salt = self.rounds
        if self.cpu:  # no client input for groups on the CPU path
            groups = [g for g in (range(self.G) if groups is None else groups)
                      if g not in self.cpu]
        pin = ri_in = abi.DRB_NONE
        if k:
            counts, ents, pool = workload.build_batch(
                self.G, k, self.seed, salt, 256, 4, groups)
            self.orc.stage_proposals(counts, k, ents, pool)
            for r, e in enumerate(self.engs):
                mp = e.cfg["max_props"]
                ec = (C.c_uint32 * self.lanes)()
                ee = (abi.Entry * (self.lanes * mp))()
                for j in range(self.lanes):
                    g = self.lane_group(r, 0, j)  # the stage slot's group
                    if g >= self.G:
                        continue
                    ec[j] = counts[g]
                    for q in range(counts[g]):
                        ee[j * mp + q] = ents[g * k + q]
                e.stage_proposals(0, ec, ee, pool)
            pin = 0
        if read_index:
            lo, hi = workload.build_read_index(self.G, self.seed, salt,
                                               salt + 30, groups)
            self.orc.stage_read_index(lo, hi)
            for r, e in enumerate(self.engs):
                el = (C.c_uint64 * self.lanes)()
                eh = (C.c_uint64 * self.lanes)()
                for j in range(self.lanes):
                    g = self.lane_group(r, 0, j)
                    if g < self.G:
                        el[j], eh[j] = lo[g], hi[g]
                e.stage_read_index(0, el, eh)
            ri_in = 0
        o = self.orc.round(tick=tick)
        outs = [e.step(tick=tick, prop_slot=pin, ri_slot=ri_in)
                for e in self.engs]
        if exchange:
            self.exchange()
        self.rounds += 1
        tot = {}
        for f in ("committed_entries", "applied_entries", "messages",
                  "ready_to_reads", "fallbacks", "errors",
                  "elections_stepped", "role_changes"):
            tot[f] = sum(getattr(x, f) for x in outs)
        return o, tot

    def check(self, groups=None, logs=True, kv=True, msgs=True, slots=None):
        errs = []
        for g in (range(self.G) if groups is None else groups):
            if g in self.cpu:
                continue
            for s in (range(self.R) if slots is None else slots):
                r, j = self.where(g, s)
                e = self.engs[r]
                a, b = e.export_replicas(j, 1)[s], self.orc.export(g, s)
                if a.flags & (abi.F_FALLBACK | abi.F_ERROR):
                    errs.append((g, s, "flags", a.flags, a.fallback_reason))
                    continue
                d = state_diff(a, b, self.R)
                if a.shard_id != b.shard_id:
                    d["shard_id"] = (a.shard_id, b.shard_id)
                if d:
                    errs.append((g, s, "state", d))
                    continue
                if logs:
                    lo = max(1, b.last_index - 8)
                    if e.export_log(j, s, lo, b.last_index) != \
                            self.orc.export_log(g, s, lo, b.last_index):
                        errs.append((g, s, "log"))
                if kv and e.kv_export(j, s) != self.orc.export_kv(g, s):
                    errs.append((g, s, "kv"))
                if msgs:
                    em = by_dest(e.export_outbox(j, s))
                    om = by_dest(self.orc.export_outbox(g, s))
                    if em != om:
                        errs.append((g, s, "msgs", em, om))
        return errs
