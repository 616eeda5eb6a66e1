"""GPU: every way a replica leaves the fast path, and the way back.

The engine's contract (include/drb_engine.h): a round that would leave the
fast path marks the replica DRB_F_FALLBACK with a reason BEFORE it mutates
anything, so the exported state is exactly the pre-round state the CPU
raft.Peer continues from; reference panics (plog.Panicf) mark DRB_F_ERROR.
Each test injects one trigger, checks the flag, the reason, the flagged
list (drb_take_flagged) and -- for fallbacks -- that the exported state
equals the oracle's state before that round.  The round-trip tests then
let the oracle (the reference step loop, standing in for the CPU
raft.Peer) step the group through the event and import it back
(drb_import_replicas / drb_import_log), after which the engine continues
bit-exact (node.go:1139-1159, peer.go:64).
"""
import pytest

from dragonboat_amd import abi, workload
from oracle import pyoracle as po
from tests.gpu_harness import Pair, state_diff

pytestmark = pytest.mark.gpu

FB = abi.FB


def _unhost(p, groups, slot):
    for g in groups:
        p.orc.set_hosted(g, slot, False)
        sts = p.eng.export_replicas(g, 1)
        sts[slot].flags &= ~abi.F_HOSTED
        p.eng.import_replicas(g, sts)


def _rehost(p, groups, slot):
    for g in groups:
        p.orc.set_hosted(g, slot, True)
        sts = p.eng.export_replicas(g, 1)
        sts[slot].flags |= abi.F_HOSTED
        p.eng.import_replicas(g, sts)


def _flagged(p):
    recs, lost = p.eng.take_flagged()
    assert lost == 0
    return {(g, s): (reason, flags) for (g, s, reason, flags, _, _) in recs}


def _assert_pre_round(p, snap, flagged):
    """Flagged (fallback) replicas export exactly their pre-round state."""
    for (g, s), (reason, flags) in flagged.items():
        a = p.eng.export_replicas(g, 1)[s]
        assert a.flags & abi.F_FALLBACK and a.fallback_reason == reason
        d = state_diff(a, snap[(g, s)], p.R)
        assert not d, ((g, s), abi.FB_NAME[reason], d)


def _steady(p, rounds, tick=True, k=1, ri=False):
    for _ in range(rounds):
        o, e = p.round(k=k, tick=tick, read_index=ri)
        assert e.fallbacks == 0 and e.errors == 0, e.to_dict()
    assert not p.check()


def _ingest(p, msgs):
    p.orc.ingest(msgs)
    marr, n, earr, pool = po.build_messages(msgs)
    acc, drop = p.eng.ingest(marr, n, earr, pool)
    assert (acc, drop) == (n, 0)


def _round_checked(p, **kw):
    """One round; returns the flagged replicas, checks the flagged ones
    against the pre-round snapshot and every other live one against the
    oracle after the round."""
    snap = p.snapshot()
    o, e = p.round(**kw)
    fl = _flagged(p)
    assert e.fallbacks == sum(1 for v in fl.values()
                              if v[1] & abi.F_FALLBACK)
    _assert_pre_round(p, snap, {k: v for k, v in fl.items()
                                if not v[1] & abi.F_APPLY_STOPPED})
    skip = {g for (g, _) in fl}
    errs = p.check(groups=[g for g in p.live_groups() if g not in skip])
    assert not errs, errs[:2]
    return fl


def _settle_and_return(p, groups, tick_rounds=45, quiet_rounds=25):
    """Step until the oracle settled every CPU group, then import them:
    ticking rounds first (elections need them), then quiet ones (a leader
    without ticks stops sending once its followers caught up)."""
    pending = set(groups)
    for r in range(tick_rounds + quiet_rounds):
        tick = r < tick_rounds
        fl = _round_checked(p, k=1, tick=tick)
        assert not fl, fl
        for g in list(pending):
            if not tick and p.settled(g):
                p.from_cpu(g)
                pending.discard(g)
        if not pending:
            return
    raise AssertionError("CPU groups did not settle: %s %s" % (
        sorted(pending), [p.orc.export(g, s).to_dict(p.R)
                          for g in sorted(pending)[:1] for s in range(p.R)]))


def test_election_fallback_and_round_trip():
    """Followers that stop hearing from their leader reach the randomized
    election timeout (raft.go:598-611): DRB_FB_ELECTION before the
    campaign.  The oracle runs the election (raft.go:1176-1217,
    2235-2253), the group comes back with its new leader at term 3, keeps
    running bit-exact, and the old leader rejoining at term 2 leaves the
    fast path on the new leader's higher-term messages (raft.go:1540-1590)
    and comes back as a follower."""
    p = Pair(G=24, R=3)
    _steady(p, 3)
    E = [1, 6, 11, 20]
    _unhost(p, E, 0)
    seen = {}
    for r in range(40):
        fl = _round_checked(p, k=1, tick=True)
        for (g, s), (reason, flags) in fl.items():
            assert g in E and s != 0, (g, s)
            assert reason == FB["ELECTION"], abi.FB_NAME[reason]
            seen[(g, s)] = reason
            if g not in p.cpu:
                p.to_cpu(g)
        if len(p.cpu) == len(E):
            break
    assert sorted(p.cpu) == E
    _settle_and_return(p, E)
    for g in E:  # a new leader at term 3 on slot 1 or 2
        sts = p.eng.export_replicas(g, 1)
        assert sts[0].term == 2 and sts[0].role == abi.LEADER
        assert {sts[1].role, sts[2].role} == {abi.LEADER, abi.FOLLOWER}
        assert sts[1].term == sts[2].term == 3
    _steady(p, 6, tick=True, ri=True)
    # the old leader rejoins: the new leaders' term-3 messages hand it to
    # the CPU path, which steps it down (becomeFollower)
    _rehost(p, E, 0)
    for r in range(6):
        fl = _round_checked(p, k=1, tick=True)
        for (g, s), (reason, _) in fl.items():
            assert g in E and s == 0
            assert reason in (FB["TERM_MISMATCH"], FB["MESSAGE_TYPE"])
            p.to_cpu(g)
        if len(p.cpu) == len(E):
            break
    assert sorted(p.cpu) == E
    _settle_and_return(p, E)
    for g in E:
        st = p.eng.export_replicas(g, 1)[0]
        assert st.role == abi.FOLLOWER and st.term == 3
    _steady(p, 8, tick=True, ri=True)


def test_check_quorum_fallback_and_round_trip():
    """A leader whose followers stopped responding loses quorum at the
    CheckQuorum tick (raft.go:623-633, 1785-1792): DRB_FB_CHECK_QUORUM;
    the oracle steps it down, the followers come back, elect a leader and
    the group returns to the engine."""
    p = Pair(G=16, R=3)
    _steady(p, 2)
    E = [3, 9]
    _unhost(p, E, 1)
    _unhost(p, E, 2)
    for r in range(30):
        fl = _round_checked(p, k=1, tick=True)
        for (g, s), (reason, _) in fl.items():
            assert (g in E and s == 0), (g, s)
            assert reason == FB["CHECK_QUORUM"], abi.FB_NAME[reason]
            p.to_cpu(g)
        if len(p.cpu) == len(E):
            break
    assert sorted(p.cpu) == E
    _rehost(p, E, 1)
    _rehost(p, E, 2)
    _settle_and_return(p, E)
    _steady(p, 8, tick=True, ri=True)


def test_term_mismatch_from_ingested_messages():
    """A higher-term message at a follower and a lower-term response at a
    leader (raft.go:1540-1590) take the replica off the fast path."""
    p = Pair(G=8, R=3)
    _steady(p, 3)
    _unhost(p, [2, 5], 2)
    st = p.eng.export_replicas(2, 1)[1]
    _ingest(p, [
        po.msg(abi.MSG["Heartbeat"], from_=3, to=2, term=5,
               commit=st.committed, shard_id=1 + 2),
        po.msg(abi.MSG["ReplicateResp"], from_=3, to=1, term=1,
               log_index=1, shard_id=1 + 5)])
    fl = _round_checked(p, k=1, tick=False)
    assert fl == {(2, 1): (FB["TERM_MISMATCH"], abi.F_FALLBACK | 1),
                  (5, 0): (FB["TERM_MISMATCH"], abi.F_FALLBACK | 1)}, fl


def test_off_path_message_type_from_ingest():
    """A RequestVote at the current term (handleNodeRequestVote,
    raft.go:1697-1722) is not a fast-path message: DRB_FB_MESSAGE_TYPE."""
    p = Pair(G=8, R=3)
    _steady(p, 2)
    _unhost(p, [4], 2)
    st = p.eng.export_replicas(4, 1)[1]
    _ingest(p, [po.msg(abi.MSG["RequestVote"], from_=3, to=2, term=2,
                       log_index=st.last_index, log_term=2, shard_id=5)])
    fl = _round_checked(p, k=1, tick=False)
    assert fl == {(4, 1): (FB["MESSAGE_TYPE"], abi.F_FALLBACK | 1)}, fl


def _stage_engine_only(p, group_entries):
    """Proposals staged on the engine alone (the oracle gets none for
    those groups): {g: [Entry dict]}."""
    mp = p.eng.cfg["max_props"]
    ep = po.EntryPool()
    counts = (po.U32 * p.G)()
    slots = [None] * (p.G * mp)
    for g, ents in group_entries.items():
        for j, e in enumerate(ents):
            slots[g * mp + j] = len(ep.items)
            ep.add(**e)
        counts[g] = len(ents)
    arr, pool, n = ep.arrays()
    eents = (abi.Entry * (p.G * mp))()
    for i, x in enumerate(slots):
        if x is not None:
            eents[i] = arr[x]
    p.eng.stage_proposals(1, counts, eents, pool)


@pytest.mark.parametrize("kind", ["session", "snappy", "no_client",
                                  "metadata"])
def test_non_fast_path_proposals_fall_back_before_append(kind):
    """Proposals the rsm fast path cannot apply (regular client session,
    a Snappy-compressed encoded Cmd, a non-empty entry without ClientID,
    a metadata entry; statemachine.go:935-969, encoded.go:55-65) make the
    leader fall back before it appends anything: DRB_FB_ENTRY_TYPE."""
    p = Pair(G=8, R=3, prop_slots=2)
    _steady(p, 2)
    cmd = bytes([0x00]) + po.pbkv_marshal(b"k" * 8, b"vvvv")
    e = po.ent(type=abi.ENTRY_ENCODED, client_id=77, cmd=cmd)
    if kind == "session":
        e["series_id"] = 5
    elif kind == "snappy":
        e["cmd"] = bytes([0x02]) + cmd[1:]  # EESnappy (encoded.go:28-33)
    elif kind == "no_client":
        e["client_id"] = 0
    else:
        e["type"] = abi.ENTRY_METADATA
    _stage_engine_only(p, {3: [e]})
    snap = p.snapshot()
    o = p.orc.round(tick=False)
    out = p.eng.step(tick=False, prop_slot=1)
    p.rounds += 1
    fl = _flagged(p)
    assert fl == {(3, 0): (FB["ENTRY_TYPE"], abi.F_FALLBACK | 1)}, fl
    _assert_pre_round(p, snap, fl)
    assert out.fallbacks == 1
    assert not p.check(groups=[g for g in range(p.G) if g != 3])


def test_oversized_cmd_falls_back_before_append():
    """A staged Cmd longer than cmd_cap (checked per entry by the device
    layout of drb_stage_proposals) sends only its group to the CPU path,
    before the leader appends: DRB_FB_CAPACITY; the other groups step."""
    p = Pair(G=8, R=3, prop_slots=2)
    _steady(p, 2)
    big = bytes([0x00]) + po.pbkv_marshal(b"k" * 8, b"v" * 64)
    assert len(big) > p.eng.cfg["cmd_cap"]
    e = po.ent(type=abi.ENTRY_ENCODED, client_id=77, cmd=big)
    _stage_engine_only(p, {5: [e]})
    snap = p.snapshot()
    p.orc.round(tick=False)
    out = p.eng.step(tick=False, prop_slot=1)
    p.rounds += 1
    fl = _flagged(p)
    assert fl == {(5, 0): (FB["CAPACITY"], abi.F_FALLBACK | 1)}, fl
    _assert_pre_round(p, snap, fl)
    assert out.fallbacks == 1
    assert not p.check(groups=[g for g in range(p.G) if g != 5])


def test_config_change_proposal_round_trip():
    """A ConfigChange proposal (AddNode of an existing member) goes to the
    CPU path before the leader appends (DRB_FB_ENTRY_TYPE); the oracle
    proposes, commits and applies it (raft.go:1794-1815,
    statemachine.go:1006-1019) and the group returns."""
    p = Pair(G=12, R=3, prop_slots=2)
    _steady(p, 2)
    cc = bytes([0x08, 0, 0x10, 0, 0x18, 2, 0x22, 15]) + \
        b"localhost:26001" + bytes([0x28, 1])
    e = po.ent(type=abi.ENTRY_CONFIG_CHANGE, cmd=cc)
    _stage_engine_only(p, {7: [e]})
    snap = p.snapshot()
    p.orc.round(tick=False)
    p.eng.step(tick=False, prop_slot=1)
    p.rounds += 1
    fl = _flagged(p)
    assert fl == {(7, 0): (FB["ENTRY_TYPE"], abi.F_FALLBACK | 1)}, fl
    _assert_pre_round(p, snap, fl)
    # the CPU raft.Peer takes the group: the pre-round state is what the
    # oracle holds, which now handles the proposal itself
    p.to_cpu(7)
    counts = (po.U32 * p.G)()
    counts[7] = 1
    arr, pool, _ = po.EntryPool([e]).arrays()
    ents = (abi.Entry * p.G)()
    ents[7] = arr[0]
    p.orc.stage_proposals(counts, 1, ents, pool)
    _settle_and_return(p, [7])
    st = p.eng.export_replicas(7, 1)[0]
    assert st.role == abi.LEADER and st.sm_index == st.last_index
    _steady(p, 6, tick=True, ri=True)


def test_lagging_follower_beyond_window_falls_back_and_returns():
    """A follower more than W entries behind rejoins: its rejection would
    lower next below the resident window (remote.go:182-198; the
    reference reads LogDB there, logentry.go:180-195), so the replica
    leaves the fast path before anything is sent (DRB_FB_CAPACITY); the
    oracle catches the follower up and the group returns."""
    p = Pair(G=10, R=3, window=8)
    _steady(p, 2, tick=False)
    E = [0, 4, 9]
    _unhost(p, E, 2)
    for r in range(12):  # the leader's window moves on without it
        fl = _round_checked(p, k=1, tick=False)
        assert not fl, fl
    _rehost(p, E, 2)
    for r in range(6):
        fl = _round_checked(p, k=1, tick=False)
        for (g, s), (reason, _) in fl.items():
            assert g in E and s in (0, 2), (g, s)
            assert reason == FB["CAPACITY"], abi.FB_NAME[reason]
            if g not in p.cpu:
                p.to_cpu(g)
        if len(p.cpu) == len(E):
            break
    assert sorted(p.cpu) == E
    _settle_and_return(p, E)
    _steady(p, 10, tick=True)


def test_readindex_queue_capacity():
    """More pending ReadIndex requests than the device queue holds
    (DRB_RI_DEPTH) hand the leader to the CPU path (DRB_FB_CAPACITY)."""
    p = Pair(G=8, R=3)
    _steady(p, 2)
    _unhost(p, [6], 1)
    _unhost(p, [6], 2)
    for r in range(8):
        fl = _round_checked(p, k=0, tick=False, read_index=True)
        if fl:
            assert fl == {(6, 0): (FB["CAPACITY"], abi.F_FALLBACK | 1)}
            st = p.eng.export_replicas(6, 1)[0]
            assert st.ri_count == abi.DRB_RI_DEPTH
            return
    raise AssertionError("no capacity fallback")


def test_snapshot_remote_and_role_fall_back():
    """A leader with a remote in the Snapshot state (remote.go:128-141)
    and a replica in the candidate role are CPU-path states."""
    p = Pair(G=8, R=3)
    _steady(p, 2, tick=False)
    sts = p.eng.export_replicas(2, 1)
    sts[0].remotes[1].state = abi.REMOTE_SNAPSHOT
    p.eng.import_replicas(2, sts)
    pre_leader = p.eng.export_replicas(2, 1)[0]
    sts = p.eng.export_replicas(5, 1)
    sts[2].role = abi.CANDIDATE
    p.eng.import_replicas(5, sts)
    pre_cand = p.eng.export_replicas(5, 1)[2]
    p.eng.step(tick=False)
    fl = _flagged(p)
    assert fl == {(2, 0): (FB["SNAPSHOT"], abi.F_FALLBACK | 1),
                  (5, 2): (FB["ROLE"], abi.F_FALLBACK | 1)}, fl
    for g, s, pre in ((2, 0, pre_leader), (5, 2, pre_cand)):
        a = p.eng.export_replicas(g, 1)[s]
        assert not state_diff(a, pre, 3)


def test_kv_full_stops_apply_after_the_round():
    """The KV table fills (KVTest has no bound; the device table does):
    the raft round completes and the apply stops at that entry
    (DRB_F_APPLY_STOPPED, DRB_FB_CAPACITY); sm_index / kv_count stay at
    the last applied entry and the rest of the state is the oracle's."""
    p = Pair(G=8, R=3, kv_slots=4)
    for r in range(12):
        snap = p.snapshot()
        o, e = p.round(k=1, tick=False)
        fl = _flagged(p)
        for (g, s), (reason, flags) in fl.items():
            assert reason == FB["CAPACITY"]
            assert flags & abi.F_APPLY_STOPPED and flags & abi.F_FALLBACK
            a, b, pre = (p.eng.export_replicas(g, 1)[s], p.orc.export(g, s),
                         snap[(g, s)])
            d = state_diff(a, b, p.R)
            assert set(d) <= {"sm_index", "sm_term", "kv_count"}, d
            assert (a.sm_index, a.kv_count) == (pre.sm_index, pre.kv_count)
            assert a.pushed_index == b.pushed_index > a.sm_index
        if fl:
            return
        assert not p.check()
    raise AssertionError("the KV table never filled")


def test_error_commit_beyond_last():
    """A Heartbeat whose commit is past the follower's log: commitTo
    panics in the reference (logentry.go:336-349) -> DRB_ERR_COMMIT."""
    p = Pair(G=4, R=3)
    _steady(p, 2, tick=False)
    _unhost(p, [1], 0)
    st = p.eng.export_replicas(1, 1)[1]
    _ingest(p, [po.msg(abi.MSG["Heartbeat"], from_=1, to=2, term=2,
                       commit=st.last_index + 5, shard_id=2)])
    with pytest.raises(po.OracleError):
        p.orc.round(tick=False)
    p.eng.step(tick=False)
    fl = _flagged(p)
    assert fl == {(1, 1): (FB["ERR_COMMIT"], abi.F_ERROR | 1)}, fl


def test_error_append_term_regress():
    """Entries whose term is below the last resident entry's:
    checkEntriesToAppend panics (entryutils.go:36-48) -> DRB_ERR_APPEND."""
    p = Pair(G=4, R=3)
    _steady(p, 3, tick=False)
    # the leader leaves this engine; its last messages still arrive (the
    # sender must not be hosted here when the transport delivers for it)
    _unhost(p, [2], 0)
    _round_checked(p, k=0, tick=False)
    st = p.eng.export_replicas(2, 1)[1]  # holds unapplied entries
    assert st.last_index >= st.marker_index
    ent = po.ent(term=1, index=st.last_index + 1, type=abi.ENTRY_ENCODED,
                 client_id=9, cmd=bytes([0]) + po.pbkv_marshal(b"a" * 8,
                                                              b"bbbb"))
    _ingest(p, [po.msg(abi.MSG["Replicate"], from_=1, to=2, term=2,
                       log_index=st.last_index, log_term=2,
                       commit=st.committed, entries=[ent], shard_id=3)])
    with pytest.raises(po.OracleError):
        p.orc.round(tick=False)
    p.eng.step(tick=False)
    fl = _flagged(p)
    assert fl == {(2, 1): (FB["ERR_APPEND"], abi.F_ERROR | 1)}, fl


def test_error_apply_pushed_index():
    """An apply cursor ahead of the committed entries: pb.EntriesToApply
    in strict mode panics (raftpb/entry.go:27-47) -> DRB_ERR_APPLY."""
    p = Pair(G=4, R=3)
    _steady(p, 2, tick=False)
    sts = p.eng.export_replicas(3, 1)
    f = sts[1]
    f.processed = f.committed - 1
    f.pushed_index = f.committed
    p.eng.import_replicas(3, sts)
    p.eng.step(tick=False)
    fl = _flagged(p)
    assert fl == {(3, 1): (FB["ERR_APPLY"], abi.F_ERROR | 1)}, fl


def test_error_readindex_index_moved_backward():
    """A queued ReadIndex whose index is ahead of the commit index a new
    request gets: readIndex.addRequest panics (readindex.go:43-66) ->
    DRB_ERR_READINDEX."""
    p = Pair(G=4, R=3)
    _steady(p, 2, tick=False)
    sts = p.eng.export_replicas(0, 1)
    ld = sts[0]
    ld.ri_count = 1
    ld.ri[0].ctx_low, ld.ri[0].ctx_high = 12345, 7
    ld.ri[0].index = ld.committed + 3
    ld.ri[0].from_ = 0
    p.eng.import_replicas(0, sts)
    lo = (po.U64 * p.G)(99, 0, 0, 0)
    hi = (po.U64 * p.G)(31, 0, 0, 0)
    p.eng.stage_read_index(0, lo, hi)
    p.eng.step(tick=False, ri_slot=0)
    fl = _flagged(p)
    assert fl == {(0, 0): (FB["ERR_READINDEX"], abi.F_ERROR | 1)}, fl


def test_remote_below_window_falls_back_before_reading():
    """A remote whose next lies below the resident window would need
    entries the reference reads from LogDB (logentry.go:180-195): the
    leader's pre-pass hands it to the CPU path (DRB_FB_CAPACITY) instead
    of reading below the window (DRB_ERR_LOG_RANGE, the invariant behind
    it, never fires)."""
    p = Pair(G=4, R=3, window=8)
    _steady(p, 14, tick=False)
    sts = p.eng.export_replicas(1, 1)
    ld = sts[0]
    ld.remotes[2].next = 2
    ld.remotes[2].match = 1
    ld.remotes[2].state = abi.REMOTE_RETRY
    p.eng.import_replicas(1, sts)
    pre = p.eng.export_replicas(1, 1)[0]
    p.eng.step(tick=True)
    fl = _flagged(p)
    assert fl == {(1, 0): (FB["CAPACITY"], abi.F_FALLBACK | 1)}, fl
    assert not state_diff(p.eng.export_replicas(1, 1)[0], pre, 3)
