"""GPU: a follower whose log diverges from its leader's is truncated and
overwritten (matchTerm / tryAppend / getConflictIndex,
logentry.go:296-379; inMemory.merge, inmemory.go:199-230).

follower_replicate's conflict branches (drb_step.hpp) run here: the
conflict at or below inMemory.markerIndex (marker and savedTo rewritten,
the window replaced from the conflict on) and the conflict above it (keep
[marker, conflict), savedTo lowered, append).  Every round compares every
field of every replica -- marker_index, saved_to, committed, applied,
sm_index included -- the resident log, the KV, the outboxes and the
ReadyToReads with the oracle cluster, which runs the reference step loop.
"""
import pytest

from dragonboat_amd import abi
from tests import scenarios as sc
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu


def _ok(p, o, e):
    assert e.fallbacks == 0 and e.errors == 0, (p.rounds, e.to_dict(),
                                                p.why())
    assert (e.committed_entries, e.messages) == (o.committed_entries,
                                                 o.messages), \
        (p.rounds, e.to_dict(), o.to_dict())
    errs = p.check()
    assert not errs, (p.rounds, errs[:2])


def _log(p, g, s, span=20):
    """(term, index) of the last `span` entries of replica (g, s)."""
    st = p.eng.export(g, s)
    lo = max(1, st.last_index - span + 1)
    return [(t[0], t[1]) for t in p.eng.export_log(g, s, lo, st.last_index)]


def test_leader_sync_follower_log():
    """LeaderSyncFollowerLog (raft_etcd_paper_test.go:690-770): six groups,
    one per follower log of the reference table.  The leader-to-be (term 8,
    LEAD_ENTS committed) campaigns on the GPU, the third replica's vote is
    ingested (the reference's nopStepper), and the new term-9 leader probes
    each follower back to the matching index and overwrites the rest: the
    shorter logs are appended to, the ones with extra entries at terms 6 /
    7 are cut at 11, and the one diverging at index 4 (terms 2-3) is
    replaced from index 4.  All of it bit-exact with the oracle every
    round; at the end every follower holds LEAD_ENTS and the no-op."""
    G = len(sc.SYNC_CASES)
    p = Pair(G=G, R=3, elections=1)
    before = {}
    for g, tt in enumerate(sc.SYNC_CASES):
        p.import_group(g, sc.sync_follower_group(
            lambda s, g=g: p.orc.export(g, s), tt))
        before[g] = _log(p, g, 1)
        assert before[g] == [(e["term"], e["index"]) for e in tt]
    assert not p.check()
    o, e = p.round(k=0, tick=True)
    _ok(p, o, e)
    for g in range(G):
        st = p.eng.export(g, 0)
        assert (st.role, st.term) == (abi.CANDIDATE, sc.LEAD_TERM + 1)
    shard = [p.eng.export(g, 0).shard_id for g in range(G)]
    acc, drop = p.ingest([sc.vote_from_hole(shard[g]) for g in range(G)])
    assert (acc, drop) == (G, 0)
    for _ in range(30):
        o, e = p.round(k=0, tick=True)
        _ok(p, o, e)
    want = [(e["term"], e["index"]) for e in sc.LEAD_ENTS] + \
        [(sc.LEAD_TERM + 1, len(sc.LEAD_ENTS) + 1)]
    for g in range(G):
        lead, fol = p.eng.export(g, 0), p.eng.export(g, 1)
        assert lead.role == abi.LEADER and fol.role == abi.FOLLOWER
        assert _log(p, g, 0) == want and _log(p, g, 1) == want, g
        assert fol.committed == fol.sm_index == lead.last_index
    # the cases that needed an overwrite (entries not in the leader's log)
    cut = [g for g in range(G) if any(x not in want for x in before[g])]
    assert cut == [2, 3, 4, 5]


def _unhost(p, groups, slot, hosted=False):
    for g in groups:
        p.orc.set_hosted(g, slot, hosted)
        sts = p.eng.export_replicas(g, 1)
        if hosted:
            sts[slot].flags |= abi.F_HOSTED
        else:
            sts[slot].flags &= ~abi.F_HOSTED
        p.eng.import_replicas(g, sts)


def _rounds(p, n, k=1, tick=True, groups=None, ri=True):
    for _ in range(n):
        o, e = p.round(k=k, tick=tick, groups=groups,
                       read_index=ri and p.rounds % 3 == 0)
        _ok(p, o, e)


@pytest.mark.parametrize("pre_vote", [0, 1])
def test_deposed_leader_log_overwritten(pre_vote):
    """LeaderElectionOverwriteNewerLogs on the GPU (raft_etcd_test.go:547
    in spirit): the leader of some groups is cut off while it takes three
    writes nobody acknowledges; its followers elect a new leader among
    themselves (with PreVote a pre-vote round first) and commit new
    entries at term 3; when the old leader returns it steps down and its
    uncommitted term-2 tail is replaced by the new leader's entries.

    E1 groups: the leader's last two writes before the cut reached the
    followers but were never acknowledged (they are kept, the conflict is
    above the old leader's marker -- the "keep [marker, ci)" branch); E2
    groups: everything before the cut was committed and applied (the
    conflict is at the marker -- the replace branch)."""
    p = Pair(G=16, R=3, elections=1, pre_vote=pre_vote)
    _rounds(p, 2)
    E1, E2 = [2, 7, 12], [4, 9]
    E = E1 + E2
    rest = [g for g in range(p.G) if g not in E]
    # two more writes for E1 only; then the leader stops while its
    # followers append the second and answer; then the whole group stops a
    # round (the answers expire): E1's followers hold two entries its
    # leader never saw committed, E2's leader committed and applied all
    _rounds(p, 2, groups=rest + E1)
    _unhost(p, E, 0)
    _rounds(p, 1, groups=rest)
    _unhost(p, E, 1)
    _unhost(p, E, 2)
    _rounds(p, 1, groups=rest)
    # the cut-off leader alone: three writes, no ticks (no CheckQuorum)
    _unhost(p, E, 0, hosted=True)
    _rounds(p, 3, tick=False, ri=False)
    old = {g: p.eng.export(g, 0) for g in E}
    old_log = {g: _log(p, g, 0, 12) for g in E}
    for g in E:
        assert old[g].role == abi.LEADER and old[g].term == 2
        assert old[g].last_index == old[g].committed + (5 if g in E1 else 3)
    # the followers alone: they time out and elect a leader at term 3
    _unhost(p, E, 0)
    _unhost(p, E, 1, hosted=True)
    _unhost(p, E, 2, hosted=True)
    for _ in range(80):
        _rounds(p, 1)
        if all(any(p.eng.export(g, s).role == abi.LEADER for s in (1, 2))
               for g in E):
            break
    _rounds(p, 2)  # writes under the new leaders
    # the old leader returns; no client writes meanwhile, so its log's
    # changed region stays resident while it is compared
    _unhost(p, E, 0, hosted=True)
    ci, new_t = {}, {}
    for _ in range(40):
        _rounds(p, 1, k=0)
        for g in E:
            if g in ci:
                continue
            ot = dict((i, t) for t, i in old_log[g])
            st = p.eng.export(g, 0)
            lo, hi = min(ot), min(max(ot), st.last_index)
            cur = dict((i, t) for t, i in (
                (e[0], e[1]) for e in p.eng.export_log(g, 0, lo, hi)))
            changed = [i for i in cur if cur[i] != ot[i]]
            if changed:
                ci[g] = min(changed)
                new_t[g] = cur[ci[g]]
        if len(ci) == len(E) and all(
                _log(p, g, 0, 8) == _log(p, g, _leader(p, g), 8) for g in E):
            break
    _rounds(p, 3)
    for g in E:
        st = p.eng.export(g, 0)
        assert st.role == abi.FOLLOWER and st.term >= 3
        # (writes go on: the follower may be a round behind the leader)
        lo = st.last_index - 7
        assert p.eng.export_log(g, 0, lo, st.last_index) == \
            p.eng.export_log(g, _leader(p, g), lo, st.last_index)
        # the conflict index: the first entry of the old leader's log that
        # changed, a term-2 entry replaced by a term >= 3 one
        assert new_t[g] >= 3 and dict(
            (i, t) for t, i in old_log[g])[ci[g]] == 2
        m = old[g].marker_index
        if g in E1:
            assert ci[g] > m, (g, ci[g], m)   # keep [marker, ci), append
        else:
            assert ci[g] == m, (g, ci[g], m)  # replace from the marker


def _leader(p, g):
    lead = [s for s in range(p.R) if p.eng.export(g, s).role == abi.LEADER]
    return lead[-1]
