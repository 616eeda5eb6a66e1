"""GPU: elections on the device (drb_config.elections).

The replicas a step round would hand to the CPU path for an election
timeout, a CheckQuorum loss, a term change, a vote message or the candidate
role are stepped by the raft launch instead: campaign (raft.go:1176-1217),
RequestVote / RequestVoteResp (raft.go:1697-1722, 2235-2253), becomeFollower
/ Candidate / Leader (raft.go:961-1050), the term gate with
dropRequestVoteFromHighTermNode and the NoOP answer to a stale leader
(raft.go:1507-1590), CheckQuorum step-down (raft.go:1785-1792).  Every
round is compared with the oracle cluster (the reference step loop) over
every field -- term, vote, role, votes, the randomized timeout and its
generator state included -- the log, the KV, the outboxes and the
ReadyToReads; no replica leaves the GPU.
"""
import pytest

from dragonboat_amd import abi
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu


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


def _rounds(p, n, stats, k=1, tick=True, ri_every=3, groups=None):
    for _ in range(n):
        o, e = p.round(k=k, tick=tick, read_index=(p.rounds % ri_every == 0),
                       groups=groups)
        assert e.fallbacks == 0 and e.errors == 0, (p.rounds, e.to_dict(),
                                                     p.why())
        assert (e.committed_entries, e.messages) == (o.committed_entries,
                                                     o.messages), \
            (p.rounds, e.to_dict(), o.to_dict())
        errs = p.check()
        assert not errs, (p.rounds, errs[:2])
        stats["slow"] += e.elections_stepped
        stats["roles"] += e.role_changes


def _roles(p, g):
    return [(st.role, st.term) for st in p.eng.export_replicas(g, 1)]


@pytest.mark.parametrize("R,pre_vote", [(3, 0), (5, 0), (3, 1), (5, 1)])
def test_leader_loss_elects_on_gpu(R, pre_vote):
    """The leader replica of some groups stops (unhosted): its followers
    time out, campaign at term 3, vote, and a new leader takes over --
    appending its term-start no-op and replicating -- all on the GPU,
    bit-exact with the oracle every round.  The old leader then returns at
    term 2: the new leader's heartbeats make it answer with NoOP or step
    down to follower at term 3 (raft.go:1540-1590)."""
    p = Pair(G=24, R=R, elections=1, pre_vote=pre_vote)
    st = {"slow": 0, "roles": 0}
    _rounds(p, 3, st)
    E = [1, 6, 11, 20]
    _unhost(p, E, 0)
    for _ in range(60):
        _rounds(p, 1, st)
        if all(abi.LEADER in [r for r, _ in _roles(p, g)[1:]] for g in E):
            break
    for g in E:
        roles = _roles(p, g)
        assert roles[0] == (abi.LEADER, 2), roles  # the stopped one
        lead = [s for s in range(1, R) if roles[s][0] == abi.LEADER]
        assert len(lead) == 1 and roles[lead[0]][1] >= 3, roles
    assert st["slow"] > 0 and st["roles"] >= len(E)
    _rounds(p, 8, st)  # writes and reads under the new leaders
    _rehost(p, E, 0)
    _rounds(p, 12, st)
    for g in E:
        roles = _roles(p, g)
        assert roles[0][0] == abi.FOLLOWER and roles[0][1] >= 3, roles
        assert sum(r == abi.LEADER for r, _ in roles) == 1, roles
    _rounds(p, 6, st)


@pytest.mark.parametrize("pre_vote", [0, 1])
def test_check_quorum_step_down_and_reelection(pre_vote):
    """A leader whose followers stopped answering loses quorum at the
    CheckQuorum tick and steps down (becomeFollower at its term); when the
    followers return the group elects again -- possibly several rounds of
    split or rejected votes, with PreVote a pre-vote round before each
    campaign (RequestPreVote at term + 1, the term unchanged until a
    quorum granted it) -- and settles with one leader."""
    p = Pair(G=16, R=3, elections=1, pre_vote=pre_vote)
    st = {"slow": 0, "roles": 0}
    _rounds(p, 2, st)
    E = [3, 9]
    _unhost(p, E, 1)
    _unhost(p, E, 2)
    # no client writes to the cut-off leader: its window would fill with
    # entries nobody acknowledges (the CPU path's, DRB_FB_CAPACITY)
    rest = [g for g in range(p.G) if g not in E]
    for _ in range(30):
        _rounds(p, 1, st, groups=rest)
        if all(_roles(p, g)[0][0] == abi.FOLLOWER for g in E):
            break
    for g in E:
        assert _roles(p, g)[0] == (abi.FOLLOWER, 2), _roles(p, g)
    _rehost(p, E, 1)
    _rehost(p, E, 2)
    for _ in range(80):
        _rounds(p, 1, st, groups=rest)
        if all(sum(r == abi.LEADER for r, _ in _roles(p, g)) == 1
               for g in E):
            break
    for g in E:
        assert sum(r == abi.LEADER for r, _ in _roles(p, g)) == 1
    _rounds(p, 8, st)
    assert st["roles"] > 0


def test_elections_engine_steady_state_matches_plain_engine():
    """With nothing to elect, an elections engine runs the same rounds as a
    plain one: no replica goes to the raft launch."""
    p = Pair(G=32, R=3, elections=1)
    st = {"slow": 0, "roles": 0}
    _rounds(p, 10, st)
    assert st == {"slow": 0, "roles": 0}


def test_role_census_counts_leaders():
    """drb_role_census: per slot, the hosted fast-path replicas by role."""
    p = Pair(G=40, R=3, elections=1)
    st = {"slow": 0, "roles": 0}
    _rounds(p, 2, st)
    c = p.eng.role_census()
    assert c[0][abi.LEADER] == 40 and c[1][abi.FOLLOWER] == 40
    _unhost(p, [5, 7], 0)
    c = p.eng.role_census()
    assert c[0][abi.LEADER] == 38


@pytest.mark.parametrize("pre_vote,listed", [(0, 0), (1, 0), (0, 1)])
def test_quiesced_groups_fail_over(pre_vote, listed):
    """Elections with Quiesce (SURVEY 8d C5's mostly idle groups, F3 + F4):
    every group goes quiet (20 x ElectionRTT idle ticks, quiesce.go:80-82)
    and then loses its leader.  A quiesced follower ticks with
    quiescedTick (raft.go:650-656): it never times out while quiet, so the
    groups stay leaderless -- until a ReadIndex at a follower ends its
    quiesce (node.handleReadIndex -> qs.record, node.go:1296-1298); its
    next tick then campaigns at once (the quiesced ticks counted), on the
    GPU, and the group elects.  Bit-exact with the oracle every checked
    round, listed rounds (C5) included."""
    p = Pair(G=16, R=3, elections=1, quiesce=True, pre_vote=pre_vote)
    st = {"slow": 0, "roles": 0}

    def rounds(n, check_every=1, **kw):
        for _ in range(n):
            o, e = p.round(k=0, tick=True, listed=bool(listed), **kw)
            assert e.fallbacks == 0 and e.errors == 0, (p.rounds, e.to_dict(),
                                                         p.why())
            assert (e.committed_entries, e.messages) == \
                (o.committed_entries, o.messages), (p.rounds, e.to_dict(),
                                                    o.to_dict())
            if p.rounds % check_every == 0:
                errs = p.check()
                assert not errs, (p.rounds, errs[:2])
            st["slow"] += e.elections_stepped
            st["roles"] += e.role_changes

    rounds(230, check_every=23)
    assert all(p.eng.export(g, s).qs_quiesced_since > 0
               for g in range(p.G) for s in range(p.R))
    E = [2, 5, 11]
    _unhost(p, E, 0)
    rounds(40, check_every=4)  # quiet: nobody notices
    for g in E:
        assert [r for r, _ in _roles(p, g)[1:]] == [abi.FOLLOWER] * 2
    assert st["slow"] == 0
    # a read at replica 3 of the leaderless groups wakes that follower
    rounds(1, read_index=True, groups=E, ri_replica=3)
    for _ in range(60):
        rounds(1)
        if all(abi.LEADER in [r for r, _ in _roles(p, g)[1:]] for g in E):
            break
    for g in E:
        roles = _roles(p, g)
        lead = [s for s in (1, 2) if roles[s][0] == abi.LEADER]
        assert len(lead) == 1 and roles[lead[0]][1] >= 3, roles
    assert st["slow"] > 0 and st["roles"] >= len(E)
    rounds(10)


@pytest.mark.parametrize("N,R,G,pre_vote", [(2, 3, 24, 0), (3, 5, 30, 1),
                                            (4, 3, 24, 0), (8, 5, 40, 0)])
def test_failover_with_replicas_spread_over_ranks(N, R, G, pre_vote):
    """Elections under C4 placement (replica slot s of group g on rank
    (g + s) mod N, drb_exchange_local moving the planes between the ranks'
    engines -- what RCCL moves between GPUs): the leader replica of some
    groups stops, its followers on other ranks time out, campaign and elect
    in their raft launches, the votes and the new leader's Replicates and
    entry rows crossing ranks (with the rterm rows of records whose term is
    not their header's).  The old leader then returns and steps down.
    Bit-exact with one oracle cluster of all G groups every round.  Client
    input goes to the groups whose leader stayed at the stage slot
    (drb_stage_proposals stages a lane's batch at slot 0's replica)."""
    from tests.gpu_harness import DistPair
    p = DistPair(G=G, R=R, N=N, max_props=2, elections=1, pre_vote=pre_vote)
    st = {"slow": 0, "roles": 0}
    E = [g for g in range(G) if g % 5 == 2]
    rest = [g for g in range(G) if g not in E]

    def rounds(n, groups=None, k=1):
        for _ in range(n):
            o, e = p.round(k=k, tick=True, read_index=(p.rounds % 3 == 0),
                           groups=groups)
            assert e["fallbacks"] == 0 and e["errors"] == 0, (p.rounds, e,
                                                              p.why())
            assert (e["committed_entries"], e["messages"]) == \
                (o.committed_entries, o.messages), (p.rounds, e, o.to_dict())
            errs = p.check()
            assert not errs, (p.rounds, errs[:2])
            st["slow"] += e["elections_stepped"]
            st["roles"] += e["role_changes"]

    rounds(3)
    for g in E:
        p.set_hosted(g, 0, False)
    for _ in range(60):
        rounds(1, groups=rest)
        if all(any(p.replica(g, s).role == abi.LEADER for s in range(1, R))
               for g in E):
            break
    for g in E:
        lead = [s for s in range(1, R) if p.replica(g, s).role == abi.LEADER]
        assert len(lead) == 1 and p.replica(g, lead[0]).term >= 3, g
    assert st["slow"] > 0 and st["roles"] >= len(E)
    rounds(4, groups=rest)
    for g in E:
        p.set_hosted(g, 0, True)
    rounds(12, groups=rest)
    for g in E:
        roles = [p.replica(g, s).role for s in range(R)]
        assert roles[0] == abi.FOLLOWER and roles.count(abi.LEADER) == 1, \
            (g, roles)
