"""GPU: nonVoting and witness members (drb_config.nonvoting_slots /
witness_slots).

A nonVoting member is replicated but not counted in the commit quorum, is
sent no ReadIndex heartbeats (their ctx), never campaigns, and forwards its
proposals and ReadIndex requests to the leader (raft.go:2396-2407,
handleNonVoting*, raft.go:2046-2082).  A witness is counted in the quorum
and votes but is sent metadata entries only (makeMetadataEntries,
raft.go:771-785), never campaigns and neither proposes nor reads
(ErrInvalidOperation, node.go:425-429).  Quorum = voting members / 2 + 1
(raft.go:385-393).  Every round is compared with the oracle cluster, whose
member kinds are pinned by the reference's KATs
(tests/test_oracle_members_kat.py): every replica field, the logs (a
witness's metadata entries), the KV, the outboxes and the ReadyToReads.
"""
import pytest

from dragonboat_amd import abi
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu

NV = 3  # the member slot of the 3+1 tests (replica ID 4)


def _round(p, stats=None, **kw):
    o, e = p.round(**kw)
    assert e.fallbacks == 0 and e.errors == 0, (p.rounds, e.to_dict(),
                                                 p.why())
    assert (e.committed_entries, e.messages, e.dropped_proposals) == \
        (o.committed_entries, o.messages, o.dropped_proposals), \
        (p.rounds, e.to_dict(), o.to_dict())
    errs = p.check()
    assert not errs, (p.rounds, errs[:2])
    if stats is not None:
        stats["committed"] += e.committed_entries
        stats["slow"] += e.elections_stepped
    return e


def _roles(p, g):
    return [x.role for x in p.eng.export_replicas(g, 1)]


def test_witness_replication_and_reads():
    """3 voters + 1 witness (quorum 3 of 4): proposals at the leader commit
    with the witness's responses counted; its log holds metadata entries;
    ReadIndex at the leader and at a follower is confirmed by a quorum that
    counts the witness."""
    G, R = 96, 4
    p = Pair(G=G, R=R, witness_slots=1 << NV)
    assert _roles(p, 0)[NV] == abi.WITNESS
    st = {"committed": 0, "slow": 0}
    for r in range(14):
        _round(p, st, k=1 + r % 2, tick=(r % 2 == 0), read_index=(r % 3 != 2),
               ri_replica=[0, 2][r % 2])
    assert st["committed"] > G * 15, st
    # the witness applied every entry it knows committed, as a no-op (no
    # KV); its commit index trails the leader's by the round in flight
    w = p.eng.export_replicas(0, 1)[NV]
    assert w.sm_index == w.committed > 0
    assert p.eng.kv_export(0, NV) == {}
    e = p.eng.export_log(0, NV, w.last_index, w.last_index)[0]
    assert e[2] == abi.ENTRY_METADATA and e[3:] == (0, 0, 0, 0, b""), e


def test_witness_cannot_propose_or_read():
    """Proposals or ReadIndex staged at a witness: ErrInvalidOperation
    (node.go:425-429, nodehost.go:823, 909) -- the round is refused."""
    G, R = 16, 4
    p = Pair(G=G, R=R, witness_slots=1 << NV, forward_proposals=1,
             max_props=1, mailbox=16)
    _round(p, k=1, tick=True)
    with pytest.raises(Exception):
        p.eng.step(prop_slot=abi.DRB_NONE, ri_slot=abi.DRB_NONE,
                   prop_replica=NV + 1)
    with pytest.raises(Exception):
        p.eng.step(prop_slot=abi.DRB_NONE, ri_slot=abi.DRB_NONE,
                   ri_replica=NV + 1)


def test_nonvoting_replication_proposals_and_reads():
    """3 voters + 1 nonVoting (quorum 2 of 3): the nonVoting is replicated
    but not counted; proposals and ReadIndex made at it are forwarded to
    the leader (handleNonVotingPropose / handleNonVotingReadIndex) and its
    ReadyToReads come back as ReadIndexResp; the leader's ReadIndex
    heartbeats skip it."""
    G, R = 96, 4
    p = Pair(G=G, R=R, nonvoting_slots=1 << NV, forward_proposals=1,
             max_props=2, mailbox=16)
    assert _roles(p, 0)[NV] == abi.NONVOTING
    st = {"committed": 0, "slow": 0}
    for r in range(16):
        _round(p, st, k=1 + r % 2, tick=(r % 2 == 0), read_index=(r % 3 != 2),
               ri_replica=[0, NV + 1, 2][r % 3],
               prop_replica=[0, NV + 1][r % 2])
    assert st["committed"] > G * 12, st
    lead, nv = p.eng.export_replicas(0, 1)[0], p.eng.export_replicas(0, 1)[NV]
    assert nv.sm_index == lead.committed
    assert p.eng.kv_export(0, NV) == p.eng.kv_export(0, 0)


@pytest.mark.parametrize("pre_vote", [0, 1])
def test_nonvoting_not_in_the_quorum(pre_vote):
    """A stopped voter: the leader, one voter and the nonVoting -- 2 of 3
    voters still commit.  Then a second voter stops: the nonVoting's
    acknowledgements do not make a quorum, nothing commits, and CheckQuorum
    steps the leader down (raft launch); with PreVote the remaining voters'
    pre-vote campaigns find no quorum either."""
    G, R = 32, 4
    p = Pair(G=G, R=R, nonvoting_slots=1 << NV, elections=1,
             pre_vote=pre_vote)
    st = {"committed": 0, "slow": 0}
    for r in range(3):
        _round(p, st, k=1, tick=True)
    for g in range(G):
        p.orc.set_hosted(g, 2, False)
    p.eng.host_slot(2, False)
    c0 = st["committed"]
    for r in range(6):
        _round(p, st, k=1, tick=(r % 2 == 0), read_index=True)
    assert st["committed"] - c0 >= G * 5, st
    for g in range(G):
        p.orc.set_hosted(g, 1, False)
    p.eng.host_slot(1, False)
    for r in range(3):  # what slot 1 acknowledged before it stopped commits
        _round(p, st, k=1, tick=True)
    c1 = p.eng.export_replicas(0, 1)[0].committed
    for r in range(30):
        _round(p, st, k=1 if r < 3 else 0, tick=True)
    sts = p.eng.export_replicas(0, 1)
    assert sts[0].committed == c1
    assert sts[NV].role == abi.NONVOTING and sts[0].role != abi.LEADER


@pytest.mark.parametrize("pre_vote", [0, 1])
@pytest.mark.parametrize("kind", ["witness", "nonvoting"])
def test_member_never_campaigns(kind, pre_vote):
    """The leader stops: a voter is elected; the member keeps its role (a
    witness votes and grants pre-votes -- the any-state RequestPreVote
    branch of the passive roles, raft.go:1670-1695 --, a nonVoting does
    neither) and follows the new leader."""
    G, R = 24, 4
    kw = {kind + "_slots": 1 << NV}
    p = Pair(G=G, R=R, elections=1, pre_vote=pre_vote, **kw)
    want = abi.WITNESS if kind == "witness" else abi.NONVOTING
    st = {"committed": 0, "slow": 0}
    for r in range(3):
        _round(p, st, k=1, tick=True)
    for g in range(G):
        p.orc.set_hosted(g, 0, False)
    p.eng.host_slot(0, False)
    elected = False
    for r in range(80):
        _round(p, st, k=0, tick=True)
        roles = [_roles(p, g) for g in range(G)]
        assert all(rs[NV] == want for rs in roles)
        if all(abi.LEADER in rs[1:NV] for rs in roles):
            elected = True
            break
    assert elected and st["slow"] > 0, st
    for r in range(6):
        _round(p, st, k=1, tick=(r % 2 == 0), read_index=True,
               ri_replica=0)


@pytest.mark.parametrize("pre_vote", [0, 1])
def test_witness_vote_makes_the_quorum(pre_vote):
    """Two voters and a witness (quorum 2 of 3): when the leader stops, the
    remaining voter wins only with the witness's pre-vote (PreVote) and
    vote -- the witness's term gate and vote handlers decide the election
    (raft.go:1507-1590, 1670-1722), bit-exact with the oracle."""
    G, R = 24, 3
    p = Pair(G=G, R=R, elections=1, witness_slots=1 << 2, pre_vote=pre_vote)
    st = {"committed": 0, "slow": 0}
    for r in range(3):
        _round(p, st, k=1, tick=True)
    for g in range(G):
        p.orc.set_hosted(g, 0, False)
    p.eng.host_slot(0, False)
    elected = False
    for r in range(80):
        _round(p, st, k=0, tick=True)
        roles = [_roles(p, g) for g in range(G)]
        assert all(rs[2] == abi.WITNESS for rs in roles)
        if all(rs[1] == abi.LEADER for rs in roles):
            elected = True
            break
    assert elected and st["slow"] > 0, st
    c0 = st["committed"]
    for r in range(6):
        _round(p, st, k=1, tick=(r % 2 == 0), read_index=True,
               ri_replica=0)
    assert st["committed"] - c0 >= G * 3, st


@pytest.mark.parametrize("kind,N", [("witness", 2), ("nonvoting", 3)])
def test_members_under_c4_placement(kind, N):
    """Replicas spread over ranks (C4 placement, drb_exchange_local's pull):
    a 4 + 1 group whose slot 4 is a witness / nonVoting; the metadata
    entries travel in the entry rows of the planes, the quorum is the
    voters'."""
    from tests.gpu_harness import DistPair
    G, R = 40, 5
    p = DistPair(G=G, R=R, N=N, max_props=2, **{kind + "_slots": 1 << 4})
    assert not p.check(), "init"
    for r in range(10):
        o, e = p.round(k=1 + r % 2, tick=(r % 2 == 0),
                       read_index=(r % 3 == 0))
        assert e["fallbacks"] == 0 and e["errors"] == 0, (r, e)
        assert (e["committed_entries"], e["messages"]) == \
            (o.committed_entries, o.messages), (r, e, o.to_dict())
        errs = p.check()
        assert not errs, (r, errs[:3])
