"""GPU: PreVote against replicas on another NodeHost.

The other NodeHost's replica is unhosted here; its messages arrive through
drb_ingest (decoded pb.Message arrays) or drb_ingest_wire (its TCP bytes,
built by the oracle codec), and the oracle cluster takes the same messages
(orc_cluster_ingest).  Covered, each bit-exact with the oracle every round:

- a RequestPreVote at term + 1 to a leader and to a follower that hear from
  their leader: dropped by the CheckQuorum lease
  (dropRequestVoteFromHighTermNode, raft.go:1507-1529);
- a RequestPreVote at a lower term: answered with NoOP (raft.go:1574-1584);
- a RequestPreVote at the current term: rejected at the receiver's term
  (handleNodeRequestPreVote, raft.go:1670-1695);
- a granted RequestPreVoteResp above the term at a follower: let through
  the term gate (isPreVoteMessageWithExpectedHigherTerm, raft.go:1531-1534)
  and ignored by the follower's handlers;
- a preVoteCandidate that a quorum of remote replicas rejects goes back to
  follower at its term (handlePreVoteCandidateRequestPreVoteResp,
  raft.go:2259-2276).
"""
import pytest

from dragonboat_amd import abi
from oracle import pyoracle as po
from tests import wire_ref as wr
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu

MSG = abi.MSG
DID = 0xD1D


def _unhost(p, groups, slot):
    for g in groups:
        p.orc.set_hosted(g, slot, False)
        sts = p.eng.export_replicas(g, 1)
        sts[slot].flags &= ~abi.F_HOSTED
        p.eng.import_replicas(g, sts)


def _deliver(p, msgs, via):
    """The same messages from unhosted replicas into both sides."""
    p.orc.ingest(msgs)
    if via == "ingest":
        marr, n, earr, pool = po.build_messages(msgs)
        p.eng.ingest(marr, n, earr, pool)
    else:
        data = wr.expected_stream(msgs, DID, b"10.0.0.9:26001")
        got = p.eng.ingest_wire(data, DID)
        assert got["accepted"] == len(msgs), got


def _round(p, k=1, groups=None, tick=True):
    o, e = p.round(k=k, tick=tick, groups=groups)
    assert e.fallbacks == 0 and e.errors == 0, (p.rounds, e.to_dict(),
                                                 p.why())
    assert (e.committed_entries, e.messages) == (o.committed_entries,
                                                 o.messages), \
        (p.rounds, e.to_dict(), o.to_dict())
    errs = p.check()
    assert not errs, (p.rounds, errs[:2])
    return e


@pytest.mark.parametrize("via", ["ingest", "wire"])
def test_prevotes_from_another_nodehost(via):
    G, R = 20, 3
    p = Pair(G=G, R=R, elections=1, pre_vote=1)
    for _ in range(3):
        _round(p)
    # slot 2 (replica 3) of every group lives on another NodeHost
    _unhost(p, range(G), 2)
    _round(p)
    msgs = []
    for g in range(G):
        lead = p.eng.export_replicas(g, 1)[0]
        t, last, sid = lead.term, lead.last_index, g + 1
        kind = g % 5
        if kind == 0:    # term + 1 at the leader: the lease drops it
            msgs.append(po.msg(MSG["RequestPreVote"], from_=3, to=1,
                               term=t + 1, log_index=last, log_term=t,
                               shard_id=sid))
        elif kind == 1:  # term + 1 at a follower in its lease: dropped
            msgs.append(po.msg(MSG["RequestPreVote"], from_=3, to=2,
                               term=t + 1, log_index=last, log_term=t,
                               shard_id=sid))
        elif kind == 2:  # a lower term: NoOP back
            msgs.append(po.msg(MSG["RequestPreVote"], from_=3, to=2,
                               term=t - 1, log_index=last, log_term=t - 1,
                               shard_id=sid))
        elif kind == 3:  # the current term: rejected at the receiver's
            msgs.append(po.msg(MSG["RequestPreVote"], from_=3, to=2,
                               term=t, log_index=last, log_term=t,
                               shard_id=sid))
        else:            # a stale granted pre-vote at a follower: ignored
            msgs.append(po.msg(MSG["RequestPreVoteResp"], from_=3, to=2,
                               term=t + 1, shard_id=sid))
    _deliver(p, msgs, via)
    e = _round(p)
    assert e.elections_stepped > 0
    for g in range(G):  # nobody moved: same term, same leader
        sts = p.eng.export_replicas(g, 1)
        assert [s.role for s in sts[:2]] == [abi.LEADER, abi.FOLLOWER], g
        assert sts[0].term == sts[1].term == 2, g
    for _ in range(4):
        _round(p)


@pytest.mark.parametrize("via", ["ingest", "wire"])
def test_prevote_candidate_rejected_by_remote_quorum(via):
    """R = 5: the leader (replica 1) stops and replicas 4, 5 live on another
    NodeHost, so the hosted followers 2, 3 time out and campaign for
    pre-votes; the remote replicas 1, 4, 5 reject them at the candidate's
    term, a rejecting quorum, and the candidate steps back to follower."""
    G, R = 12, 5
    p = Pair(G=G, R=R, elections=1, pre_vote=1)
    for _ in range(3):
        _round(p)
    for s in (0, 3, 4):
        _unhost(p, range(G), s)
    rejected = set()
    for _ in range(40):
        _round(p, k=0)
        msgs = []
        for g in range(G):
            for s in (1, 2):
                st = p.orc.export(g, s)
                if st.role == abi.PREVOTE_CANDIDATE and g not in rejected:
                    msgs += [po.msg(MSG["RequestPreVoteResp"], from_=f,
                                    to=s + 1, term=st.term, reject=True,
                                    shard_id=g + 1) for f in (1, 4, 5)]
                    rejected.add(g)
        if msgs:
            _deliver(p, msgs, via)
            _round(p, k=0)
        if len(rejected) >= G // 2:
            break
    assert rejected
    for _ in range(3):
        _round(p, k=0)
