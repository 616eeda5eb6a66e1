"""Proposals at the leader and at a follower: the reference's KATs restated.

TestProposal (raft_etcd_test.go:1056-1117): a network whose node 1
campaigns, then proposes; the proposal commits on every live peer exactly
when node 1 won the election (a candidate drops it, handleCandidatePropose
raft.go:2197-2201).  TestProposalByProxy (raft_etcd_test.go:1119-1150): the
proposal is made at follower 2, which forwards it to the leader
(handleFollowerPropose, raft.go:2103-2116) -- the path the GPU steps when
drb_round_in.prop_replica names a follower (tests/test_gpu_propose.py).
Every live peer's log is compared as ltoa (raft_etcd_test.go:100-107)
prints it: committed, processed and every entry.
"""
import pytest

from oracle import pyoracle as po
from oracle.pyoracle import ent, msg
from dragonboat_amd.abi import MSG

DATA = b"somedata"


def _ltoa(r):
    return (r.committed, r.info().processed,
            [(e["term"], e["index"], e["cmd"]) for e in r.all_entries()])


def _want(success):
    if not success:
        return (0, 0, [])
    return (2, 0, [(1, 1, b""), (1, 2, DATA)])


@pytest.mark.parametrize("peers,success", [
    ((None, None, None), True),
    ((None, None, "nop"), True),
    ((None, "nop", "nop"), False),
    ((None, "nop", "nop", None), False),
    ((None, "nop", "nop", None, None), True)])
def test_proposal(peers, success):
    net = po.Network(*[po.BlackHole() if p == "nop" else p for p in peers])
    net.send(msg(MSG["Election"], from_=1, to=1))
    net.send(msg(MSG["Propose"], from_=1, to=1, entries=[ent(cmd=DATA)]))
    want = _want(success)
    for i, p in net.peers.items():
        if isinstance(p, po.TestRaft):
            assert _ltoa(p) == want, i
    assert net.peers[1].info().term == 1


@pytest.mark.parametrize("peers", [(None, None, None), (None, None, "nop")])
def test_proposal_by_proxy(peers):
    net = po.Network(*[po.BlackHole() if p == "nop" else p for p in peers])
    net.send(msg(MSG["Election"], from_=1, to=1))
    # propose via follower 2
    net.send(msg(MSG["Propose"], from_=2, to=2, entries=[ent(cmd=DATA)]))
    want = _want(True)
    for i, p in net.peers.items():
        if isinstance(p, po.TestRaft):
            assert _ltoa(p) == want, i
    assert net.peers[1].info().term == 1


def test_follower_without_leader_drops_proposal():
    """handleFollowerPropose with leaderID == NoLeader: reportDroppedProposal,
    nothing is sent (raft.go:2104-2108)."""
    r = po.TestRaft(2, [1, 2, 3], 10, 1)
    r.become_follower(1, 0)
    r.handle(msg(MSG["Propose"], from_=2, to=2, entries=[ent(cmd=DATA)]))
    assert r.read_messages() == []
    assert r.last_index == 0


def test_follower_forwards_proposal_to_its_leader():
    """The forwarded Propose: To = leaderID, From = the follower, Term 0 (a
    request message is sent without a term, raft.go:667-687), the entries
    as proposed (no term, no index)."""
    r = po.TestRaft(2, [1, 2, 3], 10, 1)
    r.become_follower(1, 3)
    r.handle(msg(MSG["Propose"], from_=2, to=2, entries=[ent(cmd=DATA)]))
    ms = r.read_messages()
    assert len(ms) == 1
    m = ms[0]
    assert (m["type"], m["from_"], m["to"], m["term"]) == \
        (MSG["Propose"], 2, 3, 0)
    assert [(e["term"], e["index"], e["cmd"]) for e in m["entries"]] == \
        [(0, 0, DATA)]
