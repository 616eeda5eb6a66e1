"""NonVoting and witness members: the reference's KATs restated.

Sources (/root/reference/internal/raft/raft_test.go):
  :499  TestNonVotingReplication
  :534  TestNonVotingCanPropose
  :576  TestNonVotingCanReadIndexQuorum1
  :618  TestNonVotingCanReadIndexQuorum2
  :968  TestWitnessReplication
  :985  TestApplicationMessageSentToWitnessIsEmpty
  :1088 TestWitnessCannotReadIndex
They pin the oracle's member kinds (oracle/raft_oracle.c rem_kind): a
nonVoting is replicated but neither counted in the commit quorum nor sent
ReadIndex heartbeats; a witness counts in the quorum and is sent metadata
entries only (makeMetadataEntries, raft.go:771-785).  The GPU path is then
checked against this oracle (tests/test_gpu_members.py).
"""
from oracle import pyoracle as po
from oracle.pyoracle import ent, msg
from dragonboat_amd.abi import MSG, LEADER, FOLLOWER, NONVOTING, WITNESS

TR = po.TestRaft


def _nonvoting_pair():
    p1 = TR.with_kind(1, [], [1, 2], TR.NONVOTING, 10, 1)
    p2 = TR.with_kind(2, [], [1, 2], TR.NONVOTING, 10, 1)
    p1.add_node(1)
    p2.add_node(1)
    assert p1.info().role == FOLLOWER  # p1 is no longer nonVoting
    assert p2.info().role == NONVOTING
    nt = po.Network(p1, p2)
    assert p1.remote_kind(1) == TR.VOTING and p1.remote_kind(2) == \
        TR.NONVOTING
    return p1, p2, nt


def _tick_past_timeout(p1, nt=None):
    for _ in range(p1.info().randomized_election_timeout + 1):
        p1.tick()
        if nt is not None:
            nt.send(msg(MSG["NoOP"], from_=1, to=1))


def test_nonvoting_replication():  # raft_test.go:499-532
    p1, p2, nt = _nonvoting_pair()
    _tick_past_timeout(p1)
    assert p1.info().role == LEADER
    committed = p1.committed
    nt.send(msg(MSG["Propose"], from_=1, to=1,
                entries=[ent(cmd=b"test-data")]))
    assert p1.committed == committed + 1
    # the no-op blank entry appended after p1 became leader is replicated too
    assert p2.committed == committed + 1
    assert p1.remote(2).match == committed + 1


def test_nonvoting_can_propose():  # raft_test.go:534-574
    p1, p2, nt = _nonvoting_pair()
    nt.send(msg(MSG["Election"], from_=1, to=1))
    assert p1.info().role == LEADER
    _tick_past_timeout(p1, nt)
    assert p2.info().role == NONVOTING
    committed = p1.committed
    for _ in range(10):
        nt.send(msg(MSG["Propose"], from_=2, to=2,
                    entries=[ent(cmd=b"test-data")]))
    assert p1.committed == committed + 10
    assert p2.committed == committed + 10
    assert p1.remote(2).match == committed + 10


def test_nonvoting_can_read_index_quorum1():  # raft_test.go:576-616
    p1, p2, nt = _nonvoting_pair()
    nt.send(msg(MSG["Election"], from_=1, to=1))
    assert p1.info().role == LEADER
    _tick_past_timeout(p1, nt)
    committed = p1.committed
    for _ in range(10):
        nt.send(msg(MSG["Propose"], from_=2, to=2,
                    entries=[ent(cmd=b"test-data")]))
    assert p1.committed == committed + 10
    # a single voting member: ReadyToRead at once, a ReadIndexResp to the
    # nonVoting requester (raft.go:1861-1873)
    nt.send(msg(MSG["ReadIndex"], from_=2, to=2, hint=12345))
    rtr = p2.ready_to_read()
    assert len(rtr) == 1 and rtr[0][0] == p1.committed


def test_nonvoting_can_read_index_quorum2():  # raft_test.go:618-660
    p1 = TR(1, [1, 2], 10, 1)
    p2 = TR(2, [1, 2], 10, 1)
    p3 = TR.with_kind(3, [1, 2], [3], TR.NONVOTING, 10, 1)
    p1.add_nonvoting(3)
    p2.add_nonvoting(3)
    nt = po.Network(p1, p2, p3)
    nt.send(msg(MSG["Election"], from_=1, to=1))
    assert p1.info().role == LEADER
    assert p2.info().role == FOLLOWER
    assert p3.info().role == NONVOTING
    _tick_past_timeout(p1, nt)
    committed = p1.committed
    for _ in range(10):
        nt.send(msg(MSG["Propose"], from_=2, to=2,
                    entries=[ent(cmd=b"test-data")]))
    assert p1.committed == committed + 10
    nt.send(msg(MSG["ReadIndex"], from_=3, to=3, hint=12345))
    rtr = p3.ready_to_read()
    assert len(rtr) == 1 and rtr[0][0] == p1.committed


def _leader_and_witness():  # setUpLeaderAndWitness, raft_test.go:1062-1086
    leader = TR(1, [1, 2], 10, 1)
    witness = TR.with_kind(2, [], [2], TR.WITNESS, 10, 1)
    leader.add_witness(2)
    witness.add_node(1)
    assert witness.info().role == WITNESS
    nt = po.Network(leader, witness)
    assert leader.remote_kind(2) == TR.WITNESS
    nt.send(msg(MSG["Election"], from_=1, to=1))
    assert leader.info().role == LEADER
    _tick_past_timeout(leader, nt)
    assert witness.info().role == WITNESS
    return leader, witness, nt


def test_witness_replication():  # raft_test.go:968-983
    leader, witness, nt = _leader_and_witness()
    committed = leader.committed
    nt.send(msg(MSG["Propose"], from_=1, to=1,
                entries=[ent(cmd=b"test-data")]))
    assert leader.committed == committed + 1
    assert witness.committed == committed + 1
    assert leader.remote(2).match == committed + 1


def test_application_message_sent_to_witness_is_empty():
    # raft_test.go:985-1002
    _, witness, _ = _leader_and_witness()
    e = witness.all_entries()[0]
    assert (e["type"], e["term"], e["index"], e["cmd"], e["key"],
            e["client_id"]) == (3, 1, 1, b"", 0, 0)  # MetadataEntry


def test_witness_cannot_read_index():  # raft_test.go:1088-1096
    witness = TR.with_kind(1, [], [1], TR.WITNESS, 10, 1)
    nt = po.Network(witness)
    nt.send(msg(MSG["ReadIndex"], from_=1, to=1, hint=12345))
    assert witness.ready_to_read() == []
