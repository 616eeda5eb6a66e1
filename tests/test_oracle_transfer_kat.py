"""Leader-transfer known-answer tests restated from the reference's own tests.

They pin the oracle's transfer handlers (oracle/raft_oracle.c
handle_leader_transfer, handle_follower_timeout_now, the TimeoutNow trigger
in handle_leader_replicate_resp, the abort in raft_tick and the proposal
drop), which check the GPU raft launch's transfer path
(tests/test_gpu_transfer.py).

Sources (/root/reference/internal/raft/raft_etcd_test.go):
  TestLeaderTransferToUpToDateNode (:156-171), ...FromFollower (:178-192),
  ...WithPreVote (:196-221), ...WithCheckQuorum (:225-249),
  ...ToSlowFollower (:251-276), ...ToSelf (:307-314),
  ...ToNonExistingNode (:316-323), ...Timeout (:325-345),
  ...IgnoreProposal (:347-363), ...ReceiveHigherTermVote (:365-377),
  TestNewLeaderTransferCanNotOverrideOngoingLeaderTransfer (:393-411),
  TestLeaderTransferSecondTransferToSameNode (:415-433).
Not restated: TestLeaderTransferAfterSnapshot (:278-305, snapshots are not
on this path) and TestLeaderTransferRemoveNode (:379-391, membership
changes are not on this path).
"""
import pytest

from dragonboat_amd.abi import FOLLOWER, LEADER, MSG
from oracle.pyoracle import Network, ent, msg

ELECTION = MSG["Election"]
PROPOSE = MSG["Propose"]
TRANSFER = MSG["LeaderTransfer"]
TIMEOUT_NOW = MSG["TimeoutNow"]


def _check_state(r, state, lead):
    """checkLeaderTransferState (raft_etcd_test.go:145-152)."""
    st = r.info()
    assert (st.role, st.leader_id) == (state, lead)
    assert r.peek("leader_transfer_target") == 0


def _elect(nt, id=1):
    nt.send(msg(ELECTION, from_=id, to=id))
    lead = nt.peers[id]
    assert lead.info().leader_id == id
    return lead


def _propose(nt, to=1):
    nt.send(msg(PROPOSE, from_=to, to=to, entries=[ent()]))


def _transfer(nt, frm, to, target):
    nt.send(msg(TRANSFER, from_=frm, to=to, hint=target))


@pytest.mark.parametrize("via_follower", [False, True])
def test_leader_transfer_to_up_to_date_node(via_follower):
    nt = Network(None, None, None)
    lead = _elect(nt)
    # transfer leadership to 2, sent to the leader or to the target itself
    _transfer(nt, 2, 2 if via_follower else 1, 2)
    _check_state(lead, FOLLOWER, 2)
    # after some log replication, transfer leadership back to 1
    _propose(nt)
    _transfer(nt, 1, 1 if via_follower else 2, 1)
    _check_state(lead, LEADER, 1)


@pytest.mark.parametrize("pre_vote", [True, False])
def test_leader_transfer_within_lease(pre_vote):
    """...WithPreVote / ...WithCheckQuorum: the transfer's RequestVote
    carries Hint == From, which passes the voters' leader lease."""
    nt = Network(None, None, None)
    for i in (1, 2, 3):
        r = nt.peers[i]
        r.set_check_quorum(True)
        if pre_vote:
            r.set_pre_vote(True)
        r.set_randomized_election_timeout(10 + i)
    # peer 2's electionTick reaches the timeout so it can vote for peer 1
    f = nt.peers[2]
    for _ in range(10):
        f.tick()
    lead = _elect(nt)
    _transfer(nt, 2, 1, 2)
    _check_state(lead, FOLLOWER, 2)
    _propose(nt)
    _transfer(nt, 1, 2, 1)
    _check_state(lead, LEADER, 1)


def test_leader_transfer_to_slow_follower():
    nt = Network(None, None, None)
    lead = _elect(nt)
    nt.isolate(3)
    _propose(nt)
    nt.recover()
    assert lead.remote(3).match == 1
    # node 3 lacks the log: the leader waits (no Replicate is forced)
    _transfer(nt, 3, 1, 3)
    st = lead.info()
    assert (st.role, st.leader_id) == (LEADER, 1)
    assert lead.peek("leader_transfer_target") == 3  # leaderTransfering()
    lead.poke(leader_transfer_target=0)  # abortLeaderTransfer
    _propose(nt)
    _transfer(nt, 3, 1, 3)
    _check_state(lead, FOLLOWER, 3)


@pytest.mark.parametrize("target", [1, 4])
def test_leader_transfer_to_self_or_unknown_is_noop(target):
    nt = Network(None, None, None)
    lead = _elect(nt)
    _transfer(nt, target, 1, target)
    _check_state(lead, LEADER, 1)


def test_leader_transfer_timeout():
    nt = Network(None, None, None)
    lead = _elect(nt)
    nt.isolate(3)
    _transfer(nt, 3, 1, 3)
    assert lead.peek("leader_transfer_target") == 3
    for _ in range(1):  # heartbeatTimeout
        lead.tick()
    assert lead.peek("leader_transfer_target") == 3
    for _ in range(10):  # electionTimeout
        lead.tick()
    _check_state(lead, LEADER, 1)


def test_leader_transfer_ignore_proposal():
    nt = Network(None, None, None)
    lead = _elect(nt)
    nt.isolate(3)
    _transfer(nt, 3, 1, 3)
    assert lead.peek("leader_transfer_target") == 3
    _propose(nt)
    matched = lead.remote(2).match
    _propose(nt)
    assert lead.remote(2).match == matched
    assert lead.info().last_index == 1  # both proposals dropped


def test_leader_transfer_receive_higher_term_vote():
    nt = Network(None, None, None)
    lead = _elect(nt)
    nt.isolate(3)
    _transfer(nt, 3, 1, 3)
    assert lead.peek("leader_transfer_target") == 3
    nt.send(msg(ELECTION, from_=2, to=2, log_index=1, term=2))
    _check_state(lead, FOLLOWER, 2)


def test_new_transfer_cannot_override_ongoing_transfer():
    nt = Network(None, None, None)
    lead = _elect(nt)
    nt.isolate(3)
    _transfer(nt, 3, 1, 3)
    assert lead.peek("leader_transfer_target") == 3
    ot = lead.peek("election_tick")
    _transfer(nt, 1, 1, 1)
    assert lead.peek("leader_transfer_target") == 3
    assert lead.peek("election_tick") == ot


def test_second_transfer_to_same_node_keeps_timeout():
    nt = Network(None, None, None)
    lead = _elect(nt)
    nt.isolate(3)
    _transfer(nt, 3, 1, 3)
    assert lead.peek("leader_transfer_target") == 3
    for _ in range(1):  # heartbeatTimeout
        lead.tick()
    # a second request to the same node does not extend the timeout
    _transfer(nt, 3, 1, 3)
    for _ in range(10 - 1):  # electionTimeout - heartbeatTimeout
        lead.tick()
    _check_state(lead, LEADER, 1)


def test_timeout_now_campaigns_without_pre_vote():
    """handleFollowerTimeoutNow (raft.go:2172-2185) + campaign (:1192-1196):
    the target skips the PreVote round and its RequestVote names itself
    in Hint, so voters inside their lease still grant."""
    nt = Network(None, None, None, pre_vote=True, check_quorum=True)
    lead = _elect(nt)
    t = nt.peers[3]
    t.handle(msg(TIMEOUT_NOW, from_=1, to=3, term=lead.info().term))
    out = t.read_messages()
    assert {m["type"] for m in out} == {MSG["RequestVote"]}
    assert all(m["hint"] == 3 and m["term"] == 2 for m in out)
    assert t.peek("is_leader_transfer_target") == 0
