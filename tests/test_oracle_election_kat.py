"""Election known-answer tests restated from the reference's own tests.

They pin the oracle's election state machine (campaign, the vote handlers,
the term gate, CheckQuorum, PreVote; oracle/raft_oracle.c), which is the
checker of the GPU raft launch (drb_step.hpp el_*, tests/test_gpu_elections
.py, tests/test_gpu_truncation.py).

Sources (all in /root/reference/internal/raft):
  raft_etcd_test.go  TestLeaderElection (:468-508), TestLeaderCycle
                     (:510-536), TestLeaderElectionOverwriteNewerLogs
                     (:538-600), TestVoteFromAnyState (:602-670),
                     TestPastElectionTimeout (:1208-1239),
                     TestStepIgnoreOldTermMsg (:1241-1256), TestRecvMsgVote
                     (:1477-1528), TestStateTransition (:1530-1591),
                     TestLeaderSupersedingWithCheckQuorum (:1691-1731),
                     TestLeaderElectionWithCheckQuorum (:1733-1780),
                     TestFreeStuckCandidateWithCheckQuorum (:1782-1858)
  raft_test.go       TestBecomePreVoteCandidateFromCandidate (:255-267),
                     TestElectionTickResetAfterGrantVote (:1922-1940),
                     TestElectionIgnoredWhenConfigChangeIsPending
                     (:2660-2679), TestRequestVoteMessageWontResetElection-
                     Tick (:2699-2723)
The PreVote variants of TestLeaderElection and TestFreeStuckCandidateWith-
CheckQuorum are commented out in the reference (raft_etcd_test.go:472-476,
1786-1790), so they have no expected values to restate; the PreVote
elections are pinned by raft_test.go's own PreVote tests
(tests/test_oracle_raft_kat.py) and a network election below.
"""
import pytest

from dragonboat_amd.abi import (CANDIDATE, FOLLOWER, LEADER, MSG,
                                PREVOTE_CANDIDATE)
from oracle import pyoracle as po
from oracle.pyoracle import BlackHole, Network, ent, msg

ELECTION = MSG["Election"]
REQUEST_VOTE = MSG["RequestVote"]
REQUEST_VOTE_RESP = MSG["RequestVoteResp"]
REPLICATE = MSG["Replicate"]
HEARTBEAT = MSG["Heartbeat"]

ents = po.ents_with_config
voted = po.voted_with_config
NOP = BlackHole


def _state(r):
    return r.info().role


def _term(r):
    return r.info().term


@pytest.mark.parametrize("peers,state,term", [
    # raft_etcd_test.go:480-493
    ((None, None, None), LEADER, 1),
    ((None, None, NOP), LEADER, 1),
    ((None, NOP, NOP), CANDIDATE, 1),
    ((None, NOP, NOP, None), CANDIDATE, 1),
    ((None, NOP, NOP, None, None), LEADER, 1),
    # three logs further along than 0, but in the same term so rejections
    # are returned instead of the votes being ignored
    ((None, (1,), (1,), (1, 1), None), FOLLOWER, 1)])
def test_leader_election(peers, state, term):
    built = []
    for p in peers:
        if p is NOP:
            built.append(BlackHole())
        elif isinstance(p, tuple):
            built.append(ents(*p))
        else:
            built.append(p)
    nt = Network(*built)
    nt.send(msg(ELECTION, from_=1, to=1))
    sm = nt.peers[1]
    assert (_state(sm), _term(sm)) == (state, term)


def test_leader_cycle():
    # raft_etcd_test.go:510-536: each node campaigns and is elected in turn
    nt = Network(None, None, None)
    for cid in (1, 2, 3):
        nt.send(msg(ELECTION, from_=cid, to=cid))
        for pid, p in nt.peers.items():
            want = LEADER if pid == cid else FOLLOWER
            assert _state(p) == want, (cid, pid)


def test_leader_election_overwrite_newer_logs():
    # raft_etcd_test.go:538-600: node 1 won term 1 and replicated one
    # entry to node 2; node 3 won term 2 and wrote an entry nobody got;
    # nodes 4 and 5 voted for 3 at term 2.
    nt = Network(ents(1), ents(1), ents(2), voted(3, 2), voted(3, 2))
    # node 1's first campaign fails (a quorum knows term 2); its term is
    # pushed to 2
    nt.send(msg(ELECTION, from_=1, to=1))
    sm1 = nt.peers[1]
    assert (_state(sm1), _term(sm1)) == (FOLLOWER, 2)
    # the second campaign, at term 3, succeeds
    nt.send(msg(ELECTION, from_=1, to=1))
    assert (_state(sm1), _term(sm1)) == (LEADER, 3)
    # everyone now holds term 1 at index 1 and term 3 at index 2: node 3's
    # term-2 entry was overwritten by a lower-term leader's log
    for pid, p in nt.peers.items():
        es = p.all_entries()
        assert [(e["term"], e["index"]) for e in es] == [(1, 1), (3, 2)], pid


@pytest.mark.parametrize("st", range(6))
def test_vote_from_any_state(st):
    # raft_etcd_test.go:602-670 (RequestVote): every state grants a vote
    # for a higher term and becomes a follower at it
    r = po.TestRaft(1, [1, 2, 3], 10, 1)
    r.poke(term=1)
    if st == FOLLOWER:
        r.become_follower(1, 3)
    elif st == CANDIDATE:
        r.become_candidate()
    elif st == LEADER:
        r.become_candidate()
        r.become_leader()
    new_term = _term(r) + 1
    r.handle(msg(REQUEST_VOTE, from_=2, to=1, term=new_term,
                 log_term=new_term, log_index=42))
    ms = r.read_messages()
    assert len(ms) == 1
    assert ms[0]["type"] == REQUEST_VOTE_RESP and not ms[0]["reject"]
    i = r.info()
    assert (i.role, i.term, i.vote) == (FOLLOWER, new_term, 2)


@pytest.mark.parametrize("elapse,wprob,rnd", [
    # raft_etcd_test.go:1208-1239
    (5, 0, False), (10, 0.1, True), (13, 0.4, True), (15, 0.6, True),
    (18, 0.9, True), (20, 1, False)])
def test_past_election_timeout(elapse, wprob, rnd):
    # the randomized timeout is uniform over [ElectionRTT, 2 ElectionRTT)
    # (raft.go:658-661; the oracle draws it from its per-replica splitmix
    # generator, as the GPU does)
    r = po.TestRaft(1, [1], 10, 1)
    r.poke(election_tick=elapse)
    c = sum(r.draw_timeout_time_for_election() for _ in range(10000))
    got = c / 10000.0
    if rnd:
        got = int(got * 10 + 0.5) / 10.0
    assert got == wprob


def test_step_ignore_old_term_msg():
    # raft_etcd_test.go:1241-1256: a Replicate from an older term is
    # dropped by the term gate before any handler runs
    r = po.TestRaft(1, [1], 10, 1)
    r.poke(term=2)
    before = r.info()
    assert r.term_not_matched(msg(REPLICATE, term=1))
    r.handle(msg(REPLICATE, term=1))
    after = r.info()
    assert r.read_messages() == []  # no NoOP: CheckQuorum and PreVote off
    assert (after.term, after.role, after.last_index, after.committed) == \
        (before.term, before.role, before.last_index, before.committed)


@pytest.mark.parametrize("state,i,term,vote_for,wreject", [
    # raft_etcd_test.go:1477-1510
    (FOLLOWER, 0, 0, 0, True), (FOLLOWER, 0, 1, 0, True),
    (FOLLOWER, 0, 2, 0, True), (FOLLOWER, 0, 3, 0, False),
    (FOLLOWER, 1, 0, 0, True), (FOLLOWER, 1, 1, 0, True),
    (FOLLOWER, 1, 2, 0, True), (FOLLOWER, 1, 3, 0, False),
    (FOLLOWER, 2, 0, 0, True), (FOLLOWER, 2, 1, 0, True),
    (FOLLOWER, 2, 2, 0, False), (FOLLOWER, 2, 3, 0, False),
    (FOLLOWER, 3, 0, 0, True), (FOLLOWER, 3, 1, 0, True),
    (FOLLOWER, 3, 2, 0, False), (FOLLOWER, 3, 3, 0, False),
    (FOLLOWER, 3, 2, 2, False), (FOLLOWER, 3, 2, 1, True),
    (LEADER, 3, 3, 1, True), (CANDIDATE, 3, 3, 1, True)])
def test_recv_msg_vote(state, i, term, vote_for, wreject):
    # the log: entries {1: term 2, 2: term 2} in the LogDB, inMemory from 3
    db = po.LogDB([ent(term=2, index=1), ent(term=2, index=2)])
    r = po.TestRaft(1, [1, 2], 10, 1, db)
    r.poke(state=state, vote=vote_for)
    r.handle(msg(REQUEST_VOTE, from_=2, log_index=i, log_term=term))
    ms = r.read_messages()
    assert len(ms) == 1
    assert bool(ms[0]["reject"]) == wreject


@pytest.mark.parametrize("frm,to,wallow,wterm,wlead", [
    # raft_etcd_test.go:1530-1555 (the preVoteCandidate rows are commented
    # out in the reference)
    (FOLLOWER, FOLLOWER, True, 1, 0), (FOLLOWER, CANDIDATE, True, 1, 0),
    (FOLLOWER, LEADER, False, 0, 0), (CANDIDATE, FOLLOWER, True, 0, 0),
    (CANDIDATE, CANDIDATE, True, 1, 0), (CANDIDATE, LEADER, True, 0, 1),
    (LEADER, FOLLOWER, True, 1, 0), (LEADER, CANDIDATE, False, 1, 0),
    (LEADER, LEADER, True, 0, 1)])
def test_state_transition(frm, to, wallow, wterm, wlead):
    r = po.TestRaft(1, [1], 10, 1)
    r.poke(state=frm)
    try:
        if to == FOLLOWER:
            r.become_follower(wterm, wlead)
        elif to == CANDIDATE:
            r.become_candidate()
        else:
            r.become_leader()
    except po.OracleError:
        assert not wallow
        return
    assert wallow
    i = r.info()
    assert (i.term, i.leader_id) == (wterm, wlead)


def _cq_net():
    a, b, c = (po.TestRaft(i, [1, 2, 3], 10, 1) for i in (1, 2, 3))
    for x in (a, b, c):
        x.set_check_quorum(True)
    return a, b, c, Network(a, b, c)


def test_leader_superseding_with_check_quorum():
    # raft_etcd_test.go:1691-1731
    a, b, c, nt = _cq_net()
    b.set_randomized_election_timeout(10 + 1)
    for _ in range(10):
        b.tick()
    nt.send(msg(ELECTION, from_=1, to=1))
    assert _state(a) == LEADER and _state(c) == FOLLOWER
    nt.send(msg(ELECTION, from_=3, to=3))
    # b rejected c's vote: its election tick had not reached the timeout
    assert _state(c) == CANDIDATE
    for _ in range(10):
        b.tick()
    nt.send(msg(ELECTION, from_=3, to=3))
    assert _state(c) == LEADER


def test_leader_election_with_check_quorum():
    # raft_etcd_test.go:1733-1780
    a, b, c, nt = _cq_net()
    a.set_randomized_election_timeout(10 + 1)
    b.set_randomized_election_timeout(10 + 2)
    # immediately after creation votes are cast regardless of the timeout
    nt.send(msg(ELECTION, from_=1, to=1))
    assert _state(a) == LEADER and _state(c) == FOLLOWER
    a.set_randomized_election_timeout(10 + 1)
    b.set_randomized_election_timeout(10 + 2)
    for _ in range(10):
        a.tick()
    for _ in range(10):
        b.tick()
    nt.send(msg(ELECTION, from_=3, to=3))
    assert _state(a) == FOLLOWER and _state(c) == LEADER


def test_free_stuck_candidate_with_check_quorum():
    # raft_etcd_test.go:1782-1858: a candidate with a higher term disrupts
    # a leader that still holds its lease; the leader steps down to the
    # candidate's term
    a, b, c, nt = _cq_net()
    b.set_randomized_election_timeout(10 + 1)
    for _ in range(10):
        b.tick()
    nt.send(msg(ELECTION, from_=1, to=1))
    nt.isolate(1)
    nt.send(msg(ELECTION, from_=3, to=3))
    assert _state(b) == FOLLOWER and _state(c) == CANDIDATE
    assert _term(c) == _term(b) + 1
    nt.send(msg(ELECTION, from_=3, to=3))  # vote again for safety
    assert _state(b) == FOLLOWER and _state(c) == CANDIDATE
    assert _term(c) == _term(b) + 2
    nt.recover()
    nt.send(msg(HEARTBEAT, from_=1, to=3, term=_term(a)))
    # disrupt the leader so that the stuck peer is freed
    assert _state(a) == FOLLOWER
    assert _term(c) == _term(a)
    nt.send(msg(ELECTION, from_=3, to=3))
    assert _state(c) == LEADER


def test_become_pre_vote_candidate_from_candidate():
    # raft_test.go:255-267
    r = po.TestRaft(1, [1, 2, 3], 10, 1)
    r.set_pre_vote(True)
    r.become_follower(2, 3)
    r.become_candidate()
    r.become_pre_vote_candidate()
    assert _term(r) == 3 and _state(r) == PREVOTE_CANDIDATE


def test_election_tick_reset_after_grant_vote():
    # raft_test.go:1922-1940
    r = po.TestRaft(1, [1, 2], 5, 1)
    r.become_follower(2, 2)
    r.poke(election_tick=101)
    r.handle(msg(REQUEST_VOTE, from_=2, to=1, term=3))
    assert r.info().vote == 2
    assert r.peek("election_tick") == 0


def test_election_ignored_when_config_change_is_pending():
    # raft_test.go:2660-2679
    r = po.TestRaft(1, [1, 2], 5, 1)
    r.become_follower(2, 2)
    r.poke(committed=10, applied=5, config_change_hook=0)
    r.handle(msg(ELECTION))
    assert r.read_messages() == []
    assert _state(r) == FOLLOWER


def test_handle_election():
    # raft_test.go:2681-2697 (TestHandleElection)
    r = po.TestRaft(1, [1, 2], 5, 1)
    r.become_follower(2, 2)
    r.handle(msg(ELECTION))
    ms = r.read_messages()
    assert [(m["type"], m["to"]) for m in ms] == [(REQUEST_VOTE, 2)]
    assert _state(r) == CANDIDATE


def test_request_vote_message_wont_reset_election_tick():
    # raft_test.go:2699-2723: becomeFollowerKE keeps the election tick on a
    # higher-term RequestVote; any other higher-term message resets it
    r = po.TestRaft(1, [1, 2], 5, 1)
    r.become_follower(2, 2)
    r.poke(election_tick=101, election_timeout=102)
    r.term_not_matched(msg(REQUEST_VOTE, from_=2, to=1, term=3))
    assert (r.peek("election_tick"), r.peek("election_timeout")) == (101, 102)
    r.term_not_matched(msg(REPLICATE, term=5))
    assert r.peek("election_tick") == 0


def test_leader_election_with_pre_vote_network():
    # the TestLeaderElection table run with PreVote on every replica
    # (raft_test.go:3278-3296 pins one election; here the stuck and the
    # rejected cases too): a pre-vote round that fails leaves the term
    # unchanged (preVoteCampaign, raft.go:1149-1174)
    nt = Network(None, BlackHole(), BlackHole(), pre_vote=True)
    nt.send(msg(ELECTION, from_=1, to=1))
    sm = nt.peers[1]
    assert (_state(sm), _term(sm)) == (PREVOTE_CANDIDATE, 0)
    nt = Network(None, None, BlackHole(), pre_vote=True)
    nt.send(msg(ELECTION, from_=1, to=1))
    assert (_state(nt.peers[1]), _term(nt.peers[1])) == (LEADER, 1)
