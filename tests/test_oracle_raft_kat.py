"""Raft known-answer tests restated from the reference's own test files.

Sources (all in /root/reference/internal/raft):
  raft_etcd_paper_test.go  commit / replicate KATs (section 5.3, 5.4.2)
  logentry_test.go         matchTerm / upToDate / getConflictIndex /
                           commitTo / commitUpdate tables
  readindex_test.go        readIndex queue / confirm KATs
  raft_test.go:1578-1666   make / broadcast Replicate and Heartbeat
  raft_test.go:2952-3037   ReadIndex handled by the leader
They pin the oracle (oracle/*.c) to the reference's expected values; the
oracle is then the checker for the GPU path (tests/test_gpu_*.py).
"""
import pytest

from oracle import pyoracle as po
from oracle.pyoracle import ent, msg
from dragonboat_amd.abi import MSG, LEADER, FOLLOWER, CANDIDATE

REPLICATE = MSG["Replicate"]
REPLICATE_RESP = MSG["ReplicateResp"]
PROPOSE = MSG["Propose"]


def ids_by_size(n):  # raft_etcd_test.go:3043
    return list(range(1, n + 1))


def accept_and_reply(m):  # raft_etcd_paper_test.go:969-980
    assert m["type"] == REPLICATE
    return msg(REPLICATE_RESP, from_=m["to"], to=m["from_"], term=m["term"],
               log_index=m["log_index"] + len(m["entries"]))


def commit_noop_entry(r, s):  # raft_etcd_paper_test.go:938-967
    assert r.info().role == LEADER
    r.broadcast_replicate()
    for m in r.read_messages():
        assert (m["type"] == REPLICATE and len(m["entries"]) == 1 and
                m["entries"][0]["cmd"] == b"")
        r.handle(accept_and_reply(m))
    r.read_messages()
    s.append(r.entries_to_save())
    rc, term = r.term(r.last_index)
    r.commit_update(processed=r.committed, stable_log_to=r.last_index,
                    stable_log_term=term)


def _strip(e):
    return (e["term"], e["index"], e["cmd"])


def test_leader_commit_entry():  # raft_etcd_paper_test.go:411-451
    s = po.LogDB()
    r = po.TestRaft(1, [1, 2, 3], 10, 1, s)
    r.become_candidate()
    r.become_leader()
    commit_noop_entry(r, s)
    li = r.last_index
    r.handle(msg(PROPOSE, from_=1, to=1, entries=[ent(cmd=b"some data")]))
    for m in r.read_messages():
        r.handle(accept_and_reply(m))
    assert r.committed == li + 1
    assert [_strip(e) for e in r.entries_to_apply()] == \
        [(1, li + 1, b"some data")]
    msgs = sorted(r.read_messages(), key=lambda m: m["to"])
    for i, m in enumerate(msgs):
        assert m["to"] == i + 2
        assert m["type"] == REPLICATE
        assert m["commit"] == li + 1


@pytest.mark.parametrize("size,acceptors,wack", [
    (1, set(), True), (3, set(), False), (3, {2}, True), (3, {2, 3}, True),
    (5, set(), False), (5, {2}, False), (5, {2, 3}, True),
    (5, {2, 3, 4}, True), (5, {2, 3, 4, 5}, True)])
def test_leader_acknowledge_commit(size, acceptors, wack):
    # raft_etcd_paper_test.go:453-490
    s = po.LogDB()
    r = po.TestRaft(1, ids_by_size(size), 10, 1, s)
    r.become_candidate()
    r.become_leader()
    commit_noop_entry(r, s)
    li = r.last_index
    r.handle(msg(PROPOSE, from_=1, to=1, entries=[ent(cmd=b"some data")]))
    for m in r.read_messages():
        if m["to"] in acceptors:
            r.handle(accept_and_reply(m))
    assert (r.committed > li) == wack


@pytest.mark.parametrize("tt", [
    [], [ent(term=2, index=1)], [ent(term=1, index=1), ent(term=2, index=2)],
    [ent(term=1, index=1)]])
def test_leader_commit_preceding_entries(tt):
    # raft_etcd_paper_test.go:495-529
    storage = po.LogDB(tt)
    r = po.TestRaft(1, [1, 2, 3], 10, 1, storage)
    r.load_state(term=2)
    r.become_candidate()
    r.become_leader()
    r.handle(msg(PROPOSE, from_=1, to=1, entries=[ent(cmd=b"some data")]))
    for m in r.read_messages():
        r.handle(accept_and_reply(m))
    li = len(tt)
    want = [(e["term"], e["index"], b"") for e in tt] + \
        [(3, li + 1, b""), (3, li + 2, b"some data")]
    assert [_strip(e) for e in r.entries_to_apply()] == want


@pytest.mark.parametrize("ents,commit", [
    ([ent(term=1, index=1, cmd=b"some data")], 1),
    ([ent(term=1, index=1, cmd=b"some data"),
      ent(term=1, index=2, cmd=b"some data2")], 2),
    ([ent(term=1, index=1, cmd=b"some data2"),
      ent(term=1, index=2, cmd=b"some data")], 2),
    ([ent(term=1, index=1, cmd=b"some data"),
      ent(term=1, index=2, cmd=b"some data2")], 1)])
def test_follower_commit_entry(ents, commit):
    # raft_etcd_paper_test.go:532-588
    r = po.TestRaft(1, [1, 2, 3], 10, 1)
    r.become_follower(1, 2)
    r.handle(msg(REPLICATE, from_=2, to=1, term=1, entries=ents,
                 commit=commit))
    assert r.committed == commit
    assert [_strip(e) for e in r.entries_to_apply()] == \
        [_strip(e) for e in ents[:commit]]


@pytest.mark.parametrize("term,index,windex,wreject,whint", [
    (0, 0, 1, False, 0), (1, 1, 1, False, 0), (2, 2, 2, False, 0),
    (1, 2, 2, True, 2), (3, 3, 3, True, 2)])
def test_follower_check_replicate(term, index, windex, wreject, whint):
    # raft_etcd_paper_test.go:590-630
    storage = po.LogDB([ent(term=1, index=1), ent(term=2, index=2)])
    r = po.TestRaft(1, [1, 2, 3], 10, 1, storage)
    r.load_state(commit=1)
    r.become_follower(2, 2)
    r.handle(msg(REPLICATE, from_=2, to=1, term=2, log_term=term,
                 log_index=index))
    msgs = r.read_messages()
    assert len(msgs) == 1
    m = msgs[0]
    assert (m["from_"], m["to"], m["type"], m["term"], m["log_index"],
            m["reject"], m["hint"]) == (1, 2, REPLICATE_RESP, 2, windex,
                                        wreject, whint)


@pytest.mark.parametrize("index,term,ents,wents,wunstable", [
    (2, 2, [ent(term=3, index=3)],
     [(1, 1), (2, 2), (3, 3)], [(3, 3)]),
    (1, 1, [ent(term=3, index=2), ent(term=4, index=3)],
     [(1, 1), (3, 2), (4, 3)], [(3, 2), (4, 3)]),
    (0, 0, [ent(term=1, index=1)], [(1, 1), (2, 2)], []),
    (0, 0, [ent(term=3, index=1)], [(3, 1)], [(3, 1)])])
def test_follower_append_entries(index, term, ents, wents, wunstable):
    # raft_etcd_paper_test.go:636-688
    storage = po.LogDB([ent(term=1, index=1), ent(term=2, index=2)])
    r = po.TestRaft(1, [1, 2, 3], 10, 1, storage)
    r.become_follower(2, 2)
    r.handle(msg(REPLICATE, from_=2, to=1, term=2, log_term=term,
                 log_index=index, entries=ents))
    assert [(e["term"], e["index"]) for e in r.all_entries()] == wents
    assert [(e["term"], e["index"]) for e in r.entries_to_save()] == \
        wunstable


def _e(pairs):
    return [ent(term=t, index=i) for t, i in pairs]


LEAD_ENTS = _e([(1, 1), (1, 2), (1, 3), (4, 4), (4, 5), (5, 6), (5, 7),
                (6, 8), (6, 9), (6, 10)])
SYNC_CASES = [
    _e([(1, 1), (1, 2), (1, 3), (4, 4), (4, 5), (5, 6), (5, 7), (6, 8),
        (6, 9)]),
    _e([(1, 1), (1, 2), (1, 3), (4, 4)]),
    _e([(1, 1), (1, 2), (1, 3), (4, 4), (4, 5), (5, 6), (5, 7), (6, 8),
        (6, 9), (6, 10), (6, 11)]),
    _e([(1, 1), (1, 2), (1, 3), (4, 4), (4, 5), (5, 6), (5, 7), (6, 8),
        (6, 9), (6, 10), (7, 11), (7, 12)]),
    _e([(1, 1), (1, 2), (1, 3), (4, 4), (4, 5), (4, 6), (4, 7)]),
    _e([(1, 1), (1, 2), (1, 3), (2, 4), (2, 5), (2, 6), (3, 7), (3, 8),
        (3, 9), (3, 10), (3, 11)]),
]


@pytest.mark.parametrize("tt", SYNC_CASES)
def test_leader_sync_follower_log(tt):
    # raft_etcd_paper_test.go:690-770 (figure 7)
    term = 8
    lead_storage = po.LogDB(LEAD_ENTS)
    lead = po.TestRaft(1, [1, 2, 3], 10, 1, lead_storage)
    lead.load_state(commit=lead.last_index, term=term)
    follower = po.TestRaft(2, [1, 2, 3], 10, 1, po.LogDB(tt))
    follower.load_state(term=term - 1)
    n = po.Network(lead, follower, po.BlackHole())
    n.send(msg(MSG["Election"], from_=1, to=1))
    n.send(msg(MSG["RequestVoteResp"], from_=3, to=1, term=term + 1))
    n.send(msg(PROPOSE, from_=1, to=1, entries=[ent()]))
    li, fi = lead.info(), follower.info()
    assert (li.committed, li.processed) == (fi.committed, fi.processed)
    assert [_strip(e) for e in lead.all_entries()] == \
        [_strip(e) for e in follower.all_entries()]


@pytest.mark.parametrize("index,wcommit", [(1, 0), (2, 0), (3, 3)])
def test_leader_only_commits_log_from_current_term(index, wcommit):
    # raft_etcd_paper_test.go:867-899 (section 5.4.2)
    storage = po.LogDB([ent(term=1, index=1), ent(term=2, index=2)])
    r = po.TestRaft(1, [1, 2], 10, 1, storage)
    r.load_state(term=2)
    r.become_candidate()
    r.become_leader()
    r.read_messages()
    r.handle(msg(PROPOSE, from_=1, to=1, entries=[ent()]))
    r.handle(msg(REPLICATE_RESP, from_=2, to=1, term=r.info().term,
                 log_index=index))
    assert r.committed == wcommit


def test_leader_start_replication():  # raft_etcd_paper_test.go:900-935
    s = po.LogDB()
    r = po.TestRaft(1, [1, 2, 3], 10, 1, s)
    r.become_candidate()
    r.become_leader()
    commit_noop_entry(r, s)
    li = r.last_index
    r.handle(msg(PROPOSE, from_=1, to=1, entries=[ent(cmd=b"some data")]))
    assert r.last_index == li + 1
    assert r.committed == li
    msgs = sorted(r.read_messages(), key=lambda m: m["to"])
    want_ents = [dict(ent(term=1, index=li + 1, cmd=b"some data"))]
    assert len(msgs) == 2
    for to, m in zip((2, 3), msgs):
        assert (m["from_"], m["to"], m["term"], m["type"], m["log_index"],
                m["log_term"], m["commit"]) == (1, to, 1, REPLICATE, li, 1, li)
        assert m["entries"] == want_ents


@pytest.mark.parametrize("ents,logterm,index,wreject", [
    (_e([(1, 1)]), 1, 1, False), (_e([(1, 1)]), 1, 2, False),
    (_e([(1, 1), (1, 2)]), 1, 1, True),
    (_e([(1, 1)]), 2, 1, False), (_e([(1, 1)]), 2, 2, False),
    (_e([(1, 1), (1, 2)]), 2, 1, False),
    (_e([(2, 1)]), 1, 1, True), (_e([(2, 1)]), 1, 2, True),
    (_e([(2, 1), (1, 2)]), 1, 1, True)])
def test_voter(ents, logterm, index, wreject):
    # raft_etcd_paper_test.go:811-864 (election used by the setup path)
    r = po.TestRaft(1, [1, 2], 10, 1, po.LogDB(ents))
    r.handle(msg(MSG["RequestVote"], from_=2, to=1, term=3, log_term=logterm,
                 log_index=index))
    msgs = r.read_messages()
    assert len(msgs) == 1
    assert msgs[0]["type"] == MSG["RequestVoteResp"]
    assert msgs[0]["reject"] == wreject


# ---------------------------------------------------------------- entryLog
def _log_fixture():
    # logentry_test.go:409-425 (shared setup of the matchTerm/upToDate/...
    # tables): logdb holds 1..4, the in-memory part holds 5..7
    r = po.TestRaft(1, [1], 10, 1,
                    po.LogDB(_e([(1, 1), (1, 2), (2, 3), (3, 4)])))
    r.append(_e([(3, 5), (3, 6), (4, 7)]))
    return r


@pytest.mark.parametrize("index,term,match", [
    (1, 1, True), (1, 2, False), (4, 4, False), (4, 3, True), (5, 3, True),
    (5, 4, False), (7, 4, True), (8, 5, False)])
def test_log_match_term(index, term, match):  # logentry_test.go:409-447
    assert _log_fixture().match_term(index, term) == match


@pytest.mark.parametrize("index,term,ok", [
    (1, 2, False), (8, 2, False), (1, 4, False), (7, 4, True), (8, 4, True),
    (8, 5, True), (2, 5, True)])
def test_log_up_to_date(index, term, ok):  # logentry_test.go:449-487
    assert _log_fixture().up_to_date(index, term) == ok


@pytest.mark.parametrize("ents,conflict", [
    ([], 0), (_e([(2, 1)]), 1), (_e([(1, 1), (1, 2)]), 0),
    (_e([(1, 1), (2, 2)]), 2), (_e([(3, 6), (4, 7)]), 0),
    (_e([(3, 6), (5, 7)]), 7), (_e([(4, 7), (4, 8)]), 8)])
def test_log_get_conflict_index(ents, conflict):  # logentry_test.go:489-530
    assert _log_fixture().conflict_index(ents) == conflict


def test_log_commit_to():  # logentry_test.go:532-556
    r = _log_fixture()
    r.commit_to(3)
    assert r.committed == 3
    r.commit_to(2)
    assert r.committed == 3


def test_log_commit_to_panics_on_unavailable_index():  # :558-583
    with pytest.raises(po.OracleError):
        _log_fixture().commit_to(8)


def test_log_commit_update_sets_applied():  # logentry_test.go:608-618
    r = _log_fixture()
    r.commit_to(7)
    r.commit_update(processed=5)
    assert r.info().processed == 5


def test_log_commit_update_panics_when_apply_twice():  # :620-633
    r = _log_fixture()
    r.commit_to(7)
    r.commit_update(processed=6)
    with pytest.raises(po.OracleError):
        r.commit_update(processed=5)


def test_log_commit_update_panics_when_applying_not_committed():  # :635-648
    r = _log_fixture()
    r.commit_to(7)
    r.commit_update(processed=6)
    with pytest.raises(po.OracleError):
        r.commit_update(processed=12)


@pytest.mark.parametrize("index,term,committed,ok", [
    (5, 3, 5, True), (5, 4, 0, False), (7, 4, 7, True), (3, 2, 3, True)])
def test_log_try_commit_term_rule(index, term, committed, ok):
    # logentry.go:395-410 -- commit only at the leader's current term
    r = _log_fixture()
    assert r.log_try_commit(index, term) == ok
    assert r.committed == committed


# ---------------------------------------------------------------- readIndex
def ctx(v):  # readindex_test.go:20-25 getTestSystemCtx
    return (v, v + 1)


def test_same_ctx_can_not_be_added_twice():  # readindex_test.go:30-40
    r = po.ReadIndexQ()
    r.add_request(1, ctx(10001), 1)
    assert len(r) == 1
    r.add_request(2, ctx(10001), 2)
    assert len(r) == 1


def test_inconsistent_pending_queue():  # readindex_test.go:42-53
    r = po.ReadIndexQ()
    r.add_request(1, ctx(10001), 1)
    r.push_raw(ctx(10003))
    with pytest.raises(po.OracleError):
        r.add_request(2, ctx(10002), 2)


def test_read_index_request_can_be_added():  # readindex_test.go:55-84
    r = po.ReadIndexQ()
    r.add_request(1, ctx(10001), 1)
    r.add_request(2, ctx(10002), 2)
    items = r.items()
    assert len(items) == 2
    assert items[1] == (ctx(10002), 2, 2)
    assert items[-1][0] == ctx(10002)  # peepCtx


def test_read_index_checks_input_index():  # readindex_test.go:86-103
    r = po.ReadIndexQ()
    r.add_request(3, ctx(10001), 1)
    r.add_request(5, ctx(10002), 3)
    with pytest.raises(po.OracleError):
        r.add_request(4, ctx(10003), 2)


def test_add_confirmation_checks_inconsistent_pending_queue():  # :105-124
    r = po.ReadIndexQ()
    r.add_request(3, ctx(10002), 1)
    r.add_request(4, ctx(10001), 3)
    r.add_request(5, ctx(10003), 2)
    r.push_raw(ctx(10004), front=True)
    r.confirm(ctx(10001), 1, 3)
    with pytest.raises(po.OracleError):
        r.confirm(ctx(10001), 3, 3)


def test_read_index_leader_can_be_confirmed():  # readindex_test.go:126-164
    r = po.ReadIndexQ()
    r.add_request(3, ctx(10002), 1)
    r.add_request(4, ctx(10001), 3)
    r.add_request(5, ctx(10003), 2)
    assert r.confirm(ctx(10001), 1, 3) == []
    ris = r.confirm(ctx(10001), 3, 3)
    assert len(ris) == 2
    assert ris[1] == (ctx(10001), 4, 3)
    assert ris[0] == (ctx(10002), 4, 1)
    assert len(r) == 1


# ---- raft_test.go:1578-1666: make / broadcast Replicate and Heartbeat ----
HEARTBEAT = MSG["Heartbeat"]
READ_INDEX = MSG["ReadIndex"]
ENTRY_NON_CMD_FIELDS_SIZE = 128  # settings.EntryNonCmdFieldsSize (soft.go)


def size_upper_limit(cmd_len):  # Entry.SizeUpperLimit (raft_optimized.go:77)
    return ENTRY_NON_CMD_FIELDS_SIZE + cmd_len


def test_make_replicate_message():
    # raft_test.go:1578-1611
    r = po.TestRaft(1, [1, 2], 5, 1)
    r.become_candidate()
    r.become_leader()
    r.append_entries([ent(index=2, term=1, cmd=bytes(16)),
                      ent(index=3, term=1, cmd=bytes(16))])
    sz = size_upper_limit(0) + 2 * size_upper_limit(16) + 1
    m = r.make_replicate(2, 1, sz)
    assert m["type"] == REPLICATE and m["to"] == 2
    assert len(m["entries"]) == 3  # the NoOP plus the two above
    m = r.make_replicate(2, 1, size_upper_limit(0) + size_upper_limit(16))
    assert len(m["entries"]) == 2


def test_broadcast_replicate_message():
    # raft_test.go:1613-1627
    r = po.TestRaft(1, [1, 2, 3], 5, 1)
    r.become_candidate()
    r.become_leader()
    r.broadcast_replicate()
    assert sum(m["type"] == REPLICATE for m in r.read_messages()) == 2


def test_broadcast_heartbeat_message():
    # raft_test.go:1629-1643
    r = po.TestRaft(1, [1, 2, 3], 5, 1)
    r.become_candidate()
    r.become_leader()
    r.broadcast_heartbeat()
    assert sum(m["type"] == HEARTBEAT for m in r.read_messages()) == 2


def test_broadcast_heartbeat_message_with_hint():
    # raft_test.go:1645-1666
    r = po.TestRaft(1, [1, 2, 3], 5, 1)
    r.become_candidate()
    r.become_leader()
    r.broadcast_heartbeat_hint((101, 1001))
    msgs = r.read_messages()
    assert sum(m["type"] == HEARTBEAT for m in msgs) == 2
    assert all(m["hint"] == 101 and m["hint_high"] == 1001 for m in msgs)


# ---- raft_test.go:2952-3037: ReadIndex inside raft -----------------------
def test_leader_read_index_on_single_node_shard():
    # raft_test.go:2952-2976
    r = po.TestRaft(1, [1], 5, 1)
    r.become_candidate()
    r.become_leader()
    r.handle(msg(READ_INDEX, hint=101, hint_high=1002))
    assert r.read_messages() == []
    assert r.ready_to_read() == [(r.committed, (101, 1002))]
    assert r.read_index_len() == 0


def test_leader_ignore_read_index_when_shard_committed_is_unknown():
    # raft_test.go:2978-2997
    r = po.TestRaft(1, [1, 2, 3], 5, 1)
    r.become_candidate()
    r.become_leader()
    r.handle(msg(READ_INDEX, hint=101, hint_high=1002))
    assert r.read_messages() == []
    assert r.ready_to_read() == []
    assert r.read_index_len() == 0


def test_handle_leader_read_index():
    # raft_test.go:2999-3037
    r = po.TestRaft(1, [1, 2, 3], 5, 1)
    r.become_follower(1, 0)
    assert not r.has_committed_entry_at_current_term()
    r.become_candidate()
    r.become_leader()
    assert not r.has_committed_entry_at_current_term()
    rm = r.remote(2)
    po.lib().orc_remote_try_update(rm, r.last_index)
    r.set_remote(2, rm)
    assert r.try_commit()
    assert r.has_committed_entry_at_current_term()
    r.handle(msg(READ_INDEX, hint=101, hint_high=1002))
    hb = [m for m in r.read_messages() if m["type"] == HEARTBEAT and
          m["to"] in (2, 3) and m["hint"] == 101 and m["hint_high"] == 1002]
    assert len(hb) == 2
    assert r.read_index_len() == 1

# raft_test.go:3039-3063 (TestWitnessReadIndex) is not restated: witness
# members are outside the GPU fast path, which only steps
# voting members.


# ---------------------------------------------------------------- elections
# The election state machine the GPU's raft launch restates (el_*,
# drb_step.hpp) is checked against the oracle; these pin the oracle.
REQUEST_VOTE = MSG["RequestVote"]
REQUEST_VOTE_RESP = MSG["RequestVoteResp"]


def _granted(st, rid):
    return bool((st.votes >> (8 + rid - 1)) & 1)


@pytest.mark.parametrize("state", ["follower", "candidate"])
def test_nonleader_start_election(state):
    # raft_etcd_paper_test.go:141-193 (testNonleaderStartElection)
    et = 10
    r = po.TestRaft(1, [1, 2, 3], et, 1)
    if state == "follower":
        r.become_follower(1, 2)
    else:
        r.become_candidate()
    for _ in range(1, 2 * et):
        r.tick()
    st = r.info()
    assert st.term == 2 and st.role == CANDIDATE
    assert _granted(st, 1)
    msgs = sorted(r.read_messages(), key=lambda m: m["to"])
    assert [(m["from_"], m["to"], m["term"], m["type"]) for m in msgs] == [
        (1, 2, 2, REQUEST_VOTE), (1, 3, 2, REQUEST_VOTE)]


@pytest.mark.parametrize("size,votes,state", [
    # raft_etcd_paper_test.go:199-242 (TestLeaderElectionInOneRoundRPC)
    (1, {}, LEADER), (3, {2: True, 3: True}, LEADER), (3, {2: True}, LEADER),
    (5, {2: True, 3: True, 4: True, 5: True}, LEADER),
    (5, {2: True, 3: True, 4: True}, LEADER), (5, {2: True, 3: True}, LEADER),
    (3, {2: False, 3: False}, FOLLOWER),
    (5, {2: False, 3: False, 4: False, 5: False}, FOLLOWER),
    (5, {2: True, 3: False, 4: False, 5: False}, FOLLOWER),
    (3, {}, CANDIDATE), (5, {2: True}, CANDIDATE),
    (5, {2: False, 3: False}, CANDIDATE), (5, {}, CANDIDATE)])
def test_leader_election_in_one_round_rpc(size, votes, state):
    r = po.TestRaft(1, ids_by_size(size), 10, 1)
    r.handle(msg(MSG["Election"], from_=1, to=1))
    for rid, vote in votes.items():
        r.handle(msg(REQUEST_VOTE_RESP, from_=rid, to=1, term=r.info().term,
                     reject=not vote))
    st = r.info()
    assert st.role == state
    assert st.term == 1


@pytest.mark.parametrize("vote,nvote,wreject", [
    # raft_etcd_paper_test.go:244-276 (TestFollowerVote)
    (0, 1, False), (0, 2, False), (1, 1, False), (2, 2, False),
    (1, 2, True), (2, 1, True)])
def test_follower_vote(vote, nvote, wreject):
    r = po.TestRaft(1, [1, 2, 3], 10, 1)
    r.load_state(term=1, vote=vote)
    r.handle(msg(REQUEST_VOTE, from_=nvote, to=1, term=1))
    msgs = r.read_messages()
    assert [(m["from_"], m["to"], m["term"], m["type"], bool(m["reject"]))
            for m in msgs] == [(1, nvote, 1, REQUEST_VOTE_RESP, wreject)]


@pytest.mark.parametrize("term", [1, 2])
def test_candidate_fallback(term):
    # raft_etcd_paper_test.go:278-303 (TestCandidateFallback)
    r = po.TestRaft(1, [1, 2, 3], 10, 1)
    r.handle(msg(MSG["Election"], from_=1, to=1))
    assert r.info().role == CANDIDATE
    r.handle(msg(REPLICATE, from_=2, to=1, term=term))
    st = r.info()
    assert st.role == FOLLOWER and st.term == term


@pytest.mark.parametrize("active", [True, False])
def test_leader_stepdown_check_quorum(active):
    # raft_etcd_test.go:1656-1688 (TestLeaderStepdownWhenQuorumActive /
    # ...QuorumLost)
    r = po.TestRaft(1, [1, 2, 3], 5, 1)
    r.set_check_quorum(True)
    r.become_candidate()
    r.become_leader()
    for _ in range(5 + 1):
        if active:
            r.handle(msg(MSG["HeartbeatResp"], from_=2, to=1,
                         term=r.info().term))
        r.tick()
    assert r.info().role == (LEADER if active else FOLLOWER)


# ------------------------------------------------------------ PreVote
PREVOTE_CANDIDATE = 2


def test_become_pre_vote_candidate():
    # raft_test.go:269-287 (TestBecomePreVoteCandidate)
    r = po.TestRaft(1, [1, 2, 3], 10, 1)
    r.set_pre_vote(True)
    r.become_follower(2, 3)
    r.handle(msg(MSG["Election"], from_=1, to=1))
    st = r.info()
    assert st.term == 2 and st.role == PREVOTE_CANDIDATE
    assert st.leader_id == 0
    msgs = sorted(r.read_messages(), key=lambda m: m["to"])
    assert [(m["to"], m["term"], m["type"]) for m in msgs] == [
        (2, 3, MSG["RequestPreVote"]), (3, 3, MSG["RequestPreVote"])]


def test_no_op_sent_on_small_term_rejected_request_pre_vote():
    # raft_test.go:1420-1432
    r = po.TestRaft(1, [1, 2], 5, 1)
    r.set_pre_vote(True)
    r.become_follower(10, 2)
    r.handle(msg(MSG["RequestPreVote"], from_=2, to=1, term=9))
    msgs = r.read_messages()
    assert [(m["type"], m["to"], m["from_"], m["term"]) for m in msgs] == [
        (MSG["NoOP"], 2, 1, 10)]


def test_pre_vote_resp_with_higher_term():
    # raft_test.go:1434-1446
    r = po.TestRaft(1, [1, 2], 5, 1)
    r.set_pre_vote(True)
    r.become_follower(10, 2)
    r.handle(msg(MSG["RequestPreVoteResp"], from_=2, to=1, term=11))
    assert r.info().term == 10
    r.handle(msg(MSG["RequestPreVoteResp"], from_=2, to=1, term=20,
                 reject=True))
    assert r.info().term == 20


def test_election_with_pre_vote():
    # raft_test.go:3278-3296 (TestElectionWithPreVote)
    peers = [po.TestRaft(i, [1, 2, 3], 10, 1) for i in (1, 2, 3)]
    for p in peers:
        p.set_pre_vote(True)
    nt = po.Network(*peers)
    nt.send(msg(MSG["Election"], from_=1, to=1))
    assert [p.info().role for p in peers] == [LEADER, FOLLOWER, FOLLOWER]
    assert peers[0].info().term == 1  # one campaign after the PreVote round


@pytest.mark.parametrize("utd,higher,reject", [
    (True, True, False), (False, True, True), (True, False, True)])
def test_handle_node_request_pre_vote(utd, higher, reject):
    # handleNodeRequestPreVote (raft.go:1670-1695): granted at m.Term only
    # for a higher term and an up-to-date log, else rejected at r.term
    r = po.TestRaft(1, [1, 2, 3], 10, 1)
    r.set_pre_vote(True)
    r.become_follower(5, 3)
    # the follower's log: one entry at term 5
    r.handle(msg(REPLICATE, from_=3, to=1, term=5,
                 entries=[ent(term=5, index=1)]))
    r.read_messages()
    t = 6 if higher else 5
    r.handle(msg(MSG["RequestPreVote"], from_=2, to=1, term=t, log_index=1,
                 log_term=5 if utd else 4))
    msgs = r.read_messages()
    assert len(msgs) == 1
    m = msgs[0]
    assert m["type"] == MSG["RequestPreVoteResp"] and bool(m["reject"]) == reject
    assert m["term"] == (t if not reject else 5)
    assert r.info().term == 5  # a PreVote never changes the term
