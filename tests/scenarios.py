"""Replica states for scenarios the step loop only reaches through history
the steady-state setup does not have (divergent logs), shared by the
oracle-only tests and the GPU parity tests.

LeaderSyncFollowerLog (raft_etcd_paper_test.go:690-770, figure 7 of the
Raft paper): a leader-to-be at term 8 holding LEAD_ENTS, committed, and a
follower at term 7 holding one of SYNC_CASES -- shorter, longer, with
extra entries of terms 6 and 7, or diverging from index 4 at terms 2-3.
The third replica is the reference's nopStepper: not hosted, its one
message (a RequestVoteResp granting term 9) is ingested by hand.
"""
import ctypes as C

from dragonboat_amd import abi
from oracle import pyoracle as po
from oracle.pyoracle import ent


def _e(pairs):
    return [ent(term=t, index=i) for t, i in pairs]


LEAD_TERM = 8
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


def _loaded(base, log, term, commit, hosted, election_tick=0):
    """raft.loadState(pb.State{Term, Commit}) over a LogDB holding `log`
    (newEntryLog: inMemory starts after it, logentry.go:86-95), the node
    and state machine having applied everything committed."""
    st = abi.ReplicaState()
    C.memmove(C.byref(st), C.byref(base), C.sizeof(st))
    last = len(log)
    st.term, st.vote, st.leader_id = term, 0, 0
    st.role = abi.FOLLOWER
    st.committed = st.processed = st.applied = commit
    st.last_index, st.marker_index, st.saved_to = last, last + 1, last
    st.applied_to_index = st.applied_to_term = 0
    st.applied_index = st.confirmed_index = st.pushed_index = commit
    st.prev_term, st.prev_vote, st.prev_commit = term, 0, commit
    st.sm_index = commit
    st.sm_term = log[commit - 1]["term"] if commit else 0
    st.kv_count = 0
    st.election_tick = election_tick
    st.heartbeat_tick = 0
    st.votes = 0
    st.ri_count = 0
    st.flags = abi.F_HOSTED if hosted else 0
    st.fallback_reason = 0
    for s in range(abi.DRB_MAX_REPLICAS):
        st.remotes[s].match = st.remotes[s].next = 0
        st.remotes[s].state = st.remotes[s].active = 0
    return st


def sync_follower_group(base, tt):
    """[(state, log)] of the three replicas of one LeaderSyncFollowerLog
    case; base(slot) is a ReplicaState to start from (ids, seeds)."""
    lead = _loaded(base(0), LEAD_ENTS, LEAD_TERM, len(LEAD_ENTS), True)
    # its election timer fires on the next tick (n.send(Election))
    lead.election_tick = lead.randomized_election_timeout - 1
    follower = _loaded(base(1), tt, LEAD_TERM - 1, 0, True)
    hole = _loaded(base(2), tt, LEAD_TERM - 1, 0, False)
    return [(lead, LEAD_ENTS), (follower, tt), (hole, tt)]


def vote_from_hole(shard_id):
    """n.send(RequestVoteResp{From: 3, To: 1, Term: term + 1})"""
    return po.msg(abi.MSG["RequestVoteResp"], from_=3, to=1,
                  term=LEAD_TERM + 1, shard_id=shard_id)
