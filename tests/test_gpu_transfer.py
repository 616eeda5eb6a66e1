"""GPU: leader transfer on the device (drb_request_leader_transfer; SURVEY
8f F3, elections).

NodeHost.RequestLeaderTransfer (nodehost.go:1238-1251) queues a target at
one replica; its next round takes it after the proposals
(node.handleLeaderTransfer, node.go:1249-1257 -> Peer.RequestLeaderTransfer,
peer.go:106-113).  A leader records the target (handleLeaderTransfer,
raft.go:1925-1953) and drops proposals (raft.go:1796-1800) until the target
holds its whole log, then sends TimeoutNow (raft.go:873-878, 1890-1895); the
target campaigns at once, without PreVote and with Hint = itself so the
voters' CheckQuorum lease lets the vote through (raft.go:1192-1196,
1507-1529, 2172-2185).  A follower forwards the request to its leader
(raft.go:2145-2153).  An election timeout without a new leader abandons the
transfer (raft.go:622-636).  Every round is compared with the oracle
cluster over every field -- the transfer target included -- the log, the
KV, the outboxes, the ReadyToReads and the dropped-proposal count; no
replica leaves the GPU.
"""
import pytest

from dragonboat_amd import abi
from dragonboat_amd.engine import DrbError
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu


def _unhost(p, groups, slot):
    for g in groups:
        p.orc.set_hosted(g, slot, False)
        sts = p.eng.export_replicas(g, 1)
        sts[slot].flags &= ~abi.F_HOSTED
        p.eng.import_replicas(g, sts)


def _rounds(p, n, st, k=1, ri_every=3):
    for _ in range(n):
        o, e = p.round(k=k, tick=True, read_index=(p.rounds % ri_every == 0))
        assert e.fallbacks == 0 and e.errors == 0, (p.rounds, e.to_dict(),
                                                     p.why())
        assert (e.committed_entries, e.messages, e.dropped_proposals) == \
            (o.committed_entries, o.messages, o.dropped_proposals), \
            (p.rounds, e.to_dict(), o.to_dict())
        errs = p.check()
        assert not errs, (p.rounds, errs[:2])
        st["slow"] += e.elections_stepped
        st["dropped"] += e.dropped_proposals


def _request(p, slot, targets):
    bo = p.orc.request_leader_transfer(slot, targets)
    be = p.eng.request_leader_transfer(slot, targets)
    assert be == bo
    return be


def _leader(p, g):
    """The group's one leader (replica ID), 0 while it has none or two (a
    campaign in flight, a deposed leader not yet told)."""
    ls = [s for s, st in enumerate(p.eng.export_replicas(g, 1))
          if st.role == abi.LEADER]
    return ls[0] + 1 if len(ls) == 1 else 0


@pytest.mark.parametrize("R,pre_vote,at", [(3, 0, "leader"),
                                           (3, 1, "leader"),
                                           (5, 0, "follower"),
                                           (5, 1, "follower")])
def test_leader_transfer_on_gpu(R, pre_vote, at):
    """Transfers to up-to-date followers under a write + read load,
    requested at the leader or at a follower (naming itself or another
    follower); the new leaders serve, and a second transfer hands some
    groups back."""
    G = 24
    p = Pair(G=G, R=R, elections=1, pre_vote=pre_vote)
    st = {"slow": 0, "dropped": 0}
    _rounds(p, 3, st)
    # A target campaigns on TimeoutNow only when it has applied everything
    # it committed (hasConfigChangeToApply, raft.go:1611-1622, checked by
    # handleNodeElection).  Under a steady write load the TimeoutNow a
    # ReplicateResp triggers arrives with the commit that ReplicateResp
    # advanced, so the target ignores it and the transfer times out -- the
    # oracle and the GPU agree on that.  The requests therefore come after
    # two rounds without writes, and writes resume the round after.
    _rounds(p, 2, st, k=0)
    want = {}
    targets = [0] * G
    slot = 0 if at == "leader" else R - 1
    for i, g in enumerate(range(0, G, 3)):
        # leader: to replica 2..R in turn; follower: itself or replica 2
        t = (2 + i % (R - 1)) if at == "leader" else (R if i % 2 else 2)
        targets[g] = want[g] = t
    assert _request(p, slot, targets) == 0
    # a second request before the first is taken is refused (busy)
    assert _request(p, slot, targets) == len(want)
    _rounds(p, 1, st, k=0)
    for _ in range(40):
        _rounds(p, 1, st)
        if all(_leader(p, g) == t for g, t in want.items()):
            break
    for g, t in want.items():
        assert _leader(p, g) == t, (g, t)
        sts = p.eng.export_replicas(g, 1)
        assert sts[t - 1].term == 3 and all(x.transfer == 0 for x in sts)
    others = [g for g in range(G) if g not in want]
    assert all(_leader(p, g) == 1 for g in others)
    assert st["slow"] > 0 and st["dropped"] > 0
    _rounds(p, 6, st)  # writes and reads under the new leaders
    # hand half of them back to replica 1, requested at the new leader
    back = sorted(want)[::2]
    _rounds(p, 2, st, k=0)
    for s in range(1, R):
        tg = [1 if g in back and want[g] == s + 1 else 0 for g in range(G)]
        if any(tg):
            assert _request(p, s, tg) == 0
    _rounds(p, 1, st, k=0)
    for _ in range(40):
        _rounds(p, 1, st)
        if all(_leader(p, g) == 1 for g in back):
            break
    assert all(_leader(p, g) == 1 for g in back)
    _rounds(p, 4, st)


def test_leader_transfer_timeout_and_noops_on_gpu():
    """A transfer to a stopped replica: the leader drops every proposal
    while it waits and abandons the transfer after an election timeout
    (raft.go:622-636), then takes writes again.  Transfers to the leader
    itself are ignored (raft.go:1936-1939)."""
    G, R = 16, 3
    p = Pair(G=G, R=R, elections=1)
    st = {"slow": 0, "dropped": 0}
    _rounds(p, 3, st)
    E = [4, 9]
    _unhost(p, E, 2)
    _rounds(p, 2, st)
    assert _request(p, 0, [3 if g in E else 0 for g in range(G)]) == 0
    _rounds(p, 1, st)
    for g in E:
        assert p.eng.export_replicas(g, 1)[0].transfer == 3
    d0 = st["dropped"]
    last = {g: p.eng.export_replicas(g, 1)[0].last_index for g in E}
    _rounds(p, 4, st)
    assert st["dropped"] - d0 == 4 * len(E)  # one write per group per round
    for g in E:
        assert p.eng.export_replicas(g, 1)[0].last_index == last[g]
    _rounds(p, 8, st)  # the election timeout (10 ticks) passes
    for g in E:
        lead = p.eng.export_replicas(g, 1)[0]
        assert lead.role == abi.LEADER and lead.transfer == 0
        assert lead.last_index > last[g]
    # self-transfers are no-ops
    assert _request(p, 0, [1] * G) == 0
    _rounds(p, 3, st)
    assert all(_leader(p, g) == 1 for g in range(G))


def test_leader_transfer_needs_elections():
    p = Pair(G=8, R=3)
    with pytest.raises(DrbError):
        p.eng.request_leader_transfer(0, [2] * 8)
