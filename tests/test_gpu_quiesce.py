"""GPU: Quiesce bit-exact against the oracle.

quiesceState (quiesce.go:23-120) per replica: after 20 x ElectionRTT idle
ticks a replica quiesces, tells its peers (sendEnterQuiesceMessages,
node.go:993-1005) and its ticks become quiesced ticks (raft.quiescedTick,
raft.go:650-656: no heartbeats, no CheckQuorum, no election); any
non-heartbeat message wakes it (record, quiesce.go:56-74).  On the engine a
quiesced replica at rest skips tick rounds and has the skipped ticks
applied when it next runs; the exported state includes them.
"""
import pytest

from dragonboat_amd import abi, workload
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu


def _quiesced(p):
    n = 0
    for g in range(p.G):
        for st in p.eng.export_replicas(g, 1):
            n += st.qs_quiesced_since > 0
    return n


@pytest.mark.parametrize("ppm,ri,listed", [(20000, False, False),
                                           (5000, True, False),
                                           (5000, True, True)])
def test_quiesce_sparse_activity(ppm, ri, listed):
    """Sparse proposals (a seeded ppm of the groups per round) and
    ReadIndex on a few groups, a LocalTick every round, ElectionRTT 4
    (threshold 80 ticks): groups quiesce, wake on proposals / reads and
    quiesce again; every field, log, KV, message (Quiesce messages
    included) stays bit-exact -- also in listed rounds (only the replicas
    with work stepped, drb_round_in.listed)."""
    p = Pair(G=40, R=3, election_rtt=4, quiesce=True, max_props=2,
             prop_slots=2)
    peak = woke = 0
    prev = 0
    for r in range(220):
        act = workload.active_groups(p.G, p.seed, r, ppm)
        o, e = p.round(k=1, tick=True, groups=act,
                       read_index=ri and r % 7 == 3,
                       prop_slot=r % 2, listed=listed)
        assert e.fallbacks == 0 and e.errors == 0, (r, p.why())
        assert (e.committed_entries, e.applied_entries, e.messages,
                e.ready_to_reads) == (o.committed_entries, o.applied_entries,
                                      o.messages, o.ready_to_reads), r
        if r % 5 == 4 or r > 210:
            errs = p.check()
            assert not errs, (r, errs[:2])
            q = _quiesced(p)
            if q < prev:
                woke += 1
            prev = q
            peak = max(peak, q)
    assert peak >= p.R, peak     # whole groups quiesced at some point
    assert woke > 0              # and activity woke some of them


def test_quiesce_idle_then_wake_all():
    """Every group idle past the threshold: all replicas quiesce and stay
    quiesced with ticks skipped on the device; then one round of
    proposals to every group wakes them all (TestNodesCanEnterQuiesce,
    TestNodesCanExitQuiesceByMakingProposal, node_test.go:884-937)."""
    p = Pair(G=32, R=3, election_rtt=4, quiesce=True)
    for r in range(100):
        o, e = p.round(k=0, tick=True)
        assert e.fallbacks == 0 and e.errors == 0, (r, p.why())
    assert not p.check()
    assert _quiesced(p) == p.G * p.R
    for r in range(30):  # quiesced ticks only: the device skips them
        p.round(k=0, tick=True)
    assert not p.check()
    assert _quiesced(p) == p.G * p.R
    for r in range(4):
        o, e = p.round(k=1 if r == 0 else 0, tick=True)
        assert e.fallbacks == 0 and e.errors == 0, (r, p.why())
        assert not p.check(), r
    assert _quiesced(p) == 0


@pytest.mark.parametrize("listed", [False, True])
def test_quiesced_replicas_skip_tick_rounds(listed):
    """Quiesced replicas at rest do not run tick rounds at all
    (replicas_stepped), yet export the ticks they skipped; a round with a
    few proposals steps just those groups' replicas."""
    p = Pair(G=64, R=3, election_rtt=4, quiesce=True)
    for r in range(100):
        p.round(k=0, tick=True, listed=listed)
    o, e = p.round(k=0, tick=True, listed=listed)
    assert e.replicas_stepped == 0, e.to_dict()
    for r in range(5):
        o, e = p.round(k=1, tick=True, groups=[5, 40], listed=listed)
        assert e.fallbacks == 0 and e.errors == 0, p.why()
        assert e.replicas_stepped <= 2 * 3, e.to_dict()
    assert not p.check()
