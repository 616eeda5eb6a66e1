"""GPU: randomized rounds over the features together, bit-exact every round.

Each round draws, from a seeded generator: how many proposals a group
queues (0-2) and at which replica (the leader, a follower, a nonVoting --
drb_round_in.prop_replica with forward_proposals), whether a LocalTick
fires, whether a ReadIndex batch is staged and at which replica, and now
and then a replica slot of some groups stops or comes back (elections on
the GPU re-elect where a leader stopped).  Member kinds vary by case (all
voters; a witness; a nonVoting).  After every round the engine is compared
with the oracle cluster (the reference step loop: tests/gpu_harness.py):
every replica field, the logs, the KV, the outboxes and the ReadyToReads,
and the round counters.  A replica may leave the GPU only through a
capacity bound (the device ReadIndex queue, a mailbox): its group then runs
on the CPU path (the oracle) until it settles and is imported back, as in
production; an invariant error never.
"""
import os
import random

import pytest

from dragonboat_amd import abi
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu


def _set_hosted(p, groups, slot, hosted):
    for g in groups:
        p.orc.set_hosted(g, slot, hosted)
        sts = p.eng.export_replicas(g, 1)
        if hosted:
            sts[slot].flags |= abi.F_HOSTED
        else:
            sts[slot].flags &= ~abi.F_HOSTED
        p.eng.import_replicas(g, sts)


def _seeds():
    # DRB_SOAK_SEEDS="a-b" widens the run (tools, not the default suite)
    r = os.environ.get("DRB_SOAK_SEEDS")
    if r:
        a, b = (int(x) for x in r.split("-"))
        return list(range(a, b + 1))
    return [11, 12]


@pytest.mark.parametrize("case", ["voters", "witness", "nonvoting"])
@pytest.mark.parametrize("seed", _seeds())
def test_random_rounds(case, seed):
    rng = random.Random(seed * 1000 + len(case))
    G, R = 48, 4
    kw = {}
    if case != "voters":
        kw[case + "_slots"] = 1 << 3
    # (the pre-pass's per-follower mailbox bound -- the broadcasts every
    # follower gets plus what that follower's own records cause -- stays
    # within 16 on this mix: tools/mailbox_bound.py against the oracle)
    p = Pair(G=G, R=R, elections=1, forward_proposals=1, max_props=2,
             mailbox=16, **kw)
    # replica IDs (0: the leader); a witness neither proposes nor reads
    ids = [0, 1, 2, 3] + ([4] if case != "witness" else [])
    stopped = {}  # slot -> groups
    committed = fallbacks = ri_full = 0
    for rnd in range(40):
        # now and then a replica slot of a third of the groups stops, or
        # the stopped ones come back
        if rnd % 8 == 3 and not stopped:
            s = rng.choice([0, 1, 2])
            gs = [g for g in range(G) if rng.random() < 0.33]
            _set_hosted(p, gs, s, False)
            stopped[s] = gs
        elif rnd % 8 == 7 and stopped:
            for s, gs in stopped.items():
                _set_hosted(p, gs, s, True)
            stopped = {}
        # (clients reach running NodeHosts only)
        up = [i for i in ids if i == 0 or (i - 1) not in stopped]
        k = rng.choice([0, 1, 1, 2])
        o, e = p.round(k=k, tick=rng.random() < 0.7,
                       read_index=rng.random() < 0.5,
                       ri_replica=rng.choice(up),
                       prop_replica=rng.choice(up) if k else 0)
        assert e.errors == 0, (rnd, e.to_dict(), p.why())
        # a capacity bound of the device (the ReadIndex queue, a mailbox)
        # hands the group to the CPU path, as in production: the oracle --
        # the reference step loop -- steps it until it settles, then it
        # comes back (include/drb_engine.h DRB_FB_*)
        recs, lost = p.eng.take_flagged()
        assert lost == 0
        for (g, s, reason, flags, _, _) in recs:
            assert reason == abi.FB["CAPACITY"] and \
                not flags & abi.F_ERROR, (rnd, g, s, reason, flags)
            if g not in p.cpu:
                st = p.eng.export_replicas(g, 1)[s]
                ri_full += st.ri_count == abi.DRB_RI_DEPTH
                if os.environ.get("DRB_SOAK_VERBOSE") and fallbacks < 2:
                    d = st.to_dict(p.R)
                    print("fallback", rnd, g, s, {k: d[k] for k in (
                        "last_index", "committed", "ri_count", "remotes",
                        "ring_lo", "term_start") if k in d}, d["ri"])
                p.to_cpu(g)
                fallbacks += 1
        if not recs and not p.cpu:
            assert (e.committed_entries, e.messages, e.ready_to_reads,
                    e.dropped_proposals) == \
                (o.committed_entries, o.messages, o.ready_to_reads,
                 o.dropped_proposals), (rnd, e.to_dict(), o.to_dict())
        errs = p.check()  # (the groups on the GPU path)
        assert not errs, (rnd, errs[:2])
        for g in sorted(p.cpu):
            if not stopped and p.settled(g):
                p.from_cpu(g)
        committed += e.committed_entries
    assert committed > G * 10
    # the default seeds run without a single capacity fallback; wider runs
    # (DRB_SOAK_SEEDS) may meet the ReadIndex queue's depth now and then
    if not os.environ.get("DRB_SOAK_SEEDS"):
        assert fallbacks == 0, fallbacks
    assert fallbacks <= G, fallbacks  # the GPU path stays the main one
    print("soak %s/%d: %d capacity fallbacks, %d at a full ReadIndex queue"
          % (case, seed, fallbacks, ri_full))
