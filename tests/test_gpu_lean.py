"""GPU: the lean kernel of listed rounds (drb_lean.hpp).

In a listed round the heartbeat-only replicas of quiet groups -- C5's common
case: a tick, a Heartbeat or HeartbeatResp, node.qs -- go through
lean_kernel, and every other light replica is escalated, untouched, to the
full step kernel (handleFollowerHeartbeat / handleLeaderHeartbeatResp,
raft.go:1400-1409, 1910-1923, 2128; quiesce.go:40-114; raft.go:571-648).
Checked here on C5 in miniature (1-2 % of the groups proposing per round,
116 B values, EntryBatch saves, Quiesce with a short threshold so that
groups quiesce, wake and quiesce again): the engine with the lean kernel
and one with it off (drb_config.no_lean) stay identical every round --
state records, logs, KV, outboxes, saves, counters -- and both equal the
oracle.
"""
import pytest

from dragonboat_amd import workload
from dragonboat_amd.engine import Engine
from tests.gpu_harness import Pair, by_dest, state_diff

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,ppm,tick_every", [(3, 20000, 1), (3, 10000, 2),
                                              (5, 20000, 1)])
def test_lean_rounds_match_full_kernel_and_oracle(R, ppm, tick_every):
    G, VAL, ERTT = 512, 116, 4
    kw = dict(cmd_cap=144, kv_val_cap=128, kv_slots=32, max_props=2,
              save_cap=8192, prop_slots=2)
    p = Pair(G=G, R=R, election_rtt=ERTT, quiesce=True, **kw)
    full = Engine(num_groups=G, num_replicas=R, window=32,
                  election_rtt=ERTT, quiesce=1, no_lean=1, **kw)
    full.init_steady(term=2, leader_slot=0, seed=p.seed)
    stepped = lean = 0
    for r in range(160):
        act = workload.active_groups(G, p.seed, r, ppm)
        counts, ents, pool = workload.build_batch(G, 1, p.seed, r, 256, VAL,
                                                  groups=act)
        p.orc.stage_proposals(counts, 1, ents, pool)
        for e in (p.eng, full):
            e.gen_kv_proposals(r % 2, 1, 256, VAL, p.seed, r,
                               active_ppm=ppm)
        tick = r % tick_every == 0
        o = p.orc.round(tick=tick)
        a = p.eng.step(tick=tick, prop_slot=r % 2, encode_saves=True,
                       listed=True)
        b = full.step(tick=tick, prop_slot=r % 2, encode_saves=True,
                      listed=True)
        p.rounds += 1
        assert a.fallbacks == 0 and a.errors == 0, (r, p.why())
        da, db = a.to_dict(), b.to_dict()
        lean += da.pop("lean_stepped")
        assert db.pop("lean_stepped") == 0
        assert da == db, (r, da, db)
        assert (a.committed_entries, a.applied_entries, a.messages) == \
            (o.committed_entries, o.applied_entries, o.messages), r
        stepped += a.replicas_stepped
        if r % 8 == 7:
            for g in range(0, G, 3):
                sa, sb = p.eng.export_replicas(g, 1), full.export_replicas(g, 1)
                for s in range(R):
                    assert not state_diff(sa[s], sb[s], R), (r, g, s)
                    assert by_dest(p.eng.export_outbox(g, s)) == \
                        by_dest(full.export_outbox(g, s)), (r, g, s)
                    assert p.eng.export_saved(g, s) == \
                        full.export_saved(g, s), (r, g, s)
        if r % 40 == 39:
            errs = p.check()
            assert not errs, (r, errs[:2])
            assert not p.check_saves(), r
    quiesced = sum(st.qs_quiesced_since > 0 for g in range(G)
                   for st in p.eng.export_replicas(g, 1))
    # (quiesce takes 20 x ElectionRTT = 80 idle ticks: 160 rounds ticking
    # every round get there, every other round not)
    assert stepped > 0 and (quiesced > 0 or tick_every > 1), \
        (quiesced, stepped)
    # most stepped replicas of a quiet round ran the lean kernel
    assert lean > stepped // 2, (lean, stepped)
    full.close()


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_lean_rounds_random_mix(seed):
    """Random activity (0-20 % of the groups proposing), ticks on ~3 rounds
    in 4 and EntryBatch encoding switched on and off from round to round,
    with Quiesce: the round-6 shortcuts -- the quiesce base stored only by
    rounds that end quiesced and at rest, the lean ReadyToRead and save_len
    clears skipped where F_AT_REST / F_SAVE_ZERO say they are zero -- keep
    the engine equal to the oracle (state every 10 rounds, every encoded
    round's saves) and to an engine without the lean kernel."""
    import random
    rng = random.Random(seed)
    G, R, VAL, ERTT = 384, 3, 116, 4
    kw = dict(cmd_cap=144, kv_val_cap=128, kv_slots=32, max_props=2,
              save_cap=8192, prop_slots=2)
    p = Pair(G=G, R=R, election_rtt=ERTT, quiesce=True, **kw)
    full = Engine(num_groups=G, num_replicas=R, window=32,
                  election_rtt=ERTT, quiesce=1, no_lean=1, **kw)
    full.init_steady(term=2, leader_slot=0, seed=p.seed)
    lean = 0
    for r in range(150):
        ppm = rng.choice([0, 0, 2000, 20000, 200000])
        tick = rng.random() < 0.75
        enc = rng.random() < 0.7
        act = workload.active_groups(G, p.seed, r, ppm)
        counts, ents, pool = workload.build_batch(G, 1, p.seed, r, 256, VAL,
                                                  groups=act)
        p.orc.stage_proposals(counts, 1, ents, pool)
        for e in (p.eng, full):
            e.gen_kv_proposals(r % 2, 1, 256, VAL, p.seed, r,
                               active_ppm=ppm)
        o = p.orc.round(tick=tick)
        a = p.eng.step(tick=tick, prop_slot=r % 2, encode_saves=enc,
                       listed=True)
        b = full.step(tick=tick, prop_slot=r % 2, encode_saves=enc,
                      listed=True)
        p.rounds += 1
        assert a.fallbacks == 0 and a.errors == 0, (r, p.why())
        da, db = a.to_dict(), b.to_dict()
        lean += da.pop("lean_stepped")
        db.pop("lean_stepped")
        assert da == db, (r, da, db)
        assert (a.committed_entries, a.applied_entries, a.messages) == \
            (o.committed_entries, o.applied_entries, o.messages), r
        if enc:
            assert not p.check_saves(), r
            for g in range(0, G, 17):
                for s in range(R):
                    assert p.eng.export_saved(g, s) == \
                        full.export_saved(g, s), (r, g, s)
        if r % 10 == 9:
            errs = p.check()
            assert not errs, (r, errs[:2])
    assert lean > 0
    full.close()
