"""GPU: drb_step_rounds -- k rounds chunk by chunk of the groups.

Each chunk of the engine's groups runs all k rounds before the next chunk
starts (groups are independent: the reference steps each shard when it is
ready, engine.go:1316-1328).  The oracle cluster steps the same k rounds
with the same inputs round by round; after every call every replica field,
the logs, the KV, the outboxes and the ReadyToReads must be bit-exact, as
after k drb_step_round calls.  Ragged chunks (G not a multiple of the
chunk), k = 1, 2, 4, with writes, ReadIndex, ticks and served reads.
"""
import pytest

from dragonboat_amd import abi, workload
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu


def _rounds(p, k, base, reads, groups=None):
    """Stage k rounds of inputs (slot t) on both sides, step the oracle
    through them, and describe them for drb_step_rounds."""
    rs = []
    for t in range(k):
        salt = base + t
        counts, ents, pool = workload.build_batch(p.G, 1, p.seed, salt, 256,
                                                  4, groups)
        p.orc.stage_proposals(counts, 1, ents, pool)
        mp = p.eng.cfg["max_props"]
        eents = (abi.Entry * (p.G * mp))()
        for g in range(p.G):
            for j in range(counts[g]):
                eents[g * mp + j] = ents[g + j]
        p.eng.stage_proposals(t, counts, eents, pool)
        lo, hi = workload.build_read_index(p.G, p.seed, salt, salt + 30,
                                           groups)
        p.orc.stage_read_index(lo, hi)
        p.eng.stage_read_index(t, lo, hi)
        tick = (salt % 2 == 0)
        p.orc.round(tick=tick)
        if reads:
            p.orc.serve_reads(reads, 256)
        rs.append(dict(tick=tick, prop_slot=t, ri_slot=t,
                       reads_per_ctx=reads, key_space=256))
    return rs


def _sample(G, chunk):
    """Every chunk's first and last groups, and a seeded sample."""
    import random
    gs = set(random.Random(G).sample(range(G), min(G, 120)))
    for c in range(0, G, chunk):
        gs |= {c, c + 1, min(G, c + chunk) - 2, min(G, c + chunk) - 1}
    return sorted(g for g in gs if 0 <= g < G)


@pytest.mark.parametrize("G,chunk,k", [(1000, 256, 2), (1536, 512, 4),
                                       (700, 256, 1), (2048, 1024, 4),
                                       # one chunk of every group: plain
                                       # rounds from one call
                                       (1000, 1024, 4), (2048, 2048, 3)])
def test_rounds_by_chunk_match_the_oracle(G, chunk, k):
    p = Pair(G=G, R=3, prop_slots=4, ri_slots=4, max_props=1)
    sample = _sample(G, chunk)
    base = 0
    for call in range(5):
        rs = _rounds(p, k, base, reads=9 if call % 2 else 0)
        p.eng.step_rounds(rs, chunk)
        base += k
        out = p.eng.read_counters(reset=True)
        assert out.fallbacks == 0 and out.errors == 0, out.to_dict()
        assert out.round == base
        errs = p.check(groups=sample)
        assert not errs, (call, errs[:2])
    # and back to single rounds: the same engine continues bit-exact
    for r in range(3):
        o, e = p.round(k=1, tick=True, read_index=True)
        assert e.fallbacks == 0 and not p.check(groups=sample)


def test_rounds_refuses_what_it_does_not_chunk():
    p = Pair(G=256, R=3, elections=1)
    with pytest.raises(Exception, match="status -1"):
        p.eng.step_rounds([dict(tick=True)], 256)
    q = Pair(G=256, R=3)
    with pytest.raises(Exception, match="status -1"):
        q.eng.step_rounds([dict(tick=True)], 100)  # not a multiple of 256
