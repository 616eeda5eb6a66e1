"""GPU: the KV grows past kv_slots (drb_config.kv_overflow_buckets).

KVTest's state machine is a Go map (internal/tests/kvtest.go:145-162): it
never fills.  The device table is a fixed open-addressing table per
replica; with overflow buckets a full table chains 4-slot buckets from an
engine-wide pool, so the apply keeps going where the fixed table would stop
(test_gpu_fallback.py::test_kv_full_stops_apply_after_the_round).  Checked
bit-exact against the oracle every round: states, logs, the KV contents
(drb_kv_export walks the chain), messages, ReadyToReads and the reads
served in-round (lookups that miss a full table walk the chain).
"""
import pytest

from dragonboat_amd import abi
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu


def _rounds(p, rounds, val_len, key_space=64):
    total = 0
    for r in range(rounds):
        o, e = p.round(k=2, tick=(r % 3 == 0), read_index=True, reads=9,
                       read_key_space=key_space, key_space=key_space,
                       val_len=val_len)
        assert e.fallbacks == 0 and e.errors == 0, (r, p.why())
        assert (e.committed_entries, e.applied_entries, e.messages,
                e.ready_to_reads) == (o.committed_entries, o.applied_entries,
                                      o.messages, o.ready_to_reads), r
        sums, served, deferred = p.orc.serve_reads(9, key_space)
        assert (e.reads_served, e.reads_deferred) == (served, deferred), r
        esums = p.eng.export_read_sums(0, p.G)
        for i, x in enumerate(sums):
            if x is not None:
                assert esums[i] == x, (r, i)
        total += served
        errs = p.check()
        assert not errs, (r, errs[:2])
    return total


@pytest.mark.parametrize("val_len,cmd_cap,val_cap", [
    (4, 32, 4),        # C3 16 B payload, value inline
    (60, 80, 64),      # a value crossing the 64 B header window, inline
    (116, 144, 128)])  # C5 128 B payload, value out of line
def test_kv_grows_past_the_table(val_len, cmd_cap, val_cap):
    G = 16
    p = Pair(G=G, R=3, cmd_cap=cmd_cap, kv_val_cap=val_cap, kv_slots=4,
             kv_overflow_buckets=G * 3 * 16, max_props=4)
    served = _rounds(p, 30, val_len)
    assert served > 0
    # the tables overflowed: more keys than slots on every replica
    counts = [len(p.eng.kv_export(g, s)) for g in range(G) for s in range(3)]
    assert min(counts) > 4, counts
    for g in (0, G - 1):  # point lookups through the chain
        okv = p.orc.export_kv(g, 1)
        for k, x in okv.items():
            assert p.eng.kv_lookup(g, 1, k) == x, (g, k)
        assert p.eng.kv_lookup(g, 1, b"\xff" * 8) is None


@pytest.mark.parametrize("val_len,cmd_cap,val_cap", [(4, 32, 4),
                                                     (116, 144, 128)])
def test_kv_import_past_the_table(val_len, cmd_cap, val_cap):
    """drb_kv_import of more pairs than slots (the state machine a CPU
    group hands back, Pair.from_cpu): the rest go into fresh overflow
    buckets; export and lookup give back the same map, and the replicas
    keep applying on top of it in parity with the oracle."""
    G = 6
    p = Pair(G=G, R=3, cmd_cap=cmd_cap, kv_val_cap=val_cap, kv_slots=4,
             kv_overflow_buckets=G * 3 * 16, max_props=4)
    _rounds(p, 8, val_len)
    for g in range(G):
        for s in range(3):
            kv = p.orc.export_kv(g, s)
            assert len(kv) > 4, (g, s, len(kv))
            # a smaller map first, then the oracle's back: the chain is
            # replaced each time
            small = dict(list(kv.items())[:3])
            p.eng.kv_import(g, s, small)
            assert p.eng.kv_export(g, s) == small
            p.eng.kv_import(g, s, kv)
            assert p.eng.kv_export(g, s) == kv
            for k, x in kv.items():
                assert p.eng.kv_lookup(g, s, k) == x
    assert not p.check()
    _rounds(p, 8, val_len)


def test_kv_overflow_pool_exhausted_stops_apply():
    """Two buckets for the whole engine: once they are taken a full table
    stops the apply as without overflow (DRB_F_APPLY_STOPPED,
    DRB_FB_CAPACITY); the raft round itself completes."""
    p = Pair(G=8, R=3, kv_slots=4, kv_overflow_buckets=2)
    for r in range(20):
        o, e = p.round(k=1, tick=False)
        recs, _lost = p.eng.take_flagged()
        if recs:
            for (g, s, reason, flags, _rnd, _sid) in recs:
                assert reason == abi.FB["CAPACITY"], recs
                assert flags & abi.F_APPLY_STOPPED, recs
            return
        assert not p.check(), r
    raise AssertionError("the overflow pool never ran out")


@pytest.mark.parametrize("val_len,cmd_cap,val_cap,kv_slots", [
    (4, 32, 4, 64),
    (60, 80, 64, 4),       # inline values, through the chain
    (116, 144, 128, 64),   # C5 128 B: values out of line
    (116, 144, 128, 4)])
def test_read_values_whole(val_len, cmd_cap, val_cap, kv_slots):
    """drb_export_read_values: every served read's ReadLocalNode value
    whole (nodehost.go:849 -> KVTest.Lookup, kvtest.go:164-175), compared
    with the oracle's KV -- inline and out-of-line values, table and
    overflow chain."""
    import struct
    from dragonboat_amd import workload
    G, KS = 16, 64
    p = Pair(G=G, R=3, cmd_cap=cmd_cap, kv_val_cap=val_cap, kv_slots=kv_slots,
             kv_overflow_buckets=G * 3 * 16, max_props=4,
             max_reads_per_ctx=9)
    n = 0
    for r in range(12):
        o, e = p.round(k=2, tick=(r % 3 == 0), read_index=True, reads=9,
                       read_key_space=KS, key_space=KS, val_len=val_len)
        assert e.fallbacks == 0 and e.errors == 0, (r, p.why())
        got = p.eng.export_read_values(0, pool_cap=64)  # grows on ERANGE
        short = p.eng.export_read_results(0)
        assert [x[:6] for x in got] == [x[:6] for x in short], r
        for (g, index, low, j, key, found, val) in got:
            kv = p.orc.export_kv(g, 0)
            want = kv.get(struct.pack("<Q", key))
            assert val == want, (r, g, j)
            x = workload.mix64(low ^ (((j + 1) * workload.GOLDEN) &
                                      workload.MASK)) % KS
            assert key == x
        n += sum(1 for x in got if x[5])
    assert n > 100
