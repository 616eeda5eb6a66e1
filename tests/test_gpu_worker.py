"""GPU: a step worker's round outputs without a host synchronisation
(drb_worker_export / drb_worker_wait; engine.processSteps, engine.go:
1304-1364 -> node.processReadyToRead node.go:1081, pendingReadIndex.applied
request.go:930-953, pendingProposals.applied node.go:243-257).

Each round's export is enqueued behind the round and drained into pinned
host buffers on a copy stream while the next round runs; two buffer sets
alternate, as a worker would use them.  Every export is compared with the
oracle cluster: the ReadyToReads of the slot, the ReadLocalNode result of
every served read (found, length, value) and the applied entries with their
Result.Value, in group order.
"""
import struct

import pytest

from dragonboat_amd import workload
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu

READS = 9
KEYS = 16


def _read_key(low, j):
    return workload.mix64(low ^ (((j + 1) * workload.GOLDEN) &
                                 workload.MASK)) % KEYS


def _want(p, slot):
    """(ReadyToReads with their values, applied) of the oracle's last round
    for replica slot `slot`, in the export's layout."""
    reads, applied = [], []
    for g in range(p.G):
        st = p.orc.export(g, slot)
        kv = p.orc.export_kv(g, slot)
        for (index, low, high) in p.orc.export_ready(g, slot):
            vals = []
            if index <= st.sm_index:
                for j in range(READS):
                    v = kv.get(struct.pack("<Q", _read_key(low, j)))
                    vals.append(0 if v is None else
                                int.from_bytes(v[:4], "little") |
                                ((len(v) | 1 << 31) << 32))
            reads.append(((g, index, low, high), vals))
    return reads, applied


def _got(b, n_reads, n_values):
    out = []
    for i in range(n_reads):
        r = b.reads[i]
        end = b.reads[i + 1].first if i + 1 < n_reads else n_values
        vals = [b.values[j] for j in range(r.first, end)]
        out.append(((r.group, r.index, r.ctx_low, r.ctx_high), vals))
    return out


@pytest.mark.parametrize("ri_replica", [0, 2])
def test_worker_export_matches_the_oracle(ri_replica):
    G, R = 300, 3
    p = Pair(G=G, R=R, max_reads_per_ctx=READS)
    slot = 0 if ri_replica == 0 else ri_replica - 1
    bufs = [p.eng.worker_bufs(4 * G, 4 * G * READS, 4 * G) for _ in range(2)]
    pending = None
    n_app = 0
    try:
        for rnd in range(12):
            o, e = p.round(k=1 + rnd % 2, tick=(rnd % 2 == 0),
                           read_index=True, reads=READS, read_key_space=KEYS,
                           key_space=KEYS, ri_replica=ri_replica)
            assert e.fallbacks == 0 and e.errors == 0, (rnd, e.to_dict())
            b = bufs[rnd % 2]
            p.eng.worker_export(slot, b)
            want_reads, _ = _want(p, slot)
            want_app = [(a[0], a[2], a[5], a[6])
                        for a in p.eng.apply_results(slot)]
            # the previous round's export may still be draining: wait for
            # this one (which is ordered after it)
            nr, nv, na = p.eng.worker_wait(b)
            assert _got(b, nr, nv) == want_reads, rnd
            assert nv == sum(len(v) for _, v in want_reads)
            got_app = [(b.applied[i].group, b.applied[i].key,
                        b.applied[i].value, b.applied[i].ignored)
                       for i in range(na)]
            assert got_app == want_app, rnd
            n_app += na
            pending = b
        assert n_app > G * 10
    finally:
        p.eng.sync()
        for b in bufs:
            p.eng.free_worker_bufs(b)


def test_worker_export_reports_overflow():
    """A buffer smaller than the round's records: the counts are the full
    ones and drb_worker_wait says DRB_ERANGE; the first cap records are
    there."""
    G, R = 64, 3
    p = Pair(G=G, R=R, max_reads_per_ctx=READS)
    for rnd in range(3):
        p.round(k=1, tick=True, read_index=True, reads=READS,
                read_key_space=KEYS, key_space=KEYS)
    full = p.eng.worker_bufs(4 * G, 4 * G * READS, 4 * G)
    small = p.eng.worker_bufs(8, 8, 8)
    try:
        p.eng.worker_export(0, full)
        nr, nv, na = p.eng.worker_wait(full)
        p.eng.worker_export(0, small)
        with pytest.raises(Exception):
            p.eng.worker_wait(small)
        assert (small.n_reads, small.n_values, small.n_applied) == (nr, nv, na)
        assert [small.values[i] for i in range(8)] == \
            [full.values[i] for i in range(8)]
        assert [(small.applied[i].group, small.applied[i].key)
                for i in range(8)] == \
            [(full.applied[i].group, full.applied[i].key) for i in range(8)]
    finally:
        p.eng.sync()
        p.eng.free_worker_bufs(full)
        p.eng.free_worker_bufs(small)
