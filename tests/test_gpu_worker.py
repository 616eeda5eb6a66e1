"""GPU: a step worker's round outputs without a host synchronisation
(drb_worker_export / drb_worker_wait; engine.processSteps, engine.go:
1304-1364 -> node.processReadyToRead node.go:1081, pendingReadIndex.applied
request.go:930-953, pendingProposals.applied node.go:243-257).

Each round's export is enqueued behind the round and drained into pinned
host buffers on a copy stream while the next round runs; two buffer sets
alternate, as a worker would use them.  The records are the lean ones of
include/drb_engine.h (a word per lane, Index + ctx Low per ReadyToRead, 4 B
+ a nibble per served read, 4 B per applied entry).  Every export is
decoded as a host walks it and compared with the oracle cluster: the
ReadyToReads of the slot, the ReadLocalNode result of every served read
(found, length, value) and the applied entries' Result.Value, in group
order.
"""
import struct

import pytest

from dragonboat_amd import abi, workload
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu

READS = 9
KEYS = 16


def _read_key(low, j):
    return workload.mix64(low ^ (((j + 1) * workload.GOLDEN) &
                                 workload.MASK)) % KEYS


def _nibble(v):
    """include/drb_engine.h value_meta: found, and the length (5: longer
    than 4 bytes)."""
    if v is None:
        return 0
    return abi.WORKER_FOUND | (abi.WORKER_LONG if len(v) > 4 else len(v))


def _want(p, slot):
    """Per lane, the oracle's last round for replica slot `slot` in the
    export's layout: [(index, ctx_low, [(value4, nibble) per read] or None
    when not served)]."""
    out = {}
    for g in range(p.G):
        st = p.orc.export(g, slot)
        kv = p.orc.export_kv(g, slot)
        rs = []
        for (index, low, high) in p.orc.export_ready(g, slot):
            vals = None
            if index <= st.sm_index:
                vals = []
                for j in range(READS):
                    v = kv.get(struct.pack("<Q", _read_key(low, j)))
                    vals.append((0 if v is None else
                                 int.from_bytes(v[:4], "little"),
                                 _nibble(v)))
            rs.append((index, low, vals))
        if rs:
            out[g] = rs
    return out


def _got(p, b, n_reads, n_values, n_applied):
    """(reads per lane as _want, applied [(lane, value, ignored)]) decoded
    from the lanes words, as a host walks them."""
    reads, applied = {}, []
    ri = vi = ai = 0
    for g in range(p.G):
        nr, served, na = abi.worker_lane(b.lanes[g])
        rs = []
        for k in range(nr):
            r = b.reads[ri]
            ri += 1
            vals = None
            if (served >> k) & 1:
                vals = []
                for _ in range(READS):
                    nib = (b.value_meta[vi // 2] >> (4 * (vi & 1))) & 0xF
                    vals.append((b.values[vi] if nib else 0, nib))
                    vi += 1
            rs.append((r.index, r.ctx_low, vals))
        if rs:
            reads[g] = rs
        for _ in range(na):
            a = b.applied[ai]
            ai += 1
            applied.append((g, a & 0x7FFFFFFF,
                            int(bool(a & abi.WORKER_IGNORED))))
    assert (ri, vi, ai) == (n_reads, n_values, n_applied)
    return reads, applied


@pytest.mark.parametrize("ri_replica", [0, 2])
def test_worker_export_matches_the_oracle(ri_replica):
    G, R = 300, 3
    p = Pair(G=G, R=R, max_reads_per_ctx=READS)
    slot = 0 if ri_replica == 0 else ri_replica - 1
    bufs = [p.eng.worker_bufs(4 * G, 4 * G * READS, 4 * G) for _ in range(2)]
    n_app = 0
    try:
        for rnd in range(12):
            o, e = p.round(k=1 + rnd % 2, tick=(rnd % 2 == 0),
                           read_index=True, reads=READS, read_key_space=KEYS,
                           key_space=KEYS, ri_replica=ri_replica)
            assert e.fallbacks == 0 and e.errors == 0, (rnd, e.to_dict())
            b = bufs[rnd % 2]
            p.eng.worker_export(slot, b)
            want_reads = _want(p, slot)
            # drb_apply_results (pinned by test_gpu_parity): (lane, value,
            # ignored); the keys are the host's own staged proposals
            want_app = [(a[0], a[5], a[6]) for a in p.eng.apply_results(slot)]
            nr, nv, na = p.eng.worker_wait(b)
            got_reads, got_app = _got(p, b, nr, nv, na)
            assert got_reads == want_reads, rnd
            assert got_app == want_app, rnd
            n_app += na
        assert n_app > G * 10
    finally:
        p.eng.sync()
        for b in bufs:
            p.eng.free_worker_bufs(b)


def test_worker_export_refuses_a_buffer_in_flight():
    """One export in flight per buffer set: exporting into a
    buffer whose export was not waited for is DRB_EAGAIN."""
    G, R = 64, 3
    p = Pair(G=G, R=R, max_reads_per_ctx=READS)
    p.round(k=1, tick=True, read_index=True, reads=READS,
            read_key_space=KEYS, key_space=KEYS)
    b = p.eng.worker_bufs(4 * G, 4 * G * READS, 4 * G)
    try:
        p.eng.worker_export(0, b)
        with pytest.raises(Exception, match="status -6"):
            p.eng.worker_export(0, b)
        p.eng.worker_wait(b)
        p.eng.worker_export(0, b)  # waited for: accepted again
        p.eng.worker_wait(b)
    finally:
        p.eng.sync()
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
        assert [small.value_meta[i] for i in range(4)] == \
            [full.value_meta[i] for i in range(4)]
        assert [small.applied[i] for i in range(8)] == \
            [full.applied[i] for i in range(8)]
        assert [small.lanes[g] for g in range(G)] == \
            [full.lanes[g] for g in range(G)]
    finally:
        p.eng.sync()
        p.eng.free_worker_bufs(full)
        p.eng.free_worker_bufs(small)
