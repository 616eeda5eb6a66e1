"""GPU: a step worker's round outputs without a host synchronisation
(drb_worker_export / drb_worker_wait; engine.processSteps, engine.go:
1304-1364 -> node.processReadyToRead node.go:1081, pendingReadIndex.applied
request.go:930-953, pendingProposals.applied node.go:243-257).

Each round's export is enqueued behind the round and drained into pinned
host buffers on a copy stream while the next round runs; two buffer sets
alternate, as a worker would use them.  The records are the lean ones of
include/drb_engine.h: a word per lane (ReadyToReads, served mask, the
host's own proposals applied), the ctx tag per ReadyToRead, 4 B + a 2-bit
code per served read, the Index of each ReadyToRead whose reads were not
served.  Every export is decoded as a host walks it and compared with the
oracle cluster: the ReadyToReads of the slot, the ReadLocalNode result of
every served read and the applied count per lane (drb_apply_results'
entries of the host's session client), in group order.
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


def _result(v):
    """abi.worker_value's form of a KV value (None: not found)."""
    if v is None:
        return None
    v = bytes(v)
    return v if len(v) <= 4 else (v[:4], True)


def _want(p, slot):
    """Per lane, the oracle's last round for replica slot `slot` in the
    export's layout: [(ctx tag, [result per read] when served, else the
    ReadyToRead's Index)]."""
    out = {}
    for g in range(p.G):
        st = p.orc.export(g, slot)
        kv = p.orc.export_kv(g, slot)
        rs = []
        for (index, low, high) in p.orc.export_ready(g, slot):
            if index <= st.sm_index:
                rs.append((low & 0xFFFFFFFF, [
                    _result(kv.get(struct.pack("<Q", _read_key(low, j))))
                    for j in range(READS)]))
            else:
                rs.append((low & 0xFFFFFFFF, index))
        if rs:
            out[g] = rs
    return out


def _want_applied(p, slot, sess=None):
    """Per lane, how many of the last round's applied entries are the
    host's own proposals (drb_apply_results, pinned by test_gpu_parity):
    its session client's, or any client's when none is registered."""
    out = {}
    for (g, _i, _k, client, _s, _v, ignored) in p.eng.apply_results(slot):
        if not ignored and client and (sess is None or client == sess[g]):
            out[g] = out.get(g, 0) + 1
    return out


def _got(p, b, n_reads, n_values, n_deferred, lanes=None):
    """(reads per lane as _want, applied per lane) decoded from the lanes
    words, as a host walks them; lanes: the engine lanes the words are of
    (a partition's), in order."""
    reads, applied = {}, {}
    ri = vi = di = 0
    for i, g in enumerate(range(p.G) if lanes is None else lanes):
        nr, served, na = abi.worker_lane(b.lanes[i])
        rs = []
        for k in range(nr):
            tag = b.reads[ri]
            ri += 1
            if (served >> k) & 1:
                vals = []
                for _ in range(READS):
                    code = (b.value_meta[vi // 4] >> (2 * (vi & 3))) & 3
                    vals.append(abi.worker_value(code, b.values[vi]))
                    vi += 1
                rs.append((tag, vals))
            else:
                rs.append((tag, b.deferred[di]))
                di += 1
        if rs:
            reads[g] = rs
        if na:
            applied[g] = na
    assert (ri, vi, di) == (n_reads, n_values, n_deferred)
    return reads, applied


@pytest.mark.parametrize("ri_replica,host_copies", [(0, 0), (2, 0), (0, 1)])
def test_worker_export_matches_the_oracle(ri_replica, host_copies):
    """host_copies = 1: the download through hipMemcpyAsync on the worker's
    copy stream, the path an engine takes without the HSA copy engines
    (drb_config.host_copies), with the same records."""
    G, R = 300, 3
    p = Pair(G=G, R=R, max_reads_per_ctx=READS, host_copies=host_copies)
    slot = 0 if ri_replica == 0 else ri_replica - 1
    bufs = [p.eng.worker_bufs(4 * G, 4 * G * READS, 4 * G) for _ in range(2)]
    n_app = n_def = 0
    sess = None
    try:
        for rnd in range(12):
            if rnd == 6:
                # the host's NoOP sessions registered: a lane counts only
                # its session client's entries -- every third group's
                # registered client is not the one its entries carry
                sess = [workload.client_id(p.seed, g) ^ (2 if g % 3 == 0
                                                         else 0)
                        for g in range(G)]
                p.eng.set_session_clients(sess)
            o, e = p.round(k=1 + rnd % 2, tick=(rnd % 2 == 0),
                           read_index=True, reads=READS if rnd % 5 else 0,
                           read_key_space=KEYS, key_space=KEYS,
                           ri_replica=ri_replica)
            assert e.fallbacks == 0 and e.errors == 0, (rnd, e.to_dict())
            b = bufs[rnd % 2]
            p.eng.worker_export(slot, b)
            if rnd % 5:
                want_reads = _want(p, slot)
            else:  # a round without served reads: every ReadyToRead deferred
                want_reads = {g: [(lo & 0xFFFFFFFF, i) for (i, lo, _h) in
                                  p.orc.export_ready(g, slot)]
                              for g in range(G) if p.orc.export_ready(g, slot)}
            want_app = _want_applied(p, slot, sess)
            nr, nv, nd = p.eng.worker_wait(b)
            got_reads, got_app = _got(p, b, nr, nv, nd)
            assert got_reads == want_reads, rnd
            assert got_app == want_app, rnd
            n_app += sum(got_app.values())
            n_def += nd
        assert n_app > G * 8 and n_def > 0, (n_app, n_def)
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
        nr, nv, nd = p.eng.worker_wait(full)
        p.eng.worker_export(0, small)
        with pytest.raises(Exception):
            p.eng.worker_wait(small)
        assert (small.n_reads, small.n_values, small.n_deferred) == \
            (nr, nv, nd)
        assert [small.values[i] for i in range(8)] == \
            [full.values[i] for i in range(8)]
        assert [small.value_meta[i] for i in range(2)] == \
            [full.value_meta[i] for i in range(2)]
        assert [small.reads[i] for i in range(8)] == \
            [full.reads[i] for i in range(8)]
        assert [small.lanes[g] for g in range(G)] == \
            [full.lanes[g] for g in range(G)]
    finally:
        p.eng.sync()
        p.eng.free_worker_bufs(full)
        p.eng.free_worker_bufs(small)


def test_worker_export_refuses_pageable_buffers():
    """The copy engine writes the caller's buffers directly, so each must be
    pinned host memory from its first to its last byte: a
    pageable buffer, or one whose capacity runs past its pinned allocation,
    is DRB_EINVAL before anything is enqueued, and a good set still works
    after."""
    import ctypes as C
    G, R = 64, 3
    p = Pair(G=G, R=R, max_reads_per_ctx=READS)
    p.round(k=1, tick=True, read_index=True, reads=READS,
            read_key_space=KEYS, key_space=KEYS)
    b = p.eng.worker_bufs(4 * G, 4 * G * READS, 4 * G)
    # (an address, not the field: a ctypes pointer field shares its storage)
    lanes = C.cast(b.lanes, C.c_void_p).value
    cap = b.values_cap
    u32p = C.POINTER(C.c_uint32)
    try:
        page = (C.c_uint32 * G)()
        b.lanes = C.cast(page, C.POINTER(C.c_uint32))
        with pytest.raises(Exception, match="status -1"):
            p.eng.worker_export(0, b)
        b.lanes = C.cast(lanes, u32p)
        b.values_cap = cap * 64  # past the end of its pinned block
        with pytest.raises(Exception, match="status -1"):
            p.eng.worker_export(0, b)
        b.values_cap = cap
        p.eng.worker_export(0, b)
        p.eng.worker_wait(b)
    finally:
        b.lanes, b.values_cap = C.cast(lanes, u32p), cap
        p.eng.sync()
        p.eng.free_worker_bufs(b)


def test_worker_export_by_partition():
    """Step workers each export their own partition of the shards
    (drb_worker_export_part; engine.go:1036-1049 processSteps over workerID's
    shards, FixedPartitioner ShardID % 4, internal/server/partition.go:38):
    four partition exports and a whole-slot one in flight together, each
    into its own buffers, and every partition's records are the whole
    export's records of its lanes -- and the oracle's."""
    G, R, P = 301, 3, 4
    p = Pair(G=G, R=R, max_reads_per_ctx=READS)
    full = p.eng.worker_bufs(4 * G, 4 * G * READS, 4 * G)
    # lane g is ShardID g + 1: partition q holds lanes g0, g0 + 4, ...
    lanes = [[g for g in range(G) if (g + 1) % P == q] for q in range(P)]
    parts = [p.eng.worker_bufs(4 * G, 4 * G * READS, 4 * G,
                               lanes=len(lanes[q])) for q in range(P)]
    try:
        for rnd in range(8):
            o, e = p.round(k=1 + rnd % 2, tick=(rnd % 2 == 0),
                           read_index=True, reads=READS if rnd % 3 else 0,
                           read_key_space=KEYS, key_space=KEYS)
            assert e.fallbacks == 0 and e.errors == 0, (rnd, e.to_dict())
            p.eng.worker_export(0, full)
            for q in range(P):
                p.eng.worker_export(0, parts[q], P, q)
            want_app = _want_applied(p, 0)
            got_reads, got_app = _got(p, full, *p.eng.worker_wait(full))
            assert got_app == want_app, rnd
            if rnd % 3:
                assert got_reads == _want(p, 0), rnd
            for q in range(P):
                r_q, a_q = _got(p, parts[q], *p.eng.worker_wait(parts[q]),
                                lanes=lanes[q])
                assert r_q == {g: x for g, x in got_reads.items()
                               if g in lanes[q]}, (rnd, q)
                assert a_q == {g: x for g, x in got_app.items()
                               if g in lanes[q]}, (rnd, q)
    finally:
        p.eng.sync()
        for b in [full] + parts:
            p.eng.free_worker_bufs(b)
