"""GPU: two transport threads ingest at once (include/drb_engine.h
drb_ingest_wire: "may be called from several transport threads").

Each thread owns its pinned receive buffer (drb_ingest_buffer_alloc, one
per connection as the reference's TCP transport has one receive path per
connection, transport/tcp.go:500-560) and hands its own NodeHost's byte
stream to drb_ingest_wire while the other thread does the same; a third
thread launches rounds meanwhile in the second test (drb_step_round takes
the ingest lock, so a call lands wholly before or after a round).  The
messages are the PreVote cases of test_gpu_prevote.py, from replica 3 of
every group, the groups split between the two connections; the oracle
takes the same messages, and the round after is compared bit-exactly.
"""
import ctypes as C
import threading

import pytest

from dragonboat_amd import abi
from oracle import pyoracle as po
from tests import wire_ref as wr
from tests.gpu_harness import Pair
from tests.test_gpu_prevote import MSG, _round, _unhost

pytestmark = pytest.mark.gpu

DID = 0xD1D


def _msgs(p, groups):
    out = []
    for g in groups:
        lead = p.eng.export_replicas(g, 1)[0]
        t, last, sid = lead.term, lead.last_index, g + 1
        kind = g % 4
        if kind == 0:    # term + 1 at the leader: the lease drops it
            out.append(po.msg(MSG["RequestPreVote"], from_=3, to=1,
                              term=t + 1, log_index=last, log_term=t,
                              shard_id=sid))
        elif kind == 1:  # a lower term: NoOP back
            out.append(po.msg(MSG["RequestPreVote"], from_=3, to=2,
                              term=t - 1, log_index=last, log_term=t - 1,
                              shard_id=sid))
        elif kind == 2:  # the current term: rejected
            out.append(po.msg(MSG["RequestPreVote"], from_=3, to=2,
                              term=t, log_index=last, log_term=t,
                              shard_id=sid))
        else:            # a heartbeat response at the leader's term
            out.append(po.msg(MSG["HeartbeatResp"], from_=3, to=1, term=t,
                              shard_id=sid))
    return out


def _two_connections(p, G):
    halves = [list(range(0, G, 2)), list(range(1, G, 2))]
    msgs = [_msgs(p, h) for h in halves]
    streams = [wr.expected_stream(m, DID, b"10.0.0.%d:26001" % (9 + i))
               for i, m in enumerate(msgs)]
    bufs = [p.eng.ingest_buffer_alloc(len(s)) for s in streams]
    for b, s in zip(bufs, streams):
        C.memmove(b, s, len(s))
    return msgs, streams, bufs


def _ingest_both(p, streams, bufs):
    got, errs = [None, None], []
    start = threading.Barrier(2)

    def conn(i):
        try:
            start.wait()
            got[i] = p.eng.ingest_wire_pinned(bufs[i], len(streams[i]), DID)
        except Exception as ex:  # surfaced below
            errs.append(ex)

    th = [threading.Thread(target=conn, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    assert not errs, errs
    return got


def test_two_transports_ingest_concurrently():
    G, R = 64, 3
    p = Pair(G=G, R=R, elections=1, pre_vote=1)
    for _ in range(3):
        _round(p)
    _unhost(p, range(G), 2)
    _round(p)
    for rep in range(3):
        msgs, streams, bufs = _two_connections(p, G)
        got = _ingest_both(p, streams, bufs)
        for i in range(2):
            assert got[i]["accepted"] == len(msgs[i]), (rep, i, got[i])
            assert got[i]["bad"] == 0
        # the oracle takes them in any interleaving: the halves are
        # disjoint groups, so the per-group order is each connection's
        p.orc.ingest(msgs[0] + msgs[1])
        _round(p)
        _round(p)
        for b in bufs:
            p.eng.ingest_buffer_free(b)


def test_ingest_races_round_launches():
    """Rounds launch from another thread while the two connections
    ingest.  Which round each call lands before is not observable from
    here, so there is no oracle to step in lock-step; the check is that
    both calls accept every record, no round flags a replica, and every
    group keeps its leader at term 2 afterwards."""
    G, R = 64, 3
    p = Pair(G=G, R=R, elections=1, pre_vote=1)
    for _ in range(3):
        _round(p)
    _unhost(p, range(G), 2)
    _round(p)
    msgs, streams, bufs = _two_connections(p, G)
    stop = threading.Event()
    outs = []

    def rounds():
        while not stop.is_set() and len(outs) < 8:
            outs.append(p.eng.step(tick=False))

    rt = threading.Thread(target=rounds)
    rt.start()
    got = _ingest_both(p, streams, bufs)
    stop.set()
    rt.join(60)
    for i in range(2):
        assert got[i]["accepted"] == len(msgs[i]), got[i]
    assert all(o.fallbacks == 0 and o.errors == 0 for o in outs)
    e = p.eng.step(tick=False)
    assert e.fallbacks == 0 and e.errors == 0
    for g in range(G):
        sts = p.eng.export_replicas(g, 1)
        assert sts[0].role == abi.LEADER and sts[0].term == 2, \
            (g, sts[0].to_dict(R))
    for b in bufs:
        p.eng.ingest_buffer_free(b)
