"""GPU: the cross-rank exchange inside the C ABI (drb_exchange_plan,
drb_exchange_rccl, drb_exchange_rccl_roles; include/drb_engine.h), which
replaces Transport.Send -> handleRequest (transport.go:346, :305) for
GPU-resident replicas spread over ranks (C4).

- The transfer list equals the one dragonboat_amd/exchange.py builds for
  torch.distributed (plan(), fixed mode) on every rank, and the ranks' lists
  pair up: rank r's sends to q are, in order and size, q's receives from r.
- Rounds whose planes move by exactly those transfers (each send copied into
  its paired receive, as RCCL's send / recv would) stay bit-exact with one
  oracle cluster of all groups, at N = 2 and 3.
- The RCCL entry points run against a real one-rank communicator (the pool
  gives one GPU; RCCL refuses two ranks on one device): the roles all-reduce
  returns the engine's own leader slots, a one-rank placement is a no-op
  exchange, and a communicator that does not match the placement is
  refused.  The N > 1 RCCL leg itself needs a multi-GPU node.
"""
import ctypes as C

import pytest

from dragonboat_amd import abi
from dragonboat_amd import exchange as X
from dragonboat_amd.engine import DrbError, Engine
from tests.gpu_harness import DistPair

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _leader_mask(p):
    m = 0
    for e in p.engs:
        m |= e.role_slots()[0]
    return m


def _python_plan(e, world, rank, mask):
    R = e.R
    words = X.fixed_words(R, world, mask, e.cfg["mailbox"],
                          e.cfg["entry_mbox"], bool(e.cfg["elections"]))
    return [(peer, int(op == "recv"), ptr, n) for op, peer, (ptr, n) in
            X.plan(R, world, rank, words, e.plane_regions)]


def _exchange_by_plan(p, mask, counted=False):
    """Every rank's sends copied into the paired receives (one GPU); counted:
    the lists drb_exchange_plan_words makes of every rank's plane counts."""
    dev = torch.device("cuda", 0)
    for e in p.engs:
        e.sync()
    if counted:
        words = [e.plane_counts() for e in p.engs]
        plans = [e.exchange_plan_words(words) for e in p.engs]
        for r, e in enumerate(p.engs):  # the same list exchange.py builds
            assert plans[r] == [
                (peer, int(op == "recv"), ptr, n) for op, peer, (ptr, n) in
                X.plan(e.R, p.N, r, words, e.plane_regions)], r
    else:
        plans = [e.exchange_plan(mask) for e in p.engs]
    moved = 0
    for r, pr in enumerate(plans):
        for q, pq in enumerate(plans):
            if q == r:
                continue
            sends = [(ptr, n) for peer, rv, ptr, n in pr if peer == q and not rv]
            recvs = [(ptr, n) for peer, rv, ptr, n in pq if peer == r and rv]
            assert [n for _, n in sends] == [n for _, n in recvs], (r, q)
            for (sp, n), (dp, _) in zip(sends, recvs):
                X.device_bytes(dp, n, dev).copy_(X.device_bytes(sp, n, dev))
                moved += n
    torch.cuda.synchronize()
    for e in p.engs:
        e.exchange_mark()
    return moved


@pytest.mark.parametrize("N,R", [(2, 3), (3, 5)])
def test_plan_matches_exchange_py_and_pairs_up(N, R):
    p = DistPair(G=6 * N, R=R, N=N, E=4, max_props=2)
    mask = _leader_mask(p)
    assert all(e.exchange_plan(mask) == [] for e in p.engs)  # no round yet
    p.round(k=1, tick=True, exchange=False)
    for r, e in enumerate(p.engs):
        got = e.exchange_plan(mask)
        assert got == _python_plan(e, N, r, mask), r
        assert got and {x[0] for x in got} <= set(range(N)) - {r}
    _exchange_by_plan(p, mask)
    errs = p.check()
    assert not errs, errs[:2]


@pytest.mark.parametrize("N,R,counted", [(2, 3, False), (3, 5, False),
                                         (2, 3, True), (3, 5, True),
                                         (8, 5, True)])
def test_rounds_through_the_plan_stay_bit_exact(N, R, counted):
    G = 10 * N + 1  # ragged: the last rank holds fewer lanes
    p = DistPair(G=G, R=R, N=N, E=4, max_props=2)
    mask = _leader_mask(p)
    for rnd in range(8):
        o, tot = p.round(k=1 + rnd % 2, tick=rnd % 2 == 0,
                         read_index=rnd % 3 == 1, exchange=False)
        assert tot["fallbacks"] == 0 and tot["errors"] == 0, (rnd, tot)
        assert tot["committed_entries"] == o.committed_entries, rnd
        assert _exchange_by_plan(p, mask, counted) > 0
        errs = p.check()
        assert not errs, (rnd, errs[:2])


def _rccl():
    for name in ("librccl.so.1", "/opt/rocm/lib/librccl.so.1"):
        try:
            return C.CDLL(name)
        except OSError:
            pass
    pytest.skip("librccl not loadable")


def test_rccl_entry_points_on_a_one_rank_communicator():
    L = _rccl()
    comm = C.c_void_p()
    torch.cuda.set_device(0)
    dev = (C.c_int * 1)(0)
    # one rank on device 0, no bootstrap (ncclCommInitAll)
    assert L.ncclCommInitAll(C.byref(comm), 1, dev) == 0
    try:
        e = Engine(num_groups=64, num_replicas=3)
        e.init_steady(term=2, leader_slot=1)
        assert e.exchange_rccl_roles(comm.value) == 1 << 1
        e.step(tick=True)
        e.exchange_rccl(comm.value, 1 << 1)  # one rank: nothing moves
        e.step(tick=True)
        e.exchange_rccl_counted(comm.value)
        e.step(tick=True)
        assert e.read_counters().errors == 0
        # a placement of two ranks does not match a one-rank communicator
        e2 = Engine(num_groups=32, num_replicas=3, total_groups=64,
                    place_world=2, place_rank=0, entry_mbox=3)
        e2.init_steady(term=2, leader_slot=0)
        e2.step(tick=True)
        with pytest.raises(DrbError):
            e2.exchange_rccl(comm.value, 1)
        with pytest.raises(DrbError):
            e2.exchange_rccl_counted(comm.value)
        assert e2.exchange_rccl_roles(comm.value) == 1
    finally:
        L.ncclCommDestroy(comm)
