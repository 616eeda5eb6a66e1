"""C4 end to end on one MI355X with real processes: world_size 2 (and 3)
ranks, each with its own engine (replica slot s of group g on rank
(g + s) mod N), the per-round plane exchange of dragonboat_amd/exchange.py
over torch.distributed, and the result compared bit-exactly with one CPU
oracle cluster of all groups.  The ranks share one GPU here, so the
transport is gloo with host staging; on a node the same plan runs over RCCL
(backend "nccl") straight between engine memories.  A first check pins
that torch aliases engine memory (no copy) through the device views the
RCCL path hands to send/recv.
"""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

pytestmark = pytest.mark.gpu

G, R, ROUNDS = 26, 5, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_device_view_aliases_engine_memory():
    from dragonboat_amd.engine import Engine
    from dragonboat_amd import exchange as X
    e = Engine(num_groups=8, num_replicas=3, total_groups=16, place_world=2,
               place_rank=0, entry_mbox=3)
    e.init_steady(term=2, leader_slot=0)
    e.step(prop_slot=0xFFFFFFFF, tick=True)
    w = e.plane_counts()
    regs = [r for a in range(3) for b in range(3) if w[a * 3 + b]
            for r in e.plane_regions(a, b, w[a * 3 + b], 1)]
    assert regs, w
    ptr, n = regs[0]
    t = X.device_bytes(ptr, n, torch.device("cuda", 0))
    assert t.data_ptr() == ptr and t.numel() == n
    t.fill_(0x5a)
    torch.cuda.synchronize()
    h = X.device_bytes(ptr, n, torch.device("cuda", 0)).cpu()
    assert bool((h == 0x5a).all())
    e.close()


def _worker(rank, world, port, q, fixed):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ctypes as C
        from dragonboat_amd import abi, workload
        from dragonboat_amd.engine import Engine
        from dragonboat_amd.exchange import PlaneExchange
        torch.cuda.set_device(0)
        seed = 0x5EEDD8B0
        lanes = (G + world - 1) // world
        eng = Engine(num_groups=lanes, num_replicas=R, total_groups=G,
                     place_world=world, place_rank=rank, entry_mbox=3,
                     max_props=2)
        eng.init_steady(term=2, leader_slot=0, seed=seed)
        xch = PlaneExchange(eng, world, rank, torch.device("cuda", 0),
                            staged=True, fixed=fixed)
        tot = 0
        for t in range(ROUNDS):
            counts, ents, pool = workload.build_batch(G, 1, seed, t)
            ec = (C.c_uint32 * lanes)()
            ee = (abi.Entry * (lanes * 2))()
            for j in range(lanes):
                g = world * j + rank  # the leader (slot 0) at lane j
                if g < G:
                    ec[j] = counts[g]
                    ee[j * 2] = ents[g]
            eng.stage_proposals(0, ec, ee, pool)
            out = eng.step(tick=(t % 2 == 0), prop_slot=0)
            assert out.fallbacks == 0 and out.errors == 0
            tot += out.committed_entries
            xch.step()
        res = {}
        for j in range(lanes):
            st = eng.export_replicas(j, 1)
            for s in range(R):
                g = world * j + (rank - s) % world
                if g < G:
                    x = st[s]
                    res[(g, s)] = (x.term, x.committed, x.processed,
                                   x.last_index, x.sm_index, x.kv_count,
                                   x.election_tick, x.tick_count,
                                   x.applied_index, sorted(eng.kv_export(j, s).items()))
        q.put((rank, tot, res))
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fixed", [(2, False), (3, False), (2, True),
                                         (3, True)])
def test_c4_processes_exchange_planes(world, fixed):
    from dragonboat_amd import workload
    from oracle import pyoracle as po
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, fixed))
             for r in range(world)]
    for p in procs:
        p.start()
    got, total = {}, 0
    for _ in procs:
        r, tot, res = q.get(timeout=240)
        got.update(res)
        total += tot
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = po.Cluster(G, R, seed=0x5EEDD8B0)
    c.setup_steady(0)
    otot = 0
    for t in range(ROUNDS):
        counts, ents, pool = workload.build_batch(G, 1, 0x5EEDD8B0, t)
        c.stage_proposals(counts, 1, ents, pool)
        otot += c.round(tick=(t % 2 == 0)).committed_entries
    assert total == otot
    assert len(got) == G * R
    for (g, s), v in got.items():
        x = c.export(g, s)
        exp = (x.term, x.committed, x.processed, x.last_index, x.sm_index,
               x.kv_count, x.election_tick, x.tick_count, x.applied_index,
               sorted(c.export_kv(g, s).items()))
        assert v == exp, (g, s)
