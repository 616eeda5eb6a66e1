"""The N>1 path of bench.py on the CPU: world_size-2 gloo ranks, each
hosting its own shard of groups (dragonboat_amd/dist.py), agreeing on the
tick cadence and reducing counters exactly as the RCCL run does.

Each rank steps its shard with the CPU restatement (the checker), so the
test pins the sharding arithmetic: ShardIDs are disjoint across ranks,
seeds differ, and the reduced committed count equals the sum of what every
shard committed when run alone.
"""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

G, R, ROUNDS = 48, 3, 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_shard(seed, rounds=ROUNDS):
    from dragonboat_amd import workload
    from oracle import pyoracle as po
    c = po.Cluster(G, R, seed=seed)
    c.setup_steady(0)
    committed = 0
    for t in range(rounds):
        counts, ents, pool = workload.build_batch(G, 1, seed, t)
        c.stage_proposals(counts, 1, ents, pool)
        out = c.round(tick=True)
        committed += out.committed_entries
    return committed


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from dragonboat_amd import dist as ddist
    w, r, _ = ddist.env()
    dist.init_process_group("gloo", rank=r, world_size=w)
    try:
        first, seed = ddist.shard_plan(r, G)
        firsts = [None] * w
        dist.all_gather_object(firsts, (first, seed))
        committed = _run_shard(seed)
        total = ddist.reduce_sum(committed)
        te = ddist.agree_min(3 + r)
        el = ddist.reduce_max(1.5 + r)
        ddist.barrier()
        q.put((r, firsts, committed, total, te, el))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_sharding():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    firsts = res[0][1]
    assert firsts == res[1][1]
    # ShardID ranges [first, first + G) are disjoint; seeds differ
    (f0, s0), (f1, s1) = firsts
    assert f1 >= f0 + G and s0 != s1
    per_rank = [x[2] for x in res]
    assert all(c > 0 for c in per_rank)
    assert res[0][3] == res[1][3] == sum(per_rank)
    # each shard alone commits what it committed under the job
    from dragonboat_amd import dist as ddist
    for r in range(world):
        assert _run_shard(ddist.shard_plan(r, G)[1]) == per_rank[r]
    assert all(x[4] == 3 for x in res)      # tick cadence: min over ranks
    assert all(x[5] == 2.5 for x in res)    # elapsed: max over ranks
