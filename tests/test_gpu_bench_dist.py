"""bench.py --gpus N starts its own ranks (one process per GPU) when no
launcher is around it, and reports the whole job: n_gpus = N and the
committed entries of every rank summed (dragonboat shards groups
over its step workers, internal/server/partition.go:38).  The pool's boxes
have one GPU, so the two ranks share it over gloo here; on a node the same
line runs one rank per GPU over RCCL.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G, K = 4096, 4


def _bench(*extra, env=None):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(K),
           "--warmup", "2", "--groups", str(G), "--kv-fill", "0",
           "--no-wire", "--no-cpu-baseline", "--host-staged", "0",
           "--tick-every", "1"] + list(extra)
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
              "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    p = subprocess.run(cmd, cwd=ROOT, env=e, capture_output=True, text=True,
                       timeout=300)
    return p


@pytest.mark.gpu
def test_bench_gpus_2_launches_two_ranks():
    """... and, after the timed run, C4 across the two ranks through the C
    ABI's exchange lists (c4_cross: over RCCL on a node, here the gloo
    rehearsal through host memory), both the counted and the fixed step."""
    p = _bench("--gpus", "2", "--dist-backend", "gloo", "--c4-groups",
               str(G))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 only
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2
    assert res["steps"] == K
    c = res["counters"]
    # every rank commits one entry per group per round at the steady state:
    # committed_per_round is the job's total / K / world
    assert c["committed_per_round"] == G, c
    total = c["committed_per_round"] * K * res["n_gpus"]
    assert abs(res["value"] * res["ms_per_step"] * K / 1e3 - total) <= \
        1e-6 * total + 1
    assert c["fast_path_only"], c
    x = res["c4_cross"]
    assert "error" not in x, x
    assert x["world"] == 2 and x["groups"] == G
    for mode in ("counted", "fixed"):
        m = x[mode]
        assert m["committed_per_round"] == G, (mode, m)
        assert m["fallbacks_and_errors"] == 0, (mode, m)
        assert m["xchg_bytes_per_round_per_rank"] > 0, (mode, m)
    # the counted step ships what the round sent, the fixed one every slot
    assert x["counted"]["xchg_bytes_per_round_per_rank"] < \
        x["fixed"]["xchg_bytes_per_round_per_rank"]


def test_bench_rejects_gpus_unlike_world_size():
    # (no GPU needed: the check runs before anything touches one)
    p = _bench("--gpus", "2", env={"WORLD_SIZE": "1", "RANK": "0",
                                   "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr


def test_bench_local_ranks_is_the_c4_run():
    # (no GPU needed: rejected before anything touches one)
    p = _bench("--local-ranks", "2")
    assert p.returncode != 0
    assert "local-ranks" in p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["bind", "pull"])
def test_bench_c4_local_ranks(mode):
    """bench.py --workload c4 --local-ranks 4: four engines of one process
    on the one GPU, bound for the zero-copy exchange (the default: the
    receivers read the senders' outboxes, nothing is pulled) or their
    planes moved by drb_exchange_local's device pull (which reports its
    bytes); every group commits one entry a round."""
    p = _bench("--workload", "c4", "--local-ranks", "4",
               "--local-exchange", mode)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads([x for x in p.stdout.splitlines()
                      if x.startswith("{")][-1])
    assert res["config"]["local_ranks"] == 4
    assert res["counters"]["committed_per_round"] == G
    assert res["counters"]["fallbacks_and_errors"] == 0
    assert res["exchange"]["mode"] == mode
    if mode == "pull":
        assert res["exchange"]["bytes_per_round"] > 0
    else:
        assert res["exchange"]["bytes_per_round"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("xmode", ["counted", "fixed"])
def test_bench_c4_gpus_2(xmode):
    """bench.py --workload c4 --gpus 2: the replicas of every group spread
    over the two ranks, the planes moved after every round by exchange.py
    (counted by default: an all_gather of the plane words, then the planes
    at those sizes; or the fixed full-capacity step) -- through host memory
    under gloo here, RCCL on a node.  Every group commits every round and
    nothing leaves the fast path."""
    p = _bench("--workload", "c4", "--gpus", "2", "--dist-backend", "gloo",
               "--exchange", xmode)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads([x for x in p.stdout.splitlines()
                      if x.startswith("{")][-1])
    assert res["n_gpus"] == 2
    assert res["exchange"]["mode"] == xmode
    c = res["counters"]
    assert c["fallbacks"] == 0 and c["errors"] == 0, c
    assert c["committed_per_round"] > 0, c
