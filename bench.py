"""bench.py -- committed entries/sec of the batched multi-group Raft step
round on MI355X (BASELINE.json metric), plus %HBM roofline and the CPU
oracle timed on the host cores.

One step = one step round (drb_step_round) over every group on the GPU:
proposals in, replication, quorum commit, ReadIndex, KV apply, messages
out -- the dragonboat step loop for all replicas at once.

Default workload = BASELINE.json configs[2]:
1,048,576 active groups x 3 replicas per GPU, 16 B PBKV writes (k=1 per
group per round) and a 9:1 ReadIndex:write mix batched into one ReadIndex
ctx per group per round, one LocalTick per round.  Multi-GPU: groups are
sharded over ranks (weak scaling, no data-path collective).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
READS_PER_CTX = 9      # C3: 9 ReadIndex reads per write, one ctx per round
# C2/C3: fresh-key write rounds before timing, so that every replica's
# table holds (nearly) all of its group's KEY_SPACE keys -- load ~0.50 of
# 512 slots (tests/test_gpu_fullsize.py pins the timed rounds at this fill)
C3_KV_FILL = 1536
KEY_SPACE = 256        # K = 256 keys per group


def alg_bytes_per_group_round(R=3, k=1, P=16, reads=True, spread=False):
    """SURVEY.md 8(d) algorithmic bytes for one group-round (co-resident;
    spread=True adds C4's B_msg for replicas on other GPUs)."""
    e = 56 + ((P + 1 + 15) // 16) * 16          # entry record
    b_round = 96 + 48 * R + 96 * (R - 1)        # leader core, remotes, flw
    b_entries = k * e * (1 + 2 * (R - 1))       # leader write, flw r+w
    b_apply = k * R * ((P + 1) + 2 * 16)        # Cmd read + slot r/w
    b_read = (64 + 9 * 16) if reads else 0      # ctx push/confirm + lookups
    b_msg = 3 * ((R - 1) * (48 + k * e) + (R - 1) * 24) if spread else 0
    return b_round + b_entries + b_apply + b_read + b_msg


PMC_DIR = os.path.join(ROOT, "profiles")


def pmc_file(key):
    """the committed PMC summary of a workload: C3's is pmc_current.json,
    the others pmc_<workload>.json (tools/prof_workloads.sh)"""
    return os.path.join(PMC_DIR, "pmc_current.json" if key == "c3" else
                        "pmc_%s.json" % key)


def pmc_traffic(key, G, R):
    """HBM bytes per round from the committed rocprofv3 PMC passes of this
    workload (tools/pmc_summary.py over the timed rounds' step kernels):
    (FETCH_SIZE x2 + WRITE_SIZE, FETCH_SIZE + WRITE_SIZE).  The first is an
    upper bound -- the x2 correction is for coalesced 16 B/lane reads, and
    the KV's random 16 B reads are already tallied at 64 B each -- the
    second the matching lower bound.  (None, None) when no summary matches
    this configuration."""
    try:
        s = json.load(open(pmc_file(key)))
    except (OSError, ValueError):
        return None, None
    if s.get("groups") != G or s.get("replicas") != R:
        return None, None
    return s.get("round_hbm_bytes"), s.get("round_hbm_bytes_lower")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of this node; without an external "
                         "launcher, N > 1 starts N ranks itself "
                         "(torch.distributed.run); under one it must equal "
                         "WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="c3",
                    choices=["c2", "c3", "c4", "c5"],
                    help="c3: groups sharded over GPUs, replicas "
                         "co-resident (BASELINE metric); c2: 64k groups per "
                         "GPU, 16 B writes only; c4: --groups "
                         "groups in total, replica slot s of group g on "
                         "GPU (g + s) mod N, planes exchanged over RCCL; "
                         "c5: 4M groups per GPU, --active-ppm of them "
                         "proposing --payload byte entries per round, "
                         "EntriesToSave encoded as EntryBatch + CRC32")
    ap.add_argument("--payload", type=int, default=128, choices=[128, 1024],
                    help="c5 entry payload (PBKV value 116 / 1011 B)")
    ap.add_argument("--active-ppm", type=int, default=10000,
                    help="c5: groups proposing per round, per million")
    ap.add_argument("--groups", type=int, default=1 << 20,
                    help="groups per GPU (c3) / in total (c4)")
    ap.add_argument("--replicas", type=int, default=0,
                    help="default 3 (c3) / 5 (c4)")
    ap.add_argument("--k", type=int, default=1, help="writes/group/round")
    ap.add_argument("--kv-slots", type=int, default=0,
                    help="KV table slots per replica (0: the workload's)")
    ap.add_argument("--no-read-index", action="store_true")
    ap.add_argument("--kv-fill", type=int, default=-1,
                    help="c2/c3: rounds of fresh-key writes before the "
                         "timed region, so each replica's KV holds its "
                         "group's K = 256 keys (SURVEY 8d steady state); "
                         "default 1536 (255 of 256 keys expected)")
    ap.add_argument("--tick-every", type=int, default=0,
                    help="LocalTick every N rounds (0: derive from --tick-ms)")
    ap.add_argument("--tick-ms", type=float, default=1.0,
                    help="RTTMillisecond: one LocalTick per this much wall "
                         "time (nodehost.go:1824-1914)")
    ap.add_argument("--reads-mode", default="fused",
                    choices=["fused", "separate"],
                    help="served reads inside the round's kernels or as "
                         "their own launch (drb_serve_reads)")
    ap.add_argument("--reads-at", default="leader",
                    choices=["leader", "follower"],
                    help="C3: issue the ReadIndex batch at the leader or at "
                         "a follower (forwarded, raft.go:2134-2164)")
    ap.add_argument("--listed", type=int, default=-1,
                    help="step only the replicas with work, packed "
                         "(drb_round_in.listed; default: on for c5)")
    ap.add_argument("--quiesce", type=int, default=-1,
                    help="Config.Quiesce (default: on for c5, SURVEY 8d)")
    ap.add_argument("--c5-warm", type=int, default=400,
                    help="c5: rounds run before the warmup, ticking every "
                         "round, so the timed rounds see the quiesced "
                         "steady state (quiesceState: 20 x ElectionRTT = 200 "
                         "idle ticks, quiesce.go:44-82)")
    ap.add_argument("--no-lean", action="store_true",
                    help="c5: step every listed replica through the full "
                         "step kernel (drb_config.no_lean; A/B of the lean "
                         "kernel of heartbeat rounds, drb_lean.hpp)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--save", default="",
                    choices=["", "none", "entrybatch", "tan", "tanmux"],
                    help="persistence output of every round: none, "
                         "EntryBatch + CRC32 per replica, the regular "
                         "tan LogDB's log record per replica (XXH64 "
                         "chunks), or the multiplexed tan's (16 logs per "
                         "slot, records back to back); default: entrybatch "
                         "for c5, else none")
    ap.add_argument("--elections", type=int, default=0,
                    help="1: the engine runs elections on the GPU "
                         "(drb_config.elections); the timed rounds show its "
                         "steady-state cost")
    ap.add_argument("--failover", action="store_true",
                    help="with --elections, after the timed region: stop "
                         "every group's leader replica and time the rounds "
                         "until every group elected a new one on the GPU")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group backend (nccl = RCCL); gloo only to "
                         "rehearse the multi-rank control flow with several "
                         "ranks on one GPU")
    ap.add_argument("--no-wire", action="store_true",
                    help="skip the off-GPU wire encode measurement (C3)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ingest", action="store_true",
                    help="skip the receiving-side wire ingest measurement")
    ap.add_argument("--exchange", default="counted",
                    choices=["fixed", "counted"],
                    help="c4 plane exchange: sized by an all_gather of "
                         "per-plane counts (the default: about half the "
                         "fixed step's bytes, VERDICT r5) or full-capacity "
                         "planes enqueued behind the round with no host "
                         "sync (dragonboat_amd/exchange.py)")
    ap.add_argument("--read-results", type=int, default=1,
                    help="c3: the timed reads write each client's "
                         "ReadLocalNode result (drb_config.max_reads_per_"
                         "ctx); 0 keeps only the per-replica checksum")
    ap.add_argument("--local-ranks", type=int, default=0,
                    help="c4 in ONE process on one GPU: N engines (ranks of "
                         "the placement) stepped together, their planes "
                         "moved by drb_exchange_local (the device pull, no "
                         "host synchronisation)")
    ap.add_argument("--local-exchange", choices=("bind", "pull"),
                    default="bind",
                    help="--local-ranks: bind = the engines read remote "
                         "planes in the senders' outboxes (drb_exchange_"
                         "local_bind, zero-copy); pull = the device pull "
                         "copies them into the receivers' inbound planes")
    ap.add_argument("--host-staged", type=int, default=-1,
                    help="after the timed region, also time rounds whose "
                         "proposals come from host memory through "
                         "drb_stage_proposals (default: on for c2/c3, N=1)")
    ap.add_argument("--rounds-per-call", type=int, default=-1,
                    help="timed rounds per drb_step_rounds call (a chunk of "
                         "every group: plain rounds from one C call); -1: 16 "
                         "for c2, round by round otherwise")
    ap.add_argument("--chunk-ab", default="",
                    help="c3, after the timed region: A/B of drb_step_rounds "
                         "(k rounds chunk by chunk of the groups) against "
                         "plain rounds, specs CHUNK_GROUPS:K,... (e.g. "
                         "65536:4,262144:2); reported as chunk_ab, not value")
    ap.add_argument("--c4-cross", type=int, default=-1,
                    help="with --gpus N > 1 and a co-resident workload, also "
                         "time C4 across the ranks through the C ABI's RCCL "
                         "exchange (drb_exchange_rccl*; gloo: a rehearsal "
                         "through host memory); default on")
    ap.add_argument("--c4-groups", type=int, default=1 << 20,
                    help="groups of that C4 run (in total)")
    ap.add_argument("--c4-timeout", type=int, default=240,
                    help="seconds the C4 cross-GPU phase may take")
    ap.add_argument("--step-worker", type=int, default=-1,
                    help="after the timed region, also time whole step-"
                         "worker rounds: host-staged proposals, the round, "
                         "and its ReadyToReads, read results and applied "
                         "entries back in pinned host memory "
                         "(drb_worker_export; default: on for c3, N=1)")
    return ap.parse_args()


C5_VAL = {128: 116, 1024: 1011}
# C5 KV: writes uniform over the K = 256 keys of SURVEY 8d, as C3.  A
# replica's table holds C5_SLOTS keys -- a group proposes Poisson(1 % x
# rounds) times in a run, ~0.7 in the default one -- and a full table grows
# into overflow buckets (drb_config.kv_overflow_buckets, C5_OVF_PER buckets
# per replica on average, the K = 256 keys of a long run); the values live
# in one shared block pool sized for the keys the run can write
# (put_value_long: a block per distinct key, bump-allocated)
C5_KEYS = KEY_SPACE
C5_SLOTS = 32
C5_WARM_BASE = 1 << 23  # the pre-warm rounds' draws (salt = round)
C5_OVF_PER = 1 / 64


def c5_pool_blocks(G, R, rounds, active_ppm):
    """Value blocks for every distinct key a C5 run of `rounds` rounds can
    write: R replicas of each proposing group, mean + 8 sigma + slack."""
    mean = G * R * active_ppm / 1e6 * rounds
    return int(mean + 8 * mean ** 0.5) + R * 65536


def host_cores():
    """(cores this process may run on, CPUs the host shows): the affinity
    set, capped by the cgroup's CPU quota (cpu.max) where one is set -- a
    GPU box's share of its machine."""
    visible = os.cpu_count() or 1
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n), visible


def cpu_baseline(args, seconds):
    """The CPU oracle (C restatement of the reference path) on the host:
    a bounded sample of the same workload, groups split over one thread per
    core this process may use."""
    from dragonboat_amd import workload
    from oracle import pyoracle as po
    import ctypes as C
    from dragonboat_amd.abi import RoundOut
    cores, visible = host_cores()
    G = 1000 * cores  # C1 scale per core
    c = po.Cluster(G, args.replicas, logdb_keep=64)
    c.setup_steady(0)
    L = po.lib()
    seed = 0x5EEDD8B0
    parts = [(i * G // cores, (i + 1) * G // cores) for i in range(cores)]
    committed = 0
    rounds = 0
    sums = (C.c_uint64 * (G * args.replicas))()
    t_start = time.perf_counter()
    t_run = 0.0
    while time.perf_counter() - t_start < seconds:
        if args.workload == "c5":
            act = workload.active_groups(G, seed, rounds, args.active_ppm)
            counts, ents, pool = workload.build_batch(
                G, args.k, seed, rounds, C5_KEYS,
                C5_VAL[args.payload], act)
        else:
            counts, ents, pool = workload.build_batch(G, args.k, seed,
                                                      rounds)
        c.stage_proposals(counts, args.k, ents, pool)
        if not args.no_read_index:
            lo, hi = workload.build_read_index(G, seed, rounds, rounds + 30)
            c.stage_read_index(lo, hi)
        outs = [RoundOut() for _ in parts]
        tick = 1  # a CPU round takes longer than RTTMillisecond = 1 ms
        t0 = time.perf_counter()
        th = [threading.Thread(target=L.orc_cluster_round_range,
                               args=(c.p, tick, a, b, C.byref(o)))
              for (a, b), o in zip(parts, outs)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        L.orc_cluster_end_round(c.p)
        if not args.no_read_index:
            th = [threading.Thread(target=L.orc_cluster_serve_reads,
                                   args=(c.p, READS_PER_CTX, KEY_SPACE, a, b,
                                         sums, None, None))
                  for (a, b) in parts]
            for t in th:
                t.start()
            for t in th:
                t.join()
        t_run += time.perf_counter() - t0
        committed += sum(o.committed_entries for o in outs)
        rounds += 1
    return dict(value=committed / t_run if t_run else 0.0,
                unit="committed entries/s", cores=cores,
                host_cpus_visible=visible, kind="port",
                sample="%d groups x %d replicas, %d rounds of the same "
                       "workload (k=%d, %s, a LocalTick every round), CPU "
                       "restatement (oracle/), not dragonboat" % (
                           G, args.replicas, rounds, args.k,
                           "9:1 ReadIndex + 9 KV lookups per released ctx"
                           if not args.no_read_index
                           else "writes only"))


def run_c4_local(args):
    """C4 placement with every rank's engine in this process on one GPU
    (NodeHost is one process per machine): N engines hold replica slot s of
    global group g at rank (g + s) mod N, lane g // N; every round each
    engine's step is enqueued on its own stream, then drb_exchange_local
    moves the planes (a pull kernel per receiver behind cross-stream
    events).  The host never waits inside the timed loop."""
    import torch
    from dragonboat_amd import dist as ddist
    from dragonboat_amd.engine import Engine
    N, G, k = args.local_ranks, args.groups, args.k
    R = args.replicas or 5
    lanes = (G + N - 1) // N
    NP = max(8, args.steps)
    seed = ddist.BASE_SEED
    torch.cuda.set_device(0)
    engs = [Engine(num_groups=lanes, num_replicas=R, window=32, cmd_cap=32,
                   max_props=max(1, k), prop_slots=NP, ri_slots=NP, mailbox=8,
                   kv_slots=512, kv_val_cap=4, total_groups=G, place_world=N,
                   place_rank=r, entry_mbox=k + 2, device=0)
            for r in range(N)]
    for e in engs:
        e.init_steady(term=2, leader_slot=0, seed=seed)
    bind = args.local_exchange == "bind"
    if bind:
        Engine.exchange_local_bind(engs)

    def rnd(i, b, tick):
        for e in engs:
            e.step_async(tick=tick, prop_slot=b)
        Engine.exchange_local(engs)

    WARM, TIMED = 1 << 21, 1 << 22
    for i in range(args.warmup):
        for e in engs:
            e.gen_kv_proposals(0, k, KEY_SPACE, 4, seed, WARM + i)
        rnd(i, 0, True)
    for b in range(args.steps):
        for e in engs:
            e.gen_kv_proposals(b, k, KEY_SPACE, 4, seed, TIMED + b)
    for e in engs:
        e.sync()
        e.read_counters(reset=True)
        e.exchange_bytes(reset=True)
    torch.cuda.synchronize()
    K = args.steps
    te = max(1, args.tick_every or 1)
    t0 = time.perf_counter()
    for i in range(K):
        rnd(i, i, i % te == 0)
    for e in engs:
        e.sync()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    outs = [e.read_counters(reset=True) for e in engs]
    xb = [e.exchange_bytes(reset=True) for e in engs]
    committed = sum(o.committed_entries for o in outs)
    fb = sum(o.fallbacks + o.errors for o in outs)
    alg = alg_bytes_per_group_round(R, k, 16, False, True) * G
    res = {
        "metric": "committed entries/sec (node) at %d 5-replica groups spread "
                  "over %d in-process ranks on one GPU, 16B payload" % (G, N),
        "value": committed / el, "unit": "committed entries/s",
        "n_gpus": 1, "steps": K, "warmup": args.warmup,
        "ms_per_step": el * 1e3 / K, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic (SURVEY 8d seeded PBKV writes)",
        "config": {
            "workload": "C4 placement in one process: %d groups x %d "
                        "replicas, slot s of group g at local rank (g + s) "
                        "mod %d, 16B PBKV writes k=%d/group/round, tick "
                        "every %d round(s)" % (G, R, N, k, te),
            "local_ranks": N, "groups_per_rank": lanes, "replicas": R,
            "parallelism": "replicas spread over %d engines of one process "
                           "on one GPU; drb_exchange_local (%s)" % (
                               N, "zero-copy: bound engines read the senders' "
                               "outboxes" if bind else "device pull")},
        "exchange": {
            "bytes_per_round": sum(xb) / K,
            "bytes_per_round_per_rank": sum(xb) / K / N,
            "mode": args.local_exchange,
            "note": "inbound plane bytes the pull kernels moved (headers of "
                    "the round, counted records, entry rows), "
                    "drb_exchange_bytes; 0 when bound: the step kernels "
                    "read the senders' outbox planes in place"},
        "roofline": {"bound": "hbm", "alg_bytes_per_round": alg,
                     "achieved": alg / (el / K) / 1e9, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s",
                     "frac": alg / (el / K) / 1e9 / HBM_PEAK_GBS,
                     "note": "wall time per round of all N engines, "
                             "exchange included"},
        "counters": {"committed_per_round": committed / K,
                     "fallbacks_and_errors": fb,
                     "messages": sum(o.messages for o in outs)},
    }
    print(json.dumps(res))
    for e in engs:
        e.close()
    return 0


def run_c4_cross(args, world, rank, local, gloo):
    """C4 across the process group's ranks through the C ABI, beside a
    multi-GPU run of another workload: --c4-groups groups x 5 replicas,
    replica slot s of group g on rank (g + s) mod world at lane g // world,
    bench.py's C4 engine, the planes moved after every round by
    drb_exchange_rccl_counted (drb_plane_counts, an ncclAllGather of the
    words, ncclSend / ncclRecv at those sizes) and by drb_exchange_rccl (the
    fixed full-capacity step, no host round trip) -- RCCL over xGMI, what a
    Go NodeHost per GPU would call.  With the gloo backend
    (a rehearsal with the ranks on one GPU: RCCL refuses two ranks on one
    device) the same C-ABI transfer lists (drb_exchange_plan_words /
    drb_exchange_plan) move through host memory instead."""
    import ctypes as C
    import torch
    import torch.distributed as dist
    from dragonboat_amd import dist as ddist
    from dragonboat_amd import exchange as X
    from dragonboat_amd.engine import Engine
    G, R, k = args.c4_groups, 5, 1
    lanes = (G + world - 1) // world
    NP = max(8, args.steps)
    seed = ddist.BASE_SEED
    red = "cpu" if gloo else "cuda"
    dev = torch.device("cuda", local)
    eng = Engine(num_groups=lanes, num_replicas=R, window=32, cmd_cap=32,
                 max_props=k, prop_slots=NP, ri_slots=NP, mailbox=8,
                 kv_slots=512, kv_val_cap=4, total_groups=G,
                 place_world=world, place_rank=rank, entry_mbox=k + 2,
                 device=local)
    comm = None
    try:
        eng.init_steady(term=2, leader_slot=0, seed=seed)
        if gloo:
            t = torch.tensor([eng.role_slots()[0]], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.BOR)
            mask = int(t.item())
        else:
            comm = ddist.RcclComm(world, rank)
            mask = eng.exchange_rccl_roles(comm.handle)

        def xchg(mode):
            if not gloo:
                if mode == "counted":
                    eng.exchange_rccl_counted(comm.handle)
                else:
                    eng.exchange_rccl(comm.handle, mask)
                return
            if mode == "counted":
                mine = torch.tensor(eng.plane_counts(), dtype=torch.int64)
                allw = torch.empty(world * R * R, dtype=torch.int64)
                dist.all_gather_into_tensor(allw, mine)
                flat = allw.tolist()
                ops = eng.exchange_plan_words(
                    [flat[q * R * R:(q + 1) * R * R] for q in range(world)])
            else:
                eng.sync()
                ops = eng.exchange_plan(mask)
            X.run_ops_staged([("recv" if rv else "send", peer, (ptr, n))
                              for peer, rv, ptr, n in ops], dev)
            staged[0] += sum(n for _, rv, _, n in ops if rv)
            torch.cuda.current_stream(dev).synchronize()
            eng.exchange_mark()

        out = {"groups": G, "replicas": R, "lanes_per_rank": lanes,
               "world": world,
               "transport": ("gloo rehearsal: the C-ABI transfer lists "
                             "through host memory (ranks sharing one GPU)"
                             if gloo else "RCCL ncclSend / ncclRecv over "
                             "xGMI, drb_exchange_rccl_counted / "
                             "drb_exchange_rccl on the engine stream")}
        r0, WARM, TIMED = 0, 1 << 21, 1 << 22
        staged = [0]  # (gloo: the bytes received through host memory)
        for mode in ("counted", "fixed"):
            for i in range(args.warmup):
                eng.gen_kv_proposals(0, k, KEY_SPACE, 4, seed, WARM + r0 + i)
                eng.step_async(tick=True, prop_slot=0)
                xchg(mode)
            r0 += args.warmup
            K = args.steps
            for b in range(K):
                eng.gen_kv_proposals(b, k, KEY_SPACE, 4, seed, TIMED + r0 + b)
            eng.sync()
            eng.read_counters(reset=True)
            eng.exchange_bytes(reset=True)
            staged[0] = 0
            ddist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(K):
                eng.step_async(tick=True, prop_slot=i)
                xchg(mode)
            eng.sync()
            torch.cuda.synchronize()
            ddist.barrier()
            el = ddist.reduce_max(time.perf_counter() - t0, red)
            r0 += K
            o = eng.read_counters(reset=True)
            xb = ddist.reduce_max((eng.exchange_bytes(reset=True) +
                                   staged[0]) / K, red)
            committed = ddist.reduce_sum(o.committed_entries, red)
            fb = ddist.reduce_sum(o.fallbacks + o.errors, red)
            out[mode] = {
                "value": committed / el, "unit": "committed entries/s",
                "ms_per_step": el * 1e3 / K, "steps": K,
                "committed_per_round": committed / K,
                "xchg_bytes_per_round_per_rank": xb,
                "fallbacks_and_errors": fb}
        out["note"] = ("C4 beside the main workload, timed around the whole "
                       "job (the exchange included), max over ranks; "
                       "xchg_bytes: inbound plane bytes per round of the "
                       "busiest rank (drb_exchange_bytes); not `value`")
        return out
    finally:
        if comm is not None:
            comm.close()
        eng.close()


def self_launch(args):
    """bench.py --gpus N with no launcher around it: start N ranks, one
    process per GPU, as the driver's own torch.distributed.run line would,
    and exit with their status.  This process touches no GPU before the
    ranks start (nothing here imports torch.cuda state), so the ranks are
    fresh children, not an exec of a GPU-initialised process."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % args.gpus, "--master-addr=127.0.0.1",
           "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if "WORLD_SIZE" in os.environ:
        if args.gpus is not None and args.gpus != int(os.environ["WORLD_SIZE"]):
            sys.exit("bench.py: --gpus %d under a launcher with WORLD_SIZE=%s"
                     % (args.gpus, os.environ["WORLD_SIZE"]))
    elif args.gpus is not None and args.gpus > 1:
        sys.exit(self_launch(args))
    if args.local_ranks > 1:
        if args.workload != "c4" or "WORLD_SIZE" in os.environ:
            sys.exit("bench.py: --local-ranks is the one-process c4 run")
        return run_c4_local(args)
    import torch
    import torch.distributed as dist
    from dragonboat_amd import dist as ddist
    world, rank, local = ddist.env()
    red = "cuda"  # where the counter reductions run
    if world > 1 and args.dist_backend == "gloo":
        # rehearsal: ranks may share a GPU
        local = local % max(1, torch.cuda.device_count())
        dist.init_process_group("gloo")
        red = "cpu"
    elif world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    from dragonboat_amd.engine import Engine
    c4 = args.workload == "c4"
    c5 = args.workload == "c5"
    c2 = args.workload == "c2"
    c3 = args.workload == "c3"
    if c2:  # 64k groups, 16 B writes, replicas co-resident
        args.no_read_index = True
        if args.groups == 1 << 20:
            args.groups = 1 << 16
    if not args.replicas:
        args.replicas = 5 if c4 else 3
    if args.quiesce < 0:
        args.quiesce = 1 if c5 else 0
    if args.listed < 0:
        args.listed = 1 if c5 else 0
    if c5:
        args.no_read_index = True  # writes, no reads
        if args.groups == 1 << 20:
            args.groups = 4 << 20
    if not args.save:
        args.save = "entrybatch" if c5 else "none"
    saves = args.save != "none"
    G, R, k = args.groups, args.replicas, args.k
    if c4:
        args.no_read_index = True  # 16 B writes, k_w = 1
    reads = not args.no_read_index
    # staged input batches: one per timed round, every one with fresh keys,
    # all resident in HBM before the timed region
    NP = max(8, args.steps)
    if args.kv_fill < 0:
        args.kv_fill = 0 if (c4 or c5) else C3_KV_FILL
    xch = None
    if c4:  # one global set of G groups spread over the world
        lanes = (G + world - 1) // world
        seed = ddist.BASE_SEED
        eng = Engine(num_groups=lanes, num_replicas=R, window=32, cmd_cap=32,
                     max_props=max(1, k), prop_slots=NP, ri_slots=NP,
                     mailbox=8, kv_slots=512, kv_val_cap=4, total_groups=G,
                     place_world=world, place_rank=rank, entry_mbox=k + 2,
                     device=local)
        if world > 1:
            from dragonboat_amd.exchange import PlaneExchange
            xch = PlaneExchange(eng, world, rank, torch.device("cuda", local),
                                fixed=args.exchange == "fixed")
    elif c5:  # 128 B / 1 KB entries, values out of line, saves encoded
        first_shard, seed = ddist.shard_plan(rank, G)
        vlen = C5_VAL[args.payload]
        cmd_cap = ((12 + (1 if vlen < 128 else 2) + vlen) + 15) // 16 * 16
        # proposals are drawn per round (seeded Bernoulli over the groups,
        # salt = round) into two alternating staged batches
        NP = 2
        bound = 73 + cmd_cap  # EntryBatch element bound (drb_codec.hpp)
        # the KV: C5_SLOTS keys per replica, the values in one shared pool
        # sized for the keys the run writes (c5_pool_blocks)
        ks = C5_SLOTS
        c5_rounds = args.c5_warm + 2 * args.warmup + args.steps + 8
        eng = Engine(num_groups=G, num_replicas=R, window=8, cmd_cap=cmd_cap,
                     max_props=max(1, k), prop_slots=NP, ri_slots=1,
                     mailbox=8, kv_slots=ks, kv_val_cap=vlen + 13 & ~15,
                     kv_pool_blocks=c5_pool_blocks(G, R, c5_rounds * k,
                                                   args.active_ppm),
                     kv_overflow_buckets=int(G * R * C5_OVF_PER) + 1024,
                     save_cap=(4 * bound + 15) // 16 * 16 +
                     (128 if args.save in ("tan", "tanmux") else 0),
                     save_tan=int(args.save in ("tan", "tanmux")),
                     tan_multiplexed=int(args.save == "tanmux"),
                     quiesce=args.quiesce, first_shard_id=first_shard,
                     no_lean=int(args.no_lean), device=local)
    else:
        first_shard, seed = ddist.shard_plan(rank, G)
        # with --save: room for the round's EntriesToSave (a follower may
        # save the last round's entries with this round's)
        bound = 73 + 32  # EntryBatch element bound at cmd_cap 32
        eng = Engine(num_groups=G, num_replicas=R, window=32, cmd_cap=32,
                     max_props=max(1, k), prop_slots=NP, ri_slots=NP,
                     mailbox=16, kv_slots=args.kv_slots or 512, kv_val_cap=4,
                     save_cap=(((2 * k + 2) * bound + 15) // 16 * 16 + 128
                               if saves else 0),
                     save_tan=int(args.save in ("tan", "tanmux")),
                     tan_multiplexed=int(args.save == "tanmux"),
                     elections=args.elections,
                     # the timed reads leave each client's ReadLocalNode
                     # result (drb_export_read_results / the step worker)
                     max_reads_per_ctx=(READS_PER_CTX if reads and
                                        args.read_results else 0),
                     first_shard_id=first_shard, device=local)
    eng.init_steady(term=2, leader_slot=0, seed=seed)
    stream = torch.cuda.ExternalStream(eng.stream)

    tick_every = [max(1, args.tick_every)]
    # input salts: the KV fill, the warmup and the timed rounds each draw
    # batches no earlier round used (workload.py: key = f(seed, g, salt))
    FILL_SALT, WARM_SALT, TIMED_SALT = 1 << 20, 1 << 21, 1 << 22

    def stage(b, salt):
        """batch b := the seeded inputs of salt (SURVEY 8d generators)"""
        eng.gen_kv_proposals(b, k, KEY_SPACE, 4, seed, salt)
        if reads:
            eng.gen_read_index(b, seed, salt + 30)

    def step(i, b=None):
        tick = i % tick_every[0] == 0
        # with reads: ReadLocalNode for the 9 reads behind every released
        # ctx, served inside the round (drb_round_in.reads_per_ctx)
        fused = reads and args.reads_mode == "fused"
        if c5:  # this round's 1 % (an independent draw every round)
            eng.gen_kv_proposals(i % NP, k, C5_KEYS,
                                 C5_VAL[args.payload], seed,
                                 i, active_ppm=args.active_ppm)
        if b is None:
            b = i % NP
        eng.step_async(tick=tick, prop_slot=b,
                       ri_slot=b if reads else 0xFFFFFFFF,
                       reads_per_ctx=READS_PER_CTX if fused else 0,
                       key_space=KEY_SPACE, encode_saves=saves,
                       ri_replica=2 if args.reads_at == "follower" else 0,
                       listed=bool(args.listed))
        if reads and not fused:
            eng.serve_reads(READS_PER_CTX, KEY_SPACE)
        if xch is not None:  # C4: this round's cross-GPU planes
            xch.step()

    # the KV's steady state (writes uniform over K = 256 keys
    # per group): fresh-key writes through the engine's own rounds until
    # each replica's table holds (nearly) all of its group's keys
    for i in range(args.kv_fill):
        eng.gen_kv_proposals(0, k, KEY_SPACE, 4, seed, FILL_SALT + i)
        eng.step_async(tick=True, prop_slot=0)
        if i % 256 == 255:
            eng.sync()
    # warmup (ticking every round); the tick cadence then follows the
    # reference's wall-clock tick worker: one LocalTick per RTTMillisecond
    def warm_step(i):
        if not c5:
            stage(0, WARM_SALT + i)
        step(i, 0 if not c5 else None)

    quiesce_info = None
    if c5 and args.c5_warm > 0:
        # C5's steady state: at 1 % of the groups proposing per round, a
        # group stays idle for the 200 ticks quiesceState needs with
        # probability ~0.99^200 = 13 %; these rounds (their own draws, a
        # tick each) get the timed rounds past that threshold
        for j in range(args.c5_warm):
            step(C5_WARM_BASE + j)
            if j % 128 == 127:
                eng.sync()
        eng.sync()
        # the quiesced replicas on a sample of 64 runs of 64 groups
        n_q = n_s = 0
        for r0 in range(0, G - 64 + 1, max(64, G // 64))[:64]:
            for st in eng.export_replicas(r0, 64):
                n_s += 1
                n_q += st.qs_quiesced_since > 0
        quiesce_info = {"warm_rounds": args.c5_warm,
                        "quiesced_fraction": n_q / max(1, n_s),
                        "sampled_replicas": n_s}
    tw0 = time.perf_counter()
    for i in range(args.warmup):
        warm_step(i)
    eng.sync()
    warm_ms = (time.perf_counter() - tw0) * 1e3 / max(1, args.warmup)
    if args.tick_every <= 0:
        te = max(1, int(round(args.tick_ms / max(warm_ms, 1e-6))))
        tick_every[0] = ddist.agree_min(te, red)
        for i in range(args.warmup, 2 * args.warmup):
            warm_step(i)
        eng.sync()
    args.tick_every = tick_every[0]
    if not c5:  # the timed rounds' inputs, resident before timing starts
        for b in range(args.steps):
            stage(b, TIMED_SALT + b)
        eng.sync()
    kv_load = None
    if not (c4 or c5):
        # the KV occupancy the timed rounds run at: distinct keys per
        # replica over a sample of groups (drb_kv_export)
        smp = [g * (G // 64) for g in range(64)]
        nk = [len(eng.kv_export(g, s)) for g in smp for s in range(R)]
        kv_slots = args.kv_slots or 512
        kv_load = {"keys_per_replica": sum(nk) / len(nk),
                   "kv_slots": kv_slots,
                   "load": sum(nk) / len(nk) / kv_slots,
                   "fill_rounds": args.kv_fill,
                   "note": "distinct keys per replica table after the fill "
                           "and warmup rounds, 64 sampled groups x %d "
                           "replicas; the timed rounds write fresh keys "
                           "and read uniformly over the %d" % (R, KEY_SPACE)}
    eng.read_counters(reset=True)
    phase_dbg = os.environ.get("DRB_PHASE") == "1"  # timing variants only
    if phase_dbg:
        eng.debug_phase(reset=True)
    warm_flagged = len(eng.take_flagged(reset=True)[0])
    if xch is not None:
        xch.bytes_sent = 0
    K = args.steps
    # rounds per drb_step_rounds call (C2 by default: a Python call per
    # round costs more host time than the GPU's round, profiles/r06_c2)
    rpc = args.rounds_per_call if args.rounds_per_call >= 0 else \
        (16 if c2 else 0)
    fused_reads = reads and args.reads_mode == "fused"
    if rpc > 1 and (c4 or c5 or args.listed or xch is not None or
                    (reads and not fused_reads)):
        rpc = 0  # (those step round by round)
    if rpc > 1:
        def rin_main(i):
            return dict(tick=(2 * args.warmup + i) % tick_every[0] == 0,
                        prop_slot=i % NP,
                        ri_slot=i % NP if reads else 0xFFFFFFFF,
                        reads_per_ctx=READS_PER_CTX if fused_reads else 0,
                        key_space=KEY_SPACE, encode_saves=saves,
                        ri_replica=2 if args.reads_at == "follower" else 0)
        calls = [Engine.round_array([rin_main(i) for i in
                                     range(i0, min(i0 + rpc, K))])
                 for i0 in range(0, K, rpc)]
        all_groups = (G + 255) // 256 * 256
    n_ev = len(calls) if rpc > 1 else K
    ev = [(torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(n_ev)]
    ddist.barrier()
    torch.cuda.synchronize()
    eng.sync()
    t0 = time.perf_counter()
    if rpc > 1:
        for j, arr in enumerate(calls):
            ev[j][0].record(stream)
            eng.step_rounds(arr, all_groups)
            ev[j][1].record(stream)
    else:
        for i in range(K):
            ev[i][0].record(stream)
            step(2 * args.warmup + i, None if c5 else i)
            ev[i][1].record(stream)
    eng.sync()
    torch.cuda.synchronize()
    ddist.barrier()
    t1 = time.perf_counter()
    out = eng.read_counters(reset=True)
    if phase_dbg:  # cycles per stepped lane of each round phase
        for role, x in eng.debug_phase(reset=True).items():
            print("phase raw %s per round: %s" % (
                role, " ".join("%.0f" % (c / K) for c in x)), file=sys.stderr)
            if x[0]:
                print("phase %s lanes %d: %s" % (
                    role, x[0] // K, " ".join("%.0f" % (c / x[0])
                                              for c in x[1:])),
                      file=sys.stderr)
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / K
    elapsed = t1 - t0
    committed = out.committed_entries
    elapsed = ddist.reduce_max(elapsed, red)
    committed = ddist.reduce_sum(committed, red)
    value = committed / elapsed
    # algorithmic bytes of one round on this GPU (its groups; C4: its
    # share of the global groups, plus the message bytes it moves)
    g_here = G if not c4 else (G + world - 1) // world
    if c5:  # per committed entry: the round's work for its group plus the
        # EntryBatch bytes of R replicas, written and read by the CRC
        P = args.payload
        per = alg_bytes_per_group_round(R, k, P, False) / k + \
            2 * R * (P + 30)
        alg = per * out.committed_entries / K
    else:
        alg = alg_bytes_per_group_round(R, k, 16, reads, c4 and world > 1) * \
            g_here
        if saves:  # + the save bytes the round writes
            alg += out.saved_bytes / K
    achieved = alg / (kern_ms * 1e-3) / 1e9
    # the workload's committed PMC summary (C3 at the KV steady state; C4
    # at N = 1 only, its per-GPU share differs with N)
    pmc_key = ("c5_%d" % args.payload if c5 else "c4" if c4 else
               "c2" if c2 else "c3")
    traffic = (None, None) if ((c3 and args.kv_fill == 0) or
                               (c4 and world > 1)) else \
        pmc_traffic(pmc_key, G, R)
    chunk_ab = None
    if args.chunk_ab and not (c4 or c5):
        # the same rounds (the timed batches again, slot b = i % NP) as K
        # plain rounds and as K / k drb_step_rounds calls, alternated twice
        fused = reads and args.reads_mode == "fused"

        def rin(i):
            return dict(tick=True, prop_slot=i % NP,
                        ri_slot=i % NP if reads else 0xFFFFFFFF,
                        reads_per_ctx=READS_PER_CTX if fused else 0,
                        key_space=KEY_SPACE)

        def plain():
            eng.sync()
            a = time.perf_counter()
            for i in range(K):
                eng.step_async(**rin(i))
            eng.sync()
            return (time.perf_counter() - a) * 1e3 / K

        def chunked(cg, kk):
            eng.sync()
            a = time.perf_counter()
            for i in range(0, K, kk):
                eng.step_rounds([rin(i + t) for t in range(min(kk, K - i))],
                                cg)
            eng.sync()
            return (time.perf_counter() - a) * 1e3 / K

        chunk_ab = {"plain_ms": [], "note": "K rounds of the timed batches "
                    "(LocalTick every round) as plain rounds and as "
                    "drb_step_rounds(k) over chunks of chunk_groups groups "
                    "(two streams alternating chunks), alternated twice, "
                    "ms per round; not value"}
        specs = [tuple(int(x) for x in sp.split(":"))
                 for sp in args.chunk_ab.split(",") if sp]
        for rep in range(2):
            chunk_ab["plain_ms"].append(plain())
            for cg, kk in specs:
                chunk_ab.setdefault("%d:%d" % (cg, kk), []).append(
                    chunked(cg, kk))
        out2 = eng.read_counters(reset=True)
        chunk_ab["fallbacks"] = out2.fallbacks
        chunk_ab["errors"] = out2.errors
    wire = None
    if not (c4 or c5 or args.no_wire):
        # after the timed region: the last round's leader -> follower-slot-1
        # plane as dragonboat's TCP stream (drb_encode_wire), as if every
        # slot-1 replica lived on one remote NodeHost
        reps, wt = 5, []
        for _ in range(reps):
            w0 = time.perf_counter()
            wres, _ = eng.encode_wire(0, 1, 1, b"10.0.0.1:26001", fetch=False)
            eng.sync()
            wt.append(time.perf_counter() - w0)
        wms = sorted(wt)[reps // 2] * 1e3
        wire = {"plane": "slot 0 -> slot 1 (leaders -> one follower host)",
                "messages": wres["n_msgs"], "frames": wres["n_frames"],
                "bytes": wres["n_bytes"], "ms": wms,
                "GB_per_s": wres["n_bytes"] / (wms * 1e-3) / 1e9,
                "messages_per_s": wres["n_msgs"] / (wms * 1e-3),
                "note": "median of %d drb_encode_wire calls (5 kernels + one "
                        "host sync for the plan), outside the timed "
                        "region" % reps}
        if not args.no_ingest and world == 1:
            # the receiving NodeHost: a second engine hosting the follower
            # slot only takes that stream in (drb_ingest_wire: frame and
            # payload CRCs, MessageBatch / Message / Entry decode, batched
            # placement into the next round's mailbox)
            _, stream = eng.encode_wire(0, 1, 1, b"10.0.0.1:26001")
            rx = Engine(num_groups=G, num_replicas=R, window=32, cmd_cap=32,
                        max_props=1, prop_slots=1, ri_slots=1, mailbox=16,
                        kv_slots=8, kv_val_cap=4, first_shard_id=first_shard,
                        device=local)
            rx.init_steady(term=2, leader_slot=0, seed=seed)
            rx.host_slot(0, False)
            # a first call sizes the device buffers; the replicas are reset
            # (the mailbox keeps room for a second copy), then the timed call
            rx.ingest_wire(stream, deployment_id=1)
            rx.init_steady(term=2, leader_slot=0, seed=seed)
            rx.host_slot(0, False)
            rx.sync()
            i0 = time.perf_counter()
            res = rx.ingest_wire(stream, deployment_id=1)
            rx.sync()
            ims = (time.perf_counter() - i0) * 1e3
            wire["ingest"] = {
                "messages": res["messages"], "accepted": res["accepted"],
                "dropped": res["dropped"], "ms": ims,
                "messages_per_s": res["messages"] / (ims * 1e-3),
                "GB_per_s": len(stream) / (ims * 1e-3) / 1e9,
                "note": "drb_ingest_wire of that stream into a second "
                        "engine hosting replica slot 1: one upload, GPU "
                        "CRC / decode / placement (host: frame headers and "
                        "each batch's top-level walk); warm buffers, "
                        "outside the timed region"}
            rx.close()
            # the same stream from a fresh receiver's pinned receive buffer
            # (drb_ingest_buffer: where a transport reads its connection)
            rx = Engine(num_groups=G, num_replicas=R, window=32, cmd_cap=32,
                        max_props=1, prop_slots=1, ri_slots=1, mailbox=16,
                        kv_slots=8, kv_val_cap=4, first_shard_id=first_shard,
                        device=local)
            rx.init_steady(term=2, leader_slot=0, seed=seed)
            rx.host_slot(0, False)
            ptr = rx.ingest_buffer(stream)
            rx.ingest_wire_pinned(ptr, len(stream), deployment_id=1)  # sizes
            rx.init_steady(term=2, leader_slot=0, seed=seed)
            rx.host_slot(0, False)
            rx.sync()
            p0 = time.perf_counter()
            pres = rx.ingest_wire_pinned(ptr, len(stream), deployment_id=1)
            rx.sync()
            pms = (time.perf_counter() - p0) * 1e3
            wire["ingest_pinned"] = {
                "messages": pres["messages"], "accepted": pres["accepted"],
                "ms": pms, "messages_per_s": pres["messages"] / (pms * 1e-3),
                "GB_per_s": len(stream) / (pms * 1e-3) / 1e9,
                "note": "the same call with the stream already in the "
                        "receiver's pinned buffer (drb_ingest_buffer), warm "
                        "buffers, outside the timed region"}
            rx.close()
            del stream
    failover = None
    if args.failover and args.elections and not (c4 or c5):
        # every group loses its leader replica (slot 0 stops); the
        # followers time out, campaign, vote and elect on the GPU (the
        # raft launch); ticks every round, no client traffic meanwhile
        eng.read_counters(reset=True)
        eng.host_slot(0, False)
        eng.sync()
        f0 = time.perf_counter()
        nr, elected, stepped = 0, 0, 0
        while nr < 12 * 10:
            for _ in range(5):
                eng.step_async(tick=True)
            nr += 5
            cen = eng.role_census()
            elected = sum(cen[s][3] for s in range(1, R))
            if elected >= G:
                break
        eng.sync()
        fms = (time.perf_counter() - f0) * 1e3
        fo = eng.read_counters(reset=True)
        failover = {
            "groups": G, "elected": elected, "rounds": nr, "ms": fms,
            "ms_per_round": fms / nr,
            "raft_launch_replicas": fo.elections_stepped,
            "role_changes": fo.role_changes,
            "fallbacks": fo.fallbacks, "errors": fo.errors,
            "note": "drb_host_slot(0, off) then LocalTick rounds until every "
                    "group has a leader among the other slots (census every "
                    "5 rounds, included in the time); election timeouts "
                    "are randomized in [10, 20) ticks (ElectionRTT 10)"}
        eng.host_slot(0, True)
    from dragonboat_amd import abi as _abi
    host_staged = None
    step_worker = None
    if args.host_staged < 0:
        args.host_staged = int(world == 1 and not (c4 or c5) and k == 1 and
                               not args.failover)
    if args.host_staged:
        # the same rounds with this round's proposals staged from host
        # memory: the entryQueue as a host builds its per-round upload
        # (drb_stage_proposals_packed: per group a count, per entry Key /
        # ClientID / Cmd length, the Cmd bytes back to back), uploaded and
        # laid out on the device, one call a round
        import ctypes as C
        from dragonboat_amd import workload
        # each host batch built in one pinned block at the engine's layout
        # (drb_stage_packed_layout): the upload is one DMA that overlaps the
        # previous round (the staging copies run on their own stream)
        HB = 8  # host batches, cycled
        u8p, u64p, u16p = (C.POINTER(C.c_uint8), C.POINTER(C.c_uint64),
                           C.POINTER(C.c_uint16))
        hb, hp = [], []
        # one NoOP session per group (client.NewNoOPSession): registered
        # once (drb_set_session_clients), so the batches leave ClientID out
        eng.set_session_clients(workload.build_packed_np(G, seed, 0)[2])
        for b in range(HB):
            arrs = [x.view("u1") for x in workload.build_packed_np(G, seed, b)]
            n_e, plen = arrs[1].size // 8, arrs[4].size
            off, _ = eng.stage_packed_layout(n_e, plen)
            nbytes = off[3] + plen  # (no client ids: the block ends here)
            blk = torch.zeros(max(1, nbytes), dtype=torch.uint8).pin_memory()
            view = blk.numpy()
            for o, x in zip([0] + off, arrs):
                if x is not arrs[2]:
                    view[o:o + x.size] = x
            base = blk.data_ptr()
            hb.append((blk, sum(x.size for x in arrs) - arrs[2].size))
            hp.append((C.cast(base, u8p), n_e, C.cast(base + off[0], u64p),
                       None, C.cast(base + off[2], u16p),
                       C.cast(base + off[3], u8p), plen))
        KH = max(5, K)
        eng.read_counters(reset=True)
        eng.sync()
        h0 = time.perf_counter()
        for i in range(KH):
            b = i % HB
            eng.stage_proposals_packed_async(b, _abi.ENTRY_ENCODED, *hp[b])
            step(2 * args.warmup + K + i, b)
        eng.sync()
        eng.stage_wait_upload()
        hms = (time.perf_counter() - h0) * 1e3 / KH
        hout = eng.read_counters(reset=True)
        host_staged = {
            "ms_per_step": hms, "steps": KH,
            "committed_entries_per_s": hout.committed_entries / (hms * KH *
                                                                 1e-3),
            "upload_bytes_per_round": int(hb[0][1]),
            "note": "proposals staged from pinned host memory every round "
                    "in the packed form (drb_stage_proposals_packed_async: "
                    "per group a count, per entry Key, Cmd length and bytes "
                    "-- ClientID is the group's session client, registered "
                    "once by drb_set_session_clients -- one DMA on a copy "
                    "engine overlapping the previous round, + scans and a "
                    "layout kernel; the host waits for an upload at the "
                    "next call), timed around the whole loop; not `value`"}
        if args.step_worker < 0:
            args.step_worker = int(reads and not c2 and args.read_results)
        if args.step_worker:
            # engine.processSteps as a whole (engine.go:1304-1364): the
            # entry queue up, the round, and every output a step worker
            # hands to its nodes down -- processReadyToRead, the served
            # reads' results, pendingProposals.applied -- exported behind
            # each round and drained on a copy stream into pinned host
            # buffers while the next round runs (two buffer sets)
            wb = [eng.worker_bufs(2 * G, 2 * G * READS_PER_CTX, 2 * G)
                  for _ in range(2)]
            KW = max(5, K)
            WW = max(2, args.warmup)

            def worker_loop(n, r0):
                # a step worker's iteration: the round (its proposals
                # staged one iteration ahead), the export behind it, the
                # next round's entry queue up while it runs, then the
                # outputs of the round before it (their copy ran beside
                # this round)
                got = [0, 0, 0, 0]
                marks = []
                eng.stage_proposals_packed_async(0, _abi.ENTRY_ENCODED,
                                                 *hp[0])
                pc = time.perf_counter
                for i in range(n):
                    t = [pc()]
                    step(r0 + i, i % HB)
                    t.append(pc())
                    eng.worker_export(0, wb[i % 2])
                    t.append(pc())
                    if i + 1 < n:
                        b1 = (i + 1) % HB
                        eng.stage_proposals_packed_async(
                            b1, _abi.ENTRY_ENCODED, *hp[b1])
                    t.append(pc())
                    if i >= 1:
                        n3 = eng.worker_wait(wb[(i - 1) % 2])
                        got = [d + x for d, x in zip(got, n3 + (1,))]
                    t.append(pc())
                    marks.append(t[-1])
                    phases.append([b - a for a, b in zip(t, t[1:])])
                n3 = eng.worker_wait(wb[(n - 1) % 2])
                eng.stage_wait_upload()
                return [d + x for d, x in zip(got, n3 + (1,))], marks

            r0 = 2 * args.warmup + K + KH
            phases = []
            worker_loop(WW, r0)  # untimed: first copies, host pages
            phases = []
            eng.read_counters(reset=True)
            eng.sync()
            w0 = time.perf_counter()
            down, marks = worker_loop(KW, r0 + WW)
            wms = (time.perf_counter() - w0) * 1e3 / KW
            its = sorted((b - a) * 1e3 for a, b in zip([w0] + marks, marks))
            wout = eng.read_counters(reset=True)
            for bw in wb:
                eng.free_worker_bufs(bw)
            # the lean records (include/drb_engine.h): a word per lane, a
            # 4 B ctx tag per ReadyToRead, 4 B + 2 bits per served read, 8 B
            # per ReadyToRead not served (over the exports waited for)
            dbytes = (down[3] * G * 4 + down[0] * 4 + down[1] * 4 +
                      (down[1] + 3 * down[3]) // 4 + down[2] * 8) / down[3]
            step_worker = {
                "ms_per_step": wms, "steps": KW, "warmup": WW,
                "iteration_ms_median": its[len(its) // 2],
                "iteration_ms_max": its[-1],
                # host time per call, medians: the round's launches, the
                # export, the next round's staging (waits for its upload),
                # the wait for the previous export's copies
                "host_ms": dict(zip(
                    ("round", "export", "stage", "wait"),
                    (round(sorted(x)[len(x) // 2] * 1e3, 4)
                     for x in zip(*phases)))),
                "committed_entries_per_s": wout.committed_entries /
                (wms * KW * 1e-3),
                "upload_bytes_per_round": int(hb[0][1]),
                "download_bytes_per_round": int(dbytes),
                "ready_to_reads_per_round": down[0] / KW,
                "read_results_per_round": down[1] / KW,
                "deferred_per_round": down[2] / KW,
                "note": "whole step-worker rounds timed around the loop: "
                        "packed proposals from pinned host memory (staged "
                        "one round ahead), the round with its 9 reads per "
                        "released ctx, then drb_worker_export of slot 0's "
                        "ReadyToReads, read results and applied counts "
                        "in the lean records (compaction behind the "
                        "round, exact-size copy-engine transfers into "
                        "pinned host buffers beside the next round); "
                        "drb_worker_wait of the previous round's export "
                        "every iteration; not `value`"}
        del hb, hp
    # the replicas that left the fast path during the run, by reason
    # (drb_take_flagged): a run with any is not a pure fast-path number
    flagged, lost = eng.take_flagged(reset=True)
    by_reason = {}
    for (_, _, reason, flags, _, _) in flagged:
        name = _abi.FB_NAME.get(reason, str(reason))
        if flags & _abi.F_APPLY_STOPPED:
            name += "/apply"
        by_reason[name] = by_reason.get(name, 0) + 1
    if lost:
        by_reason["unlisted"] = lost
    if out.fallbacks or out.errors:
        print("WARNING: fallbacks=%d errors=%d %s" % (
            out.fallbacks, out.errors, by_reason), file=sys.stderr)
    if rank == 0:
        if c5:
            sv = ("EntryBatch + CRC32 of EntriesToSave" if args.save ==
                  "entrybatch" else "tan log records (XXH64) of every "
                  "Update" if args.save == "tan" else "multiplexed tan log "
                  "records (XXH64) of every Update" if args.save == "tanmux"
                  else "no saves")
            metric = ("committed entries/sec (node) at %d 3-replica groups, "
                      "%d B payload, %g %% active per round, %s; %%HBM BW" % (
                          G, args.payload, args.active_ppm / 1e4, sv))
            wl = ("C5: %d groups x %d replicas per GPU, %d B PBKV writes "
                  "over %d keys per group (values out of line), %d ppm of "
                  "the groups proposing per "
                  "round (independent seeded draw each round, generated "
                  "inside the timed loop), %s, tick "
                  "every %d round(s); Quiesce %s%s" % (
                      G, R, args.payload, C5_KEYS,
                      args.active_ppm, sv, args.tick_every,
                      "on" if args.quiesce else "off",
                      ", listed rounds" if args.listed else ""))
            par = "groups sharded, replicas co-resident"
        elif c4:
            metric = ("committed entries/sec (node) at %d 5-replica groups "
                      "spread over %d GPU(s), 16B payload; %%HBM BW" % (
                          G, world))
            wl = ("C4: %d groups x %d replicas in total, replica slot s of "
                  "group g on GPU (g + s) mod %d, 16B PBKV writes "
                  "k=%d/group/round, tick every %d round(s)" % (
                      G, R, world, k, args.tick_every))
            par = ("replicas spread over GPUs; one plane exchange per round "
                   "(RCCL send/recv over xGMI)" if world > 1 else
                   "replicas co-resident (N=1)")
        elif c2:
            metric = ("committed entries/sec (node) at %d active 3-replica "
                      "groups, 16B payload, replicas co-resident; %%HBM BW"
                      % G)
            wl = ("C2: %d active groups x %d replicas per GPU, 16B PBKV "
                  "writes k=%d/group/round, tick every %d round(s)" % (
                      G, R, k, args.tick_every))
            par = "groups sharded, replicas co-resident"
        else:
            metric = ("committed entries/sec (node) at 1M active 3-replica "
                      "groups, 16B payload; %HBM BW")
            wl = ("C3: %d active groups x %d replicas per GPU, 16B PBKV "
                  "writes k=%d/group/round%s, tick every %d round(s)" % (
                      G, R, k, (", 9:1 ReadIndex:write at the %s" %
                                args.reads_at) if reads else "",
                      args.tick_every))
            par = "groups sharded, replicas co-resident"
        res = {
            "metric": metric,
            "value": value,
            "unit": "committed entries/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / K,
            "higher_is_better": True,
            "scaling": "strong" if c4 else "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (SURVEY 8d seeded PBKV writes%s)" % (
                " + ReadIndex" if reads else ""),
            "config": {
                "workload": wl,
                "groups_per_gpu": g_here, "replicas": R,
                "parallelism": par,
                "rounds_per_call": max(1, rpc)},
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic[0],
                "traffic_lower": traffic[1],
                "traffic_source": os.path.relpath(pmc_file(pmc_key), ROOT) +
                                  " (rocprofv3, "
                                  "the timed rounds' step kernels, bytes per "
                                  "round): traffic = FETCH_SIZE x2 + "
                                  "WRITE_SIZE, an upper bound (the x2 is for "
                                  "coalesced reads; a random 16 B KV read is "
                                  "tallied at 64 B already), traffic_lower = "
                                  "FETCH_SIZE + WRITE_SIZE",
                "alg_bytes_per_launch": alg,
                "kernel_ms": kern_ms},
            "counters": {"committed_per_round": committed / K / world,
                         "messages": out.messages,
                         "ready_to_reads": out.ready_to_reads,
                         "reads_served": out.reads_served,
                         "reads_deferred": out.reads_deferred,
                         "fallbacks": out.fallbacks, "errors": out.errors,
                         "fallbacks_by_reason": by_reason,
                         "fast_path_only": not (out.fallbacks or
                                                out.errors),
                         "flagged_in_warmup": warm_flagged,
                         "replicas_stepped_per_round":
                             out.replicas_stepped / K,
                         "lean_stepped_per_round": out.lean_stepped / K,
                         "saved_entries": out.saved_entries,
                         "saved_bytes": out.saved_bytes},
        }
        if c5:
            if quiesce_info is not None:
                quiesce_info["stepped_fraction"] = \
                    out.replicas_stepped / K / (G * R)
                res["quiesce"] = quiesce_info
            # C5's rounds are mostly heartbeats of the groups that do not
            # propose (past the pre-warm ~13 % of them are quiesced and
            # skipped by the listed rounds): a second figure counts, on top
            # of the entry bytes, each stepped replica's 64 B state record read + write
            # and each message's 16 B record written + read
            hb = (out.replicas_stepped * 128 + out.messages * 32) / K
            ach2 = (alg + hb) / (kern_ms * 1e-3) / 1e9
            res["roofline"]["with_heartbeats"] = {
                "alg_bytes_per_launch": alg + hb, "achieved": ach2,
                "frac": ach2 / HBM_PEAK_GBS,
                "model": "entry bytes + 128 B per stepped replica + 32 B "
                         "per message"}
        if args.save in ("tan", "tanmux"):
            res["counters"].update(
                log_records=out.log_records, log_syncs=out.log_syncs,
                log_new=out.log_new)
        if saves:
            res["config"]["save"] = {
                "entrybatch": "EntriesToSave as one EntryBatch + CRC32 per "
                              "replica per round (encode_saves)",
                "tan": "each replica's pb.Update as the regular tan LogDB's "
                       "log record (Update.MarshalTo in 32 KiB-block chunks "
                       "with XXH64 checksums, db.write skip / sync, "
                       "k_tan_select / k_tan_write)",
                "tanmux": "each replica's pb.Update as a record of the "
                          "multiplexed tan LogDB (16 logs per slot, key = "
                          "ShardID % 16, records back to back in group "
                          "order, k_tanm_chain)"}[args.save]
        if wire is not None:
            res["wire"] = wire
        if host_staged is not None:
            res["host_staged"] = host_staged
        if step_worker is not None:
            res["step_worker"] = step_worker
        if chunk_ab is not None:
            res["chunk_ab"] = chunk_ab
        if failover is not None:
            res["failover"] = failover
        if args.elections:
            res["config"]["elections"] = "on the GPU (drb_config.elections)"
        if kv_load is not None:
            res["kv_load"] = kv_load
        if xch is not None:
            res["exchange"] = {"mode": args.exchange,
                               "bytes_sent_per_round_rank0":
                               xch.bytes_sent / K,
                               "note": "the tests run this exchange over "
                                       "gloo with host staging (one-GPU "
                                       "boxes); this line is its first "
                                       "RCCL run"}
        if not args.no_cpu_baseline and world == 1:
            # (rank 0 at N = 1 only: the scaling runs keep their ranks' time)
            res["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    if args.c4_cross < 0:
        args.c4_cross = int(world > 1 and not c4)
    if args.c4_cross and world > 1:
        # C4 through the C ABI's cross-GPU exchange, after the timed run.
        # A watchdog ends the phase if the exchange hangs (ncclCommAbort,
        # then the line without it), so the main measurement still lands.
        done = threading.Event()
        cross = {}

        def watchdog():
            if done.wait(args.c4_timeout):
                return
            if rank == 0:
                res["c4_cross"] = {"error": "timed out after %d s" %
                                   args.c4_timeout}
                print(json.dumps(res), flush=True)
            os._exit(0 if rank == 0 else 3)
        threading.Thread(target=watchdog, daemon=True).start()
        try:
            cross = run_c4_cross(args, world, rank, local,
                                 args.dist_backend == "gloo")
        except Exception as ex:  # (reported in the line, not fatal to it)
            cross = {"error": "%s: %s" % (type(ex).__name__, ex)}
        done.set()
        if rank == 0:
            res["c4_cross"] = cross
    if rank == 0:
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
