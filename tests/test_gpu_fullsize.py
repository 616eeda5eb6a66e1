"""GPU: parity at the BASELINE sizes, on a sample of the groups.

The engine runs the full configuration of a bench workload -- C3
(1,048,576 groups x 3, 16 B, 9:1 ReadIndex with the reads served in the
round), C4's replica count co-resident (1,048,576 x 5), C5 (4,194,304 x 3,
128 B and 1 KB payloads, 1 % active per round, EntryBatch + CRC32, Quiesce,
listed rounds) -- from the same device input generators bench.py uses.  The
oracle simulates only a sample of ~1000 global group ids (including the
first and the last), with the same per-group seeds (oracle/, gids; groups
are independent, tests/test_oracle_cluster.py pins that), and the sampled
groups must match bit-exactly: every replica field, the resident log, the
KV contents, the outbox, the served-read checksums and the EntriesToSave
bytes + CRC.
"""
import random
import struct

import pytest

import bench
from dragonboat_amd import workload
from dragonboat_amd.engine import Engine
from oracle import pyoracle as po
from tests.gpu_harness import by_dest, state_diff

pytestmark = pytest.mark.gpu

SEED = 0x5EEDD8B0


def _sample(G, n=1000):
    rng = random.Random(G * 7 + 1)
    return sorted(set([0, 1, 2, G // 2, G - 2, G - 1] +
                      rng.sample(range(G), n)))


def _compare(eng, orc, gids, R, logs=True, saves=False):
    errs = []
    for i, g in enumerate(gids):
        est = eng.export_replicas(g, 1)
        for s in range(R):
            a, b = est[s], orc.export(i, s)
            d = state_diff(a, b, R)
            if a.shard_id != b.shard_id or a.flags != b.flags:
                d["ids"] = ((a.shard_id, a.flags), (b.shard_id, b.flags))
            if d:
                errs.append((g, s, "state", d))
                continue
            if logs:
                lo = max(1, b.last_index - 6)
                if eng.export_log(g, s, lo, b.last_index) != \
                        orc.export_log(i, s, lo, b.last_index):
                    errs.append((g, s, "log"))
            if eng.kv_export(g, s) != orc.export_kv(i, s):
                errs.append((g, s, "kv"))
            if by_dest(eng.export_outbox(g, s)) != \
                    by_dest(orc.export_outbox(i, s)):
                errs.append((g, s, "msgs"))
            if saves and eng.export_saved(g, s) != orc.export_saved(i, s):
                errs.append((g, s, "saved"))
        if len(errs) > 4:
            break
    return errs


def test_fullsize_c3_sampled():
    """C3 as bench.py runs it: first bench.py's own fill of fresh-key
    writes (C3_KV_FILL rounds: each replica's KV holds nearly all of its
    group's 256 keys, load ~0.50 -- SURVEY 8d's steady state, the table the
    timed rounds probe), then rounds whose inputs -- a write with fresh
    keys and a ReadIndex ctx per group -- come from the device generators,
    a LocalTick every round, 9 served reads per ctx, which find their
    key."""
    G, R, NP, FILL = 1 << 20, 3, 8, bench.C3_KV_FILL
    # bench.py's C3 engine: the timed reads leave every client's result
    eng = Engine(num_groups=G, num_replicas=R, window=32, cmd_cap=32,
                 max_props=1, prop_slots=NP, ri_slots=NP, mailbox=16,
                 kv_slots=512, kv_val_cap=4,
                 max_reads_per_ctx=bench.READS_PER_CTX)
    eng.init_steady(term=2, leader_slot=0, seed=SEED)
    gids = _sample(G)
    n = len(gids)
    orc = po.Cluster(n, R, seed=SEED, gids=gids)
    orc.setup_steady(0)
    for r in range(FILL):
        salt = (1 << 20) + r
        counts, ents, pool = workload.build_batch(n, 1, SEED, salt,
                                                  gids=gids)
        orc.stage_proposals(counts, 1, ents, pool)
        eng.gen_kv_proposals(0, 1, 256, 4, SEED, salt)
        orc.round(tick=True)
        e = eng.step(tick=True, prop_slot=0)
        assert e.fallbacks == 0 and e.errors == 0, (r, e.to_dict())
    errs = _compare(eng, orc, gids, R)
    assert not errs, ("fill", errs[:3])
    keys = [len(orc.export_kv(i, s)) for i in range(0, n, 50)
            for s in range(R)]
    # ~ 256 (1 - e^(-1536/256)) = 255.4 keys per replica
    assert sum(keys) / len(keys) >= 250, sum(keys) / len(keys)
    found = total = 0
    for r in range(24):
        b, salt = r % NP, (1 << 22) + r
        eng.gen_kv_proposals(b, 1, 256, 4, SEED, salt)
        eng.gen_read_index(b, SEED, salt + 30)
        counts, ents, pool = workload.build_batch(n, 1, SEED, salt,
                                                  gids=gids)
        orc.stage_proposals(counts, 1, ents, pool)
        lo, hi = workload.build_read_index(n, SEED, salt + 30, salt + 30,
                                           gids=gids)
        orc.stage_read_index(lo, hi)
        o = orc.round(tick=True)
        e = eng.step(tick=True, prop_slot=b, ri_slot=b, reads_per_ctx=9,
                     key_space=256)
        assert e.fallbacks == 0 and e.errors == 0, (r, e.to_dict())
        if r >= 3:
            assert e.committed_entries == G, (r, e.committed_entries)
        sums, served, deferred = orc.serve_reads(9, 256)
        esum = eng.export_read_sums(0, G)
        for i, g in enumerate(gids):
            for s in range(R):
                x = sums[i * R + s]
                if x is not None:
                    assert esum[g * R + s] == x, (r, g, s)
        if r % 4 == 3:  # the ReadLocalNode results of the sampled groups
            _compare_read_results(eng, orc, gids, r)
        if r % 8 == 7:
            errs = _compare(eng, orc, gids, R)
            assert not errs, (r, errs[:3])
    # the reads of a ctx look up keys that are (nearly always) present
    for i in range(0, n, 97):
        kv = orc.export_kv(i, 0)
        for rr in range(4):
            lo, _ = workload.read_index_ctx(SEED, gids[i], rr, rr)
            for j in range(9):
                key = workload.mix64(lo ^ ((j + 1) * workload.GOLDEN &
                                           workload.MASK)) % 256
                total += 1
                found += key.to_bytes(8, "little") in kv
    assert found > 0.7 * total


def _compare_read_results(eng, orc, gids, rnd, slot=0, reads=9, keys=256):
    """drb_export_read_results of the sampled groups against the oracle:
    per served read of every ReadyToRead whose index the replica applied,
    the key, found, length and value (request.go:930-953 ->
    nodehost.go:849 -> KVTest.Lookup, kvtest.go:164-175)."""
    for i in range(0, len(gids), 7):
        g = gids[i]
        got = eng.export_read_results(slot, g, 1)
        st = orc.export(i, slot)
        kv = orc.export_kv(i, slot)
        want = []
        for (index, low, high) in orc.export_ready(i, slot):
            if index > st.sm_index:
                continue
            for j in range(reads):
                key = workload.mix64(low ^ (((j + 1) * workload.GOLDEN) &
                                            workload.MASK)) % keys
                v = kv.get(struct.pack("<Q", key))
                want.append((g, index, low, j, key, int(v is not None),
                             len(v) if v is not None else 0,
                             int.from_bytes((v or b"")[:4], "little")))
        assert got == want, (rnd, g, got[:2], want[:2])


def test_fullsize_five_replicas_sampled():
    """C4's 5-replica groups at 1,048,576 lanes, co-resident (N = 1)."""
    G, R, NP = 1 << 20, 5, 8
    eng = Engine(num_groups=G, num_replicas=R, window=32, cmd_cap=32,
                 max_props=1, prop_slots=NP, ri_slots=NP, mailbox=16,
                 kv_slots=512, kv_val_cap=4)
    eng.init_steady(term=2, leader_slot=0, seed=SEED)
    for b in range(NP):
        eng.gen_kv_proposals(b, 1, 256, 4, SEED, b)
    gids = _sample(G, 600)
    n = len(gids)
    orc = po.Cluster(n, R, seed=SEED, gids=gids)
    orc.setup_steady(0)
    for r in range(20):
        b = r % NP
        counts, ents, pool = workload.build_batch(n, 1, SEED, b, gids=gids)
        orc.stage_proposals(counts, 1, ents, pool)
        o = orc.round(tick=(r % 2 == 0))
        e = eng.step(tick=(r % 2 == 0), prop_slot=b)
        assert e.fallbacks == 0 and e.errors == 0, (r, e.to_dict())
    errs = _compare(eng, orc, gids, R)
    assert not errs, errs[:3]


def _c5_engine(G, R, payload, rounds, active_ppm, kv_slots=None,
               ovf_buckets=None, save_extra=0, **kw):
    """bench.py's C5 engine (bench.py main): kv_slots = C5_SLOTS, overflow
    buckets G*R*C5_OVF_PER + 1024 from one engine-wide pool, the values in
    one shared block pool sized by c5_pool_blocks for the rounds run."""
    vlen = bench.C5_VAL[payload]
    cmd_cap = ((12 + (1 if vlen < 128 else 2) + vlen) + 15) // 16 * 16
    bound = 73 + cmd_cap
    eng = Engine(num_groups=G, num_replicas=R, window=8, cmd_cap=cmd_cap,
                 max_props=1, prop_slots=2, ri_slots=1, mailbox=8,
                 kv_slots=kv_slots or bench.C5_SLOTS,
                 kv_val_cap=vlen + 13 & ~15,
                 kv_pool_blocks=bench.c5_pool_blocks(G, R, rounds,
                                                     active_ppm),
                 kv_overflow_buckets=(ovf_buckets if ovf_buckets is not None
                                      else int(G * R * bench.C5_OVF_PER) +
                                      1024),
                 save_cap=(4 * bound + 15) // 16 * 16 + save_extra, quiesce=1,
                 **kw)
    return eng, vlen


def _c5_run(eng, orc, gids, R, vlen, rounds, active_ppm, check_every):
    n = len(gids)
    for r in range(rounds):
        act = workload.active_groups(n, SEED, r, active_ppm, gids=gids)
        counts, ents, pool = workload.build_batch(n, 1, SEED, r,
                                                  bench.C5_KEYS, vlen,
                                                  groups=act, gids=gids)
        orc.stage_proposals(counts, 1, ents, pool)
        eng.gen_kv_proposals(r % 2, 1, bench.C5_KEYS, vlen, SEED, r,
                             active_ppm=active_ppm)
        o = orc.round(tick=True)
        e = eng.step(tick=True, prop_slot=r % 2, encode_saves=True,
                     listed=True)
        assert e.fallbacks == 0 and e.errors == 0, (r, e.to_dict())
        if r % check_every == check_every - 1 or r == rounds - 1:
            errs = _compare(eng, orc, gids, R, saves=True)
            assert not errs, (r, errs[:3])


@pytest.mark.parametrize("payload,rounds", [(128, 240), (1024, 40)])
def test_fullsize_c5_sampled(payload, rounds):
    """C5 as bench.py runs it, with bench.py's own engine arguments:
    4,194,304 groups, a fresh seeded 1 % of them proposing each round
    (device generator, salt = round) over the 256-key space, values out of
    line in the shared pool, KV overflow buckets, EntriesToSave encoded,
    Quiesce on, listed rounds."""
    G, R = 4 << 20, 3
    eng, vlen = _c5_engine(G, R, payload, rounds, 10000)
    eng.init_steady(term=2, leader_slot=0, seed=SEED)
    gids = _sample(G, 1000)
    orc = po.Cluster(len(gids), R, seed=SEED, gids=gids, quiesce=True)
    orc.setup_steady(0)
    _c5_run(eng, orc, gids, R, vlen, rounds, 10000, 60)
    n = len(gids)
    qs = sum(orc.export(i, s).qs_quiesced_since > 0
             for i in range(n) for s in range(R))
    if rounds > 220:
        assert qs > 0  # some sampled groups went quiet past the threshold


def test_fullsize_c5_overflow_chains():
    """The KV overflow chains at full size: 4-slot tables at 4,194,304
    groups x 3 and a quarter of the groups proposing every round, so that
    most replicas hold several times their table's keys -- chains of
    buckets bump-allocated from the one engine-wide pool by 12.6 M
    replicas at once (kvtest.go:145-162: KVTest's map grows).  Every
    sampled replica's whole KV (table and chain) equals the oracle's."""
    G, R, rounds, ppm = 4 << 20, 3, 40, 250000
    eng, vlen = _c5_engine(G, R, 128, rounds, ppm, kv_slots=4,
                           ovf_buckets=3 * G * R)
    eng.init_steady(term=2, leader_slot=0, seed=SEED)
    gids = _sample(G, 600)
    orc = po.Cluster(len(gids), R, seed=SEED, gids=gids, quiesce=True)
    orc.setup_steady(0)
    _c5_run(eng, orc, gids, R, vlen, rounds, ppm, 20)
    sizes = [len(eng.kv_export(g, s)) for g in gids for s in range(R)]
    chained = sum(x > 4 for x in sizes)
    assert chained > len(sizes) // 2, (chained, len(sizes))
    assert max(sizes) >= 12, max(sizes)  # chains of two buckets and more


def test_fullsize_failover_sampled():
    """Elections on the GPU at the C3 size: 1,048,576 groups x 3 with
    writes and reads, then every group's leader replica (slot 0) stops; the
    followers elect new leaders through the raft launch while the client
    queue keeps proposing (dropped while a group has no leader), and the
    sampled groups match the oracle bit-exactly throughout -- terms, votes,
    roles, randomized timeouts and their generator state, logs, KV,
    outboxes."""
    G, R, NP = 1 << 20, 3, 8
    eng = Engine(num_groups=G, num_replicas=R, window=32, cmd_cap=32,
                 max_props=1, prop_slots=NP, ri_slots=NP, mailbox=16,
                 kv_slots=512, kv_val_cap=4, elections=1)
    eng.init_steady(term=2, leader_slot=0, seed=SEED)
    for b in range(NP):
        eng.gen_kv_proposals(b, 1, 256, 4, SEED, b)
        eng.gen_read_index(b, SEED, b + 30)
    gids = _sample(G, 800)
    n = len(gids)
    orc = po.Cluster(n, R, seed=SEED, gids=gids)
    orc.setup_steady(0)
    slow = 0
    for r in range(200):
        if r == 6:  # the leaders stop
            eng.host_slot(0, False)
            for i in range(n):
                orc.set_hosted(i, 0, False)
        b = r % NP
        counts, ents, pool = workload.build_batch(n, 1, SEED, b, gids=gids)
        orc.stage_proposals(counts, 1, ents, pool)
        lo, hi = workload.build_read_index(n, SEED, b + 30, b + 30,
                                           gids=gids)
        orc.stage_read_index(lo, hi)
        o = orc.round(tick=True)
        e = eng.step(tick=True, prop_slot=b, ri_slot=b)
        if e.fallbacks or e.errors:
            recs, _ = eng.take_flagged(cap=4096)
            hist = {}
            for (g, s, reason, flags, _r, _sh) in recs:
                hist[(s, reason, flags)] = hist.get((s, reason, flags), 0) + 1
            st = [eng.export_replicas(g, 1)[s].to_dict(R)
                  for (g, s, *_x) in recs[:2]]
            raise AssertionError((r, e.to_dict(), hist, st))
        slow += e.elections_stepped
        if r % 15 == 14:
            errs = _compare(eng, orc, gids, R)
            assert not errs, (r, errs[:3])
        if r >= 40 and r % 10 == 9:
            cen = eng.role_census()
            if sum(cen[s][3] for s in (1, 2)) == G:  # every group re-elected
                break
    assert sum(cen[s][3] for s in (1, 2)) == G, cen
    errs = _compare(eng, orc, gids, R)
    assert not errs, errs[:3]
    assert slow > 0


def test_fullsize_c5_tan_sampled():
    """C5 at 128 B with the tan LogDB records (save_tan): 4,194,304 groups,
    1 % proposing per round, Quiesce, listed rounds.  The oracle's tan db of
    every sampled replica takes that replica's Update every round; at the
    check rounds the GPU's record of the round -- bytes, offset, sync, log
    -- and its writer position equal the oracle's."""
    G, R = 4 << 20, 3
    # bench.py's C5 engine with --save tan (its save_cap + 128)
    eng, vlen = _c5_engine(G, R, 128, 48, 10000, save_extra=128, save_tan=1)
    eng.init_steady(term=2, leader_slot=0, seed=SEED)
    gids = _sample(G, 500)
    n = len(gids)
    orc = po.Cluster(n, R, seed=SEED, gids=gids, quiesce=True)
    orc.setup_steady(0)
    dbs = [[po.TanDB() for _ in range(R)] for _ in range(n)]
    checked = 0
    for r in range(48):
        act = workload.active_groups(n, SEED, r, 10000, gids=gids)
        counts, ents, pool = workload.build_batch(n, 1, SEED, r,
                                                  bench.C5_KEYS, vlen,
                                                  groups=act, gids=gids)
        orc.stage_proposals(counts, 1, ents, pool)
        eng.gen_kv_proposals(r % 2, 1, bench.C5_KEYS, vlen, SEED, r,
                             active_ppm=10000)
        o = orc.round(tick=True)
        e = eng.step(tick=True, prop_slot=r % 2, encode_saves=True,
                     listed=True)
        assert e.fallbacks == 0 and e.errors == 0, (r, e.to_dict())
        check = r % 12 == 11
        for i, g in enumerate(gids):
            for s in range(R):
                want = orc.tan_write(i, s, dbs[i][s])
                if not check:
                    continue
                rec, data = eng.export_tan(g, s)
                where = (r, g, s, rec, want)
                if want is None:
                    assert not rec["flags"] & 1, where
                    continue
                assert (rec["offset"], rec["len"], rec["log"],
                        bool(rec["flags"] & 2)) == \
                    (want["off"], want["len"], want["log"], want["sync"]), where
                f = dbs[i][s].file(want["log"])
                assert data == f[want["off"]:want["off"] + want["len"]], where
                assert eng.tan_get(g, s)[0] == want["offset"], where
                checked += 1
    assert checked > 0


def _compare_spread(engs, orc, gids, R, N):
    """_compare for C4's placement: replica slot s of global group g lives on
    rank (g + s) mod N at lane g // N."""
    errs = []
    for i, g in enumerate(gids):
        for s in range(R):
            e, j = engs[(g + s) % N], g // N
            a, b = e.export_replicas(j, 1)[s], orc.export(i, s)
            d = state_diff(a, b, R)
            if a.shard_id != b.shard_id or a.flags != b.flags:
                d["ids"] = ((a.shard_id, a.flags), (b.shard_id, b.flags))
            if d:
                errs.append((g, s, "state", d))
                continue
            lo = max(1, b.last_index - 6)
            if e.export_log(j, s, lo, b.last_index) != \
                    orc.export_log(i, s, lo, b.last_index):
                errs.append((g, s, "log"))
            if e.kv_export(j, s) != orc.export_kv(i, s):
                errs.append((g, s, "kv"))
            if by_dest(e.export_outbox(j, s)) != \
                    by_dest(orc.export_outbox(i, s)):
                errs.append((g, s, "msgs"))
        if len(errs) > 4:
            break
    return errs


def _exchange_by_plan(engs, mask, counted=False):
    """drb_exchange_plan's transfers of every rank (counted: drb_exchange_
    plan_words over every rank's drb_plane_counts, the step of
    drb_exchange_rccl_counted), each send copied into its paired receive
    (what RCCL's send / recv do between GPUs)."""
    import torch
    from dragonboat_amd import exchange as X
    dev = torch.device("cuda", 0)
    for e in engs:
        e.sync()
    if counted:
        words = [e.plane_counts() for e in engs]
        plans = [e.exchange_plan_words(words) for e in engs]
    else:
        plans = [e.exchange_plan(mask) for e in engs]
    moved = 0
    for r, pr in enumerate(plans):
        for q, pq in enumerate(plans):
            if q == r:
                continue
            sends = [(p, n) for peer, rv, p, n in pr if peer == q and not rv]
            recvs = [(p, n) for peer, rv, p, n in pq if peer == r and rv]
            assert [n for _, n in sends] == [n for _, n in recvs], (r, q)
            for (sp, n), (dp, _) in zip(sends, recvs):
                X.device_bytes(dp, n, dev).copy_(X.device_bytes(sp, n, dev))
                moved += n
    torch.cuda.synchronize()
    for e in engs:
        e.exchange_mark()
    return moved


@pytest.mark.parametrize("mode", ["local", "plan", "counted", "bound"])
def test_fullsize_c4_spread_sampled(mode):
    """C4 at its configured size and placement: 1,048,576 groups x 5
    replicas over 8 ranks -- replica slot s of group g on rank (g + s) mod
    8 at lane g // 8 -- as 8 engines of one process on the one GPU, with
    bench.py's C4 engine arguments (mailbox 8, entry_mbox k + 2, the device
    input generators).  After every round the planes move either by
    drb_exchange_local (the device pull; "bound": nothing moves, the
    receivers read the senders' outboxes, drb_exchange_local_bind), by
    drb_exchange_plan's transfer
    list (the fixed-capacity step of drb_exchange_rccl) or by
    drb_exchange_plan_words over every rank's counts (the counted step of
    drb_exchange_rccl_counted), each send copied into its paired receive as
    RCCL would.  ~1000 sampled groups match one oracle cluster every few
    rounds: every replica field, log, KV and outbox.  The counted step ships
    at most 230 MB per rank per round (the fixed one 419 MB)."""
    G, R, N, NP, k = 1 << 20, 5, 8, 8, 1
    lanes = G // N
    engs = [Engine(num_groups=lanes, num_replicas=R, window=32, cmd_cap=32,
                   max_props=k, prop_slots=NP, ri_slots=NP, mailbox=8,
                   kv_slots=512, kv_val_cap=4, total_groups=G,
                   place_world=N, place_rank=r, entry_mbox=k + 2)
            for r in range(N)]
    try:
        for e in engs:
            e.init_steady(term=2, leader_slot=0, seed=SEED)
        if mode == "bound":
            Engine.exchange_local_bind(engs)
        mask = 0
        for e in engs:
            mask |= e.role_slots()[0]
        gids = _sample(G, 1000)
        n = len(gids)
        orc = po.Cluster(n, R, seed=SEED, gids=gids)
        orc.setup_steady(0)
        moved = 0
        for r in range(16):
            b, salt = r % NP, (1 << 22) + r
            counts, ents, pool = workload.build_batch(n, k, SEED, salt,
                                                      gids=gids)
            orc.stage_proposals(counts, k, ents, pool)
            for e in engs:
                e.gen_kv_proposals(b, k, 256, 4, SEED, salt)
            tick = r % 3 != 2
            orc.round(tick=tick)
            outs = [e.step(tick=tick, prop_slot=b) for e in engs]
            assert sum(o.fallbacks + o.errors for o in outs) == 0, \
                (r, [o.to_dict() for o in outs if o.fallbacks or o.errors])
            if r >= 3:
                assert sum(o.committed_entries for o in outs) == G, r
            if mode in ("local", "bound"):
                Engine.exchange_local(engs)
            else:
                m = _exchange_by_plan(engs, mask, counted=mode == "counted")
                if mode == "counted" and r >= 3:
                    assert m / N <= 230e6, (r, m / N)
                moved += m
            if r % 5 == 4 or r == 15:
                errs = _compare_spread(engs, orc, gids, R, N)
                assert not errs, (r, errs[:3])
        assert mode in ("local", "bound") or moved > 0
    finally:
        for e in engs:
            e.close()
