"""GPU parity: the HIP step round against the CPU oracle, bit-exact.

Every test drives dragonboat_amd (through the C ABI) and the oracle with
the same seeded inputs (SURVEY 8d workload) and compares the full
per-replica state, resident log, KV contents, sent messages and
ReadyToReads after every round (tests/gpu_harness.py).
"""
import ctypes as C

import pytest

from dragonboat_amd import abi
from dragonboat_amd.engine import Engine
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu


def _run(pair, rounds, k=1, tick_every=1, ri_every=0, check_every=1):
    for r in range(rounds):
        tick = tick_every and (r % tick_every == 0)
        ri = bool(ri_every) and (r % ri_every == 0)
        o, e = pair.round(k=k, tick=tick, read_index=ri)
        assert (e.committed_entries, e.applied_entries, e.messages,
                e.ready_to_reads, e.dropped_read_indexes) == \
            (o.committed_entries, o.applied_entries, o.messages,
             o.ready_to_reads, o.dropped_read_indexes), (r, e.to_dict(),
                                                         o.to_dict())
        assert e.fallbacks == 0 and e.errors == 0, e.to_dict()
        if check_every and r % check_every == 0:
            errs = pair.check()
            assert not errs, (r, errs[:3])


def test_init_steady_matches_oracle_setup():
    p = Pair(G=64, R=3)
    errs = p.check(msgs=False, ready=False)
    assert not errs, errs[:3]


@pytest.mark.parametrize("R", [1, 2, 3, 5])
def test_init_steady_all_sizes(R):
    p = Pair(G=16, R=R)
    assert not p.check(msgs=False, ready=False)


def test_write_rounds_r3():
    _run(Pair(G=96, R=3), rounds=12, k=1, tick_every=0)


def test_write_rounds_with_ticks_r3():
    _run(Pair(G=96, R=3), rounds=25, k=1, tick_every=1)


def test_write_rounds_batched_k3():
    _run(Pair(G=64, R=3), rounds=12, k=3, tick_every=2)


@pytest.mark.parametrize("R", [1, 5])
def test_write_rounds_other_sizes(R):
    _run(Pair(G=64, R=R), rounds=15, k=1, tick_every=1)


def test_read_index_mix_c3():
    # 9:1 ReadIndex:write batched into one ctx per group per round
    _run(Pair(G=64, R=3), rounds=20, k=1, tick_every=1, ri_every=1)


def test_idle_groups_and_ragged_proposals():
    p = Pair(G=80, R=3)
    for r in range(14):
        groups = [g for g in range(p.G) if (g * 7 + r) % 3 != 0]
        o, e = p.round(k=2 if r % 2 else 1, tick=(r % 3 == 0),
                       read_index=(r % 4 == 1), groups=groups)
        assert e.fallbacks == 0 and e.errors == 0
        assert (e.committed_entries, e.messages) == \
            (o.committed_entries, o.messages)
        errs = p.check()
        assert not errs, (r, errs[:3])


def test_empty_rounds_then_resume():
    p = Pair(G=32, R=3)
    for r in range(6):
        p.round(k=0, tick=False)
    assert not p.check()
    _run(p, rounds=6, k=1, tick_every=1)


def test_lagging_follower_catches_up_via_reject_and_retry():
    # follower slot 2 of every group stops stepping for a few rounds (its
    # messages are lost), then rejoins: the leader's optimistic Replicate is
    # rejected (raft.go:1465-1470), decreaseTo/Retry (remote.go:182-198)
    # probes back and the follower catches up (logentry.go:296-310).
    p = Pair(G=48, R=3)
    _run(p, rounds=3, k=1, tick_every=0)
    for g in range(p.G):
        p.orc.set_hosted(g, 2, False)
    sts = p.eng.export_replicas(0, p.G)
    for i in range(2, len(sts), 3):
        sts[i].flags &= ~abi.F_HOSTED
    p.eng.import_replicas(0, sts)
    for r in range(5):
        p.round(k=1, tick=False)
        assert not p.check(groups=range(0, p.G, 7))
    for g in range(p.G):
        p.orc.set_hosted(g, 2, True)
    sts = p.eng.export_replicas(0, p.G)
    for i in range(2, len(sts), 3):
        sts[i].flags |= abi.F_HOSTED
    p.eng.import_replicas(0, sts)
    _run(p, rounds=10, k=1, tick_every=2)


def test_served_reads_c3():
    """ReadLocalNode for the 9 reads behind every released ReadIndex ctx
    (request.go:930-953 -> kvtest.go:164-175), drb_serve_reads vs oracle."""
    p = Pair(G=64, R=3)
    total = 0
    for r in range(12):
        o, e = p.round(k=1, tick=True, read_index=True)
        assert e.ready_to_reads == o.ready_to_reads
        p.eng.serve_reads(9, 256)
        got = p.eng.read_counters(reset=True)
        sums, served, deferred = p.orc.serve_reads(9, 256)
        assert (got.reads_served, got.reads_deferred) == (served, deferred)
        esums = p.eng.export_read_sums(0, p.G)
        for i, x in enumerate(sums):
            if x is not None:
                assert esums[i] == x, (r, i)
        total += served
    assert total >= 9 * p.G * 8


@pytest.mark.gpu
@pytest.mark.parametrize("key_space", [256, 200])
def test_served_reads_in_round(key_space):
    """The same reads served inside the step round (drb_round_in.
    reads_per_ctx), against the oracle's serve after its round; the key
    space 200 (not a power of two) takes the modulo path."""
    p = Pair(G=96, R=3)
    total = 0
    for r in range(10):
        o, e = p.round(k=1, tick=(r % 3 != 1), read_index=(r % 4 != 3),
                       reads=9, read_key_space=key_space)
        assert e.ready_to_reads == o.ready_to_reads
        sums, served, deferred = p.orc.serve_reads(9, key_space)
        assert (e.reads_served, e.reads_deferred) == (served, deferred), r
        esums = p.eng.export_read_sums(0, p.G)
        for i, x in enumerate(sums):
            if x is not None:
                assert esums[i] == x, (r, i)
        total += served
    assert total >= 9 * p.G * 5
    assert not p.check()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 3])
def test_entries_to_save_entrybatch_crc(k):
    """SaveRaftState input (engine.go:1343): every replica's EntriesToSave
    encoded on the GPU as EntryBatch bytes (entrybatch.go:25-58, colfer
    Entry raft_optimized.go:166-300) with CRC32-IEEE, byte-identical to the
    oracle codec; the CRC also checked against zlib."""
    import zlib
    p = Pair(G=40, R=3, save_cap=1024, max_props=4)
    n = 0
    for r in range(8):
        o, e = p.round(k=k if r % 3 != 2 else 0, tick=(r % 2 == 0),
                       read_index=(r % 3 == 0), encode_saves=True)
        assert e.fallbacks == 0 and e.errors == 0, e.to_dict()
        assert not p.check_saves(), r
        for g in range(0, p.G, 7):
            for s in range(3):
                b, crc = p.eng.export_saved(g, s)
                assert crc == (zlib.crc32(b) if b else 0)
                n += len(b) > 0
        assert e.saved_bytes == sum(len(p.eng.export_saved(g, s)[0])
                                    for g in range(p.G) for s in range(3))
    assert n > 0
    assert not p.check()


@pytest.mark.gpu
def test_batched_logdb_records_match_oracle():
    """save_batched (A26 -> F2): every round and replica, the GPU's batched
    LogDB records (batchedEntries.record, logdb/batch.go:288-346: split at
    index / 48, the first merged with the batch's earlier saves, then
    compactBatchFields) equal the oracle's restatement fed the oracle's
    EntriesToSave, byte for byte with their CRC32, across the batch
    boundaries at 48 and 96 with 1-3 proposals a round."""
    import zlib
    from oracle import pyoracle as po
    p = Pair(G=12, R=3, window=64, save_cap=8192, max_props=4,
             save_batched=1)
    db = po.BatchDB()
    first = p.eng.cfg["first_shard_id"]
    n_recs = merged = 0
    for r in range(45):
        o, e = p.round(k=1 + r % 3, tick=(r % 2 == 0),
                       read_index=(r % 5 == 0), encode_saves=True)
        assert e.fallbacks == 0 and e.errors == 0, (r, e.to_dict())
        for g in range(p.G):
            for s in range(p.R):
                ob, _ = p.orc.export_saved(g, s)
                ents = po.entrybatch_unmarshal(ob) if ob else []
                want = [(b, v, zlib.crc32(v)) for b, v in
                        db.record(first + g, s + 1, ents)] if ents else []
                got = p.eng.export_save_records(g, s)
                assert got == want, (r, g, s)
                n_recs += len(got)
                merged += sum(len(po.entrybatch_unmarshal(v)) > 1
                              for _, v, _ in got)
    assert n_recs and merged


@pytest.mark.gpu
def test_entries_to_save_capacity_falls_back():
    """A save buffer too small for the round's bound hands the replica to
    the CPU path before it mutates (DRB_FB_CAPACITY)."""
    p = Pair(G=8, R=3, save_cap=128, max_props=4)
    o, e = p.round(k=3, encode_saves=True)
    assert e.fallbacks > 0
    st = p.eng.export_replicas(0, 1)
    assert st[0].flags & abi.F_FALLBACK
    assert st[0].fallback_reason == abi.FB["CAPACITY"]


@pytest.mark.gpu
@pytest.mark.parametrize("N,R,G,counted", [
    (8, 5, 44, False), (2, 3, 30, False), (3, 5, 31, False),
    (4, 3, 20, False), (8, 5, 44, True), (3, 5, 31, True),
    (8, 5, 44, "bound"), (3, 5, 31, "bound"), (2, 3, 30, "bound")])
def test_replicas_spread_over_ranks_c4(N, R, G, counted):
    """C4 placement: replica slot s of group g on rank
    (g + s) mod N; every cross-rank message and its entries travel in the
    mailbox planes moved between the ranks' engines (drb_plane_regions --
    what RCCL moves between GPUs, here drb_exchange_local on one GPU: the
    full-capacity planes behind cross-stream events, or the counted sizes
    with host synchronisation) -- or, engines bound for the zero-copy
    exchange ("bound", drb_exchange_local_bind), read by the receivers in
    the senders' outboxes.  Bit-exact against one oracle cluster of all G
    groups."""
    from tests.gpu_harness import DistPair
    p = DistPair(G=G, R=R, N=N, max_props=4, counted=counted is True,
                 bound=counted == "bound")
    assert not p.check(), "init"
    for r in range(12):
        k = 1 if r % 5 != 4 else (3 if r % 2 else 0)
        o, e = p.round(k=k, tick=(r % 2 == 0), read_index=(r % 3 == 0))
        assert e["fallbacks"] == 0 and e["errors"] == 0, (r, e)
        assert (e["committed_entries"], e["applied_entries"], e["messages"],
                e["ready_to_reads"]) == \
            (o.committed_entries, o.applied_entries, o.messages,
             o.ready_to_reads), (r, e, o.to_dict())
        errs = p.check()
        assert not errs, (r, errs[:3])


@pytest.mark.gpu
def test_bound_engines_take_no_other_exchange():
    """Engines bound for the zero-copy exchange (drb_exchange_local_bind)
    read their remote planes in their peers' outboxes: nothing may be
    delivered into the inbound copies they no longer read -- ingest, the
    counted local exchange, inbound plane regions are DRB_EINVAL -- a
    second bind is refused, and rounds stay bit-exact after the refusals."""
    from dragonboat_amd.engine import DrbError
    from tests.gpu_harness import DistPair
    p = DistPair(G=20, R=3, N=2, max_props=4, bound=True)
    o, e = p.round(k=1, tick=True)
    assert e["fallbacks"] == 0 and not p.check()
    eng = p.engs[0]
    marr = (abi.Message * 1)()
    earr = (abi.Entry * 1)()
    pool = (C.c_uint8 * 16)()
    with pytest.raises(DrbError, match="status -1"):
        eng.ingest_ex(marr, 0, earr, pool)
    with pytest.raises(DrbError, match="status -1"):
        Engine.exchange_local(p.engs, counted=True)
    with pytest.raises(DrbError, match="status -1"):
        eng.plane_regions(1, 0, 0xffffffff, 1)
    with pytest.raises(DrbError, match="status -1"):
        Engine.exchange_local_bind(p.engs)
    for r in range(4):
        o, e = p.round(k=1, tick=r % 2 == 0)
        assert e["fallbacks"] == 0 and e["errors"] == 0, (r, e)
        assert e["committed_entries"] == o.committed_entries, r
    assert not p.check()


def _long_payload_rounds(p, val_len, rounds=8, encode=False, device_gen=False):
    from dragonboat_amd import workload
    for r in range(rounds):
        k = 1 if r % 4 != 3 else 2
        if device_gen:  # the bench's on-device generator, same definition
            counts, ents, pool = workload.build_batch(p.G, k, p.seed, r, 256,
                                                      val_len)
            p.orc.stage_proposals(counts, k, ents, pool)
            p.eng.gen_kv_proposals(0, k, 256, val_len, p.seed, r)
            o = p.orc.round(tick=(r % 2 == 0))
            e = p.eng.step(tick=(r % 2 == 0), prop_slot=0,
                           encode_saves=encode)
            p.rounds += 1
        else:
            o, e = p.round(k=k, tick=(r % 2 == 0), read_index=(r % 3 == 0),
                           val_len=val_len, encode_saves=encode)
        assert e.fallbacks == 0 and e.errors == 0, (r, p.why())
        assert (e.committed_entries, e.applied_entries, e.messages) == \
            (o.committed_entries, o.applied_entries, o.messages), r
        errs = p.check()
        assert not errs, (r, errs[:2])
        if encode:
            assert not p.check_saves(), r


@pytest.mark.gpu
@pytest.mark.parametrize("val_len,cmd_cap,val_cap", [
    (116, 144, 124),     # C5 128 B payload, value inline (9-chunk slots)
    (116, 144, 128),     # the same value out of line
    (1011, 1040, 1024),  # C5 1 KB payload, out of line
    (60, 80, 64)])       # a value crossing the 64 B header window, inline
def test_long_payloads_kv_apply(val_len, cmd_cap, val_cap):
    """SURVEY 8d C5 payloads: PBKV values of 116 / 1011 bytes (2-byte
    length varint), applied from the resident window 16 B at a time into
    inline slots or out-of-line value blocks; bit-exact KV, logs and the
    EntryBatch + CRC of every round's EntriesToSave."""
    p = Pair(G=24, R=3, cmd_cap=cmd_cap, kv_val_cap=val_cap, kv_slots=64,
             max_props=4, save_cap=8192)
    _long_payload_rounds(p, val_len, encode=True)


@pytest.mark.gpu
@pytest.mark.parametrize("val_len,cmd_cap,val_cap", [(4, 32, 4),
                                                     (1011, 1040, 1024)])
def test_device_generator_matches_workload(val_len, cmd_cap, val_cap):
    """drb_gen_kv_proposals (what bench.py stages) builds exactly the
    proposals of dragonboat_amd/workload.py (the SURVEY 8d definition)."""
    p = Pair(G=40, R=3, cmd_cap=cmd_cap, kv_val_cap=val_cap, kv_slots=64,
             max_props=4)
    _long_payload_rounds(p, val_len, rounds=5, device_gen=True)


@pytest.mark.gpu
@pytest.mark.parametrize("val_len,cmd_cap,val_cap,listed", [
    (116, 144, 128, False), (1011, 1040, 1024, False),
    (116, 144, 128, True)])
def test_c5_sparse_activity_idle_rounds(val_len, cmd_cap, val_cap, listed):
    """C5 in miniature: a seeded 10 % of the groups propose per round
    (drb_gen_kv_proposals_active), 128 B / 1 KB payloads, EntriesToSave
    encoded with CRC, ticks only every 4th round -- replicas at rest skip
    the idle rounds; state, logs, KV, messages and saves stay bit-exact."""
    from dragonboat_amd import workload
    p = Pair(G=64, R=3, cmd_cap=cmd_cap, kv_val_cap=val_cap, kv_slots=32,
             max_props=2, save_cap=8192, prop_slots=2)
    for r in range(16):
        act = workload.active_groups(p.G, p.seed, r, 100000)
        counts, ents, pool = workload.build_batch(p.G, 1, p.seed, r, 256,
                                                  val_len, groups=act)
        p.orc.stage_proposals(counts, 1, ents, pool)
        p.eng.gen_kv_proposals(r % 2, 1, 256, val_len, p.seed, r,
                               active_ppm=100000)
        tick = r % 4 == 0
        o = p.orc.round(tick=tick)
        e = p.eng.step(tick=tick, prop_slot=r % 2, encode_saves=True,
                       listed=listed)
        p.rounds += 1
        assert e.fallbacks == 0 and e.errors == 0, (r, p.why())
        assert (e.committed_entries, e.applied_entries, e.messages) == \
            (o.committed_entries, o.applied_entries, o.messages), r
        errs = p.check()
        assert not errs, (r, errs[:2])
        assert not p.check_saves(), r


@pytest.mark.gpu
@pytest.mark.parametrize("R,at", [(3, 2), (3, 3), (5, 4)])
def test_follower_read_index(R, at):
    """ReadIndex issued at a follower (SURVEY 8d C3 follower variant):
    handleFollowerReadIndex forwards the ctx to the leader
    (raft.go:2134-2144), the leader's handleLeaderReadIndex queues it with
    the follower as requester and confirms it by heartbeat quorum
    (raft.go:1842-1876, 1955-1974), the ReadIndexResp comes back
    (raft.go:2155-2164) and the follower serves the reads in-round."""
    p = Pair(G=48, R=R)
    total = 0
    for r in range(14):
        o, e = p.round(k=1, tick=(r % 2 == 0), read_index=True,
                       ri_replica=at, reads=9)
        assert e.fallbacks == 0 and e.errors == 0, (r, p.why())
        assert (e.committed_entries, e.messages, e.ready_to_reads,
                e.dropped_read_indexes) == \
            (o.committed_entries, o.messages, o.ready_to_reads,
             o.dropped_read_indexes), (r, e.to_dict(), o.to_dict())
        sums, served, deferred = p.orc.serve_reads(9, 256)
        assert (e.reads_served, e.reads_deferred) == (served, deferred), r
        esums = p.eng.export_read_sums(0, p.G)
        for i, x in enumerate(sums):
            if x is not None:
                assert esums[i] == x, (r, i)
        total += e.ready_to_reads
        errs = p.check()
        assert not errs, (r, errs[:2])
    assert total >= p.G * 8


@pytest.mark.gpu
def test_apply_results_and_durable_commit():
    """drb_apply_results: per applied entry the Key / ClientID / SeriesID
    and KVTest's Result.Value = len(payload) (kvtest.go:161) that
    pendingProposals.applied completes the proposal with (node.go:243-257),
    checked against the entries the oracle applied (its log from the
    previous sm index).  drb_commit_round gates the next round under a
    durable LogDB (engine.go:1343-1359)."""
    from dragonboat_amd.engine import DrbError
    p = Pair(G=32, R=3, durable_log=1)
    seen = 0
    for r in range(8):
        prev = {(g, s): p.orc.export(g, s).sm_index
                for g in range(p.G) for s in range(3)}
        o, e = p.round(k=1 if r % 3 else 2, tick=(r % 2 == 0))
        assert e.fallbacks == 0 and e.errors == 0
        for s in range(3):
            got = p.eng.apply_results(s)
            exp = []
            for g in range(p.G):
                now = p.orc.export(g, s).sm_index
                for t in p.orc.export_log(g, s, prev[(g, s)] + 1, now):
                    term, index, typ, key, cid, sid, _, cmd = t
                    ign = int(cid == 0)
                    val = 0 if ign else (len(cmd) - 1 if typ == 2 else
                                         len(cmd))
                    exp.append((g, index, key, cid, sid, val, ign))
            assert got == exp, (r, s, got[:3], exp[:3])
            seen += len(got)
        # the next round waits for this one's persistence
        with pytest.raises(DrbError):
            p.eng.step(tick=False)
        p.eng.commit_round(p.eng.round)
        assert p.eng.committed_round == p.eng.round
        assert not p.check()
    assert seen > 3 * p.G * 6
