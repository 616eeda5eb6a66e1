"""The CPU restatement of the step loop (node_test.go:274-353) over a
cluster of groups: steady-state properties the reference guarantees, and
the synthetic workload definition it is fed.

These pin the checker the GPU parity tests compare against:
  * steady setup = the state a CPU election + config-change bootstrap leaves
    (raft.go:1049 noop at term 2 after R config-change entries),
  * k proposals per round commit on the leader two rounds later and on the
    followers three rounds later (Replicate -> Resp -> commit -> Heartbeat /
    Replicate carrying Commit),
  * every replica's KV equals the last-writer-wins map of the applied PBKV
    writes (kvtest.go:145-162),
  * ReadIndex ctx are released to the leader with the committed index at
    their arrival (raft.go:1842-1876, readindex.go:77-115).
"""
import struct

import pytest

from dragonboat_amd import abi, workload
from oracle import pyoracle as po

SEED = 0x5EEDD8B0


def expected_kv(G, rounds, k, seed=SEED, key_space=256, val_len=4):
    kv = [dict() for _ in range(G)]
    for s in range(rounds):
        for g in range(G):
            for j in range(k):
                p = workload.proposal(seed, g, s, j, key_space, val_len)
                key, val = po.pbkv_unmarshal(p["cmd"][1:])
                kv[g][key] = val
    return kv


def run(G, R, rounds, k=1, reads=False, tick=True, drain=4):
    c = po.Cluster(G, R, seed=SEED)
    c.setup_steady(0)
    outs = []
    for t in range(rounds + drain):
        if t < rounds:
            counts, ents, pool = workload.build_batch(G, k, SEED, t)
            c.stage_proposals(counts, k, ents, pool)
            if reads:
                lo, hi = workload.build_read_index(G, SEED, t, t + 30)
                c.stage_read_index(lo, hi)
        outs.append(c.round(tick=tick))
    return c, outs


@pytest.mark.parametrize("R", [1, 3, 5])
def test_steady_setup(R):
    c = po.Cluster(4, R, seed=SEED)
    c.setup_steady(0)
    for g in range(4):
        for s in range(R):
            st = c.export(g, s)
            assert st.term == 2 and st.leader_id == 1 and st.vote == 1
            assert st.last_index == R + 1 == st.committed == st.applied
            assert st.role == (abi.LEADER if s == 0 else abi.FOLLOWER)
        log = c.export_log(g, 0, 1, R + 1)
        assert [e[2] for e in log[:R]] == [abi.ENTRY_CONFIG_CHANGE] * R
        assert log[R][0] == 2 and log[R][3] == 0  # noop at term 2, key 0


@pytest.mark.parametrize("R,k", [(3, 1), (3, 3), (5, 1), (1, 2)])
def test_writes_commit_and_apply_everywhere(R, k):
    G, rounds = 16, 8
    c, outs = run(G, R, rounds, k=k)
    total = sum(o.committed_entries for o in outs)
    assert total == G * rounds * k
    kv = expected_kv(G, rounds, k)
    for g in range(G):
        for s in range(R):
            st = c.export(g, s)
            assert st.last_index == R + 1 + rounds * k
            assert st.committed == st.applied == st.last_index
            assert st.sm_index == st.last_index
            assert st.kv_count == rounds * k
            assert c.export_kv(g, s) == kv[g]


def test_commit_pipeline_latency():
    """Leader commits round t's write in round t+2 (R=3)."""
    c, outs = run(8, 3, 1, drain=4)
    assert [o.committed_entries for o in outs] == [0, 0, 8, 0, 0]


def test_read_index_released_at_leader():
    G = 8
    c = po.Cluster(G, 3, seed=SEED)
    c.setup_steady(0)
    lo, hi = workload.build_read_index(G, SEED, 0, 30)
    c.stage_read_index(lo, hi)
    # round 0: queued + Heartbeat{Hint=ctx}; round 1: HeartbeatResp echoes
    # it; round 2: quorum confirms and the leader releases it
    outs = [c.round(tick=False) for _ in range(3)]
    assert [o.ready_to_reads for o in outs] == [0, 0, G]
    for g in range(G):
        rtr = c.export_ready(g, 0)
        assert rtr == [(4, lo[g], hi[g])]  # committed index at arrival


def test_deterministic():
    a, oa = run(8, 3, 5, reads=True)
    b, ob = run(8, 3, 5, reads=True)
    assert [o.to_dict() for o in oa] == [o.to_dict() for o in ob]
    for g in range(8):
        for s in range(3):
            assert a.export(g, s).to_dict(3) == b.export(g, s).to_dict(3)


def test_workload_definition():
    """Encoded NoOP-session entry, Cmd = 00 || PBKV{k8, v}."""
    p = workload.proposal(SEED, 7, 3, 0, 256, 4)
    assert p["type"] == abi.ENTRY_ENCODED
    assert p["key"] & 1 and p["client_id"] & 1
    assert p["client_id"] == workload.client_id(SEED, 7)
    cmd = p["cmd"]
    assert len(cmd) == 17 and cmd[0] == 0
    assert cmd[1:3] == b"\x0a\x08" and cmd[11:13] == b"\x12\x04"
    key, val = po.pbkv_unmarshal(cmd[1:])
    assert struct.unpack("<Q", key)[0] < 256 and len(val) == 4
    assert po.pbkv_marshal(key, val) == cmd[1:]
    lo, hi = workload.read_index_ctx(SEED, 7, 3, 33)
    assert lo & 1 and hi == 33
    # splitmix64 reference value (Steele et al.; seed 0 -> first output)
    assert workload.mix64(0) == 0xE220A8397B1DCDAF


def test_oracle_saved_entrybatch_decodes_to_the_round_entries():
    """The oracle's SaveRaftState output (EntryBatch of EntriesToSave +
    CRC32) decodes back to entries with contiguous indexes at the leader's
    term, and the CRC is zlib's crc32 (Go crc32.ChecksumIEEE)."""
    import zlib
    from dragonboat_amd import workload
    c = po.Cluster(6, 3, seed=7)
    c.setup_steady(0)
    seen = 0
    for r in range(5):
        counts, ents, pool = workload.build_batch(6, 2, 7, r)
        c.stage_proposals(counts, 2, ents, pool)
        c.round(tick=(r % 2 == 0))
        for g in range(6):
            for s in range(3):
                b, crc = c.export_saved(g, s)
                if not b:
                    continue
                assert crc == zlib.crc32(b)
                es = po.entrybatch_unmarshal(b)
                idx = [e["index"] for e in es]
                assert idx == list(range(idx[0], idx[0] + len(idx)))
                assert all(e["term"] == 2 for e in es)
                assert po.entrybatch_marshal(es) == b
                seen += 1
    assert seen >= 6 * 3 * 3


# ---- Quiesce at the node level (node_test.go:858-1000) -----------------
def _quiesced(c):
    return [c.export(g, s).qs_quiesced_since > 0
            for g in range(c.G) for s in range(c.R)]


def _idle(c, n):
    for _ in range(n):
        c.round(tick=True)


def test_quiesce_can_be_disabled():
    """TestRaftNodeQuiesceCanBeDisabled (node_test.go:858-882)."""
    c = po.Cluster(2, 3, quiesce=False)
    c.setup_steady(0)
    _idle(c, 2 * 200 + 1)
    assert not any(_quiesced(c))


def test_nodes_can_enter_quiesce():
    """TestNodesCanEnterQuiesce (node_test.go:884-905): threshold() =
    20 x ElectionRTT idle ticks, then every replica stays quiesced."""
    c = po.Cluster(2, 3, quiesce=True)
    c.setup_steady(0)
    _idle(c, 2 * 200 + 1)
    assert all(_quiesced(c))
    _idle(c, 3 * 200 + 1)
    assert all(_quiesced(c))
    # quiesced ticks: no heartbeats, no LocalTick-driven messages
    o = c.round(tick=True)
    assert o.messages == 0


def test_nodes_exit_quiesce_by_proposal_and_read_index():
    """TestNodesCanExitQuiesceByMakingProposal / ...ByReadIndex
    (node_test.go:907-972)."""
    for how in ("propose", "read"):
        c = po.Cluster(2, 3, quiesce=True)
        c.setup_steady(0)
        _idle(c, 2 * 200 + 1)
        assert all(_quiesced(c))
        if how == "propose":
            counts, ents, pool = workload.build_batch(2, 1, 7, 1)
            c.stage_proposals(counts, 1, ents, pool)
        else:
            lo, hi = workload.build_read_index(2, 7, 1, 31)
            c.stage_read_index(lo, hi)
        for _ in range(4):
            c.round(tick=True)
        assert not any(_quiesced(c)), how


def test_sampled_cluster_matches_full_cluster():
    """A cluster simulating only some global group ids (the full-size
    parity tests' oracle) steps those groups exactly like a cluster of
    all the groups does: groups are independent."""
    G, gids, seed = 40, [0, 3, 17, 39], 0x5EEDD8B0
    full = po.Cluster(G, 3, seed=seed)
    samp = po.Cluster(len(gids), 3, seed=seed, gids=gids)
    full.setup_steady(0)
    samp.setup_steady(0)
    for r in range(12):
        for c, n, kw in ((full, G, {}), (samp, len(gids), {"gids": gids})):
            counts, ents, pool = workload.build_batch(n, 1, seed, r, **kw)
            c.stage_proposals(counts, 1, ents, pool)
            if r % 3 == 1:
                lo, hi = workload.build_read_index(n, seed, r, r + 30, **kw)
                c.stage_read_index(lo, hi)
            c.round(tick=(r % 2 == 0))
        for i, g in enumerate(gids):
            for s in range(3):
                a, b = full.export(g, s), samp.export(i, s)
                assert a.to_dict(3) == b.to_dict(3), (r, g, s)
                assert full.export_outbox(g, s) == samp.export_outbox(i, s)
                assert full.export_kv(g, s) == samp.export_kv(i, s)


# ------------------------------------------------ divergent logs (import)
@pytest.mark.parametrize("case", range(6))
def test_leader_sync_follower_log_in_cluster(case):
    """LeaderSyncFollowerLog (raft_etcd_paper_test.go:690-770) through the
    cluster's step loop: the states are imported (orc_cluster_import, the
    oracle side of drb_import_replicas / drb_import_log), the leader-to-be
    times out, the hole's vote is ingested, and after the rounds the
    follower's log equals the leader's -- LEAD_ENTS plus the term-9 no-op
    -- with every entry committed and applied on both."""
    from tests import scenarios as sc
    c = po.Cluster(1, 3, seed=SEED, election_rtt=10)
    c.setup_steady(0)
    reps = sc.sync_follower_group(lambda s: c.export(0, s),
                                  sc.SYNC_CASES[case])
    for s, (st, log) in enumerate(reps):
        c.import_replica(0, s, st, log)
        assert c.export(0, s).last_index == len(log)
    c.round(tick=True)
    assert (c.export(0, 0).role, c.export(0, 0).term) == \
        (abi.CANDIDATE, sc.LEAD_TERM + 1)
    c.ingest([sc.vote_from_hole(c.export(0, 0).shard_id)])
    for _ in range(30):  # the probe walks back one index a Replicate
        c.round(tick=True)
    lead, fol = c.export(0, 0), c.export(0, 1)
    assert lead.role == abi.LEADER and fol.role == abi.FOLLOWER
    assert lead.last_index == fol.last_index == len(sc.LEAD_ENTS) + 1
    assert lead.committed == fol.committed == lead.last_index
    assert fol.sm_index == fol.committed
    want = [(e["term"], i + 1) for i, e in enumerate(sc.LEAD_ENTS)] + \
        [(sc.LEAD_TERM + 1, len(sc.LEAD_ENTS) + 1)]
    for s in (0, 1):
        got = [(e[0], e[1]) for e in c.export_log(0, s, 1, lead.last_index)]
        assert got == want, (s, got)
