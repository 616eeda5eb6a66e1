"""GPU wire path (drb_encode_wire) against the oracle, byte for byte.

For each (sender slot, receiver slot) plane the engine encodes the last
round's messages of every group as the TCP stream dragonboat's transport
writes to the NodeHost hosting the receivers (framed MessageBatches,
transport.go:443-508, tcp.go:142-178).  The expected stream is built from
the ORACLE cluster's outboxes (tests/wire_ref.py), so the check covers the
messages themselves, the Message / colfer Entry encoding, the batch cut
and both CRCs.
"""
import pytest

from oracle import pyoracle as po
from tests import wire_ref as wr
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu

SRC = b"gpu-node-7.example:26001"


def _check_planes(p, did, limits, planes=None):
    planes = planes or [(a, b) for a in range(p.R) for b in range(p.R)
                        if a != b]
    for frm, to in planes:
        msgs = wr.plane_messages(p.orc.export_outbox, p.G, frm, to)
        for lim in limits:
            res, data = p.eng.encode_wire(frm, to, did, SRC, max_batch=lim)
            exp = wr.expected_stream(msgs, did, SRC,
                                     lim or wr.MAX_MSG_BATCH)
            assert res["n_msgs"] == len(msgs), (frm, to, lim)
            assert res["n_bytes"] == len(exp), (frm, to, lim)
            if data != exp:
                i = next(k for k in range(min(len(data), len(exp)))
                         if data[k] != exp[k])
                raise AssertionError((frm, to, lim, "first diff at", i,
                                      data[max(0, i - 8):i + 8].hex(),
                                      exp[max(0, i - 8):i + 8].hex()))
            assert res["n_frames"] == len(
                wr.split_batches(msgs, lim or wr.MAX_MSG_BATCH))


def test_wire_before_any_round_is_empty():
    p = Pair(G=8, R=3)
    res, data = p.eng.encode_wire(0, 1, 1, SRC)
    assert res == {"n_msgs": 0, "n_frames": 0, "n_bytes": 0} and data == b""


def test_wire_write_rounds_r3():
    """Replicate / ReplicateResp / Heartbeat(+Resp) / ReadIndex planes at
    the default 64 MiB cut and at cuts that force every batch shape."""
    p = Pair(G=40, R=3)
    for r in range(6):
        k = 1 if r % 3 else 3
        o, e = p.round(k=k, tick=(r % 2 == 0), read_index=(r % 3 == 1))
        assert e.fallbacks == 0 and e.errors == 0
        _check_planes(p, did=0x1234567890 + r,
                      limits=[0, 1, 500, 2000] if r < 5 else [0])


def test_wire_r5_and_large_ids():
    """R=5, a 64-bit DeploymentId and 1-2 byte varint shard ids."""
    p = Pair(G=150, R=5)
    for r in range(3):
        p.round(k=2, tick=True, read_index=(r == 1))
        _check_planes(p, did=(1 << 63) + 5, limits=[0, 3000],
                      planes=[(0, 1), (0, 4), (3, 0)])


def test_wire_long_payloads():
    """C5 payloads: 116 / 1011-byte PBKV values in the Replicate entries."""
    for val_len, cmd_cap, val_cap in [(116, 144, 128), (1011, 1040, 1024)]:
        p = Pair(G=24, R=3, cmd_cap=cmd_cap, kv_val_cap=val_cap, kv_slots=64,
                 max_props=4)
        for r in range(3):
            p.round(k=1 + (r == 2), tick=(r % 2 == 0), val_len=val_len)
            _check_planes(p, did=9, limits=[0, 4096],
                          planes=[(0, 1), (2, 0)])


def test_wire_idle_and_ragged_groups():
    """Groups without messages leave no gap; an empty plane is empty."""
    p = Pair(G=64, R=3)
    p.round(k=1, tick=True)
    groups = [g for g in range(64) if g % 7 in (1, 4)]
    p.round(k=1, tick=False, groups=groups)
    _check_planes(p, did=3, limits=[0, 700])
    p.round(k=0, tick=False)   # nothing sent at all
    _check_planes(p, did=3, limits=[0])


def test_wire_large_plane_properties():
    """64k groups (C2 size): the stream parses, every frame's header and
    payload CRC verify with zlib, and the decoded messages equal the
    engine's own outboxes on sampled groups."""
    from dragonboat_amd.engine import Engine
    G = 65536
    eng = Engine(num_groups=G, num_replicas=3)
    eng.init_steady(term=2, leader_slot=0, seed=0x5EEDD8B0)
    for r in range(3):
        eng.gen_kv_proposals(0, 1, 256, 4, 0x5EEDD8B0, r)
        eng.step(tick=True, prop_slot=0)
    res, data = eng.encode_wire(0, 1, 42, SRC, max_batch=4 << 20)
    assert res["n_frames"] > 1 and res["n_bytes"] == len(data)
    msgs = []
    for pl in wr.parse_stream(data):
        ms, did, src, bv = po.messagebatch_unmarshal(pl, cap=1 << 17)
        assert (did, src, bv) == (42, SRC, 210)
        msgs += ms
    assert len(msgs) == res["n_msgs"]
    by_shard = {}
    for m in msgs:
        by_shard.setdefault(m["shard_id"], []).append(m)
    first = eng.cfg.get("first_shard_id", 1)
    for g in list(range(0, G, 4099)) + [G - 1]:
        exp = [wr.tuple_to_msg(t) for t in eng.export_outbox(g, 0)
               if t[2] == 2]
        assert by_shard.get(first + g, []) == exp, g


class TwoNodes:
    """Two engines as two NodeHosts joined by the wire path: `lead` hosts
    replica slot 0 (the leaders) of every group, `foll` hosts the other
    slots.  After each round every plane crosses as a TCP byte stream
    (drb_encode_wire -> drb_ingest_wire); one oracle cluster with every
    replica co-resident is the reference."""

    def __init__(self, G, R=3, seed=0x5EEDD8B0, did=0xD1D, by_slot=False):
        from dragonboat_amd import abi
        from dragonboat_amd.engine import Engine
        self.G, self.R, self.seed, self.did = G, R, seed, did
        self.orc = po.Cluster(G, R, seed=seed)
        self.orc.setup_steady(0)
        self.lead = Engine(num_groups=G, num_replicas=R)
        self.foll = Engine(num_groups=G, num_replicas=R)
        for eng, mine in ((self.lead, {0}), (self.foll, set(range(1, R)))):
            eng.init_steady(term=2, leader_slot=0, seed=seed)
            if by_slot:  # drb_host_slot: one call per slot, no round trip
                for s in range(R):
                    if s not in mine:
                        eng.host_slot(s, False)
                continue
            sts = eng.export_replicas(0, G)
            for i in range(len(sts)):
                if i % R not in mine:
                    sts[i].flags &= ~abi.F_HOSTED
            eng.import_replicas(0, sts)
        self.rounds = 0
        self.wire_bytes = 0

    def round(self, k=1, tick=False, read_index=False):
        from dragonboat_amd import abi, workload
        pin = ri_in = abi.DRB_NONE
        if k:
            counts, ents, pool = workload.build_batch(
                self.G, k, self.seed, self.rounds, 256, 4, None)
            self.orc.stage_proposals(counts, k, ents, pool)
            mp = self.lead.cfg["max_props"]
            eents = (abi.Entry * (self.G * mp))()
            for g in range(self.G):
                for j in range(counts[g]):
                    eents[g * mp + j] = ents[g * k + j]
            self.lead.stage_proposals(0, counts, eents, pool)
            pin = 0
        if read_index:
            lo, hi = workload.build_read_index(self.G, self.seed, self.rounds,
                                               self.rounds + 30, None)
            self.orc.stage_read_index(lo, hi)
            self.lead.stage_read_index(0, lo, hi)
            ri_in = 0
        o = self.orc.round(tick=tick)
        a = self.lead.step(tick=tick, prop_slot=pin, ri_slot=ri_in)
        b = self.foll.step(tick=tick)
        self.rounds += 1
        for s in range(1, self.R):
            self._cross(self.lead, self.foll, 0, s)
            self._cross(self.foll, self.lead, s, 0)
        return o, a, b

    def _cross(self, src, dst, frm, to):
        res, data = src.encode_wire(frm, to, self.did, SRC)
        self.wire_bytes += len(data)
        if self.rounds % 2:  # every other round through the pinned
            # receive buffer a transport reads its connection into
            ptr = dst.ingest_buffer(data)
            got = dst.ingest_wire_pinned(ptr, len(data), self.did)
        else:
            got = dst.ingest_wire(data, self.did)
        assert got["bad"] == 0 and got["consumed"] == len(data), got
        assert got["messages"] == res["n_msgs"] == got["accepted"], got

    def check(self):
        errs = []
        from tests.gpu_harness import by_dest, state_diff
        for g in range(self.G):
            for s in range(self.R):
                eng = self.lead if s == 0 else self.foll
                a, b = eng.export_replicas(g, 1)[s], self.orc.export(g, s)
                d = state_diff(a, b, self.R)
                if d:
                    errs.append((g, s, "state", d))
                    continue
                if eng.kv_export(g, s) != self.orc.export_kv(g, s):
                    errs.append((g, s, "kv"))
                em = by_dest(eng.export_outbox(g, s))
                om = by_dest(self.orc.export_outbox(g, s))
                if em != om:
                    errs.append((g, s, "msgs", em, om))
                if eng.export_ready(g, s) != self.orc.export_ready(g, s):
                    errs.append((g, s, "ready"))
        return errs


@pytest.mark.parametrize("R,by_slot", [(3, False), (5, False), (3, True)])
def test_two_nodehosts_over_the_wire(R, by_slot):
    """Leaders on one engine, followers on another, every message crossing
    as dragonboat TCP bytes: bit-exact with one co-resident oracle cluster
    (writes, ticks, ReadIndex).  by_slot: hosting set with drb_host_slot
    instead of an export/import of every replica record."""
    t = TwoNodes(G=32, R=R, by_slot=by_slot)
    for r in range(8):
        o, a, b = t.round(k=1 + (r % 3 == 2), tick=(r % 2 == 0),
                          read_index=(r % 3 == 1))
        for x in (a, b):
            assert x.fallbacks == 0 and x.errors == 0, (r, x.to_dict())
        assert a.committed_entries + b.committed_entries == \
            o.committed_entries, r
        errs = t.check()
        assert not errs, (r, errs[:2])
    assert t.wire_bytes > 0


def test_ingest_wire_filters_and_bad_frames():
    """transport.go:305-316: a batch of another deployment (or BinVer) is
    dropped whole; tcp.go:180-237: a corrupted frame stops the stream
    (ErrBadMessage), frames before it are delivered."""
    t = TwoNodes(G=16)
    t.round(k=1, tick=True)
    # the round's wire traffic was delivered by round(); make a fresh
    # stream of the same round and deliver it with the wrong deployment
    res, data = t.lead.encode_wire(0, 1, t.did + 1, SRC)
    got = t.foll.ingest_wire(data, t.did)
    assert got["accepted"] == 0 and got["dropped"] == res["n_msgs"] > 0
    # two frames (one message each, max_batch=1), the second corrupted
    res, data = t.lead.encode_wire(0, 1, t.did, SRC, max_batch=1)
    frames = wr.parse_stream(data)
    first = 20 + len(frames[0])
    bad = bytearray(data)
    bad[first + 25] ^= 0x40
    got = t.foll.ingest_wire(bytes(bad), t.did)
    assert got["bad"] == 1 and got["frames"] == 1
    assert got["consumed"] == first and got["messages"] == 1
    # a snapshot-chunk frame (method 200) is skipped, not fatal
    chunk = b"\xae\x7d" + po.request_header_encode(200, 3, wr.zlib.crc32(
        b"abc")) + b"abc"
    got = t.foll.ingest_wire(chunk + data[:first], t.did)
    assert got["bad"] == 0 and got["snapshots"] == 1 and got["frames"] == 2


@pytest.mark.parametrize("kind", ["witness", "nonvoting"])
def test_wire_planes_with_member_kinds(kind):
    """A 3 + 1 group: the leader's plane to a witness carries metadata
    entries (makeMetadataEntries, raft.go:771-785), the one to a nonVoting
    the entries whole; both byte for byte against the oracle's outbox."""
    p = Pair(G=32, R=4, **{kind + "_slots": 1 << 3})
    for r in range(4):
        o, e = p.round(k=1 + r % 2, tick=(r % 2 == 0), read_index=(r == 2))
        assert e.fallbacks == 0 and e.errors == 0
        _check_planes(p, did=77, limits=[0, 2000],
                      planes=[(0, 3), (3, 0), (0, 1)])


def test_ingest_wire_wide_steps_and_warm_reruns():
    """drb_ingest_wire's element steps go up as 2 B while every Requests
    element is under 64 KB, else as 4 B: a 70 KB Replicate in a frame of
    another deployment (dropped whole, transport.go:305-316) ahead of a
    round's stream.  Then warm calls whose per-piece speculation fails (a
    corrupted frame, tcp.go:180-237) and rounds after them: every replica
    bit-exact with the oracle cluster."""
    from dragonboat_amd import abi
    t = TwoNodes(G=16)
    t.round(k=1, tick=True)
    big = po.msg(abi.MSG["Replicate"], from_=1, to=2, term=2, log_index=1,
                 entries=[po.ent(term=2, index=2, cmd=b"\x5a" * 70000)],
                 shard_id=1)
    frame = po.wire_frame(po.messagebatch_marshal([big], t.did + 1, SRC))
    assert len(frame) > 70000
    cross = t._cross

    def cross_with_big(src, dst, frm, to):
        if frm != 0:
            return cross(src, dst, frm, to)
        res, data = src.encode_wire(frm, to, t.did, SRC)
        got = dst.ingest_wire(frame + data, t.did)
        assert got["bad"] == 0 and got["consumed"] == len(frame) + len(data)
        assert got["accepted"] == res["n_msgs"] == got["messages"], got
        assert got["dropped"] == 1, got

    t._cross = cross_with_big
    o, a, b = t.round(k=2, tick=False, read_index=True)
    t._cross = cross
    errs = t.check()
    assert not errs, errs[:2]
    # a corrupted first frame on the warm engine: the speculation does not
    # hold, nothing is delivered, and its pass leaves no trace
    res, data = t.lead.encode_wire(0, 1, t.did, SRC, max_batch=1)
    bad = bytearray(data)
    bad[25] ^= 0x40
    got = t.foll.ingest_wire(bytes(bad), t.did)
    assert got["bad"] == 1 and got["frames"] == 0 and got["messages"] == 0
    assert got["accepted"] == 0, got
    for r in range(3):
        t.round(k=1, tick=True, read_index=r == 1)
    errs = t.check()
    assert not errs, errs[:2]


def test_ingest_wire_first_call_without_a_whole_frame():
    """A fresh receiver's first drb_ingest_wire calls hold no whole frame:
    an empty stream, then a cut inside the first request header, then one
    inside the first payload (the call the round-4 crash came from: the
    upload pipeline's first event recorded before any piece existed,
    DESIGN §7a).  Nothing is consumed; the whole stream then goes in and
    the round after it stays bit-exact with the oracle cluster."""
    from dragonboat_amd import abi
    t = TwoNodes(G=16)
    hb = po.msg(abi.MSG["Heartbeat"], from_=1, to=2, term=2, shard_id=1)
    data = po.wire_frame(po.messagebatch_marshal([hb] * 4, t.did, SRC))
    assert len(data) > 40
    for cut in (0, 9, 40):
        got = t.foll.ingest_wire(data[:cut], t.did)
        assert got["consumed"] == 0 and got["messages"] == 0, (cut, got)
        assert got["bad"] == 0 and got["accepted"] == 0, (cut, got)
    o, a, b = t.round(k=1, tick=True)
    errs = t.check()
    assert not errs, errs[:2]
    got = t.foll.ingest_wire_pinned(t.foll.ingest_buffer(data[:30]), 30,
                                    t.did)
    assert got["consumed"] == 0 and got["messages"] == 0, got
