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
