"""pb.Message / pb.MessageBatch wire codec and the TCP frame of the oracle.

Pinning: the reference ships no byte-level fixture for Message or
MessageBatch (its tests only round-trip, raftpb/raft_test.go:389-411), so
the oracle's gogo-proto encoder (raftpb/message.go:32-124,
messagebatch.go:23-70) is checked against an independent proto2 encoder:
google.protobuf with descriptors built here from the field numbers and
wire types of those MarshalTo functions.  gogo's non-nullable scalar fields
are always emitted, which is proto2 with every field explicitly set.
Entries are colfer bytes (raft_optimized.go:166-300, pinned by the golden
WAL fixture in test_oracle_codec.py), modelled as `repeated bytes` 11.
The TCP request header (tcp.go:64-112) is checked field by field with
struct/zlib.
"""
import random
import struct
import zlib

import pytest

from oracle import pyoracle as po
from oracle.pyoracle import ent, msg

pb = pytest.importorskip("google.protobuf")
from google.protobuf import descriptor_pb2, descriptor_pool  # noqa: E402
from google.protobuf import message_factory  # noqa: E402

U64 = descriptor_pb2.FieldDescriptorProto.TYPE_UINT64
U32 = descriptor_pb2.FieldDescriptorProto.TYPE_UINT32
BOOL = descriptor_pb2.FieldDescriptorProto.TYPE_BOOL
BYTES = descriptor_pb2.FieldDescriptorProto.TYPE_BYTES
STR = descriptor_pb2.FieldDescriptorProto.TYPE_STRING
MSG = descriptor_pb2.FieldDescriptorProto.TYPE_MESSAGE
OPT = descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL
REP = descriptor_pb2.FieldDescriptorProto.LABEL_REPEATED


def _classes():
    f = descriptor_pb2.FileDescriptorProto(name="drbwire.proto",
                                           package="w", syntax="proto2")

    def add(name, fields):
        m = f.message_type.add(name=name)
        for num, fname, typ, lab, tn in fields:
            fd = m.field.add(name=fname, number=num, type=typ, label=lab)
            if tn:
                fd.type_name = ".w." + tn

    # membership.go:29-148 (maps empty)
    add("Membership", [(1, "config_change_id", U64, OPT, None)])
    # snapshot.go:72-150 (Files empty, Checksum nil)
    add("Snapshot", [(2, "filepath", STR, OPT, None),
                     (3, "file_size", U64, OPT, None),
                     (4, "index", U64, OPT, None),
                     (5, "term", U64, OPT, None),
                     (6, "membership", MSG, OPT, "Membership"),
                     (9, "dummy", BOOL, OPT, None),
                     (10, "shard_id", U64, OPT, None),
                     (11, "type", U64, OPT, None),
                     (12, "imported", BOOL, OPT, None),
                     (13, "on_disk_index", U64, OPT, None),
                     (14, "witness", BOOL, OPT, None)])
    # message.go:32-90
    add("Message", [(1, "type", U64, OPT, None), (2, "to", U64, OPT, None),
                    (3, "from", U64, OPT, None),
                    (4, "shard_id", U64, OPT, None),
                    (5, "term", U64, OPT, None),
                    (6, "log_term", U64, OPT, None),
                    (7, "log_index", U64, OPT, None),
                    (8, "commit", U64, OPT, None),
                    (9, "reject", BOOL, OPT, None),
                    (10, "hint", U64, OPT, None),
                    (11, "entries", BYTES, REP, None),
                    (12, "snapshot", MSG, OPT, "Snapshot"),
                    (13, "hint_high", U64, OPT, None)])
    # messagebatch.go:23-51
    add("MessageBatch", [(1, "requests", MSG, REP, "Message"),
                         (2, "deployment_id", U64, OPT, None),
                         (3, "source_address", STR, OPT, None),
                         (4, "bin_ver", U32, OPT, None)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(f)
    get = message_factory.GetMessageClass
    return (get(pool.FindMessageTypeByName("w.Message")),
            get(pool.FindMessageTypeByName("w.MessageBatch")))


PMessage, PBatch = _classes()


def _fill(pm, m):
    pm.type = m["type"]
    setattr(pm, "to", m["to"])
    setattr(pm, "from", m["from_"])
    pm.shard_id = m["shard_id"]
    pm.term = m["term"]
    pm.log_term = m["log_term"]
    pm.log_index = m["log_index"]
    pm.commit = m["commit"]
    pm.reject = bool(m["reject"])
    pm.hint = m["hint"]
    for e in m["entries"]:
        pm.entries.append(po.entry_marshal(e))
    s = pm.snapshot
    s.filepath = ""
    s.file_size = s.index = s.term = 0
    s.membership.config_change_id = 0
    s.dummy = False
    s.shard_id = s.type = 0
    s.imported = False
    s.on_disk_index = 0
    s.witness = False
    pm.hint_high = m["hint_high"]
    return pm


def _independent_message(m):
    return _fill(PMessage(), m).SerializeToString()


def _independent_batch(msgs, did, src, bv):
    b = PBatch()
    for m in msgs:
        _fill(b.requests.add(), m)
    b.deployment_id = did
    b.source_address = src.decode()
    b.bin_ver = bv
    return b.SerializeToString()


def _rand_u64(rng):
    # spread over varint lengths 1..10
    return rng.getrandbits(rng.choice([0, 1, 7, 8, 14, 21, 35, 49, 56, 63,
                                       64]))


def _rand_entry(rng):
    return ent(term=_rand_u64(rng), index=_rand_u64(rng),
               type=rng.choice([0, 1, 2, 3]), key=_rand_u64(rng),
               client_id=_rand_u64(rng), series_id=_rand_u64(rng),
               responded_to=_rand_u64(rng),
               cmd=bytes(rng.getrandbits(8)
                         for _ in range(rng.choice([0, 1, 17, 200]))))


def _rand_msg(rng):
    return msg(rng.choice([12, 13, 17, 18, 19, 20, 1, 7]),
               from_=_rand_u64(rng), to=_rand_u64(rng),
               shard_id=_rand_u64(rng), term=_rand_u64(rng),
               log_term=_rand_u64(rng), log_index=_rand_u64(rng),
               commit=_rand_u64(rng), reject=rng.random() < 0.3,
               hint=_rand_u64(rng), hint_high=_rand_u64(rng),
               entries=[_rand_entry(rng)
                        for _ in range(rng.choice([0, 0, 1, 3]))])


def test_heartbeat_wire_size():
    """a Heartbeat without entries is ~52 B on the wire."""
    m = msg(17, from_=1, to=2, shard_id=1000, term=2, commit=100)
    b = po.message_marshal(m)
    assert b == _independent_message(m)
    assert len(b) == 49  # 10 one-byte varint fields + ShardID 1000 + 26 + 2
    # the empty Snapshot field is the fixed 26 bytes 0x62 0x18 <24 B>
    i = b.index(b"\x62\x18")
    assert b[i + 2:i + 26] == bytes.fromhex(
        "120018002000280032020800480050005800600068007000")


@pytest.mark.parametrize("seed", range(8))
def test_message_matches_independent_proto2(seed):
    rng = random.Random(seed)
    for _ in range(40):
        m = _rand_msg(rng)
        assert po.message_marshal(m) == _independent_message(m)


@pytest.mark.parametrize("seed", range(4))
def test_messagebatch_matches_independent_and_roundtrips(seed):
    rng = random.Random(100 + seed)
    msgs = [_rand_msg(rng) for _ in range(rng.choice([0, 1, 5, 30]))]
    did = _rand_u64(rng)
    src = b"10.0.0.%d:26000" % rng.randrange(256)
    b = po.messagebatch_marshal(msgs, did, src)
    assert b == _independent_batch(msgs, did, src, 210)
    got, gdid, gsrc, gbv = po.messagebatch_unmarshal(b)
    assert (gdid, gsrc, gbv) == (did, src, 210)
    assert got == msgs
    # byte-identical re-encode
    assert po.messagebatch_marshal(got, gdid, gsrc, gbv) == b


def test_messagebatch_unmarshal_rejects_truncation_and_snapshots():
    rng = random.Random(7)
    msgs = [_rand_msg(rng) for _ in range(4)]
    b = po.messagebatch_marshal(msgs, 5, b"a:1")
    for cut in (1, 7, len(b) // 2, len(b) - 1):
        with pytest.raises(ValueError):
            po.messagebatch_unmarshal(b[:cut] + b"\xff")
    # a Message carrying a non-empty Snapshot is off this path
    pm = _fill(PMessage(), msgs[0])
    pm.snapshot.index = 9
    pbb = PBatch()
    pbb.requests.append(pm)
    with pytest.raises(NotImplementedError):
        po.messagebatch_unmarshal(pbb.SerializeToString())


def test_request_header_and_frame():
    payload = po.messagebatch_marshal(
        [msg(17, from_=1, to=2, shard_id=3, term=2, commit=9)], 1, b"x:1")
    fr = po.wire_frame(payload)
    assert fr[:2] == b"\xae\x7d"
    h = fr[2:20]
    method, size = struct.unpack(">HQ", h[:10])
    (hcrc,) = struct.unpack(">I", h[10:14])
    (pcrc,) = struct.unpack(">I", h[14:18])
    assert (method, size) == (100, len(payload))
    assert pcrc == zlib.crc32(payload)
    assert hcrc == zlib.crc32(h[:10] + b"\0\0\0\0" + h[14:])
    assert fr[20:] == payload
    assert po.request_header_decode(h) == (100, len(payload), pcrc)
    bad = bytearray(h)
    bad[3] ^= 1
    assert po.request_header_decode(bytes(bad)) is None
    # snapshotType is accepted, anything else is not (tcp.go:101-104)
    assert po.request_header_decode(po.request_header_encode(200, 1, 2)) == \
        (200, 1, 2)
    assert po.request_header_decode(po.request_header_encode(7, 1, 2)) is None
