"""raftpb codec parity pinned by the reference's own byte-level fixture.

tests/golden/v2_rocksdb_wal_puts.json holds the Put values of the RocksDB
WAL shipped with the reference (internal/logdb/testdata/
v2-rocksdb-batched.tar.bz2, logdb-2/000003.log; extraction script
tests/golden/extract_rocksdb_wal.py).  Those values are EntryBatch records
written by dragonboat itself (internal/logdb/batch.go), so decoding and
re-encoding them must be byte-identical (raftpb/raft_optimized.go,
raftpb/entrybatch.go).  CRC32-IEEE is pinned by the standard check value
and zlib.crc32 (the same polynomial as Go's crc32.ChecksumIEEE).
"""
import json
import os
import random
import zlib

import pytest

from oracle import pyoracle as po
from oracle.pyoracle import ent

GOLD = os.path.join(os.path.dirname(__file__), "golden",
                    "v2_rocksdb_wal_puts.json")


def _batches():
    with open(GOLD) as f:
        puts = json.load(f)["puts"]
    # keys with prefix 0x0707 are entry-batch records (internal/logdb/keys.go)
    return [bytes.fromhex(p["value"]) for p in puts
            if p["key"].startswith("0707")]


def test_golden_batches_present():
    bs = _batches()
    assert len(bs) == 3
    assert len(bs[0]) == 36 and bs[0][:2] == b"\x0a\x22"


def test_golden_entrybatch_decode_values():
    last = _batches()[-1]
    ents = po.entrybatch_unmarshal(last)
    assert [(e["term"], e["index"], e["type"]) for e in ents] == \
        [(1, 1, 1), (2, 2, 0), (2, 3, 0)]
    # bootstrap ConfigChange{AddNode, ReplicaID 1, "localhost:26000",
    # Initialize} (peer.go:404-428, configchange.go:28-56)
    assert ents[0]["cmd"] == bytes.fromhex("0800100018012" "20f") + \
        b"localhost:26000" + b"\x28\x01"
    # leader no-op (raft.go:1049)
    assert ents[1]["cmd"] == b"" and ents[1]["client_id"] == 0
    # a NoOP-session proposal with 64-bit random Key / ClientID encoded in
    # the 0x80-tagged big-endian form (raft_optimized.go:166-186)
    assert ents[2]["key"] == 0x51141BD43FED56D4
    assert ents[2]["client_id"] == 0x2E83CD4D80F8CC7B
    assert ents[2]["series_id"] == 0 and ents[2]["cmd"] == bytes(128)


@pytest.mark.parametrize("i", range(3))
def test_golden_entrybatch_roundtrip_bytes(i):
    raw = _batches()[i]
    ents = po.entrybatch_unmarshal(raw)
    assert po.entrybatch_marshal(ents) == raw


def test_configchange_marshal_matches_golden():
    import ctypes as C
    buf = (C.c_uint8 * 64)()
    n = po.lib().orc_configchange_marshal_addnode(1, b"localhost:26000", buf)
    ents = po.entrybatch_unmarshal(_batches()[0])
    assert bytes(buf[:n]) == ents[0]["cmd"]


def test_entry_size_matches_marshal_random():
    rng = random.Random(11)
    for _ in range(500):
        def rv():
            return rng.choice([0, 1, 127, 128, (1 << 49) - 1, 1 << 49,
                               rng.getrandbits(64), rng.getrandbits(20)])
        e = ent(term=rv(), index=rv(), type=rng.choice([0, 1, 2, 3, 200]),
                key=rv(), client_id=rv(), series_id=rv(), responded_to=rv(),
                cmd=bytes(rng.getrandbits(8) for _ in range(
                    rng.choice([0, 1, 17, 127, 128, 300]))))
        b = po.entry_marshal(e)
        assert len(b) == po.entry_size(e)
        d, n = po.entry_unmarshal(b)
        assert n == len(b)
        assert d == e


def test_entry_unmarshal_rejects_truncation():
    b = po.entry_marshal(ent(term=5, index=9, key=1 << 60, cmd=b"abc"))
    for cut in range(1, len(b)):
        with pytest.raises(ValueError):
            po.entry_unmarshal(b[:cut])


def test_crc32_check_value():
    assert po.crc32_ieee(b"123456789") == 0xCBF43926
    assert po.crc32_ieee(b"") == 0


def test_crc32_matches_zlib():
    rng = random.Random(5)
    for n in (1, 3, 16, 17, 63, 64, 65, 1000, 4096):
        d = bytes(rng.getrandbits(8) for _ in range(n))
        assert po.crc32_ieee(d) == zlib.crc32(d)
    for raw in _batches():
        assert po.crc32_ieee(raw) == zlib.crc32(raw)


def test_pbkv_16_byte_layout():
    # internal/tests/kvpb/kv.go:26-40 -- the SURVEY 8d 16 B command
    key, val = b"K" * 8, b"v" * 4
    b = po.pbkv_marshal(key, val)
    assert b == b"\x0a\x08" + key + b"\x12\x04" + val
    assert len(b) == 16
    assert po.pbkv_unmarshal(b) == (key, val)


def test_pbkv_last_field_wins_and_skips_unknown():
    b = (b"\x0a\x01a\x12\x01b" + b"\x18\x05" + b"\x0a\x02cc")
    assert po.pbkv_unmarshal(b) == (b"cc", b"b")
