"""The oracle's tan LogDB write path (oracle/tan_oracle.c) pinned by the
reference's own record tests (internal/tan/record_test.go), its Update
round-trip cases (raftpb/update_test.go:23-45) and the python xxhash
package for XXH64 (cespare/xxhash/v2 v2.1.2 is not in the reference tree;
tan's getCRC is the low 32 bits of its Sum64, internal/tan/crc.go:21-23).
"""
import random
import struct

import numpy as np
import pytest
import xxhash

from oracle import pyoracle as po

B = 32768  # blockSize (record.go:128)
HDR = 7    # legacyHeaderSize (record.go:130)


# ---------------------------------------------------------------- XXH64
def test_xxh64_matches_xxhash_package():
    rng = random.Random(7)
    for n in list(range(0, 130)) + [255, 256, 1000, 4096, 32761, 40000]:
        data = bytes(rng.getrandbits(8) for _ in range(n))
        assert po.xxh64(data) == xxhash.xxh64_intdigest(data), n
    # the published XXH64 check values (seed 0)
    assert po.xxh64(b"") == 0xEF46DB3751D8E999
    assert po.xxh64(b"a") == xxhash.xxh64_intdigest(b"a")


# ---------------------------------------------------------------- writer
def _records(lengths):
    """makeTestRecords (record_test.go:292-336): record i repeats byte i."""
    return [bytes([i & 0xFF]) * n for i, n in enumerate(lengths)]


def _write(recs):
    w = po.TanWriter()
    offs = []
    for r in recs:
        w.write_record(r)
        offs.append(w.last_record_offset())
    w.close()
    return w.bytes(), offs


def test_last_record_offset():
    # TestLastRecordOffset (record_test.go:744-767)
    recs = _records([B * 3, 3 * (B - HDR) - 2 * B - 2 * HDR, B - HDR, B - HDR,
                     B // 2])
    _, offs = _write(recs)
    assert offs == [0, 98332, 131072, 163840, 196608]


def test_no_last_record_offset():
    # TestNoLastRecordOffset (record_test.go:769-794)
    w = po.TanWriter()
    assert w.last_record_offset() == -1
    w.flush()
    assert w.last_record_offset() == -1
    w.write_record(b"testrecord")
    assert w.last_record_offset() == 0


def test_reader_offset():
    # TestReaderOffset (record_test.go:623-652)
    recs = _records([B * 2, 400, 500, 600, 700, 800, 9000, 1000])
    data, offs = _write(recs)
    got = po.tan_read(data)
    assert [o for o, _ in got] == offs
    assert [p for _, p in got] == recs


def _roundtrip(recs):
    data, _ = _write(recs)
    got = po.tan_read(data)
    assert [p for _, p in got] == list(recs)
    return data


def test_basic():
    # TestBasic (record_test.go:140-146)
    _roundtrip([b"a" * 1000, b"b" * 97270, b"c" * 8000])


def test_many():
    # TestMany (record_test.go:105-119)
    _roundtrip([b"%d." % i for i in range(100000)])


def test_random_lengths():
    # TestRandom (record_test.go:121-138): 100 records of up to 2 blocks +
    # 16 bytes.  Go's math/rand stream is not reproduced; numpy draws the
    # same shape of lengths.
    rng = np.random.default_rng(0)
    recs = [bytes([(i + 1) & 0xFF]) * int(rng.integers(0, 2 * B + 16))
            for i in range(100)]
    _roundtrip(recs)


def _big(partial, n):
    return (partial * (n // len(partial) + 1))[:n]


def test_boundary():
    # TestBoundary (record_test.go:148-158), every 4th length each way
    for i in range(B - 16, B + 16, 4):
        s0 = _big(b"abcd", i)
        for j in range(B - 16, B + 16, 4):
            s1 = _big(b"ABCDE", j)
            _roundtrip([s0, s1])
            _roundtrip([s0, b"", s1])
            _roundtrip([s0, b"x", s1])


def test_size():
    # TestSize (record_test.go:796-810)
    w = po.TanWriter()
    rng = random.Random(3)
    for _ in range(100):
        w.write_record(bytes(rng.randrange(8 << 10)))
        w.flush()
        assert len(w.bytes()) == w.size()


def test_chunk_layout_and_padding():
    """fillHeader (record.go:468-487): CRC = low 32 bits of XXH64 over the
    type byte and payload, little-endian length, FULL/FIRST/MIDDLE/LAST
    types; a header that does not fit in a block leaves zero padding."""
    data, _ = _write([b"\x11" * (B - HDR - 3), b"\x22" * 10])
    # record 0 fills the block up to 3 bytes: record 1 starts a new block
    assert data[B - 3:B] == b"\0\0\0"
    crc, ln, typ = struct.unpack_from("<IHB", data, 0)
    assert (ln, typ) == (B - HDR - 3, 1)
    assert crc == xxhash.xxh64_intdigest(data[6:HDR + ln]) & 0xFFFFFFFF
    crc, ln, typ = struct.unpack_from("<IHB", data, B)
    assert (ln, typ) == (10, 1)
    # a record spanning three blocks: FIRST, MIDDLE, LAST
    data, _ = _write([b"\x33" * (2 * B)])
    assert [data[6], data[B + 6], data[2 * B + 6]] == [2, 3, 4]
    # corrupting a checksum is detected (record.go:260-266)
    bad = bytearray(data)
    bad[0] ^= 1
    with pytest.raises(po.OracleError):
        po.tan_read(bytes(bad))


# ---------------------------------------------------------------- Update
def _uvarint(b, i):
    x = s = 0
    while True:
        c = b[i]
        i += 1
        x |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return x, i


def _decode_update(b):
    """Update.Unmarshal (raftpb/update.go:183-229), independent of the
    oracle; the Entries through the oracle's colfer decoder (pinned by the
    reference WAL fixture, test_oracle_codec.py)."""
    shard, i = _uvarint(b, 0)
    replica, i = _uvarint(b, i)
    state = None
    if b[i] == 1:
        (n,) = struct.unpack_from("<I", b, i + 1)
        st = b[i + 5:i + 5 + n]
        vals, j = [], 0
        for tag in (0x08, 0x10, 0x18):
            assert st[j] == tag
            v, j = _uvarint(st, j + 1)
            vals.append(v)
        assert j == n
        state = tuple(vals)
        i += 5 + n
    else:
        i += 1
    (cnt,) = struct.unpack_from("<I", b, i)
    i += 4
    ents = []
    for _ in range(cnt):
        (n,) = struct.unpack_from("<I", b, i)
        e, used = po.entry_unmarshal(b[i + 4:i + 4 + n])
        assert used == n
        ents.append(e)
        i += 4 + n
    assert b[i] == 0  # empty Snapshot
    assert i + 1 == len(b)
    return shard, replica, state, ents


def test_update_marshal_roundtrip():
    # TestUpdateMarshalAndUnmarshal (raftpb/update_test.go:23-45), the
    # cases without a Snapshot (snapshots are not on the GPU path)
    cases = [
        (0, 0, None, [po.ent(index=100, term=200, cmd=b"test-data"),
                      po.ent(index=200, term=300)]),
        (0, 0, (100, 200, 300), []),
        (7, 3, (1 << 40, 2, 1 << 63), [po.ent(index=5, term=9, key=1 << 60,
                                              client_id=77, type=1,
                                              cmd=bytes(range(200)))]),
    ]
    for shard, replica, state, ents in cases:
        b = po.update_marshal(shard, replica, state, ents)
        s2, r2, st2, e2 = _decode_update(b)
        assert (s2, r2, st2) == (shard, replica, state)
        assert len(e2) == len(ents)
        for a, e in zip(e2, ents):
            for k, v in e.items():
                assert a[k] == v, (k, a, e)
    # exact bytes of the state-only case
    assert po.update_marshal(1, 2, (3, 4, 5), []) == bytes(
        [1, 2, 1, 6, 0, 0, 0, 0x08, 3, 0x10, 4, 0x18, 5, 0, 0, 0, 0, 0])


# ---------------------------------------------------------------- db.write
def test_db_write_rules():
    """db.write (internal/tan/db.go:97-130): an Update whose State equals
    the stored one and that saves nothing is not written; sync on entries
    or a term / vote change; the stored state becomes the Update's own,
    empty included."""
    db = po.TanDB()
    e = [po.ent(term=2, index=5, cmd=b"\0abc")]
    assert db.write(1, 1, None, []) is None           # empty == empty
    w = db.write(1, 1, (2, 1, 4), [])                 # first state
    assert w["sync"] and w["off"] == 0 and w["len"] > 0
    w = db.write(1, 1, (2, 1, 5), [])                 # commit only
    assert not w["sync"]
    w = db.write(1, 1, (2, 1, 5), e)                  # entries
    assert w["sync"]
    # an Update without State after a stored state: written, and the
    # state sync compares Term 0 with 2 (stateSyncChange)
    w = db.write(1, 1, None, [])
    assert w is not None and w["sync"]
    assert db.write(1, 1, None, []) is None           # stored empty now
    w = db.write(1, 1, (3, 0, 5), [])
    assert w["sync"]
    recs = po.tan_read(db.file(0))
    assert len(recs) == 5
    assert recs[-1][1] == po.update_marshal(1, 1, (3, 0, 5), [])
    # appended bytes are exactly the file's tail
    f = db.file(0)
    assert f[w["off"]:w["off"] + w["len"]] == f[-w["len"]:]
    assert w["offset"] == len(f)


def test_db_switches_log_at_max_size():
    """makeRoomForWrite (db.go:175-180): once the offset reaches
    MaxLogFileSize the next write goes to a new log at offset 0."""
    db = po.TanDB(max_log_size=4096)
    cmd = bytes(1000)
    logs, prev = [], 0
    for i in range(12):
        w = db.write(9, 2, (2, 1, i + 1), [po.ent(term=2, index=i + 1,
                                                   cmd=cmd)])
        assert w["new_log"] == (prev >= 4096)
        assert (w["off"] == 0) == (i == 0 or w["new_log"])
        logs.append(w["log"])
        prev = w["offset"]
    # ~1.04 KB records: four fit below 4096, the fifth starts a new log
    assert logs == [0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2]
    for lg in range(3):
        recs = po.tan_read(db.file(lg))
        assert len(recs) == logs.count(lg)


def test_multiplexed_db_keeps_state_per_node():
    """A multiplexed log (db_keeper.go:84-123) holds the records of many
    shards; db.write's skip and sync (db.go:108-114) use each node's own
    stored State (nodeStates.getState(ShardID, ReplicaID)): the same State
    from another shard is still written and synced, a repeat from the same
    node is skipped."""
    db = po.TanDB()
    a = db.write(1, 1, (2, 1, 5), [])
    assert a and a["sync"] and a["off"] == 0
    b = db.write(17, 1, (2, 1, 5), [])  # same key 1, another shard
    assert b and b["sync"] and b["off"] == a["off"] + a["len"]
    assert db.write(1, 1, (2, 1, 5), []) is None
    c = db.write(17, 1, (2, 1, 6), [])  # commit only: written, no sync
    assert c and not c["sync"]
    recs = po.tan_read(db.file(0))
    assert [r[0] for r in recs] == [0, a["len"], a["len"] + b["len"]]
