"""Extract the reference's own byte-level LogDB fixture.

Source (data file shipped with the reference, read only as data):
  /root/reference/internal/logdb/testdata/v2-rocksdb-batched.tar.bz2
  member .../logdb-2/000003.log  (a RocksDB WAL, 675 bytes)

It is used by the reference test TestV2DataCanBeHandled
(nodehost_test.go:4674-4720).  The WAL holds raw raftpb.EntryBatch / Entry
values written by dragonboat's batched LogDB (internal/logdb/batch.go), so
its Put values pin the Entry colfer codec (raft_optimized.go:84-656) and the
EntryBatch codec (entrybatch.go:25-146) byte for byte.

Run once in the build container (the GPU box has no /root/reference):
  python tests/golden/extract_rocksdb_wal.py
writes tests/golden/v2_rocksdb_logdb2_000003.log and
tests/golden/v2_rocksdb_wal_puts.json (key/value hex of every Put).
"""
import json
import os
import struct
import tarfile

SRC = "/root/reference/internal/logdb/testdata/v2-rocksdb-batched.tar.bz2"
MEMBER_SUFFIX = "logdb-2/000003.log"
HERE = os.path.dirname(os.path.abspath(__file__))


def _varint(buf, i):
    shift = 0
    v = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if b < 0x80:
            return v, i
        shift += 7


def wal_records(raw):
    """RocksDB log format: 32 KiB blocks of {crc32c u32, len u16, type u8}."""
    out = []
    pending = b""
    block = 32768
    pos = 0
    while pos + 7 <= len(raw):
        left = block - (pos % block)
        if left < 7:
            pos += left
            continue
        _crc, ln, typ = struct.unpack_from("<IHB", raw, pos)
        data = raw[pos + 7 : pos + 7 + ln]
        pos += 7 + ln
        if typ == 0 and ln == 0:
            continue
        if typ == 1:  # FULL
            out.append(data)
        elif typ == 2:  # FIRST
            pending = data
        elif typ == 3:  # MIDDLE
            pending += data
        elif typ == 4:  # LAST
            out.append(pending + data)
            pending = b""
    return out


def write_batch_puts(rec):
    """WriteBatch: seq u64, count u32, then tagged records."""
    _seq, count = struct.unpack_from("<QI", rec, 0)
    i = 12
    puts = []
    for _ in range(count):
        tag = rec[i]
        i += 1
        if tag == 0x1:  # kTypeValue
            kl, i = _varint(rec, i)
            key = rec[i : i + kl]
            i += kl
            vl, i = _varint(rec, i)
            val = rec[i : i + vl]
            i += vl
            puts.append((key, val))
        elif tag == 0x0:  # kTypeDeletion
            kl, i = _varint(rec, i)
            i += kl
        else:
            raise ValueError("unsupported WriteBatch tag %d" % tag)
    return puts


def main():
    with tarfile.open(SRC) as t:
        m = [x for x in t.getmembers() if x.name.endswith(MEMBER_SUFFIX)][0]
        raw = t.extractfile(m).read()
    with open(os.path.join(HERE, "v2_rocksdb_logdb2_000003.log"), "wb") as f:
        f.write(raw)
    puts = []
    for rec in wal_records(raw):
        for k, v in write_batch_puts(rec):
            puts.append({"key": k.hex(), "value": v.hex()})
    with open(os.path.join(HERE, "v2_rocksdb_wal_puts.json"), "w") as f:
        json.dump({"source": SRC + "::" + m.name, "puts": puts}, f, indent=1)
    print("%d bytes, %d puts" % (len(raw), len(puts)))


if __name__ == "__main__":
    main()
