"""GPU parity of the tan LogDB records (save_tan, drb_tan.hpp; SURVEY 8f
F2): every round, every replica's record -- what db.write
(internal/tan/db.go:97-130) appends to that replica's log: the marshalled
pb.Update (raftpb/update.go:128-169) in 32 KiB-block chunks with XXH64
checksums (internal/tan/record.go:468-591, crc.go:21-23) -- equals, byte
for byte, what the oracle's tan restatement (oracle/tan_oracle.c, pinned in
tests/test_oracle_tan.py) writes for the oracle cluster's own Updates, with
the same offsets, sync decisions and log switches; and every log the GPU
builds reads back record by record through the record reader.
"""
import pytest

from dragonboat_amd import abi
from oracle import pyoracle as po
from tests.gpu_harness import Pair


def _check_round(p, dbs, logs, r):
    """Compare every replica's record of the round; append the GPU's bytes
    to its log images."""
    n = 0
    for g in range(p.G):
        for s in range(p.R):
            want = p.orc.tan_write(g, s, dbs[g][s])
            rec, data = p.eng.export_tan(g, s)
            where = (r, g, s, rec, want)
            if want is None:
                assert not rec["flags"] & abi.TAN_WRITTEN, where
                assert rec["len"] == 0, where
                continue
            assert rec["flags"] & abi.TAN_WRITTEN, where
            assert (rec["offset"], rec["len"], rec["log"]) == \
                (want["off"], want["len"], want["log"]), where
            assert bool(rec["flags"] & abi.TAN_SYNC) == want["sync"], where
            assert bool(rec["flags"] & abi.TAN_NEW_LOG) == want["new_log"], \
                where
            f = dbs[g][s].file(want["log"])
            assert data == f[want["off"]:want["off"] + want["len"]], where
            img = logs.setdefault((g, s, rec["log"]), bytearray())
            assert len(img) == rec["offset"], where
            img += data
            n += 1
    return n


def _read_back(logs, dbs):
    """Every GPU-built log is the oracle's file and reads back cleanly."""
    for (g, s, lg), img in logs.items():
        assert bytes(img) == dbs[g][s].file(lg), (g, s, lg)
        recs = po.tan_read(bytes(img))
        assert recs and recs[0][0] == 0


@pytest.mark.gpu
def test_tan_records_match_oracle():
    """16 B payloads, ragged proposals (0-3 a round), ticks, ReadIndex:
    Updates with entries, with a State only, and with neither (messages
    only: written once after a stored State, then skipped -- db.go:108-114),
    and a 1 KiB MaxLogFileSize so logs switch every dozen rounds."""
    p = Pair(G=12, R=3, save_cap=4096, max_props=4, save_tan=1,
             tan_max_log=1024)
    dbs = [[po.TanDB(1024) for _ in range(p.R)] for _ in range(p.G)]
    logs = {}
    written = 0
    for r in range(40):
        k = (0, 1, 3, 0, 2)[r % 5]
        o, e = p.round(k=k, tick=(r % 2 == 0), read_index=(r % 3 == 0),
                       encode_saves=True)
        assert e.fallbacks == 0 and e.errors == 0, (r, e.to_dict())
        n = _check_round(p, dbs, logs, r)
        assert e.log_records == n, (r, e.to_dict())
        written += n
    _read_back(logs, dbs)
    assert written > 0
    assert any(lg > 0 for (_, _, lg) in logs)  # logs switched
    st = p.eng.tan_get(0, 0)
    assert st[0] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("val_len,cmd_cap,val_cap", [(116, 144, 128),
                                                     (1011, 1040, 1024)])
def test_tan_records_long_payloads(val_len, cmd_cap, val_cap):
    """C5 payloads (128 B / 1 KB): records of several KB that cross 32 KiB
    blocks (FIRST / MIDDLE / LAST chunks, zero padding where a header does
    not fit), 64 KiB logs."""
    p = Pair(G=16, R=3, cmd_cap=cmd_cap, kv_val_cap=val_cap, kv_slots=64,
             max_props=4, save_cap=8192, save_tan=1, tan_max_log=1 << 16)
    dbs = [[po.TanDB(1 << 16) for _ in range(p.R)] for _ in range(p.G)]
    logs = {}
    for r in range(24):
        o, e = p.round(k=(1, 4, 2)[r % 3], tick=(r % 3 == 0),
                       encode_saves=True, val_len=val_len)
        assert e.fallbacks == 0 and e.errors == 0, (r, e.to_dict())
        _check_round(p, dbs, logs, r)
    _read_back(logs, dbs)
    if val_len < 1000:
        return
    # some record spans a block boundary
    spans = 0
    for (g, s, lg), img in logs.items():
        for b in range(32768, len(img), 32768):
            spans += img[b + 6] in (3, 4)  # MIDDLE / LAST chunk at a block
    assert spans > 0


@pytest.mark.gpu
def test_tan_writer_position_roundtrip():
    """drb_tan_set / drb_tan_get hand a replica's tan writer position over
    (a group returning from the CPU raft.Peer): the next record continues
    the CPU db's log at its offset, with its stored state."""
    p = Pair(G=4, R=3, save_cap=4096, max_props=4, save_tan=1)
    dbs = [[po.TanDB() for _ in range(p.R)] for _ in range(p.G)]
    # the CPU side wrote 3 records to replica (2, 1)'s log
    pre = dbs[2][1]
    for i in range(3):
        pre.write(p.eng.cfg["first_shard_id"] + 2, 2, (2, 1, i + 1), [])
    off = pre.last()["offset"]
    p.eng.tan_set(2, 1, off, 0, True)
    assert p.eng.tan_get(2, 1) == (off, 0, 1)
    logs = {(2, 1, 0): bytearray(pre.file(0))}
    for r in range(6):
        o, e = p.round(k=1, tick=(r % 2 == 0), encode_saves=True)
        assert e.fallbacks == 0 and e.errors == 0
        _check_round(p, dbs, logs, r)
    _read_back(logs, dbs)
    rec, _ = p.eng.export_tan(2, 1)
    assert rec["offset"] > off


def _mux_round(p, dbs, r):
    """One round of the multiplexed tan: every log (slot, key) takes its
    groups' Updates in group order; each record and each log's staged
    bytes equal the oracle db's."""
    first = p.eng.cfg["first_shard_id"]
    n = 0
    for s in range(p.R):
        for c in range(16):
            db = dbs[s][c]
            before = db.last()["offset"]  # the writer's, before the round
            pieces, syncs, fresh = [], False, False
            for g in range(p.G):
                if (first + g) % 16 != c:
                    continue
                want = p.orc.tan_write(g, s, db)
                rec, data = p.eng.export_tan(g, s)
                where = (r, s, c, g, rec, want)
                if want is None:
                    assert not rec["flags"] & abi.TAN_WRITTEN, where
                    continue
                assert rec["flags"] & abi.TAN_WRITTEN, where
                assert (rec["offset"], rec["len"], rec["log"]) == \
                    (want["off"], want["len"], want["log"]), where
                assert bool(rec["flags"] & abi.TAN_SYNC) == want["sync"]
                assert bool(rec["flags"] & abi.TAN_NEW_LOG) == \
                    want["new_log"], where
                f = db.file(want["log"])
                assert data == f[want["off"]:want["off"] + want["len"]], where
                pieces.append(data)
                syncs |= want["sync"]
                fresh |= want["new_log"]
                n += 1
            lg, staged = p.eng.export_tan_log(s, c)
            where = (r, s, c, lg)
            assert staged == b"".join(pieces), where
            assert lg["start_offset"] == before, where
            end = db.last()["offset"]
            assert lg["end_offset"] == end, where
            assert bool(lg["flags"] & abi.TAN_SYNC) == syncs, where
            assert bool(lg["flags"] & abi.TAN_NEW_LOG) == fresh, where
            if pieces:
                assert p.eng.tan_get(next(
                    g for g in range(p.G) if (first + g) % 16 == c), s)[0] \
                    == end, where
    return n


@pytest.mark.gpu
@pytest.mark.parametrize("val_len,cmd_cap,val_cap,max_log", [
    (4, 32, 4, 2048), (1011, 1040, 1024, 1 << 16)])
def test_tan_multiplexed_matches_oracle(val_len, cmd_cap, val_cap, max_log):
    """tan_multiplexed (CreateLogMultiplexedTan): 16 logs per slot shared by
    the shards with the same ShardID % 16, each replica's skip / sync from
    its own stored State; a round's records of one log back to back in
    group order at the offsets the oracle's shared db gives them -- block
    padding, FIRST / MIDDLE / LAST chunks (1 KB payloads in 64 KiB logs)
    and log switches inside a round (2 KiB logs) included."""
    kw = dict(cmd_cap=cmd_cap, kv_val_cap=val_cap) if val_len > 4 else {}
    if val_len > 4:
        kw.update(kv_slots=64)
    p = Pair(G=40, R=3, save_cap=8192, max_props=4, save_tan=1,
             tan_multiplexed=1, tan_max_log=max_log, **kw)
    dbs = [[po.TanDB(max_log) for _ in range(16)] for _ in range(p.R)]
    written = 0
    for r in range(30):
        k = (0, 1, 3, 0, 2)[r % 5]
        rkw = dict(val_len=val_len) if val_len > 4 else {}
        o, e = p.round(k=k, tick=(r % 2 == 0), read_index=(r % 3 == 0),
                       encode_saves=True, **rkw)
        assert e.fallbacks == 0 and e.errors == 0, (r, e.to_dict())
        n = _mux_round(p, dbs, r)
        assert e.log_records == n, (r, e.to_dict())
        written += n
    assert written > 0
    assert any(db.last()["log"] > 0 for row in dbs for db in row)
