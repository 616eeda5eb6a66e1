"""Batched LogDB records (SURVEY 8 A26 -> F2) restated in the oracle
(oracle/logdb_oracle.c) and pinned by the reference's own tables and data:

  internal/logdb/batch_test.go:29-247   batch ids, compaction, restore, merge
  internal/logdb/batch_test.go:249-342  record-level merges
  internal/logdb/testdata/v2-rocksdb-batched.tar.bz2 (tests/golden/
  v2_rocksdb_wal_puts.json): the three EntryBatch records of shard 2 /
  replica 1, batch 0, written by three successive saves -- reproduced byte
  for byte from the entries they hold.
"""
import json
import os

import pytest

from oracle import pyoracle as po

BATCH = 48  # settings.Hard.LogDBEntryBatchSize (hard.go:125)
GOLDEN = os.path.join(os.path.dirname(__file__), "golden",
                      "v2_rocksdb_wal_puts.json")


@pytest.mark.parametrize("low,high,blow,bhigh", [
    (2, 3, 0, 1), (1, BATCH, 0, 1), (BATCH, 2 * BATCH, 1, 2),
    (1, BATCH + 1, 0, 2), (BATCH, 2 * BATCH + 1, 1, 3),
    (BATCH + 1, 2 * BATCH, 1, 2), (BATCH + 1, 2 * BATCH + 1, 1, 3)])
def test_get_batch_id_range(low, high, blow, bhigh):
    # batch_test.go:29-52
    assert po.batch_id_range(low, high) == (blow, bhigh)


def test_not_compacted_when_index_has_gap():
    # batch_test.go:54-74
    ents = [(2, i) for i in range(1, BATCH) if i != BATCH // 2]
    assert po.batch_compact(ents) == ents


def test_not_compacted_when_multiple_terms():
    # batch_test.go:76-97
    ents = [(2 if i in (BATCH - 1, BATCH - 2) else 1, i)
            for i in range(1, BATCH)]
    assert po.batch_compact(ents) == ents


def test_can_be_compacted_and_restored():
    # batch_test.go:99-130
    ents = [(1, i) for i in range(1, BATCH)]
    c = po.batch_compact(ents)
    assert c[0] == (1, 1) and all(x == (0, 0) for x in c[1:])
    assert po.batch_compact(c, restore=True) == ents


def test_not_compacted_batch_is_not_restored():
    # batch_test.go:132-149
    ents = [(1, i) for i in range(1, BATCH)]
    assert po.batch_compact(ents, restore=True) == ents


@pytest.mark.parametrize("restore", [False, True])
@pytest.mark.parametrize("ents", [[], [(0, 0)]])
def test_compact_restore_panic_when_batch_too_small(restore, ents):
    # batch_test.go:151-167
    with pytest.raises(po.OracleError):
        po.batch_compact(ents, restore=restore)


def test_merge_first_batch_panics():
    # batch_test.go:169-186
    with pytest.raises(po.OracleError):
        po.batch_merged_first([], [(1, 1)])
    with pytest.raises(po.OracleError):
        po.batch_merged_first([(1, 1)], [])
    with pytest.raises(po.OracleError):
        po.batch_merged_first([(1, BATCH)], [(1, 2 * BATCH)])


def test_incoming_batch_more_recent_than_last_batch():
    # batch_test.go:188-193
    eb = [(1, 2 * BATCH)]
    assert po.batch_merged_first(eb, [(1, BATCH)]) == eb


@pytest.mark.parametrize("ebf,ebl,lbf,lbl,mf,ml,new", [
    (1, 10, 2, 10, 1, 10, 1), (1, 10, 2, 11, 1, 10, 1),
    (1, 10, 2, 9, 1, 10, 1), (2, 10, 2, 10, 2, 10, 2),
    (2, 10, 2, 9, 2, 10, 2), (2, 10, 2, 11, 2, 10, 2),
    (2, 10, 1, 10, 1, 10, 2), (3, 10, 1, 3, 1, 10, 3),
    (3, 10, 1, 2, 1, 10, 3), (3, 10, 1, 4, 1, 10, 3)])
def test_get_merged_first_batch(ebf, ebl, lbf, lbl, mf, ml, new):
    # batch_test.go:195-247
    eb = [(2, i) for i in range(ebf, ebl + 1)]
    lb = [(1, i) for i in range(lbf, lbl + 1)]
    m = po.batch_merged_first(eb, lb)
    assert m[0][1] == mf and m[-1][1] == ml
    assert all(t == 2 for t, i in m if i >= new)


def _decode(value):
    return po.entrybatch_unmarshal(value)


def test_entry_batch_will_not_be_merged_to_previous_batch():
    # batch_test.go:249-292
    db = po.BatchDB()
    db.record(0, 4, [po.ent(term=1, index=1)])
    recs = db.record(0, 4, [po.ent(term=1, index=1 + BATCH)])
    assert [b for b, _ in recs] == [1]
    ents = _decode(recs[0][1])
    assert [(e["term"], e["index"]) for e in ents] == [(1, 1 + BATCH)]


def test_entry_batch_merged_not_last_batch():
    # batch_test.go:294-342
    db = po.BatchDB()
    db.record(0, 4, [po.ent(term=1, index=i) for i in range(1, BATCH + 4)])
    recs = db.record(0, 4, [po.ent(term=2, index=i)
                            for i in range(BATCH - 4, BATCH + 3)])
    assert [b for b, _ in recs] == [0, 1]
    ents = _decode(recs[0][1])
    assert [e["index"] for e in ents] == list(range(1, BATCH))
    assert [e["term"] for e in ents] == \
        [1 if i < BATCH - 4 else 2 for i in range(1, BATCH)]


def test_save_entries_across_multiple_batches():
    # batch_test.go:344-: saves [1], [2], [3 .. 49]; batch 0 holds 1..47
    # compacted (one term, contiguous), batch 1 holds 48 and 49
    db = po.BatchDB()
    db.record(0, 4, [po.ent(term=1, index=1)])
    db.record(0, 4, [po.ent(term=1, index=2)])
    recs = db.record(0, 4, [po.ent(term=1, index=i)
                            for i in range(3, BATCH + 2)])
    assert [b for b, _ in recs] == [0, 1]
    e0 = _decode(recs[0][1])
    assert len(e0) == BATCH - 1
    assert (e0[0]["term"], e0[0]["index"]) == (1, 1)
    assert all((e["term"], e["index"]) == (0, 0) for e in e0[1:])
    e1 = _decode(recs[1][1])
    assert [(e["term"], e["index"]) for e in e1] == [(1, BATCH), (0, 0)]


def test_golden_wal_batch_records():
    """The reference's own WAL: three saves of shard 2 / replica 1 each
    rewrote the batch-0 record, which grew 1 -> 2 -> 3 entries (different
    terms, so never compacted).  The oracle reproduces all three values
    from the entries, one save at a time."""
    puts = json.load(open(GOLDEN))["puts"]
    # the EntryBatch key of shard 2, replica 1, batch 0 as the WAL holds it
    key = "07070000000000000000000200000000000000010000000000000000"
    vals = [bytes.fromhex(p["value"]) for p in puts if p["key"] == key]
    assert len(vals) == 3
    last = _decode(vals[-1])
    db = po.BatchDB()
    for i, want in enumerate(vals):
        recs = db.record(2, 1, [last[i]])
        assert recs == [(0, want)], i
