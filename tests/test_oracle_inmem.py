"""inMemory known-answer tests restated from
/root/reference/internal/raft/inmemory_test.go:260-548.

They pin the oracle's inMemory (oracle/raft_oracle.c im_*, inmemory.go)
to the reference's expected values; the GPU path's resident window
follows the same rules (drb_step.hpp append / saved / applied markers) and
is checked against the oracle in tests/test_gpu_*.py.
"""
import pytest

from oracle import pyoracle as po


def E(*pairs):
    return [po.ent(index=i, term=t) for i, t in pairs]


@pytest.mark.parametrize("shrunk", [False, True])
def test_inmem_merge_full_append(shrunk):
    # inmemory_test.go:261-291 (testInMemMergeFullAppend)
    im = po.InMem(5, E((5, 5), (6, 6), (7, 7)), shrunk=shrunk)
    im.merge(E((8, 8), (9, 9)))
    info = im.info()
    assert info["shrunk"] == shrunk
    assert info["n"] == 5 and info["marker_index"] == 5
    assert im.last_index() == (9, True)


def test_inmem_merge_replace():
    # inmemory_test.go:293-318
    im = po.InMem(5, E((5, 5), (6, 6), (7, 7)), shrunk=True)
    im.merge(E((2, 2), (3, 3)))
    info = im.info()
    assert not info["shrunk"]
    assert info["n"] == 2 and info["marker_index"] == 2
    assert im.last_index() == (3, True)


def test_inmem_merge_with_hole_cause_panic():
    # inmemory_test.go:320-340
    im = po.InMem(5, E((5, 5), (6, 6), (7, 7)))
    with pytest.raises(po.OracleError):
        im.merge(E((9, 9), (10, 10)))


def test_inmem_merge():
    # inmemory_test.go:342-373
    im = po.InMem(5, E((5, 5), (6, 6), (7, 7)), shrunk=True)
    im.merge(E((6, 7), (7, 10)))
    info = im.info()
    assert not info["shrunk"]
    assert info["n"] == 3 and info["marker_index"] == 5
    assert im.last_index() == (7, True)
    assert im.term(6) == (7, True)
    assert im.term(7) == (10, True)


def test_inmem_entries_to_save_return_not_saved_entries():
    # inmemory_test.go:375-407
    im = po.InMem(5, E((5, 5), (6, 6), (7, 7)), saved_to=4)
    assert im.entries_to_save() == (3, 5)
    for saved_to, want in ((5, 2), (7, 0), (8, 0)):
        im = po.InMem(5, E((5, 5), (6, 6), (7, 7)), saved_to=saved_to)
        assert im.entries_to_save()[0] == want, saved_to


@pytest.mark.parametrize("index,term,saved_to", [
    (4, 1, 4), (8, 1, 4), (6, 7, 4), (6, 6, 6)])
def test_inmem_saved_log_to_updates_saved_to(index, term, saved_to):
    # inmemory_test.go:409-435
    im = po.InMem(5, E((5, 5), (6, 6), (7, 7)), saved_to=4)
    im.saved_log_to(index, term)
    assert im.info()["saved_to"] == saved_to


def test_inmem_set_saved_to_when_restoring_snapshot():
    # inmemory_test.go:437-450
    im = po.InMem(5, E((5, 5)), saved_to=4)
    im.restore(100, 10)
    assert im.info()["saved_to"] == 100


def test_inmem_merge_set_saved_to():
    # inmemory_test.go:452-511
    six = E((6, 6), (7, 8))
    im = po.InMem(6, E((6, 6), (7, 7)), saved_to=5)
    im.merge(six)
    assert im.info()["saved_to"] == 5
    full = E((5, 5), (6, 6), (7, 7), (8, 8), (9, 9), (10, 10))
    im = po.InMem(5, full, saved_to=4)
    im.merge(six)
    assert im.info()["saved_to"] == 4
    im = po.InMem(5, full, saved_to=6)
    im.merge(six)
    assert im.info()["saved_to"] == 5
    im = po.InMem(6, E((6, 6), (7, 7)), saved_to=5)
    im.merge(E((8, 8), (9, 9)))
    assert im.info()["saved_to"] == 5


@pytest.mark.parametrize("applied_to,length,first_index", [
    (4, 6, 5), (5, 5, 6), (11, 6, 5), (6, 4, 7), (10, 0, 11)])
def test_applied_log_to(applied_to, length, first_index):
    # inmemory_test.go:513-548
    im = po.InMem(5, E((5, 5), (6, 6), (7, 7), (8, 8), (9, 9), (10, 10)),
                  saved_to=4)
    im.applied_log_to(applied_to)
    info = im.info()
    assert info["n"] == length
    if length:
        assert info["first"] == first_index
