"""remote flow-control KATs restated from internal/raft/remote_test.go.

These pin the oracle's restatement of remote.go:103-213 (SURVEY 8a A9,
A14, A15) to the reference's own expected values.
"""
import pytest

from oracle import pyoracle as po
from dragonboat_amd.abi import (REMOTE_REPLICATE, REMOTE_RETRY,
                                REMOTE_SNAPSHOT, REMOTE_WAIT)

L = po.lib


def test_remote_become_retry():  # remote_test.go:104-113
    r = po.new_remote(state=REMOTE_REPLICATE)
    L().orc_remote_become_retry(r)
    assert r.next == r.match + 1 and r.state == REMOTE_RETRY


def test_remote_become_retry_from_snapshot():  # remote_test.go:115-138
    r = po.new_remote(state=REMOTE_SNAPSHOT, snapshot_index=100)
    L().orc_remote_become_retry(r)
    assert (r.next, r.state, r.snapshot_index) == (101, REMOTE_RETRY, 0)
    r = po.new_remote(state=REMOTE_SNAPSHOT, match=10, snapshot_index=0)
    L().orc_remote_become_retry(r)
    assert (r.next, r.state, r.snapshot_index) == (11, REMOTE_RETRY, 0)


@pytest.mark.parametrize("st", [REMOTE_REPLICATE, REMOTE_RETRY,
                                REMOTE_SNAPSHOT])
def test_remote_become_snapshot(st):  # remote_test.go:140-156
    r = po.new_remote(state=st, match=10, next=11)
    L().orc_remote_become_snapshot(r, 12)
    assert (r.state, r.match, r.snapshot_index) == (REMOTE_SNAPSHOT, 10, 12)


def test_remote_become_replication():  # remote_test.go:158-167
    r = po.new_remote(state=REMOTE_RETRY, match=10, next=11)
    L().orc_remote_become_replicate(r)
    assert (r.state, r.match, r.next) == (REMOTE_REPLICATE, 10, 11)


def test_remote_progress():  # remote_test.go:169-189
    r = po.new_remote(state=REMOTE_REPLICATE, match=10, next=11)
    assert L().orc_remote_progress(r, 12) == 0
    assert (r.next, r.match) == (13, 10)
    r = po.new_remote(state=REMOTE_RETRY, match=10, next=11)
    assert L().orc_remote_is_paused(r) == 0
    L().orc_remote_progress(r, 12)
    assert L().orc_remote_is_paused(r) == 1
    assert (r.next, r.match) == (11, 10)


def test_remote_progress_in_snapshot_state_panics():  # :191-200
    r = po.new_remote(state=REMOTE_SNAPSHOT, match=10, next=11)
    assert L().orc_remote_progress(r, 12) == -1


def test_remote_panic_when_in_invalid_state():  # :202-211
    r = po.new_remote(state=100)
    assert L().orc_remote_is_paused(r) == -1


@pytest.mark.parametrize("st,exp", [(REMOTE_RETRY, 0), (REMOTE_WAIT, 1),
                                    (REMOTE_REPLICATE, 0),
                                    (REMOTE_SNAPSHOT, 1)])
def test_remote_is_paused(st, exp):  # remote_test.go:213-229
    assert L().orc_remote_is_paused(po.new_remote(state=st)) == exp


@pytest.mark.parametrize("st,match,next_,si,exp_st,exp_next", [
    (REMOTE_RETRY, 10, 12, 0, REMOTE_REPLICATE, 11),
    (REMOTE_REPLICATE, 10, 12, 0, REMOTE_REPLICATE, 12),
    (REMOTE_SNAPSHOT, 10, 12, 8, REMOTE_RETRY, 11),
    (REMOTE_SNAPSHOT, 10, 11, 12, REMOTE_SNAPSHOT, 11),
])
def test_remote_responded_to(st, match, next_, si, exp_st, exp_next):
    # remote_test.go:231-260
    r = po.new_remote(state=st, match=match, next=next_, snapshot_index=si)
    L().orc_remote_responded_to(r)
    assert (r.state, r.next) == (exp_st, exp_next)


MATCH, NEXT = 10, 20


@pytest.mark.parametrize("index,paused,exp_match,exp_next,exp_paused,upd", [
    (NEXT, False, NEXT, NEXT + 1, False, True),
    (NEXT, True, NEXT, NEXT + 1, False, True),
    (NEXT - 2, False, NEXT - 2, NEXT, False, True),
    (NEXT - 2, True, NEXT - 2, NEXT, False, True),
    (NEXT - 1, False, NEXT - 1, NEXT, False, True),
    (NEXT - 1, True, NEXT - 1, NEXT, False, True),
    (MATCH - 1, False, MATCH, NEXT, False, False),
    (MATCH - 1, True, MATCH, NEXT, True, False),
])
def test_remote_try_update(index, paused, exp_match, exp_next, exp_paused,
                           upd):  # remote_test.go:262-303
    r = po.new_remote(match=MATCH, next=NEXT)
    if paused:
        L().orc_remote_retry_to_wait(r)
    assert bool(L().orc_remote_try_update(r, index)) == upd
    assert (r.next, r.match) == (exp_next, exp_match)
    if exp_paused:
        assert r.state == REMOTE_WAIT


@pytest.mark.parametrize("match,next_,rejected,decreased,exp_next", [
    (10, 15, 9, False, 15), (10, 15, 10, False, 15), (10, 15, 12, True, 11)])
def test_remote_decrease_to_in_replicate_state(match, next_, rejected,
                                               decreased, exp_next):
    # remote_test.go:305-324
    r = po.new_remote(match=match, next=next_, state=REMOTE_REPLICATE)
    assert bool(L().orc_remote_decrease_to(r, rejected, 100)) == decreased
    assert r.next == exp_next


@pytest.mark.parametrize("match,next_,rejected,last,decreased,exp_next", [
    (10, 15, 20, 100, False, 15), (10, 15, 14, 100, True, 14),
    (10, 15, 14, 10, True, 11)])
@pytest.mark.parametrize("st", [REMOTE_RETRY, REMOTE_SNAPSHOT])
def test_remote_decrease_to_not_replicate_state(match, next_, rejected, last,
                                                decreased, exp_next, st):
    # remote_test.go:326-355
    r = po.new_remote(match=match, next=next_, state=st)
    L().orc_remote_retry_to_wait(r)
    assert bool(L().orc_remote_decrease_to(r, rejected, last)) == decreased
    assert r.next == exp_next
    if decreased:
        assert r.state != REMOTE_WAIT


def test_remote_try_update_cause_resume():  # remote_test.go:357-374
    r = po.new_remote(next=5)
    L().orc_remote_retry_to_wait(r)
    L().orc_remote_decrease_to(r, 4, 4)
    assert r.state != REMOTE_WAIT
    L().orc_remote_retry_to_wait(r)
    L().orc_remote_try_update(r, 5)
    assert r.state != REMOTE_WAIT


@pytest.mark.parametrize("vals", [[1, 1, 1], [1, 1, 2], [1, 2, 2], [2, 3, 1],
                                  [3, 2, 1], [3, 3, 1]])
def test_unrolled_bubble_sort_match_value(vals):
    # raft_test.go:2242-2265
    assert po.sort_match_values(vals) == sorted(vals)


def test_sort_match_values_general_sizes():
    # sortMatchValues falls back to sort.Slice for len != 1, 3
    import random
    rng = random.Random(7)
    for n in (1, 2, 4, 5, 7, 8):
        v = [rng.randrange(20) for _ in range(n)]
        assert po.sort_match_values(v) == sorted(v)
