"""GPU: the round's ReadyToReads and served-read results as batched outputs
(SURVEY 8b "Step": SoA views of the Update's ReadyToReads; 8b "Apply":
ReadLocalNode).

drb_export_ready_to_reads_batch is node.processReadyToRead for a whole
step worker's groups (node.go:1081 -> pendingReadIndex.addReady,
request.go:883); drb_export_read_results returns what each client's
ReadLocalNode (nodehost.go:849 -> KVTest.Lookup, kvtest.go:164-175) got for
the reads served behind those ReadyToReads (pendingReadIndex.applied,
request.go:930-953).  Both are compared with the oracle cluster at the C3
shape (3 replicas, one ReadIndex ctx per group per round, 9 reads per ctx,
16 B writes), with the reads issued at the leader and at a follower.
"""
import struct

import pytest

from dragonboat_amd import workload
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu

READS = 9
KEYS = 16  # a small key space: most reads find their key


def _read_key(low, j, key_space):
    x = workload.mix64(low ^ (((j + 1) * workload.GOLDEN) & workload.MASK))
    return x % key_space


@pytest.mark.parametrize("ri_replica", [0, 2])
def test_batched_ready_to_reads_and_read_results(ri_replica):
    G, R = 300, 3
    p = Pair(G=G, R=R, max_reads_per_ctx=READS)
    slot = 0 if ri_replica == 0 else ri_replica - 1
    n_rtr = n_res = found = 0
    for rnd in range(14):
        o, e = p.round(k=1, tick=(rnd % 2 == 0), read_index=True,
                       reads=READS, read_key_space=KEYS, key_space=KEYS,
                       ri_replica=ri_replica)
        assert e.fallbacks == 0 and e.errors == 0, (rnd, e.to_dict())
        # ReadyToReads: the whole slot in one call == per replica, oracle
        batch = p.eng.export_ready_batch(slot)
        want = {g: p.orc.export_ready(g, slot) for g in range(G)}
        want = {g: x for g, x in want.items() if x}
        assert batch == want, rnd
        n_rtr += sum(len(x) for x in batch.values())
        # a sub-range of groups
        sub = p.eng.export_ready_batch(slot, 100, 57)
        assert sub == {g: x for g, x in want.items() if 100 <= g < 157}
        # the served reads: one result per read of every ctx whose index
        # the replica applied, in group, ctx, read order
        res = p.eng.export_read_results(slot)
        sums, served, deferred = p.orc.serve_reads(READS, KEYS)
        assert len(res) == served == e.reads_served, rnd
        assert e.reads_deferred == deferred, rnd
        esums = p.eng.export_read_sums(0, G)
        for i, x in enumerate(sums):
            if x is not None:
                assert esums[i] == x, (rnd, i)
        exp = []
        for g in range(G):
            st = p.orc.export(g, slot)
            kv = p.orc.export_kv(g, slot)
            for (index, low, high) in want.get(g, []):
                if index > st.sm_index:
                    continue  # deferred: no result yet
                for j in range(READS):
                    key = _read_key(low, j, KEYS)
                    v = kv.get(struct.pack("<Q", key))
                    exp.append((g, index, low, j, key, int(v is not None),
                                len(v) if v is not None else 0,
                                int.from_bytes((v or b"")[:4], "little")))
        assert res == exp, rnd
        n_res += len(res)
        found += sum(r[5] for r in res)
    assert n_rtr > G and n_res > G * READS and found > n_res // 5


def test_read_results_need_the_buffer():
    """Without drb_config.max_reads_per_ctx there is no result buffer (the
    served reads only fold into drb_export_read_sums)."""
    p = Pair(G=8, R=3)
    p.round(k=1, read_index=True, reads=READS)
    with pytest.raises(Exception):
        p.eng.export_read_results(0)
