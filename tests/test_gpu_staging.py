"""GPU: the host entry queue staged in its packed form
(drb_stage_proposals_packed: per group a count, per entry Key / ClientID /
Cmd length, the Cmd bytes back to back) lays out the same staged
proposals as drb_stage_proposals of the drb_entry rows (queue.go:60 ->
node.handleProposals, node.go:1275): rounds fed either way stay bit-exact
with the oracle.  Also the capacity path: a Cmd longer than cmd_cap is
staged as one the leader cannot take (DRB_FB_CAPACITY before appending)."""
import ctypes as C

import pytest

from dragonboat_amd import abi, workload
from dragonboat_amd.engine import DrbError
from tests.gpu_harness import Pair

pytestmark = pytest.mark.gpu


def _stage_packed(p, k, salt, groups=None, key_space=256, val_len=4,
                  slot=0, pipelined=False):
    counts, ents, pool = workload.build_batch(p.G, k, p.seed, salt,
                                              key_space, val_len, groups)
    p.orc.stage_proposals(counts, k, ents, pool)
    arrs = workload.pack_batch(p.G, k, counts, ents, pool)
    if pipelined:
        # drb_stage_proposals_packed_async: these arrays stay in use until
        # the next call returns (the caller keeps them)
        p.eng.stage_proposals_packed_async(slot, abi.ENTRY_ENCODED, *arrs)
    else:
        p.eng.stage_proposals_packed(slot, abi.ENTRY_ENCODED, *arrs)
    return arrs


@pytest.mark.parametrize("k,val_len,pipelined", [(1, 4, False), (3, 4, False),
                                                 (2, 16, False), (1, 4, True),
                                                 (3, 16, True)])
def test_packed_staging_matches_oracle(k, val_len, pipelined):
    G = 96
    p = Pair(G=G, R=3, max_props=4, cmd_cap=32, kv_val_cap=16, prop_slots=2)
    held = None
    for rnd in range(10):
        groups = None if rnd % 3 else [g for g in range(G) if g % 4]
        cur = _stage_packed(p, k, rnd, groups, val_len=val_len,
                            slot=rnd % 2 if pipelined else 0,
                            pipelined=pipelined)
        held = (held, cur)[1]  # the previous call's arrays are free now
        o = p.orc.round(tick=rnd % 2 == 0)
        e = p.eng.step(tick=rnd % 2 == 0,
                       prop_slot=rnd % 2 if pipelined else 0)
        p.rounds += 1
        assert e.fallbacks == 0 and e.errors == 0, (rnd, e.to_dict())
        assert e.committed_entries == o.committed_entries
        errs = p.check()
        assert not errs, (rnd, errs[:2])
    p.eng.stage_wait_upload()
    del held


def test_packed_staging_rejects_bad_sums():
    p = Pair(G=8, R=3)
    cnt = (C.c_uint8 * 8)(*([1] * 8))
    keys = (C.c_uint64 * 8)(*range(1, 9))
    lens = (C.c_uint16 * 8)(*([4] * 8))
    pool = (C.c_uint8 * 32)()
    with pytest.raises(DrbError):  # 7 entries declared, 8 counted
        p.eng.stage_proposals_packed(0, abi.ENTRY_ENCODED, cnt, 7, keys, keys,
                                     lens, pool, 32)
    with pytest.raises(DrbError):  # lengths add up to 32, pool says 31
        p.eng.stage_proposals_packed(0, abi.ENTRY_ENCODED, cnt, 8, keys, keys,
                                     lens, pool, 31)
    cnt[3] = 9  # more than max_props
    with pytest.raises(DrbError):
        p.eng.stage_proposals_packed(0, abi.ENTRY_ENCODED, cnt, 16, keys,
                                     keys, lens, pool, 32)
