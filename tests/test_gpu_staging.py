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


class _Pinned:
    """A pinned host block (drb_host_alloc): the staged upload then runs on
    the engine's own SDMA engine (drb_hsa.hpp)."""

    def __init__(self, eng, nbytes):
        from dragonboat_amd.engine import lib
        self.eng, self.p = eng, C.c_void_p()
        assert lib().drb_host_alloc(eng.h, max(1, nbytes),
                                    C.byref(self.p)) == 0
        self.addr = self.p.value

    def __del__(self):
        from dragonboat_amd.engine import lib
        lib().drb_host_free(self.eng.h, self.p)


def _one_block(eng, arrs, pinned=False):
    """The packed arrays copied into one block at drb_stage_packed_layout's
    offsets (the one-DMA upload)."""
    cnt, n, keys, cids, lens, pb, plen = arrs
    off, nbytes = eng.stage_packed_layout(n, plen)
    if pinned:
        blk = _Pinned(eng, nbytes)
        base = blk.addr
    else:
        blk = (C.c_uint8 * max(1, nbytes))()
        base = C.addressof(blk)
    C.memmove(base, cnt, C.sizeof(cnt))
    for o, a, sz in ((off[0], keys, 8 * n), (off[1], cids, 8 * n),
                     (off[2], lens, 2 * n), (off[3], pb, plen)):
        if a is not None:  # (no client ids: the session clients')
            C.memmove(base + o, a, sz)

    def at(o, t):
        return C.cast(base + o, C.POINTER(t))
    return blk, (at(0, C.c_uint8), n, at(off[0], C.c_uint64),
                 None if cids is None else at(off[1], C.c_uint64),
                 at(off[2], C.c_uint16), at(off[3], C.c_uint8), plen)


def _stage_packed(p, k, salt, groups=None, key_space=256, val_len=4,
                  slot=0, pipelined=False, one_block=False, sess=False):
    counts, ents, pool = workload.build_batch(p.G, k, p.seed, salt,
                                              key_space, val_len, groups)
    p.orc.stage_proposals(counts, k, ents, pool)
    arrs = workload.pack_batch(p.G, k, counts, ents, pool)
    if sess:  # each group's entries carry its registered session client
        arrs = arrs[:3] + (None,) + arrs[4:]
    if one_block:  # (the block stays alive with p until the next batch)
        p._keep, arrs = _one_block(p.eng, arrs, one_block == "pinned")
    if pipelined:
        # drb_stage_proposals_packed_async: these arrays stay in use until
        # the next call returns (the caller keeps them)
        p.eng.stage_proposals_packed_async(slot, abi.ENTRY_ENCODED, *arrs)
    else:
        p.eng.stage_proposals_packed(slot, abi.ENTRY_ENCODED, *arrs)
    return arrs


@pytest.mark.parametrize("k,val_len,pipelined,one_block,sess",
                         [(1, 4, False, False, False),
                          (3, 4, False, False, False),
                          (2, 16, False, False, False),
                          (1, 4, True, False, False),
                          (3, 16, True, False, False),
                          (2, 4, False, "pageable", False),
                          (3, 16, True, "pageable", False),
                          (2, 4, False, "pinned", False),
                          (3, 16, True, "pinned", False),
                          # client ids left out: drb_set_session_clients
                          (1, 4, False, False, True),
                          (3, 16, True, "pageable", True),
                          (2, 4, True, "pinned", True)])
def test_packed_staging_matches_oracle(k, val_len, pipelined, one_block,
                                       sess):
    G = 96
    p = Pair(G=G, R=3, max_props=4, cmd_cap=32, kv_val_cap=16, prop_slots=2)
    if sess:  # (workload.proposal: one NoOP session per group)
        p.eng.set_session_clients([workload.client_id(p.seed, g)
                                   for g in range(G)])
    held = None
    for rnd in range(10):
        groups = None if rnd % 3 else [g for g in range(G) if g % 4]
        cur = _stage_packed(p, k, rnd, groups, val_len=val_len,
                            slot=rnd % 2 if pipelined else 0,
                            pipelined=pipelined, one_block=one_block,
                            sess=sess)
        cur = (cur, getattr(p, "_keep", None))
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
    cnt0 = (C.c_uint8 * 8)(*([1] * 8))
    keys0 = (C.c_uint64 * 8)(*range(1, 9))
    lens0 = (C.c_uint16 * 8)(*([4] * 8))
    with pytest.raises(DrbError):  # no client ids, no session clients
        p.eng.stage_proposals_packed(0, abi.ENTRY_ENCODED, cnt0, 8, keys0,
                                     None, lens0, (C.c_uint8 * 32)(), 32)
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


def test_sdma_upload_lays_out_the_same_batch():
    """A batch of ≥ 8 MB built in one pinned block goes up on the engine's
    own SDMA engine (hsa_amd_memory_async_copy_on_engine, drb_hsa.hpp); the
    same batch in a pageable block goes through hipMemcpyAsync, the path
    the oracle tests above pin.  Two engines from the same state, one round
    each: the same commits, and every sampled replica's state and log
    equal."""
    import numpy as np
    from dragonboat_amd.engine import Engine
    from tests.gpu_harness import state_diff
    G, R, seed = 262144, 3, 0x5EEDD8B0
    arrs = [x.view("u1") for x in workload.build_packed_np(G, seed, 7)]
    n, plen = arrs[1].size // 8, arrs[4].size
    engs, keep = [], []
    # (pinned on SDMA, pageable, pinned with host_copies: hipMemcpyAsync,
    # the path without the HSA copy engines)
    for pinned, hc in ((True, 0), (False, 0), (True, 1)):
        e = Engine(num_groups=G, num_replicas=R, window=32, cmd_cap=32,
                   max_props=1, prop_slots=2, host_copies=hc)
        e.init_steady(term=2, leader_slot=0, seed=seed)
        off, nbytes = e.stage_packed_layout(n, plen)
        assert nbytes >= 8 << 20
        if pinned:
            blk = _Pinned(e, nbytes)
            base = blk.addr
        else:
            blk = np.zeros(nbytes, dtype=np.uint8)
            base = blk.ctypes.data
        view = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(base))
        for o, x in zip([0] + off, arrs):
            view[o:o + x.size] = x
        ptr = [C.cast(base + o, t) for o, t in zip(
            [0] + off, [C.POINTER(C.c_uint8), C.POINTER(C.c_uint64),
                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint16),
                        C.POINTER(C.c_uint8)])]
        e.stage_proposals_packed(0, abi.ENTRY_ENCODED, ptr[0], n, ptr[1],
                                 ptr[2], ptr[3], ptr[4], plen)
        committed = 0
        for r in range(3):  # the batch, then rounds that commit it
            out = e.step(tick=r == 0, prop_slot=0 if r == 0 else abi.DRB_NONE)
            assert out.fallbacks == 0 and out.errors == 0
            committed += out.committed_entries
        engs.append((e, committed))
        keep.append(blk)
    (a, ca) = engs[0]
    for (b, cb) in engs[1:]:
        assert ca == cb and ca > 0
        for g0 in range(0, G, 8191):
            sa, sb = a.export_replicas(g0, 1), b.export_replicas(g0, 1)
            for s in range(R):
                assert not state_diff(sa[s], sb[s], R), (g0, s)
                li = sa[s].last_index
                assert a.export_log(g0, s, max(1, li - 2), li) == \
                    b.export_log(g0, s, max(1, li - 2), li), (g0, s)
