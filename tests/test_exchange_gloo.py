"""The C4 exchange step (dragonboat_amd/exchange.py) on the CPU: world_size
2 and 3 gloo ranks move mailbox planes exactly as the RCCL run does.

Each rank holds fake outbox/inbox planes in host memory, sized per plane by
a summary word the way drb_plane_regions sizes the engine's (Replicate
records, other records, entry rows, c1 / header-only flags).  The routing is the engine's own
(drb_place_peer from the C ABI library, no device needed); the send/recv
lists come from exchange.plan and run as one gloo batch_isend_irecv.
After the step, inbox plane (a, b) of every rank must hold the bytes rank
(rank - d) wrote into its outbox plane (a, b), d = (b - a) mod N.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

R, LANES = 5, 24


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


C1, HDR = 1 << 18, 1 << 19


def _word(rank, a, b):
    rng = np.random.default_rng(rank * 1000 + a * 10 + b)
    kr, ko = int(rng.integers(0, 4)), int(rng.integers(0, 4))
    E = int(rng.integers(0, 3)) if a == 0 else 0
    fl = (C1 if rng.integers(0, 2) else 0) | \
        (HDR if rng.integers(0, 4) == 0 else 0)
    return kr | (ko << 5) | (E << 10) | fl if (kr or ko or E or fl & HDR) \
        else 0


def _layout(word):
    """(buffer slot, bytes) of the regions drb_plane_regions lists."""
    kr, ko, E = word & 0x1f, (word >> 5) & 0x1f, (word >> 10) & 0xff
    s = []
    for c in ((0, 1) if word & C1 else (0,)):
        if kr:
            s.append((2 * c, kr * LANES * 16))
        if ko:
            s.append((2 * c + 1, ko * LANES * 16))
    if kr or ko or word & HDR:
        s.append((4, LANES * 16))
    if kr:
        s.append((5, LANES * 8))
    if E:
        s += [(6, LANES * 8), (7, E * 5 * LANES * 16)]
    return s


class FakePlanes:
    """Host-memory planes with the engine's region sizing."""

    def __init__(self, rank):
        self.out, self.inb = {}, {}
        for a in range(R):
            for b in range(R):
                rng = np.random.default_rng(7 + rank * 100 + a * 10 + b)
                self.out[(a, b)] = [
                    rng.integers(0, 256, n, dtype=np.uint8)
                    for n in self._sizes(13 | (13 << 5) | (3 << 10) | C1)]
                self.inb[(a, b)] = [np.zeros_like(x) for x in self.out[(a, b)]]

    @staticmethod
    def _sizes(word):
        return [n for _, n in _layout(word)]

    def _pick(self, word, bufs):
        # the full-capacity buffers in region order; take the first n bytes
        return [bufs[i] for i, _ in _layout(word)]

    def regions(self, a, b, word, direction):
        bufs = self._pick(word, (self.out if direction == 0 else
                                 self.inb)[(a, b)])
        return [(x.ctypes.data, n) for x, n in zip(bufs, self._sizes(word))]


def _worker(rank, world, port, q, fixed):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dragonboat_amd import exchange as X
        fp = FakePlanes(rank)
        if fixed:  # full-capacity planes: no sizes are exchanged
            words = X.fixed_words(R, world, 0b101, 13, 3)
        else:
            mine = [_word(rank, a, b) if X.place_peer(world, rank, a, b, 0)
                    >= 0 else 0 for a in range(R) for b in range(R)]
            t = torch.tensor(mine, dtype=torch.int64)
            allw = torch.empty(world * R * R, dtype=torch.int64)
            dist.all_gather_into_tensor(allw, t)
            flat = allw.tolist()
            words = [flat[k * R * R:(k + 1) * R * R] for k in range(world)]
        ops = X.plan(R, world, rank, words, fp.regions)
        X.run_ops(ops, X.host_bytes)
        got = {k: [x.copy() for x in v] for k, v in fp.inb.items()}
        q.put((rank, words, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fixed", [(2, False), (3, False), (3, True)])
def test_plane_exchange_gloo(world, fixed):
    from dragonboat_amd import exchange as X
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, fixed))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, words, got = q.get(timeout=240)
        res[r] = (words, got)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    moved = 0
    for r in range(world):
        words, got = res[r]
        for a in range(R):
            for b in range(R):
                src = X.place_peer(world, r, a, b, 1)
                if src < 0:
                    assert all(not x.any() for x in got[(a, b)])
                    continue
                w = words[src][a * R + b]
                sent = FakePlanes(src)
                exp = sent._pick(w, sent.out[(a, b)])
                dst = FakePlanes(r)._pick(w, got[(a, b)])
                for e, d, n in zip(exp, dst, FakePlanes._sizes(w)):
                    assert (d[:n] == e[:n]).all(), (r, a, b)
                    moved += n
    assert moved > 0


def test_full_word_layout():
    """A full-capacity word lists every record position of both chunks,
    the header, the max LogIndex word and E entry rows (drb_plane_regions
    sizing, restated by _layout)."""
    from dragonboat_amd import exchange as X
    w = X.full_word(13, 3)
    assert _layout(w) == [(0, 13 * LANES * 16), (2, 13 * LANES * 16),
                          (4, LANES * 16), (5, LANES * 8), (6, LANES * 8),
                          (7, 3 * 5 * LANES * 16)]
    # a follower-only sender: every record position as "other" records
    # (positions MB - Ko .. MB - 1 = all of them) and the header
    w = X.full_word(13, 3, leader_sender=False)
    assert _layout(w) == [(1, 13 * LANES * 16), (3, 13 * LANES * 16),
                          (4, LANES * 16)]
    # leaders at slot 0: planes (0, b) and (a, 0) only
    ws = X.fixed_words(R, 2, 1, 13, 3)
    assert ws[0] == ws[1]
    for a in range(R):
        for b in range(R):
            w = ws[0][a * R + b]
            assert bool(w) == (a != b and 0 in (a, b)), (a, b)


def test_fixed_words_with_elections():
    """With elections roles change on the device (the raft launch), so the
    fixed mode moves every remote plane at full capacity -- Replicates and
    responses alike -- with the rterm rows of the records that carry a term
    of their own (DRB_PLANE_TOTHER, drb_plane_regions)."""
    from dragonboat_amd import exchange as X
    ws = X.fixed_words(R, 2, 1, 13, 3, elections=True)
    for a in range(R):
        for b in range(R):
            w = ws[0][a * R + b]
            assert bool(w) == (a != b), (a, b)
            if w:
                assert w == X.full_word(13, 3) | X.PLANE_TOTHER
                assert (w & 0x1f) == 13 and ((w >> 5) & 0x1f) == 0
