"""Cross-rank mailbox exchange for replicas spread over GPUs.

After every round each rank's engine holds, per remote (sender slot,
receiver slot) plane, the records, headers and entry rows its replicas sent
to replicas on other ranks (include/drb_engine.h, drb_plane_*).  One
exchange step per round moves them, in one of two modes:

fixed (the default on RCCL): every remote plane moves at its full capacity
  -- the mailbox's MB record positions (both chunks), the header, the max
  LogIndex + n word, the entry-row base and E entry rows -- which the
  leader's and the follower's pre-pass already bound (DRB_FB_CAPACITY
  before a round could exceed them).  The receiver reads only what the
  plane's header counts (stale positions are never read), so no sizes are
  exchanged: the sends and receives are enqueued on the engine stream
  right behind the round (torch's NCCL work waits on it, and the next
  round waits on the work), with no host synchronisation at all;

counted: 1. drb_plane_counts (a stream sync): per plane a word {records K,
  entry rows E, flags}; 2. all_gather of those words, so every receiver
  knows the sizes its senders will ship; 3. the regions at those sizes.
  Fewer bytes, one host round trip per round.

Both post one batched group of point-to-point send/recv (RCCL over xGMI
when the backend is "nccl"), plane regions straight out of / into engine
memory.

This replaces the reference's Transport.Send -> handleRequest path
(internal/transport/transport.go:346, :305) for GPU-resident replicas.
The send and receive lists are built in the same (from, to, region) order
on every rank, so each pair of ranks posts matching operations in the same
order.
"""
import ctypes as C

import torch
import torch.distributed as dist

from . import engine as _engine


class _DevView:
    """A device byte range as an object torch can alias (no copy)."""

    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {
            "shape": (int(nbytes),), "typestr": "|u1",
            "data": (int(ptr), False), "version": 3, "strides": None}


def device_bytes(ptr, nbytes, device):
    return torch.as_tensor(_DevView(ptr, nbytes), device=device)


def host_bytes(ptr, nbytes):
    buf = (C.c_uint8 * int(nbytes)).from_address(int(ptr))
    return torch.frombuffer(buf, dtype=torch.uint8)


def place_peer(world, rank, a, b, direction):
    """Rank plane (a, b) goes to (0) / comes from (1); -1 when local."""
    return _engine.lib().drb_place_peer(world, rank, a, b, direction)


PLANE_TOTHER = 1 << 20  # include/drb_engine.h DRB_PLANE_TOTHER


def full_word(mailbox, entry_mbox, leader_sender=True, elections=False):
    """The summary word of a plane at full capacity (drb_plane_regions):
    every record position, both chunks, the header, and -- when the sender
    slot may hold leaders -- the max LogIndex word and every entry row.  A
    follower-only sender slot sends responses (other records) only.  With
    elections every plane can carry both kinds, and the rterm rows of the
    records the raft launch wrote with a term of their own."""
    if leader_sender or elections:
        w = (mailbox & 0x1f) | ((entry_mbox & 0xff) << 10) | (1 << 18) | \
            (1 << 19)
        # (positions [0, mailbox) hold both kinds: Replicates from the
        # bottom, the others from the top)
        return w | (PLANE_TOTHER if elections else 0)
    return ((mailbox & 0x1f) << 5) | (1 << 18) | (1 << 19)


def fixed_words(R, world, leader_mask, mailbox, entry_mbox, elections=False):
    """Per-rank plane words of the fixed mode: plane (a, b) moves when a or
    b is a leader slot on some rank (leader_mask: the OR over the ranks of
    drb_role_slots), at full capacity.  With elections roles change on the
    device, so every plane moves."""
    row = []
    for a in range(R):
        for b in range(R):
            la, lb = (leader_mask >> a) & 1, (leader_mask >> b) & 1
            row.append(0 if a == b or not (la or lb or elections) else
                       full_word(mailbox, entry_mbox, bool(la), elections))
    return [row for _ in range(world)]


def plan(R, world, rank, words, regions):
    """[(op, peer, (ptr, nbytes))] for this rank's exchange step.

    words[q][a * R + b]: rank q's summary word of plane (a, b);
    regions(a, b, word, direction) -> [(ptr, nbytes)] of this rank."""
    ops = []
    for a in range(R):
        for b in range(R):
            if a == b:
                continue
            dst = place_peer(world, rank, a, b, 0)
            if dst < 0:
                continue
            src = place_peer(world, rank, a, b, 1)
            ws = words[rank][a * R + b]
            if ws:
                ops += [("send", dst, r) for r in regions(a, b, ws, 0)]
            wr = words[src][a * R + b]
            if wr:
                ops += [("recv", src, r) for r in regions(a, b, wr, 1)]
    return ops


def run_ops(ops, to_tensor, group=None):
    p2p = []
    for op, peer, (ptr, nbytes) in ops:
        t = to_tensor(ptr, nbytes)
        fn = dist.isend if op == "send" else dist.irecv
        p2p.append(dist.P2POp(fn, t, peer, group))
    if p2p:
        for req in dist.batch_isend_irecv(p2p):
            req.wait()


def run_ops_staged(ops, device, group=None):
    """The same step for a backend without device tensors (gloo): each
    region goes through host memory."""
    sends, recvs = [], []
    p2p = []
    for op, peer, (ptr, nbytes) in ops:
        d = device_bytes(ptr, nbytes, device)
        h = torch.empty(int(nbytes), dtype=torch.uint8)
        if op == "send":
            h.copy_(d)
            p2p.append(dist.P2POp(dist.isend, h, peer, group))
        else:
            recvs.append((d, h))
            p2p.append(dist.P2POp(dist.irecv, h, peer, group))
    if p2p:
        for req in dist.batch_isend_irecv(p2p):
            req.wait()
    for d, h in recvs:
        d.copy_(h)


def run_ops_on_stream(ops, to_tensor, stream, group=None):
    """The batch enqueued behind `stream` (the engine's): NCCL's work waits
    on the stream, and the stream waits on the work; the host does not."""
    with torch.cuda.stream(stream):
        p2p = [dist.P2POp(dist.isend if op == "send" else dist.irecv,
                          to_tensor(ptr, nbytes), peer, group)
               for op, peer, (ptr, nbytes) in ops]
        if p2p:
            for req in dist.batch_isend_irecv(p2p):
                req.wait()  # stream-side for NCCL


class PlaneExchange:
    """The exchange step of one rank's engine (torch.distributed group).
    staged=True moves the regions through host memory (gloo); fixed=True
    ships full-capacity planes with no host round trip (module doc)."""

    def __init__(self, eng, world, rank, device, group=None, staged=False,
                 fixed=None):
        self.eng, self.world, self.rank = eng, world, rank
        self.device, self.group, self.staged = device, group, staged
        self.fixed = (not staged) if fixed is None else fixed
        self.bytes_sent = 0
        self._stream = None if staged else torch.cuda.ExternalStream(
            eng.stream, device=device)
        self.leader_mask = 0
        if self.fixed:
            self.refresh_roles()

    def refresh_roles(self):
        """Collective: the OR of every rank's leader slots.  Call on every
        rank after importing replicas (roles change only there)."""
        dev = "cpu" if self.staged else self.device
        t = torch.tensor([self.eng.role_slots()[0]], dtype=torch.int64,
                         device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.BOR, group=self.group)
        self.leader_mask = int(t.item())

    def words(self):
        R = self.eng.R
        if self.fixed:
            return fixed_words(R, self.world, self.leader_mask,
                               self.eng.cfg["mailbox"],
                               self.eng.cfg["entry_mbox"],
                               bool(self.eng.cfg["elections"]))
        mine = self.eng.plane_counts()  # synchronises the engine stream
        dev = "cpu" if self.staged else self.device
        t = torch.tensor(mine, dtype=torch.int64, device=dev)
        allw = torch.empty(self.world * R * R, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(allw, t, group=self.group)
        flat = allw.tolist()
        return [flat[q * R * R:(q + 1) * R * R] for q in range(self.world)]

    def step(self):
        R = self.eng.R
        ops = plan(R, self.world, self.rank, self.words(),
                   self.eng.plane_regions)
        self.bytes_sent += sum(n for op, _, (_, n) in ops if op == "send")
        if self.staged:
            self.eng.sync()
            run_ops_staged(ops, self.device, self.group)
            torch.cuda.current_stream(self.device).synchronize()
        elif self.fixed:
            run_ops_on_stream(ops, lambda p, n: device_bytes(p, n,
                                                             self.device),
                              self._stream, self.group)
        else:
            run_ops(ops, lambda p, n: device_bytes(p, n, self.device),
                    self.group)
            torch.cuda.current_stream(self.device).synchronize()
        # transports may ingest into the remote planes again (drb_ingest
        # returns DRB_EAGAIN between a round and its exchange)
        self.eng.exchange_mark()
