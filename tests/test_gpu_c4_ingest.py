"""GPU: another NodeHost's replica talking to engines whose replicas are
spread over ranks (C4 placement; SURVEY 8b Inbound, nodehost.go:2072-2122).

Replica slot s of global group g lives on rank (g + s) mod N at lane g / N;
one slot of every group runs on a CPU NodeHost instead -- here the oracle
cluster, which steps every replica and is the reference.  After each round
the messages that replica sent go to the engine of each receiver's rank,
through drb_ingest (decoded pb.Message arrays) or drb_ingest_wire (the TCP
bytes of its connection, built by the oracle codec); a rank drops the ones
for replicas it does not host.  A plane whose sender slot belongs to
another rank is written into the receiver's inbound copies (mbox_in, ...)
and a Replicate's entries into that plane's entry rows -- exercised with
the CPU replica as the leader (its Replicates carry the entries) and as a
follower.  Every hosted replica is compared with the oracle every round.
"""
import pytest

from dragonboat_amd import abi
from dragonboat_amd.engine import DrbError
from oracle import pyoracle as po
from tests import wire_ref as wr
from tests.gpu_harness import DistPair

pytestmark = pytest.mark.gpu
DID = 0xD1D


def _host_elsewhere(p, slot):
    """Replica `slot` of every group leaves the engines (it runs on the CPU
    NodeHost: the oracle keeps stepping it)."""
    for r, e in enumerate(p.engs):
        sts = e.export_replicas(0, p.lanes)
        for j in range(p.lanes):
            sts[j * p.R + slot].flags &= ~abi.F_HOSTED
        e.import_replicas(0, sts)


def _cpu_sends(p, slot):
    """{rank: [msg]}: what the CPU replicas sent this round, by the rank of
    each receiver (group-major, send order within a destination)."""
    out = {r: [] for r in range(p.N)}
    for g in range(p.G):
        for t in p.orc.export_outbox(g, slot):
            m = wr.tuple_to_msg(t)
            out[(g + m["to"] - 1) % p.N].append(m)
    return out


@pytest.mark.parametrize("N,R,cpu_slot,via", [
    (2, 3, 0, "ingest"), (3, 3, 0, "wire"), (4, 5, 0, "ingest"),
    (2, 3, 2, "wire"), (3, 5, 4, "ingest")])
def test_cpu_nodehost_with_replicas_spread_over_ranks(N, R, cpu_slot, via):
    G = 8 * N
    # entry rows deep enough for a lagging follower's catch-up
    p = DistPair(G=G, R=R, N=N, E=8, max_props=2)
    _host_elsewhere(p, cpu_slot)
    mine = [s for s in range(R) if s != cpu_slot]
    sent = 0
    for r in range(10):
        o, e = p.round(k=1 + (r % 4 == 3), tick=(r % 2 == 0),
                       read_index=(cpu_slot != 0 and r % 3 == 0))
        assert e["fallbacks"] == 0 and e["errors"] == 0, (r, e, p.why())
        for rank, msgs in _cpu_sends(p, cpu_slot).items():
            if not msgs:
                continue
            sent += len(msgs)
            eng = p.engs[rank]
            if via == "ingest":
                marr, n, earr, pool = po.build_messages(msgs)
                acc, drop = eng.ingest(marr, n, earr, pool)
                assert (acc, drop) == (len(msgs), 0), (r, rank, acc, drop)
            else:
                got = eng.ingest_wire(wr.expected_stream(msgs, DID, b"cpu:1"),
                                      DID)
                assert got["accepted"] == len(msgs), (r, rank, got)
        errs = p.check(slots=mine)
        assert not errs, (r, errs[:2])
    assert sent > 0
    if cpu_slot == 0:  # the GPU followers applied what the CPU leader sent
        assert all(p.replica(g, s).sm_index == p.orc.export(g, s).sm_index > 3
                   for g in range(G) for s in mine)


def test_messages_for_other_ranks_are_dropped():
    """A rank takes only messages for replicas it hosts (the receiver's
    rank is (g + slot) mod N)."""
    p = DistPair(G=8, R=3, N=2, E=4)
    _host_elsewhere(p, 2)
    p.round(k=1, tick=True)
    msgs = [po.msg(abi.MSG["HeartbeatResp"], from_=3, to=1, term=2,
                   shard_id=1 + g) for g in range(8)]
    # group g's replica 1 (slot 0) is on rank g % 2: half of them are here
    acc, drop = p.engs[0].ingest(*po.build_messages(msgs))
    assert (acc, drop) == (4, 4)


@pytest.mark.parametrize("via", ["ingest", "wire"])
def test_ingest_waits_for_the_exchange(via):
    """Between a round's launch and its plane exchange the inbound planes
    still belong to the exchange: a transport's ingest then is refused with
    DRB_EAGAIN and places nothing (otherwise the exchange's copy of the
    plane's header would overwrite what it wrote); the same messages after
    the exchange land and are stepped bit-exact."""
    G, N, R = 16, 2, 3
    p = DistPair(G=G, R=R, N=N, E=8, max_props=2)
    _host_elsewhere(p, 0)  # the CPU NodeHost holds the leaders
    mine = [1, 2]
    refused = 0
    for r in range(8):
        o, e = p.round(k=1, tick=(r % 2 == 0), exchange=False)
        assert e["fallbacks"] == 0 and e["errors"] == 0, (r, e, p.why())
        sends = _cpu_sends(p, 0)
        for rank, msgs in sends.items():
            if not msgs:
                continue
            eng = p.engs[rank]
            with pytest.raises(DrbError, match="status -6"):
                if via == "ingest":
                    eng.ingest(*po.build_messages(msgs))
                else:
                    eng.ingest_wire(wr.expected_stream(msgs, DID, b"cpu:1"),
                                    DID)
            refused += 1
        p.exchange()
        for rank, msgs in sends.items():
            if not msgs:
                continue
            eng = p.engs[rank]
            if via == "ingest":
                acc, drop = eng.ingest(*po.build_messages(msgs))
            else:
                got = eng.ingest_wire(wr.expected_stream(msgs, DID, b"cpu:1"),
                                      DID)
                acc, drop = got["accepted"], got["dropped"]
            assert (acc, drop) == (len(msgs), 0), (r, rank, acc, drop)
        errs = p.check(slots=mine)
        assert not errs, (r, errs[:2])
    assert refused > 0
    assert all(p.replica(g, s).sm_index == p.orc.export(g, s).sm_index > 3
               for g in range(G) for s in mine)


@pytest.mark.parametrize("via", ["ingest", "wire"])
def test_entry_rows_overflow_goes_to_the_cpu_path(via):
    """The CPU NodeHost's leader sends Replicates whose entries a remote
    plane's entry rows cannot hold (entry_mbox = 1 row, two-entry rounds).
    The reference's inbox takes them (message.go:105-120); the engine hands
    each receiver's group to the CPU path (DRB_FB_CAPACITY) with the
    message instead of dropping it, the oracle -- which received exactly
    the engine's stream -- steps the group until it settles, and it comes
    back (drb_import_*).  The other groups stay bit-exact every round."""
    G, N, R = 16, 2, 3
    p = DistPair(G=G, R=R, N=N, E=1, max_props=2)
    _host_elsewhere(p, 0)  # the CPU NodeHost holds the leaders
    mine = [1, 2]
    went, came, diverted = set(), set(), 0
    for r in range(18):
        now = set()
        # (the last rounds without ticks: the CPU groups settle and return)
        o, e = p.round(k=2 if r in (2, 5) else 1, tick=(r % 2 == 0 and r < 14))
        assert e["fallbacks"] == 0 and e["errors"] == 0, (r, e, p.why())
        for rank, msgs in _cpu_sends(p, 0).items():
            if not msgs:
                continue
            eng = p.engs[rank]
            if via == "ingest":
                got = eng.ingest_ex(*po.build_messages(msgs))
                div = [po.msg_tuple(m) for m, f in zip(msgs, got["status"])
                       if f == abi.ING_DIVERTED]
            else:
                data = wr.expected_stream(msgs, DID, b"cpu:1")
                got = eng.ingest_wire(data, DID)
                div = [wr.message_tuple(data[o:o + n])
                       for o, n, f in eng.ingest_wire_cpu()]
            assert got["dropped"] == 0, (r, rank, got)
            assert got["accepted"] + got["diverted"] == len(msgs), got
            assert len(div) == got["diverted"]
            diverted += got["diverted"]
            for (j, s, reason, flags, _, _) in eng.take_flagged()[0]:
                assert reason == abi.FB["CAPACITY"], (j, s, reason)
                g = p.lane_group(rank, s, j)
                # the receiver's CPU inbox: what was placed, then the
                # diverted messages -- the CPU leader's sends to it
                inbox = [m for m in eng.export_inbox(j, s) if m[1] == 1] + \
                    [d for d in div if d[0] == g + 1 and d[2] == s + 1]
                want = [t for t in p.orc.export_outbox(g, 0) if t[2] == s + 1]
                assert inbox == want, (r, g, s)
                now.add(g)
        for g in sorted(now - p.cpu):
            p.to_cpu(g)
        went |= now
        errs = p.check(slots=mine)
        assert not errs, (r, errs[:2])
        for g in sorted(p.cpu):
            if p.settled(g):
                p.from_cpu(g)
                came.add(g)
    assert diverted and went and came == went and not p.cpu, \
        (diverted, went, came, p.cpu)
    assert all(p.replica(g, s).sm_index == p.orc.export(g, s).sm_index > 3
               for g in range(G) for s in mine)
