"""CPU checks of the expected-stream builder the GPU wire tests use
(tests/wire_ref.py): the processMessages batch cut and the frame parser,
on messages the oracle cluster sends."""
from oracle import pyoracle as po
from tests import wire_ref as wr


def _cluster_plane(G=12, rounds=3):
    from dragonboat_amd import workload
    c = po.Cluster(G, 3, seed=0x5EEDD8B0)
    c.setup_steady(0)
    for r in range(rounds):
        counts, ents, pool = workload.build_batch(G, 2, 0x5EEDD8B0, r, 256,
                                                  4, None)
        c.stage_proposals(counts, 2, ents, pool)
        c.round(tick=True)
    return wr.plane_messages(c.export_outbox, G, 0, 1)


def test_split_rule_cases():
    msgs = _cluster_plane()
    assert msgs and all(m["to"] == 2 for m in msgs)
    ul = [wr.size_upper_limit(m) for m in msgs]
    # one batch when the limit is never reached
    assert wr.split_batches(msgs) == [msgs]
    # a limit below any single message: every message alone
    assert wr.split_batches(msgs, 1) == [[m] for m in msgs]
    # twoBatch: the message that reaches the limit travels alone
    lim = ul[0] + ul[1] + 1
    b = wr.split_batches(msgs, lim)
    assert b[0] == msgs[:2] and b[1] == [msgs[2]]
    assert sum(len(x) for x in b) == len(msgs)


def test_expected_stream_parses_back():
    msgs = _cluster_plane()
    for lim in (wr.MAX_MSG_BATCH, 1, 700):
        data = wr.expected_stream(msgs, 77, b"10.1.2.3:63000", lim)
        got = []
        for p in wr.parse_stream(data):
            ms, did, src, bv = po.messagebatch_unmarshal(p)
            assert (did, src, bv) == (77, b"10.1.2.3:63000", 210)
            got += ms
        assert got == msgs
