"""Expected TCP byte streams for drb_encode_wire, built from the oracle.

Transport.processMessages (internal/transport/transport.go:443-508) with
the send queue drained in one go: requests accumulate while the running
sum of Message.SizeUpperLimit (raft_optimized.go:1210-1221) stays below
MaxMessageBatchSize; the request that reaches it travels alone in a second
batch (`twoBatch`), unless it is the first of the batch.  Each batch is
framed by writeMessage (tcp.go:142-178).  Test infrastructure only.
"""
import struct
import zlib

from oracle import pyoracle as po

MAX_MSG_BATCH = 64 * 1024 * 1024  # settings/hard.go:95 (LargeEntitySize)
ENTRY_NON_CMD = 16 * 8            # settings/soft.go:20


def tuple_to_msg(t):
    es = [po.ent(term=e[0], index=e[1], type=e[2], key=e[3], client_id=e[4],
                 series_id=e[5], responded_to=e[6], cmd=e[7]) for e in t[11]]
    return po.msg(t[3], from_=t[1], to=t[2], term=t[4], log_term=t[5],
                  log_index=t[6], commit=t[7], reject=bool(t[8]), hint=t[9],
                  hint_high=t[10], entries=es, shard_id=t[0])


def size_upper_limit(m):
    """Message.SizeUpperLimit with the empty Snapshot (24 B)."""
    return 16 * 12 + 24 + sum(16 + ENTRY_NON_CMD + len(e["cmd"])
                              for e in m["entries"])


def split_batches(msgs, max_batch=MAX_MSG_BATCH):
    out, s, n = [], 0, len(msgs)
    while s < n:
        sz, j = 0, s
        while j < n:
            sz += size_upper_limit(msgs[j])
            if sz >= max_batch:
                break
            j += 1
        if j >= n:
            out.append(msgs[s:])
            s = n
        elif j == s:
            out.append(msgs[s:s + 1])
            s += 1
        else:
            out.append(msgs[s:j])
            out.append(msgs[j:j + 1])
            s = j + 1
    return out


def plane_messages(outbox_of, G, frm, to):
    """Messages replica slot frm sent to slot to, group-major."""
    res = []
    for g in range(G):
        for t in outbox_of(g, frm):
            if t[2] == to + 1:
                res.append(tuple_to_msg(t))
    return res


def expected_stream(msgs, deployment_id, source, max_batch=MAX_MSG_BATCH,
                    bin_ver=po.TRANSPORT_BIN_VERSION):
    return b"".join(
        po.wire_frame(po.messagebatch_marshal(b, deployment_id, source,
                                              bin_ver))
        for b in split_batches(msgs, max_batch))


def _varint(d, i):
    v = s = 0
    while True:
        b = d[i]
        i += 1
        v |= (b & 0x7f) << s
        s += 7
        if b < 0x80:
            return v, i


def message_tuple(data):
    """pb.Message.Unmarshal (raft.pb.go field numbers, message.go:6-20) of
    one marshalled Requests element, as abi.message_to_tuple: an
    independent proto2 walk, colfer entries through the oracle codec."""
    f = dict(type=0, to=0, from_=0, shard_id=0, term=0, log_term=0,
             log_index=0, commit=0, reject=0, hint=0, hint_high=0)
    names = {1: "type", 2: "to", 3: "from_", 4: "shard_id", 5: "term",
             6: "log_term", 7: "log_index", 8: "commit", 9: "reject",
             10: "hint", 13: "hint_high"}
    ents, i = [], 0
    while i < len(data):
        key, i = _varint(data, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(data, i)
            f[names[fn]] = v
        else:
            assert wt == 2, (fn, wt)
            n, i = _varint(data, i)
            if fn == 11:
                e, used = po.entry_unmarshal(data[i:i + n])
                assert used == n
                ents.append(e)
            i += n
    m = po.msg(f["type"], from_=f["from_"], to=f["to"], term=f["term"],
               log_term=f["log_term"], log_index=f["log_index"],
               commit=f["commit"], reject=bool(f["reject"]), hint=f["hint"],
               hint_high=f["hint_high"], entries=ents, shard_id=f["shard_id"])
    return po.msg_tuple(m)


def parse_stream(data):
    """Splits a stream into payloads, checking magic, the header CRC and
    the payload CRC with zlib (independent of the oracle)."""
    out, i = [], 0
    while i < len(data):
        assert data[i:i + 2] == b"\xae\x7d", i
        h = data[i + 2:i + 20]
        method, size = struct.unpack(">HQ", h[:10])
        hcrc, pcrc = struct.unpack(">II", h[10:18])
        assert method == 100
        assert hcrc == zlib.crc32(h[:10] + b"\0\0\0\0" + h[14:]), i
        payload = data[i + 20:i + 20 + size]
        assert len(payload) == size
        assert pcrc == zlib.crc32(payload), i
        out.append(payload)
        i += 20 + size
    return out
