"""CPU: the host part of drb_ingest_wire under AddressSanitizer and UBSan.

drb_wirehost.hpp is the host's share of the receive path (tcp.go:180-237
readMessage's frame headers; MessageBatch.Unmarshal's top-level walk,
raft_optimized.go:1056-1207; the payload CRC folded from 16 KB chunk CRCs;
the 2-byte step packing).  tests/native/wirewalk.cpp drives it, built here
with -fsanitize=address,undefined, over:

- the planes of an oracle cluster as dragonboat's TCP stream (R = 3 and 5,
  16 B to 1 KB payloads, batch cuts that force every batch shape), compared
  with an independent Python walk: every frame, its CRC, DeploymentId,
  BinVer and the offset of every Requests element;
- a Requests element over 64 KB (4-byte steps, a 3-byte length varint);
- every truncation of a stream, over-long and unterminated varints, element
  lengths past the frame's end, truncated fixed-width fields, flipped bytes
  and seeded random payloads behind valid headers: no sanitizer report, and
  what is delivered is only whole, intact frames.

Round 4's one host crash in this path (a test's segfault inside
drb_ingest_wire) was an out-of-bounds read: the first call of an engine with
a stream holding no whole frame recorded st.ev[0] of an empty event vector
(DESIGN.md §7a); drb_ingest_wire now creates that event before any piece.
"""
import os
import random
import shutil
import struct
import subprocess
import zlib

import pytest

from dragonboat_amd import abi, workload
from oracle import pyoracle as po
from tests import wire_ref as wr

HERE = os.path.dirname(os.path.abspath(__file__))
DID = 0xD1D


@pytest.fixture(scope="module")
def walker(tmp_path_factory):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("wirewalk") / "wirewalk")
    subprocess.check_call([
        gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
        "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-pthread",
        "-o", out, os.path.join(HERE, "native", "wirewalk.cpp")])
    return out


def run_walk(walker, data, tmp_path, name="s.bin"):
    p = tmp_path / name
    p.write_bytes(data)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([walker, str(p)], capture_output=True, text=True,
                       env=env, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    assert "runtime error" not in r.stderr, r.stderr[-3000:]
    frames, walked, bad = [], None, None
    for line in r.stdout.splitlines():
        w = line.split()
        if w[0] == "frame":
            off, size, method, crc_ok, scan_ok, did, bv, wide = map(int, w[1:9])
            frames.append(dict(off=off, size=size, method=method,
                               crc_ok=crc_ok, scan_ok=scan_ok, did=did, bv=bv,
                               wide=wide, steps=[int(x) for x in w[9:]]))
        else:
            walked, bad = int(w[1]), int(w[3])
    return frames, walked, bad


# ----------------------------------------------- independent Python walk
def _varint(b, i):
    v = s = 0
    while True:
        if i >= len(b) or s > 63:
            raise ValueError("varint")
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, i


def py_frames(data):
    """(payload offset, payload, method) of the whole, intact frames."""
    out, i = [], 0
    while i + 20 <= len(data) and data[i:i + 2] == b"\xae\x7d":
        h = data[i + 2:i + 20]
        method, size = struct.unpack(">HQ", h[:10])
        hcrc, pcrc = struct.unpack(">II", h[10:18])
        if hcrc != zlib.crc32(h[:10] + b"\0\0\0\0" + h[14:]) or size == 0 \
                or size > len(data) - i - 20 or method not in (100, 200):
            break
        out.append((i + 20, data[i + 20:i + 20 + size], method, pcrc))
        i += 20 + size
    return out


def py_batch(p):
    """MessageBatch top-level fields: Requests element tag offsets,
    DeploymentId, BinVer (raft.proto field numbers 1, 2, 4)."""
    elems, did, bv, i = [], 0, 0, 0
    while i < len(p):
        at = i
        key, i = _varint(p, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(p, i)
            v &= (1 << 64) - 1
            if f == 2:
                did = v
            elif f == 4:
                bv = v
        elif wt in (1, 5):
            i += 8 if wt == 1 else 4
            if i > len(p):
                raise ValueError("fixed")
        elif wt == 2:
            n, i = _varint(p, i)
            if n > len(p) - i:
                raise ValueError("length")
            if f == 1:
                elems.append(at)
            i += n
        else:
            raise ValueError("wire type")
    return elems, did, bv


def check_valid(walker, data, tmp_path):
    frames, walked, bad = run_walk(walker, data, tmp_path)
    want = py_frames(data)
    assert (walked, bad) == (len(data), 0)
    assert len(frames) == len(want)
    for f, (off, payload, method, pcrc) in zip(frames, want):
        assert (f["off"], f["size"], f["method"]) == (off, len(payload),
                                                      method)
        assert f["crc_ok"] == 1 and zlib.crc32(payload) == pcrc
        assert f["scan_ok"] == 1
        elems, did, bv = py_batch(payload)
        at, got = 0, []
        for s in f["steps"]:
            at += s
            got.append(at)
        assert got == elems
        assert (f["did"], f["bv"]) == (did, bv)
        assert f["wide"] == int(any(b - a >= 1 << 16 for a, b in
                                    zip([0] + elems, elems)))
    return frames


def cluster_planes(R, val_len, rounds=4, G=24):
    orc = po.Cluster(G, R)
    orc.setup_steady(0)
    msgs = []
    for r in range(rounds):
        counts, ents, pool = workload.build_batch(G, 1 + r % 2, 0x5EEDD8B0,
                                                  r, 256, val_len)
        orc.stage_proposals(counts, 1 + r % 2, ents, pool)
        lo, hi = workload.build_read_index(G, 0x5EEDD8B0, r, r + 30)
        orc.stage_read_index(lo, hi)
        orc.round(tick=r % 2 == 0)
        for to in range(1, R):
            msgs += wr.plane_messages(orc.export_outbox, G, 0, to)
        msgs += wr.plane_messages(orc.export_outbox, G, 1, 0)
    return msgs


@pytest.mark.parametrize("R,val_len", [(3, 4), (5, 60), (3, 1011)])
def test_cluster_streams(walker, tmp_path, R, val_len):
    msgs = cluster_planes(R, val_len)
    assert msgs
    for cut in (wr.MAX_MSG_BATCH, 4096, 1500, 700):
        data = wr.expected_stream(msgs, DID, b"10.0.0.9:26001", cut)
        frames = check_valid(walker, data, tmp_path)
        if cut == 700:
            assert len(frames) > 4


def test_element_over_64k(walker, tmp_path):
    big = po.msg(abi.MSG["Replicate"], from_=1, to=2, term=2, log_index=7,
                 log_term=2, commit=6, shard_id=3,
                 entries=[po.ent(term=2, index=8, type=2, key=5, client_id=9,
                                 cmd=bytes(range(256)) * 280)])
    small = po.msg(abi.MSG["HeartbeatResp"], from_=2, to=1, term=2,
                   shard_id=3)
    data = wr.expected_stream([small, big, small], DID, b"a:1")
    frames = check_valid(walker, data, tmp_path)
    assert frames[0]["wide"] == 1


def test_every_truncation(walker, tmp_path):
    msgs = cluster_planes(3, 4, rounds=2, G=6)
    data = wr.expected_stream(msgs, DID, b"x:1", 600)
    whole = py_frames(data)
    ends = [off + len(p) for off, p, _, _ in whole]
    cuts = sorted(set(list(range(0, 48)) + ends +
                      [e - 1 for e in ends] +
                      random.Random(7).sample(range(len(data)), 40)))
    for c in cuts:
        frames, walked, bad = run_walk(walker, data[:c], tmp_path)
        n_whole = sum(1 for e in ends if e <= c)
        assert len(frames) == n_whole, c
        assert walked == (ends[n_whole - 1] if n_whole else 0)
        assert bad == 0, c  # a cut frame is still arriving, not bad
        assert all(f["crc_ok"] and f["scan_ok"] for f in frames)


def _frame(payload, method=100, good_crc=True):
    h = struct.pack(">HQ", method, len(payload))
    pcrc = zlib.crc32(payload) ^ (0 if good_crc else 1)
    hdr = h + b"\0\0\0\0" + struct.pack(">I", pcrc)
    hcrc = zlib.crc32(hdr)
    return b"\xae\x7d" + h + struct.pack(">I", hcrc) + struct.pack(">I", pcrc)


def test_malformed_payloads(walker, tmp_path):
    ok = po.messagebatch_marshal([po.msg(abi.MSG["Heartbeat"], from_=1, to=2,
                                         term=2, shard_id=1)], DID, b"s:1")
    bad_payloads = [
        b"\x0a" + b"\xff" * 11,                 # over-long length varint
        b"\x0a\xff\xff",                         # unterminated varint
        b"\x0a\x20" + b"\x00" * 5,               # element past the end
        b"\x0a\x81\x01" + b"\x00" * 10,          # 2-byte length, too long
        b"\x10" + b"\xff" * 10 + b"\x01",       # over-long DeploymentId
        b"\x19" + b"\x00" * 3,                   # fixed64 field cut short
        b"\x1d\x00",                              # fixed32 field cut short
        b"\x0b\x00",                              # group wire type
        b"\x00\x00",                              # field 0
        b"\xff" * 16,                             # garbage tag
        ok + b"\x0a",                             # trailing bare tag
        ok[:-1],                                  # cut element
    ]
    for p in bad_payloads:
        data = _frame(ok) + ok + _frame(p) + p + _frame(ok) + ok
        frames, walked, bad = run_walk(walker, data, tmp_path)
        assert (walked, bad) == (len(data), 0)
        assert [f["scan_ok"] for f in frames] == [1, 0, 1], p
        assert all(f["crc_ok"] for f in frames)
    # a payload CRC that does not match, a header CRC that does not
    data = _frame(ok, good_crc=False) + ok
    frames, walked, bad = run_walk(walker, data, tmp_path)
    assert [f["crc_ok"] for f in frames] == [0]
    hdr = bytearray(_frame(ok) + ok)
    hdr[5] ^= 1
    frames, walked, bad = run_walk(walker, bytes(hdr), tmp_path)
    assert (frames, walked, bad) == ([], 0, 1)
    # a tail shorter than a header: still arriving if its magic is sound,
    # bad if not
    whole = _frame(ok) + ok
    for tail, want in ((b"\xae", 0), (b"\xae\x7d\x00", 0), (b"\xae\x00", 1),
                       (b"\x00", 1), (b"\xae\x7d" + b"\x00" * 17, 0)):
        frames, walked, bad = run_walk(walker, whole + tail, tmp_path)
        assert (len(frames), walked, bad) == (1, len(whole), want), tail


def test_random_payloads(walker, tmp_path):
    """Seeded fuzz: random bytes, flipped bytes of a real batch and random
    varint soup behind valid headers; a sanitizer report fails the run."""
    rng = random.Random(0x5EED)
    msgs = cluster_planes(3, 60, rounds=2, G=4)
    real = po.messagebatch_marshal(msgs[:20], DID, b"f:1")
    parts = []
    for k in range(300):
        kind = k % 3
        if kind == 0:
            p = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 200)))
        elif kind == 1:
            b = bytearray(real)
            for _ in range(rng.randrange(1, 6)):
                b[rng.randrange(len(b))] = rng.randrange(256)
            p = bytes(b)
        else:
            p = b"".join(bytes([rng.choice([0x0a, 0x10, 0x12, 0x20, 0x80,
                                            0xff, 0x01])])
                         for _ in range(rng.randrange(1, 64)))
        parts.append(_frame(p) + p)
    data = b"".join(parts)
    frames, walked, bad = run_walk(walker, data, tmp_path)
    assert (len(frames), walked, bad) == (300, len(data), 0)
    for f, part in zip(frames, parts):
        p = part[20:]
        try:
            elems, did, bv = py_batch(p)
            ok = True
        except ValueError:
            ok = False
        if f["scan_ok"]:  # what the walk accepts, the independent one does
            assert ok
            at, got = 0, []
            for s in f["steps"]:
                at += s
                got.append(at)
            assert got == elems and (f["did"], f["bv"]) == (did, bv)
