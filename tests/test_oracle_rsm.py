"""rsm known-answer tests restated from the reference's own test files:

  internal/rsm/encoded_test.go:34-96     GetPayload / GetEncoded round trips
  internal/rsm/statemachine_test.go:316  TestUpdatesCanBeBatched
  internal/rsm/statemachine_test.go:1048 testHandleSnappyEncodedEntry
  internal/rsm/statemachine_test.go:1086 TestHandleUpate
  internal/rsm/statemachine_test.go:1425 TestNoOPSessionAllowEntryToBeAppliedTwice

They pin the oracle's apply path (oracle/node_oracle.c get_payload /
sm_handle, statemachine.go + encoded.go + KVTest).  The snappy block
decoder restates github.com/golang/snappy v0.0.4 (a go.mod dependency not
vendored under /root/reference); the encoder below is the literal-only
form golang/snappy's Encode emits for inputs shorter than its 17-byte
minNonLiteralBlockSize, so the encoded bytes of these KATs are exact.

Regular client sessions (register / series != NoOP) are not on the GPU
fast path: the oracle raises for them and the GPU leader falls back before
appending (DRB_FB_ENTRY_TYPE, tests/test_gpu_fallback.py "session").
"""
import os

import pytest

from oracle import pyoracle as po
from dragonboat_amd.abi import (ENTRY_APPLICATION, ENTRY_CONFIG_CHANGE,
                                ENTRY_ENCODED)

# encoded.go:31-47
EEV0, EE_NO_COMPRESSION, EE_SNAPPY, EE_HAS_SESSION = 0, 0, 1 << 1, 1
NO_COMPRESSION, SNAPPY = 0, 1          # dio.CompressionType
SERIES_ID_FOR_REGISTER = (1 << 64) - 2  # client/session.go
NOOP_SERIES_ID = 0


def uvarint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def snappy_literal_block(src):
    """golang/snappy Encode for len(src) < 17: uvarint(len) + one literal."""
    assert 0 < len(src) < 17
    return uvarint(len(src)) + bytes([(len(src) - 1) << 2]) + src


def snappy_max_encoded_len(n):  # golang/snappy MaxEncodedLen
    return 32 + n + n // 6


def get_encoded(ct, cmd):
    """GetEncoded / getEncoded (encoded.go:73-112), header via
    getEncodedHeader (:114-125)."""
    if not cmd:
        raise ValueError("empty payload")
    if ct == NO_COMPRESSION:
        return bytes([EEV0 | EE_NO_COMPRESSION]) + cmd
    return bytes([EEV0 | EE_SNAPPY]) + snappy_literal_block(cmd)


def parse_encoded_header(cmd):  # encoded.go:119-125
    h = cmd[0]
    return h & 0xF0, h & 0x0E, (h & 1) == 1


def pbkv(k, v):
    return po.pbkv_marshal(k, v)


def test_get_entry_payload():
    # encoded_test.go:34-45
    e1 = bytes([1, 2, 3, 4, 5])
    assert po.get_payload(ENTRY_APPLICATION, e1) == e1
    e2 = bytes([1, 2, 3])
    assert po.get_payload(ENTRY_CONFIG_CHANGE, e2) == e2
    e3 = bytes(range(1, 10))
    assert po.get_payload(ENTRY_ENCODED, get_encoded(SNAPPY, e3)) == e3


L1 = snappy_max_encoded_len(16)


@pytest.mark.parametrize("ct,src,dst", [
    (NO_COMPRESSION, 16, 0), (NO_COMPRESSION, 16, 1), (NO_COMPRESSION, 16, 16),
    (NO_COMPRESSION, 16, 17), (SNAPPY, 16, 0), (SNAPPY, 16, 1),
    (SNAPPY, 16, 16), (SNAPPY, 16, L1), (SNAPPY, 16, L1 - 1),
    (SNAPPY, 16, L1 + 1), (SNAPPY, 16, 128)])
def test_get_v0_encoded_payload(ct, src, dst):
    # encoded_test.go:47-96; dst only decides whether GetEncoded reuses the
    # caller's buffer, the encoded bytes are the same for every row
    data = os.urandom(src)
    result = get_encoded(ct, data)
    ver, got_ct, has_session = parse_encoded_header(result)
    assert ver == EEV0 and not has_session
    assert got_ct == (EE_NO_COMPRESSION if ct == NO_COMPRESSION else EE_SNAPPY)
    assert po.get_payload(ENTRY_ENCODED, result) == data


def test_snappy_copy_elements():
    """Copy elements with 1- and 2-byte offsets, including an overlapping
    copy (golang/snappy decode.go); decoded "abcd" * 5 + "xyz" + "xyzxyz"."""
    want = b"abcd" * 5 + b"xyzxyzxyz"
    blk = uvarint(len(want))
    blk += bytes([3 << 2]) + b"abcd"                  # literal "abcd"
    blk += bytes([((8 - 4) << 2) | 1, 4])             # copy1 len 8 off 4
    blk += bytes([((8 - 1) << 2) | 2, 4, 0])          # copy2 len 8 off 4
    blk += bytes([2 << 2]) + b"xyz"                   # literal "xyz"
    blk += bytes([((6 - 4) << 2) | 1, 3])             # overlapping copy
    assert po.get_payload(ENTRY_ENCODED, bytes([EE_SNAPPY]) + blk) == want


@pytest.mark.parametrize("cmd", [
    bytes([0x10, 1, 2]),          # version 1
    bytes([EE_HAS_SESSION, 1]),   # v0 with the session flag
    bytes([0x04, 1, 2]),          # compression type 2 (unknown)
    b"",                          # empty encoded Cmd
])
def test_get_payload_panics(cmd):
    # encoded.go:127-160: plog.Panicf / panic on these headers
    with pytest.raises(po.OracleError):
        po.get_payload(ENTRY_ENCODED, cmd)


def test_updates_can_be_batched():
    # statemachine_test.go:316-356: three NoOP-session entries at 235..237
    sm = po.StateMachine(234, 0)
    ents = [po.ent(client_id=123, series_id=NOOP_SERIES_ID, index=i, term=1)
            for i in (235, 236, 237)]
    assert sm.handle(ents) == 3
    assert sm.last_applied == 237


@pytest.mark.parametrize("ct", [SNAPPY, NO_COMPRESSION])
def test_handle_snappy_encoded_entry(ct):
    # statemachine_test.go:1048-1079
    data = pbkv(b"test-key", b"test-value")
    if ct == SNAPPY:  # > 16 bytes: build a valid block by hand (literals)
        blk = uvarint(len(data))
        for i in range(0, len(data), 16):
            chunk = data[i:i + 16]
            blk += bytes([(len(chunk) - 1) << 2]) + chunk
        cmd = bytes([EE_SNAPPY]) + blk
    else:
        cmd = get_encoded(ct, data)
    sm = po.StateMachine(234, 0)
    e = po.ent(type=ENTRY_ENCODED, client_id=123, series_id=NOOP_SERIES_ID,
               index=235, term=1, cmd=cmd)
    assert sm.handle([e]) == 1
    assert sm.last_applied == 235
    assert sm.lookup(b"test-key") == b"test-value"


def test_handle_update():
    # statemachine_test.go:1086-1117.  The register entry (235) opens a
    # regular client session, which is not on the fast path: the oracle
    # raises and the GPU falls back (DRB_FB_ENTRY_TYPE).  The update
    # itself, carried as a NoOP-session entry, stores the pair.
    sm = po.StateMachine(234, 0)
    with pytest.raises(po.OracleError):
        sm.handle([po.ent(client_id=123, series_id=SERIES_ID_FOR_REGISTER,
                          index=235, term=1)])
    sm = po.StateMachine(235, 1)
    data = pbkv(b"test-key", b"test-value")
    assert sm.handle([po.ent(client_id=123, series_id=NOOP_SERIES_ID,
                             cmd=data, index=236, term=1)]) == 1
    assert sm.last_applied == 236
    assert sm.lookup(b"test-key") == b"test-value"
    with pytest.raises(po.OracleError):  # series 2 = a regular session
        po.StateMachine(236, 1).handle([po.ent(client_id=123, series_id=2,
                                               cmd=data, index=237, term=1)])


def test_noop_session_allow_entry_to_be_applied_twice():
    # statemachine_test.go:1425-1445
    sm = po.StateMachine(789, 1)
    data = pbkv(b"test-key", b"test-value")
    sm.handle([po.ent(client_id=12345, series_id=NOOP_SERIES_ID, index=790,
                      term=1, cmd=data)])
    assert sm.last_applied == 790
    count = sm.count
    sm.handle([po.ent(client_id=12345, series_id=NOOP_SERIES_ID, index=791,
                      term=1, cmd=data)])
    assert sm.last_applied == 791
    assert sm.count != count
