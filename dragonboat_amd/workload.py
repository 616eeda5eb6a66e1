"""Synthetic inputs of SURVEY.md 8(d), defined bit-exactly.

The same definition is implemented on the device by drb_gen_kv_proposals /
drb_gen_read_index (dragonboat_amd/csrc/drb_engine.hip); this module builds
the identical records on the host so tests can stage them through
drb_stage_proposals and compare.

Per group g, batch salt s, proposal j (k per group per round):
  r0 = mix64(seed ^ (g * GOLDEN) ^ (s << 32) ^ (j << 16))
  r1 = mix64(r0); r2 = mix64(r1)
  Entry.Key      = r0 | 1                   (request.go:1047, non-zero)
  Entry.ClientID = mix64(seed ^ CLIENT ^ g) | 1   NoOP session
  SeriesID = RespondedTo = 0, Type = EncodedEntry (encoded.go:83-93)
  Cmd = 0x00 || PBKV{key = LE64(r1 % key_space), val = bytes of r2 chain}
"""
import struct

import ctypes as C

from .abi import ENTRY_ENCODED, Entry

MASK = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
CLIENT = 0xC11E47C11E47C11E
RI_SALT = 0x5EAD1DE85EAD1DE8
ACTIVE_SALT = 0xAC71BE5EAC71BE5E


def mix64(z):
    z = (z + GOLDEN) & MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return z ^ (z >> 31)


def client_id(seed, g):
    return mix64(seed ^ CLIENT ^ g) | 1


def varint(n):
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7f) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def pbkv16(key8, val):
    """PBKV{Key, Val} (internal/tests/kvpb/kv.go) -- 16 B at the default
    4-byte value; longer values take a multi-byte length varint."""
    return b"\x0a" + varint(len(key8)) + key8 + b"\x12" + varint(len(val)) \
        + val


def proposal(seed, g, s, j, key_space, val_len):
    r0 = mix64(seed ^ ((g * GOLDEN) & MASK) ^ ((s << 32) & MASK) ^ (j << 16))
    r1 = mix64(r0)
    r2 = mix64(r1)
    key8 = struct.pack("<Q", r1 % key_space)
    vb = b""
    x = r2
    while len(vb) < val_len:
        vb += struct.pack("<Q", x)
        x = mix64(x)
    cmd = b"\x00" + pbkv16(key8, vb[:val_len])
    return dict(key=r0 | 1, client_id=client_id(seed, g), series_id=0,
                responded_to=0, type=ENTRY_ENCODED, cmd=cmd)


def build_batch(num_groups, k, seed, salt, key_space=256, val_len=4,
                groups=None, gids=None):
    """Returns (counts[u32 G], ents[Entry G*k], pool).  gids: entry i
    carries the proposals of global group gids[i] (a sampled cluster)."""
    counts = (C.c_uint32 * num_groups)()
    ents = (Entry * max(1, num_groups * k))()
    pool = bytearray()
    gs = range(num_groups) if groups is None else groups
    for g in gs:
        counts[g] = k
        gg = g if gids is None else gids[g]
        for j in range(k):
            p = proposal(seed, gg, salt, j, key_space, val_len)
            ents[g * k + j] = Entry(0, 0, p["key"], p["client_id"], 0, 0,
                                    p["type"], len(p["cmd"]), len(pool))
            pool += p["cmd"]
    pbuf = (C.c_uint8 * max(1, len(pool))).from_buffer_copy(bytes(pool) or
                                                           b"\0")
    return counts, ents, pbuf


def _mix64_np(z):
    import numpy as np
    z = z + np.uint64(GOLDEN)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def build_batch_np(num_groups, seed, salt, key_space=256):
    """build_batch(num_groups, 1, seed, salt, key_space, 4) vectorised with
    numpy (the bench's host-staged rounds at 1M groups): the same Entry
    rows and Cmd pool, 17 B per group (0x00 || PBKV{8 B key, 4 B value})."""
    import numpy as np
    with np.errstate(over="ignore"):
        g = np.arange(num_groups, dtype=np.uint64)
        r0 = _mix64_np(np.uint64(seed) ^ (g * np.uint64(GOLDEN)) ^
                       np.uint64((salt << 32) & MASK))
        r1 = _mix64_np(r0)
        r2 = _mix64_np(r1)
        cid = _mix64_np(np.uint64(seed ^ CLIENT) ^ g) | np.uint64(1)
    ents = np.zeros(num_groups, dtype=np.dtype(
        [("term", "<u8"), ("index", "<u8"), ("key", "<u8"),
         ("client_id", "<u8"), ("series_id", "<u8"), ("responded_to", "<u8"),
         ("type", "<u4"), ("cmd_len", "<u4"), ("cmd_off", "<u8")]))
    assert ents.dtype.itemsize == C.sizeof(Entry)
    ents["key"] = r0 | np.uint64(1)
    ents["client_id"] = cid
    ents["type"] = ENTRY_ENCODED
    ents["cmd_len"] = 17
    ents["cmd_off"] = g * np.uint64(17)
    pool = np.zeros((num_groups, 17), dtype=np.uint8)
    pool[:, 1:3] = (0x0A, 8)
    pool[:, 3:11] = (r1 % np.uint64(key_space)).view(np.uint8).reshape(-1, 8)
    pool[:, 11:13] = (0x12, 4)
    pool[:, 13:17] = r2.view(np.uint8).reshape(-1, 8)[:, :4]
    counts = np.ones(num_groups, dtype=np.uint32)
    return counts, ents, pool.reshape(-1)


def read_index_ctx(seed, g, salt, high):
    """pendingReadIndex.genCtx (request.go:864-875): Low random non-zero."""
    low = mix64(seed ^ RI_SALT ^ ((g * GOLDEN) & MASK) ^ (salt << 40)) | 1
    return low, high


def build_read_index(num_groups, seed, salt, high, groups=None, gids=None):
    lo = (C.c_uint64 * num_groups)()
    hi = (C.c_uint64 * num_groups)()
    gs = range(num_groups) if groups is None else groups
    for g in gs:
        lo[g], hi[g] = read_index_ctx(seed, g if gids is None else gids[g],
                                      salt, high)
    return lo, hi


def active_groups(num_groups, seed, salt, active_ppm, gids=None):
    """The seeded Bernoulli subset of groups that propose in batch `salt`
    (drb_gen_kv_proposals_active; SURVEY 8d C5: 1 % active per round);
    with gids, the indices i whose global group gids[i] is active."""
    if active_ppm >= 1000000:
        return list(range(num_groups))
    return [g for g in range(num_groups)
            if mix64(seed ^ ACTIVE_SALT ^
                     (((g if gids is None else gids[g]) * GOLDEN) & MASK) ^
                     ((salt << 24) & MASK)) % 1000000 < active_ppm]


def pack_batch(num_groups, k, counts, ents, pool):
    """A build_batch batch (NoOP-session entries) in the packed form of
    drb_stage_proposals_packed: (counts u8[G], keys u64[n], clients u64[n],
    lens u16[n], pool bytes), entries group by group."""
    cnt = (C.c_uint8 * max(1, num_groups))()
    keys, cids, lens, out = [], [], [], bytearray()
    pb = bytes(pool)
    for g in range(num_groups):
        cnt[g] = counts[g]
        for j in range(counts[g]):
            e = ents[g * k + j]
            keys.append(e.key)
            cids.append(e.client_id)
            lens.append(e.cmd_len)
            out += pb[e.cmd_off:e.cmd_off + e.cmd_len]
    n = len(keys)
    return (cnt, n, (C.c_uint64 * max(1, n))(*keys),
            (C.c_uint64 * max(1, n))(*cids), (C.c_uint16 * max(1, n))(*lens),
            (C.c_uint8 * max(1, len(out))).from_buffer_copy(bytes(out) or
                                                            b"\0"), len(out))


def build_packed_np(num_groups, seed, salt, key_space=256):
    """build_batch_np's batch in the packed form (numpy arrays): what a
    host uploads per round with drb_stage_proposals_packed."""
    import numpy as np
    counts, ents, pool = build_batch_np(num_groups, seed, salt, key_space)
    return (counts.astype(np.uint8), np.ascontiguousarray(ents["key"]),
            np.ascontiguousarray(ents["client_id"]),
            ents["cmd_len"].astype(np.uint16), pool)
