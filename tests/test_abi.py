"""The C-ABI boundary without a GPU: include/drb_engine.h, the ctypes
mirror (dragonboat_amd/abi.py, engine.SIGNATURES) and the built engine
library must agree symbol-for-symbol and byte-for-byte.

No compute call is made here -- loading the library needs no device.
"""
import ctypes as C
import os
import re
import subprocess

import pytest

from dragonboat_amd import abi, engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "drb_engine.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"^[A-Za-z_][\w \*]*?\b(drb_\w+)\s*\(", src,
                          flags=re.M))


def test_header_declares_every_binding():
    assert header_functions() == set(engine.SIGNATURES)


def test_library_exports_every_declared_symbol():
    if not os.path.exists(engine.LIB_PATH):
        from dragonboat_amd import build
        build.build()
    L = C.CDLL(engine.LIB_PATH)
    missing = [n for n in header_functions() if not hasattr(L, n)]
    assert not missing
    out = subprocess.run(["nm", "-D", "--defined-only", engine.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert header_functions() <= exported


def test_library_loads_through_binding():
    lib = engine.lib()
    for name in engine.SIGNATURES:
        assert getattr(lib, name).argtypes is not None


STRUCTS = {
    "drb_remote_state": abi.RemoteState,
    "drb_read_status": abi.ReadStatus,
    "drb_replica_state": abi.ReplicaState,
    "drb_entry": abi.Entry,
    "drb_message": abi.Message,
    "drb_ready_to_read": abi.ReadyToRead,
    "drb_config": abi.Config,
    "drb_round_in": abi.RoundIn,
    "drb_round_out": abi.RoundOut,
    "drb_wire_cfg": abi.WireCfg,
    "drb_wire_out": abi.WireOut,
    "drb_wire_in": abi.WireIn,
    "drb_flagged": abi.Flagged,
    "drb_apply_result": abi.ApplyResult,
    "drb_save_record": abi.SaveRecord,
    "drb_tan_record": abi.TanRecord,
    "drb_tan_state": abi.TanState,
    "drb_tan_log": abi.TanLog,
    "drb_wire_cpu": abi.WireCpu,
    "drb_worker_bufs": abi.WorkerBufs,
    "drb_region": abi.Region,
    "drb_xfer": abi.Xfer,
}
# ctypes field names that differ from the C member name
RENAMED = {"from_": "from"}


def test_struct_layout_matches_header(tmp_path):
    """gcc compiles the header as plain C and prints sizeof/offsetof."""
    lines = ['#include <stdio.h>', '#include <stddef.h>',
             '#include "drb_engine.h"', 'int main(void) {']
    for cname, cls in STRUCTS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in cls._fields_:
            m = RENAMED.get(f, f)
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));'
                         % (cname, f, cname, m))
    lines.append('return 0; }')
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I",
                    os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    got = dict(ln.split() for ln in
               subprocess.run([str(exe)], capture_output=True, text=True,
                              check=True).stdout.splitlines())
    for cname, cls in STRUCTS.items():
        assert int(got[cname]) == C.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert int(got["%s.%s" % (cname, f)]) == getattr(cls, f).offset, \
                (cname, f)


def test_constants_match_header():
    src = open(HEADER).read()
    for name, val in [("DRB_MAX_REPLICAS", abi.DRB_MAX_REPLICAS),
                      ("DRB_RI_DEPTH", abi.DRB_RI_DEPTH)]:
        assert re.search(r"#define %s %d\b" % (name, val), src)
    enum = dict(re.findall(r"DRB_MSG_(\w+) = (\d+)", src))
    camel = {k.replace("_", "").lower(): v for k, v in abi.MSG.items()}
    assert len(enum) == len(abi.MSG)
    for k, v in enum.items():
        assert camel[k.replace("_", "").lower()] == int(v), k


def test_engine_without_gpu_fails_loudly():
    """No CPU fallback: creating an engine without a device is an error."""
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(engine.DrbError):
        engine.Engine(num_groups=64, num_replicas=3)


@pytest.mark.parametrize("kw", [
    # the plane summary word carries E in 8 bits (DRB_PLANE_E)
    dict(num_groups=64, num_replicas=3, place_world=2, place_rank=0,
         entry_mbox=256, window=512),
    dict(num_groups=64, num_replicas=3, place_world=2, place_rank=2,
         entry_mbox=3),
    # batched LogDB records merge from the window: window >= 64, save_cap
    dict(num_groups=64, num_replicas=3, save_batched=1, save_cap=4096),
    dict(num_groups=64, num_replicas=3, save_batched=1, window=64),
    dict(num_groups=64, num_replicas=3, window=48),  # not a power of two
    dict(num_groups=64, num_replicas=3, save_cap=1000),  # not 16 B aligned
    # tan records go to the save buffer; one persistence format at a time
    dict(num_groups=64, num_replicas=3, save_tan=1),
    dict(num_groups=64, num_replicas=3, save_tan=1, save_batched=1,
         save_cap=4096, window=64),
    # the multiplexed tan: a tan option; keys are ShardIDs of one rank
    dict(num_groups=64, num_replicas=3, tan_multiplexed=1, save_cap=4096),
    dict(num_groups=64, num_replicas=3, save_tan=1, tan_multiplexed=1,
         save_cap=4096, place_world=2, place_rank=0, entry_mbox=64),
    # forwarded proposals: 4-bit entry counts, co-resident planes
    dict(num_groups=64, num_replicas=3, forward_proposals=1, max_props=16),
    dict(num_groups=64, num_replicas=3, forward_proposals=1, place_world=2,
         place_rank=0, entry_mbox=4),
    dict(num_groups=64, num_replicas=3, host_copies=2),  # a 0/1 switch
])
def test_create_rejects_invalid_config(kw):
    """drb_engine_create validates the configuration before it touches a
    device: DRB_EINVAL, on a box with or without a GPU."""
    with pytest.raises(engine.DrbError) as ei:
        engine.Engine(**kw)
    assert "status %d" % abi.DRB_EINVAL in str(ei.value)
