"""Builds the HIP engine (gfx950) into dragonboat_amd/_lib/libdrb_engine.so.

hipcc cross-compiles for gfx950 without a GPU; the .so is built in-tree so
it travels to the GPU box with the repository snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIBDIR, "libdrb_engine.so")
SOURCES = ["drb_engine.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def _deps():
    """Every source and header the engine includes (all of csrc/)."""
    inc = os.path.join(os.path.dirname(HERE), "include", "drb_engine.h")
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC))
            if f.endswith((".hip", ".hpp"))] + [inc]


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in _deps())


def build(force=False, verbose=False, out=None, defines=()):
    """Builds the engine; `out`/`defines` build a tuning variant elsewhere."""
    if out is not None:
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC",
               "-shared", "-Wno-pass-failed", "-o", out] + \
            ["-D" + d for d in defines] + \
            [os.path.join(CSRC, f) for f in SOURCES]
        subprocess.check_call(cmd)
        return out
    if not force and up_to_date():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC",
           "-shared", "-Wno-pass-failed", "-o", tmp] + \
        [os.path.join(CSRC, f) for f in SOURCES]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
