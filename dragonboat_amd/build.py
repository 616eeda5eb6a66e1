"""Builds the HIP engine (gfx950) into dragonboat_amd/_lib/libdrb_engine.so.

hipcc cross-compiles for gfx950 without a GPU; the .so is built in-tree so
it travels to the GPU box with the repository snapshot.

The step kernel has 72 instantiations (R = 1..8 replicas per group x nine
kinds, drb_launch.hpp, the lean kernel's two among them).  Each is its own translation unit
(drb_step_inst.hip compiled with -DDRB_INST_R / -DDRB_INST_KIND), so the
objects build in parallel and only the ones whose sources changed rebuild;
the engine's host code and auxiliary kernels are drb_engine.hip.
"""
import hashlib
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIBDIR, "libdrb_engine.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC",
         "-Wno-pass-failed"]
NUM_KINDS = 9
# the LOCAL kinds 9-12 (drb_launch.hpp), for these R only
LOCAL_KINDS, LOCAL_R = (9, 10, 11, 12), (3, 5)
# the headers a step-kernel instantiation includes
STEP_DEPS = ["drb_step_inst.hip", "drb_step.hpp", "drb_lean.hpp",
             "drb_launch.hpp",
             "drb_layout.hpp", "drb_msg.hpp", "drb_codec.hpp", "drb_ring.hpp"]
# the tan record kernels' (drb_tan_inst.hip)
TAN_DEPS = ["drb_tan_inst.hip", "drb_tan.hpp", "drb_launch.hpp",
            "drb_layout.hpp", "drb_codec.hpp", "drb_ring.hpp"]


def _inc():
    return os.path.join(os.path.dirname(HERE), "include", "drb_engine.h")


def _deps():
    """Every source and header the engine includes (all of csrc/)."""
    return [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC))
            if f.endswith((".hip", ".hpp"))] + [_inc()]


def _units(defines):
    """(object name, source, extra defines, dependencies) of every TU."""
    step_deps = [os.path.join(CSRC, f) for f in STEP_DEPS] + [_inc()]
    tan_deps = [os.path.join(CSRC, f) for f in TAN_DEPS] + [_inc()]
    units = [("drb_engine.o", "drb_engine.hip", [], _deps()),
             ("tan_write.o", "drb_tan_inst.hip", ["DRB_TAN_KERNELS=2"],
              tan_deps),
             ("tan_select.o", "drb_tan_inst.hip", ["DRB_TAN_KERNELS=1"],
              tan_deps)]
    for r in range(1, 9):
        for k in list(range(NUM_KINDS)) + \
                (list(LOCAL_KINDS) if r in LOCAL_R else []):
            units.append(("step_r%d_k%d.o" % (r, k), "drb_step_inst.hip",
                          ["DRB_INST_R=%d" % r, "DRB_INST_KIND=%d" % k],
                          step_deps))
    return units


def _stale(obj, deps):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in _deps())


def _compile(args):
    obj, src, defs, verbose = args
    tmp = obj + ".tmp"
    cmd = [HIPCC] + FLAGS + ["-c", "-o", tmp] + ["-D" + d for d in defs] + \
        [os.path.join(CSRC, src)]
    t0 = time.time()
    subprocess.check_call(cmd)
    os.replace(tmp, obj)
    # dated when the compile started: a source edited meanwhile is newer
    os.utime(obj, (t0, t0))
    if verbose:
        print("%6.1f s  %s" % (time.time() - t0, os.path.basename(obj)),
              file=sys.stderr)
    return obj


def build(force=False, verbose=False, out=None, defines=(), jobs=None,
          variant_r=(3,)):
    """Builds the engine; `out`/`defines` build a tuning variant elsewhere:
    the step kernels of R in variant_r with the defines (their objects in a
    directory of their own, keyed by the defines), everything else from the
    in-tree build."""
    target = LIB if out is None else out
    t_start = time.time()
    if out is None and not force and up_to_date():
        return LIB
    key = hashlib.sha1(" ".join(sorted(defines)).encode()).hexdigest()[:10]
    main_dir = os.path.join(LIBDIR, "obj")
    var_dir = os.path.join(LIBDIR, "obj_" + key)
    for d in (main_dir, var_dir if defines else main_dir):
        os.makedirs(d, exist_ok=True)
    todo, objs = [], []
    for name, src, defs, deps in _units(defines):
        var = bool(defines) and any(name.startswith("step_r%d_" % r)
                                    for r in variant_r)
        obj = os.path.join(var_dir if var else main_dir, name)
        objs.append(obj)
        if force or _stale(obj, deps):
            todo.append((obj, src, (list(defines) if var else []) + defs,
                         verbose))
    jobs = jobs or int(os.environ.get("DRB_BUILD_JOBS", 0)) or \
        max(1, min(16, os.cpu_count() or 1))
    # the longest translation units first
    first = ("tan_write.o", "tan_select.o", "drb_engine.o")
    todo.sort(key=lambda t: (not t[0].endswith(first), t[0]))
    if todo:
        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(_compile, todo))
    tmp = target + ".tmp"
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-fPIC", "-shared", "-o", tmp] + \
        objs + ["-lhsa-runtime64", "-lrccl"]
    if verbose:
        print(" ".join(cmd[:6]) + " <%d objects>" % len(objs), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, target)
    os.utime(target, (t_start, t_start))  # (as the objects, _compile)
    return target


if __name__ == "__main__":
    # python build.py [--force] [-v] [--variant NAME [--r=R] -DX=1 ...]: a
    # variant goes to _lib/variants/NAME.so (bench.py loads it with
    # DRB_ENGINE_LIB; in-tree, so it travels to the GPU box)
    args = sys.argv[1:]
    if "--variant" in args:
        i = args.index("--variant")
        name, defs = args[i + 1], [a[2:] for a in args[i + 2:]
                                   if a.startswith("-D")]
        out = os.path.join(LIBDIR, "variants", name + ".so")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        vr = tuple(int(a[4:]) for a in args if a.startswith("--r="))
        print(build(verbose="-v" in args, out=out, defines=defs,
                    variant_r=vr or (3,)))
    else:
        print(build(force="--force" in args, verbose="-v" in args))
