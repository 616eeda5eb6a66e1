"""Per-kernel wave-state breakdown from rocprofv3 SQ counter passes.

SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY and SQ_ACTIVE_INST_* count
quad-cycles summed over the kernel's waves (MI355X_MICROARCH.md, PMC
slots): WAIT_ANY (parked at s_waitcnt / barrier) + WAIT_INST_ANY (issue
stall) + ACTIVE_INST_ANY ~= WAVE_CYCLES.  The fractions below are of
SQ_WAVE_CYCLES, per kernel, averaged over the last N dispatches (the timed
rounds).

usage: python tools/stall_summary.py <out.json> --last N <pass dir>...
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d, per):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                  recursive=True)
    if not f:
        raise SystemExit("no counter_collection.csv under %s" % d)
    rows = defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        rows[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in rows.items():
        per[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--last", type=int, default=20)
    ap.add_argument("--workload", default="")
    a = ap.parse_args()
    per = {}
    for d in a.dirs:
        load(d, per)
    kernels = {}
    for (name, ctr), vals in per.items():
        v = vals[-a.last:] if a.last else vals
        kernels.setdefault(name, {})[ctr] = sum(v) / len(v)
    for name, k in kernels.items():
        wc = k.get("SQ_WAVE_CYCLES")
        if not wc:
            continue
        fr = {}
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                  "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA",
                  "SQ_WAIT_INST_LDS"):
            if c in k:
                fr[c] = k[c] / wc
        k["frac_of_wave_cycles"] = fr
        if "SQ_WAVES" in k and k["SQ_WAVES"]:
            k["wave_cycles_per_wave"] = 4 * wc / k["SQ_WAVES"]
        if "SQ_BUSY_CYCLES" in k and "GRBM_GUI_ACTIVE" in k:
            k["note"] = "SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE are per-XCD sums"
    out = {"workload": a.workload, "last": a.last,
           "units": "SQ_* cycle counters are quad-cycles summed over waves "
                    "(x4 = shader cycles); SQ_INSTS_* are instruction counts "
                    "summed over waves",
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for name, k in sorted(kernels.items()):
        if "frac_of_wave_cycles" in k:
            print(name[:60], json.dumps({c.replace("SQ_", ""): round(x, 3)
                                         for c, x in
                                         k["frac_of_wave_cycles"].items()}))


if __name__ == "__main__":
    main()
