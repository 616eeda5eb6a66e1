"""Summarise rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, collected in
separate runs) into HBM bytes per launch of the round's kernels.

Correction (MI355X_MICROARCH.md, HBM section; re-checked for our access
shapes by tools/calib_hbm.hip -> profiles/calib/): FETCH_SIZE counts half
the bytes of coalesced reads -> x2; WRITE_SIZE is exact for coalesced
stores.  Both counters are in KiB.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json>
       [--groups G --replicas R --workload TEXT]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROUND_KERNELS = ("step_kernel", "lean_kernel", "k_serve_reads")


def load(d):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f:
        raise SystemExit("no counter_collection.csv under %s" % d)
    per = defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("out")
    ap.add_argument("--groups", type=int, default=1 << 20)
    ap.add_argument("--replicas", type=int, default=3)
    ap.add_argument("--workload", default="")
    ap.add_argument("--last", type=int, default=0,
                    help="average only the last N launches of each kernel "
                         "(the timed rounds, after a KV fill's rounds)")
    a = ap.parse_args()
    fetch, write = load(a.fetch), load(a.write)
    if a.last:
        for per in (fetch, write):
            for key in per:
                per[key] = per[key][-a.last:]
    kernels = {}
    for (name, ctr), vals in list(fetch.items()) + list(write.items()):
        k = kernels.setdefault(name, {})
        k[ctr] = sum(vals) / len(vals) * 1024.0
        k["launches_" + ctr] = len(vals)
    round_bytes = round_lower = 0.0
    for name, k in kernels.items():
        k["hbm_bytes"] = 2.0 * k.get("FETCH_SIZE", 0.0) + k.get("WRITE_SIZE",
                                                                 0.0)
        if any(t in name for t in ROUND_KERNELS):
            round_bytes += k["hbm_bytes"]
            round_lower += k.get("FETCH_SIZE", 0.0) + k.get("WRITE_SIZE", 0.0)
    out = {"groups": a.groups, "replicas": a.replicas,
           "workload": a.workload,
           "round_hbm_bytes": round_bytes,
           "bytes_per_group_round": round_bytes / a.groups,
           "round_hbm_bytes_lower": round_lower,
           "bytes_per_group_round_lower": round_lower / a.groups,
           "correction": "FETCH_SIZE x2 + WRITE_SIZE (KiB -> B)",
           "bound_note": "round_hbm_bytes = FETCH_SIZE x2 + WRITE_SIZE is an "
                         "upper bound: the x2 correction is calibrated for "
                         "coalesced 16 B/lane reads (MI355X_MICROARCH.md), "
                         "while a random 16 B read (the KV probes) is tallied "
                         "at its full 64 B already (profiles/r02_kvline/"
                         "calib.log); FETCH_SIZE + WRITE_SIZE "
                         "(round_hbm_bytes_lower) is the matching lower bound",
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps({k: out[k] for k in ("round_hbm_bytes",
                                          "bytes_per_group_round")}))


if __name__ == "__main__":
    main()
