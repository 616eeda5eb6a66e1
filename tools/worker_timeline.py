"""The step-worker loop as rocprofv3 saw it (--kernel-trace
--memory-copy-trace): for the last N rounds of the loop (each starts with
the export's k_worker_count), every kernel and copy relative to the round's
first dispatch, with its queue, then the period between exports, the
exports' D2H copy time per round and the mean step kernel.  Shows whether
the copies of round t overlap round t + 1 and what they cost its kernels.

usage: python tools/worker_timeline.py <trace dir> [N] [out.txt]
"""
import csv
import glob
import sys


def load(d):
    kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    ev = []
    for r in csv.DictReader(open(kt)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = name.replace("void ", "").replace("drb::", "")
        if name.startswith("step_kernel"):
            name = "step_kernel " + ("leader" if "<3, true" in name
                                     else "follower")
        name = name.split("(")[0].split("<")[0]
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   "K", name[:28], q))
    mc = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
    if mc:
        for r in csv.DictReader(open(mc[0])):
            kind = r.get("Direction") or r.get("Operation") or "copy"
            nbytes = r.get("Bytes") or r.get("Size") or ""
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "C", ("%s %s" % (kind, nbytes))[:28],
                       r.get("Stream_Id", "?")))
    ev.sort()
    return ev


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    out = open(sys.argv[3], "w") if len(sys.argv) > 3 else sys.stdout
    ev = load(d)
    counts = [i for i, e in enumerate(ev) if e[3].startswith("k_worker_count")]
    if len(counts) < n + 1:
        print("no step-worker loop in the trace", file=out)
        return
    # a round: from the first event after the previous export's count
    # kernel's round started, i.e. between consecutive k_worker_count
    spans = []
    for a, b in zip(counts[-n - 1:-1], counts[-n:]):
        t0 = ev[a][0]
        seg = [e for e in ev if t0 <= e[0] < ev[b][0]]
        spans.append((t0, seg))
    for t0, seg in spans:
        print("--- round from %.3f ms" % (t0 / 1e6), file=out)
        for s, e, k, name, q in seg:
            print("  %8.1f %8.1f us  %s q%-3s %s" % ((s - t0) / 1e3,
                                                 (e - s) / 1e3, k, q, name),
                  file=out)
    # per-loop-iteration summary: iteration period and the drain's span
    per = []
    for i in range(len(counts) - n, len(counts)):
        per.append(ev[counts[i]][0])
    periods = [(b - a) / 1e3 for a, b in zip(per, per[1:])]
    d2h = []
    for a, b in zip(per, per[1:]):
        d2h.append(sum(e[1] - e[0] for e in ev if a <= e[0] < b and
                       e[2] == "C" and "DEVICE_TO_HOST" in e[3]) / 1e3)
    steps = [(e[1] - e[0]) / 1e3 for e in ev[-4 * n * 40:]
             if e[3].startswith("step_kernel")]
    print("period between exports (us): %s" %
          ", ".join("%.0f" % p for p in periods), file=out)
    print("D2H copy time per period (us): %s" %
          ", ".join("%.0f" % x for x in d2h), file=out)
    if steps:
        print("step kernels in the window: %d, mean %.0f us" %
              (len(steps), sum(steps) / len(steps)), file=out)


if __name__ == "__main__":
    main()
