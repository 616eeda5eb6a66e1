"""Busy time of a rocprofv3 kernel trace's tail: over the span of the last
N dispatches of <kernel substring>, the union of all kernel intervals
(GPU busy with at least one kernel) and the sum of their durations (> the
union where kernels overlap), per kernel name.
usage: python tools/trace_union.py <trace dir> <kernel substring> <N>"""
import csv
import glob
import sys
from collections import defaultdict

d, key, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
       r["Kernel_Name"].split("(")[0][:70]) for r in csv.DictReader(open(f))]
iv.sort()
marks = [s for s, e, k in iv if key in k]
t0 = marks[-n]
tail = [x for x in iv if x[0] >= t0]
t1 = max(e for s, e, k in tail)
busy, cur_s, cur_e = 0, None, None
for s, e, k in tail:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
per = defaultdict(lambda: [0, 0])
for s, e, k in tail:
    per[k][0] += 1
    per[k][1] += e - s
print("span %.1f us, busy (union) %.1f us, kernel sum %.1f us" % (
    (t1 - t0) / 1e3, busy / 1e3, sum(v[1] for v in per.values()) / 1e3))
for k, (c, t) in sorted(per.items(), key=lambda x: -x[1][1]):
    print("%-70s %5d %10.1f us" % (k, c, t / 1e3))
