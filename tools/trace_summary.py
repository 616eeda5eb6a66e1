"""Average duration of the last N dispatches of each kernel in a rocprofv3
kernel trace (the timed rounds of a bench run, after its KV fill rounds).
usage: python tools/trace_summary.py <trace dir> <N> [out.csv]"""
import csv
import glob
import sys
from collections import defaultdict

d, n = sys.argv[1], int(sys.argv[2])
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
per = defaultdict(list)
for r in csv.DictReader(open(f)):
    per[r["Kernel_Name"]].append(
        (int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
rows = []
for k, v in per.items():
    v.sort()
    last = v[-n:]
    avg = sum(e - s for s, e in last) / len(last) / 1e3
    rows.append((avg * len(last), k, len(v), len(last), avg))
rows.sort(reverse=True)
out = open(sys.argv[3], "w") if len(sys.argv) > 3 else None
if out:
    out.write("kernel,dispatches,averaged,avg_us\n")
for _, k, tot, m, avg in rows:
    line = "%s,%d,%d,%.1f" % (k.split("(")[0][:90], tot, m, avg)
    print(line)
    if out:
        out.write('"%s",%d,%d,%.2f\n' % (k, tot, m, avg))
