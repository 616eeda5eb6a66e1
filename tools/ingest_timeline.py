# usage: python tools/ingest_timeline.py <0|1>  (run in the directory holding p0/ p1/ run_results.db of rocprofv3 --kernel-trace --memory-copy-trace):
# the kernels and copies of the last drb_ingest_wire call in a bench run, relative to its first event
import sqlite3, sys
z = sys.argv[1]
c = sqlite3.connect(f"p{z}/run_results.db")
ev = [(s, e, n.split('(')[0].split('<')[0][:34], 'K', st) for s, e, n, st in c.execute("select start,end,name,stream_id from kernels")]
ev += [(s, e, n[:20] + " %dB" % sz, 'C', st) for s, e, n, sz, st in c.execute("select start,end,name,size,stream_id from memory_copies")]
ev.sort()
t0 = [x for x in ev if 'k_host_slot' in x[2]][-1][1]
win = [x for x in ev if x[0] >= t0]
t1 = win[0][0]
for s, e, n, k, st in win[:200]:
    if 'k_ing_elems' in n: continue
    print("%8.3f %8.3f %7.3f st%-3s %s" % ((s - t1) / 1e6, (e - t1) / 1e6, (e - s) / 1e6, st, n))
