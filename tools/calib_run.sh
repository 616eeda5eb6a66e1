#!/bin/bash
# GPU: tools/_bin/calib (tools/calib_hbm.hip) timed, then its FETCH_SIZE and
# WRITE_SIZE passes, summarised per kernel (raw KiB -> bytes per launch).
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-calib}; mkdir -p "$o"
export TMPDIR=/tmp
tools/gpu_step.sh 120 "$o/calib.log" tools/_bin/calib || exit 1
cat "$o/calib.log"
tools/gpu_step.sh 120 "$o/fetch.log" timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d "$o/fetch" -o run --output-format csv -- tools/_bin/calib || exit 1
tools/gpu_step.sh 120 "$o/write.log" timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d "$o/write" -o run --output-format csv -- tools/_bin/calib || exit 1
python - "$o" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for c in ("fetch", "write"):
    f = glob.glob(o + "/" + c + "/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])].append(float(r["Counter_Value"]) * 1024)
    for k, v in sorted(acc.items()):
        print(c, k[0][-40:], k[1], [round(x / 1e6, 1) for x in v], "MB")
PY
