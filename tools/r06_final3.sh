#!/bin/bash
# round 6, last build: C3 at the KV steady state (line, trace, PMC), the
# C5 lines and their PMC passes, C4 local ranks
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06_final3}; mkdir -p $o
tools/prof_steady.sh ${1:-r06_final3}/c3 || exit 1
tools/prof_workloads.sh ${1:-r06_final3}/pmc c5_128 c5_1024 || exit 1
for w in "c5_128 --workload c5 --payload 128" "c5_1024 --workload c5 --payload 1024" "c4l8 --workload c4 --local-ranks 8"; do
  set -- $w; n=$1; shift
  tools/gpu_step.sh 400 $o/bench_$n.log python bench.py "$@" --no-cpu-baseline || exit 1
  grep -E '^\{' $o/bench_$n.log > $o/bench_$n.json
done
python - <<PY
import json, glob
for f in sorted(glob.glob("$o/bench*.json")) + ["$o/c3/bench.json"]:
    d = json.load(open(f)); r = d.get("roofline", {})
    print(f.split("/")[-1], round(d["ms_per_step"], 4), round(d["value"] / 1e6, 1), r.get("frac"))
PY
head -4 $o/c3/kernels_last20.txt
