#!/bin/bash
# round 6 final measurements: the default bench line with its kernel trace
# and HBM PMC passes (C3), the PMC passes of the other workloads (their
# roofline.traffic), and the other workloads' lines
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r06_final}
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_prof.sh $tag --no-tests || exit 1
python tools/trace_summary.py $o/trace 20 $o/kernels_last20.csv > $o/kernels_last20.txt
head -6 $o/kernels_last20.txt
tools/prof_workloads.sh $tag/pmc c2 c4 c5_128 c5_1024 || exit 1
for w in "c5_128 --workload c5 --payload 128" "c5_1024 --workload c5 --payload 1024" "c2 --workload c2" "c4 --workload c4" "c4l8 --workload c4 --local-ranks 8"; do
  set -- $w; n=$1; shift
  tools/gpu_step.sh 400 $o/bench_$n.log python bench.py "$@" --no-cpu-baseline || exit 1
  grep -E '^\{' $o/bench_$n.log > $o/bench_$n.json
done
python - <<PY
import json, glob
for f in sorted(glob.glob("$o/bench*.json")):
    d = json.load(open(f)); r = d.get("roofline", {})
    print(f.split("/")[-1], round(d["ms_per_step"], 4), round(d["value"] / 1e6, 1), r.get("frac"))
PY
