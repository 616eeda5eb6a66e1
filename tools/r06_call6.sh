#!/bin/bash
# round 6: compacting proposal generator, one-pass active scan, lean/full
# launches on two streams (DRB_LEAN_SPLIT, A/B) -- parity, C5 A/B, trace
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_m; mkdir -p $o
tools/gpu_tests.sh r06_m 900 tests/test_gpu_lean.py tests/test_gpu_quiesce.py \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "c5 or quiesce or lean or generator or sparse or idle" || exit 1
for rep in 1 2; do
  for x in 0 1 2 3; do
    DRB_LEAN_SPLIT=$x tools/gpu_step.sh 300 $o/c5_x${x}_$rep.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 || exit 1
  done
done
tools/r06_c5trace.sh r06_m/c5trace || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_m/c5_x*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); c = d["counters"]
            print(f.split("/")[-1], round(d["ms_per_step"], 4), c["fallbacks"], c.get("lean_stepped_per_round"))
PY
