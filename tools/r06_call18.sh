#!/bin/bash
# round 6: the lean kernel takes replicas with uncommitted or in-memory
# applied entries (nothing to save or apply) -- parity, C5, escalations
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_y; mkdir -p $o
tools/gpu_tests.sh r06_y 1000 tests/test_gpu_lean.py tests/test_gpu_quiesce.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "lean or quiesce or sparse or idle or c5" || exit 1
for rep in 1 2; do
  tools/gpu_step.sh 300 $o/c5_$rep.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
  tools/gpu_step.sh 300 $o/c5k_$rep.log python bench.py --workload c5 --payload 1024 --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
done
DRB_ENGINE_LIB=dragonboat_amd/_lib/variants/leanwhy.so DRB_PHASE=1 tools/gpu_step.sh 300 $o/c5_why.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
grep phase $o/c5_why.log
tools/r06_c5trace.sh r06_y/c5trace || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_y/c5*_?.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); c = d["counters"]
            print(f.split("/")[-1], round(d["ms_per_step"], 4), c["fallbacks"], c.get("lean_stepped_per_round"), c.get("replicas_stepped_per_round"))
PY
