#!/bin/bash
# round 6: three-class active lists (proposing lanes first) -- parity, C5 A/B
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_v; mkdir -p $o
tools/gpu_tests.sh r06_v 900 tests/test_gpu_lean.py tests/test_gpu_quiesce.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "lean or quiesce or sparse or idle or c5" || exit 1
for rep in 1 2; do
  for v in cls nocls; do
    if [ $v = cls ]; then unset DRB_AB_NOCLASS; else export DRB_AB_NOCLASS=1; fi
    tools/gpu_step.sh 300 $o/c5_${v}_$rep.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
    tools/gpu_step.sh 300 $o/c5k_${v}_$rep.log python bench.py --workload c5 --payload 1024 --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
  done
done
unset DRB_AB_NOCLASS
tools/r06_c5trace.sh r06_v/c5trace || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_v/c5*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d["counters"]["fallbacks"])
PY
