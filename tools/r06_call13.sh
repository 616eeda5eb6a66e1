#!/bin/bash
# round 6: one-pass scatter (parity + C5), lean kernel occupancy variants
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_t; mkdir -p $o
tools/gpu_tests.sh r06_t 600 tests/test_gpu_lean.py tests/test_gpu_quiesce.py tests/test_gpu_parity.py -k "lean or quiesce or sparse or idle" || exit 1
for rep in 1 2; do
  for v in main fw4 fw6 lw5 lw3; do
    if [ $v = main ]; then L=""; else L=dragonboat_amd/_lib/variants/$v.so; fi
    DRB_ENGINE_LIB=$L tools/gpu_step.sh 300 $o/c5_${v}_$rep.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 || exit 1
  done
done
tools/r06_c5trace.sh r06_t/c5trace || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_t/c5_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d["counters"]["fallbacks"])
PY
