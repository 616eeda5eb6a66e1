#!/bin/bash
# round 6: relaxed lean eligibility against the strict one (variant), C5,
# alternated on one box
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_z; mkdir -p $o
for rep in 1 2 3; do
  for v in relaxed strict; do
    if [ $v = relaxed ]; then L=""; else L=dragonboat_amd/_lib/variants/strict.so; fi
    DRB_ENGINE_LIB=$L tools/gpu_step.sh 300 $o/c5_${v}_$rep.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 || exit 1
  done
done
for v in relaxed strict; do
  if [ $v = relaxed ]; then L=""; else L=dragonboat_amd/_lib/variants/strict.so; fi
  DRB_ENGINE_LIB=$L tools/gpu_step.sh 300 $o/c5k_${v}.log python bench.py --workload c5 --payload 1024 --no-cpu-baseline --host-staged 0 --step-worker 0 || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_z/c5*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); c = d["counters"]
            print(f.split("/")[-1], round(d["ms_per_step"], 4), c["fallbacks"], c.get("lean_stepped_per_round"))
PY
