#!/bin/bash
# round 6 against round 5 on one box: C3 (and C5 128 B) with the round-5
# library (commit 0529422, built in-tree as a variant) and the current one,
# alternated
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_u; mkdir -p $o
for rep in 1 2; do
  for v in cur r05; do
    if [ $v = cur ]; then L=""; else L=dragonboat_amd/_lib/variants/r05.so; fi
    DRB_ENGINE_LIB=$L tools/gpu_step.sh 400 $o/c3_${v}_$rep.log python bench.py --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
  done
done
for rep in 1 2; do
  for v in cur r05; do
    if [ $v = cur ]; then L=""; else L=dragonboat_amd/_lib/variants/r05.so; fi
    DRB_ENGINE_LIB=$L tools/gpu_step.sh 400 $o/c5_${v}_$rep.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_u/c*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d["counters"]["fallbacks"], d["roofline"].get("kernel_ms"))
PY
