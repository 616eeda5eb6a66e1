#!/bin/bash
# round 6: 32 x 32 -> 64 row products in the layout's index helpers
# (DRB_IX32) -- parity, then C3 / C5 / C4 against the 64-bit form, alternated
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_w; mkdir -p $o
tools/gpu_tests.sh r06_w 900 tests/test_gpu_parity.py tests/test_gpu_lean.py tests/test_gpu_worker.py tests/test_gpu_staging.py || exit 1
for rep in 1 2; do
  for v in ix32 ix64; do
    if [ $v = ix32 ]; then L=""; else L=dragonboat_amd/_lib/variants/ix64.so; fi
    DRB_ENGINE_LIB=$L tools/gpu_step.sh 400 $o/c3_${v}_$rep.log python bench.py --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
    DRB_ENGINE_LIB=$L tools/gpu_step.sh 400 $o/c5_${v}_$rep.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_w/c*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d["counters"]["fallbacks"], round(d["roofline"]["kernel_ms"], 4))
PY
