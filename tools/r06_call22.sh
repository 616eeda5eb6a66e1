#!/bin/bash
# round 6: lazy quiesce base / rtr_count clears in the lean and EXT paths --
# parity (quiesce, lean, parity listed, fullsize c5), then C5 against the
# eager form (variant), alternated
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-r06_q2}; mkdir -p $o
tools/gpu_tests.sh ${1:-r06_q2} 1000 tests/test_gpu_lean.py tests/test_gpu_quiesce.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_worker.py -k "lean or quiesce or sparse or idle or c5 or worker or save or tan or batched" || exit 1
for rep in 1 2 3; do
  for v in lazy eager; do
    if [ $v = lazy ]; then L=""; else L=dragonboat_amd/_lib/variants/eager.so; fi
    DRB_ENGINE_LIB=$L tools/gpu_step.sh 300 $o/c5_${v}_$rep.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 || exit 1
  done
done
python - "${1:-r06_q2}" <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/%s/c5*.log" % __import__("sys").argv[1])):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); c = d["counters"]
            print(f.split("/")[-1], round(d["ms_per_step"], 4), c["fallbacks"], c.get("lean_stepped_per_round"))
PY
