#!/bin/bash
# round 6: LOCAL step instantiations (no remote-plane paths compiled in)
# for co-resident engines -- C3 and C5 against the build before them
# (nopeers variant), alternated; the parity tests of the co-resident paths
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_r; mkdir -p $o
tools/gpu_tests.sh r06_r 900 tests/test_gpu_parity.py tests/test_gpu_lean.py tests/test_gpu_quiesce.py || exit 1
for rep in 1 2; do
  tools/gpu_step.sh 400 $o/c3_local_$rep.log python bench.py --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
  DRB_ENGINE_LIB=dragonboat_amd/_lib/variants/nopeers.so tools/gpu_step.sh 400 $o/c3_old_$rep.log python bench.py --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
  tools/gpu_step.sh 400 $o/c5_local_$rep.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 || exit 1
  DRB_ENGINE_LIB=dragonboat_amd/_lib/variants/nopeers.so tools/gpu_step.sh 400 $o/c5_old_$rep.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_r/c*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d["counters"]["fallbacks"])
PY
