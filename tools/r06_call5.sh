#!/bin/bash
# round 6: lean follower with a single load round trip -- parity, C5 bench,
# C5 kernel trace
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_l; mkdir -p $o
tools/gpu_tests.sh r06_l 600 tests/test_gpu_lean.py || exit 1
tools/gpu_step.sh 400 $o/bench_c5_128.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 || exit 1
grep -E '^\{' $o/bench_c5_128.log > $o/bench_c5_128.json
tools/r06_c5trace.sh r06_l/c5trace || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06_l/bench_c5_128.json")); c = d["counters"]
print("c5", round(d["ms_per_step"], 4), c["fallbacks"], c.get("lean_stepped_per_round"), c.get("replicas_stepped_per_round"))
PY
