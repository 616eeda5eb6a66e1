#!/bin/bash
# round 6: the lean kernel (all loads first) -- parity, then C5 A/B and trace
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_j; mkdir -p $o
tools/gpu_tests.sh r06_j 900 tests/test_gpu_lean.py tests/test_gpu_quiesce.py \
  "tests/test_gpu_parity.py::test_c5_sparse_activity_idle_rounds" || exit 1
B="python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline"
tools/gpu_step.sh 400 $o/c5_lean.log $B || exit 1
tools/gpu_step.sh 400 $o/c5_full.log $B --no-lean || exit 1
for f in c5_lean c5_full; do tail -1 $o/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["counters"]; print(round(d["ms_per_step"],4), c["fallbacks"], c["replicas_stepped_per_round"], c["lean_stepped_per_round"])'; done
tools/r06_c5trace.sh r06_j/c5trace
