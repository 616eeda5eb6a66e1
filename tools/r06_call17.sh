#!/bin/bash
# round 6: bench.py's multi-rank lines under gloo (counted default), smoke
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_x; mkdir -p $o
tools/gpu_tests.sh r06_x 900 tests/test_gpu_bench_dist.py || exit 1
tools/gpu_step.sh 120 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tail -1 $o/smoke.log
