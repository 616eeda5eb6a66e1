#!/bin/bash
# round 6: the whole GPU suite and smoke() on the current build
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_s; mkdir -p $o
tools/gpu_tests.sh r06_s 1050 tests/ -m gpu || exit 1
tools/gpu_step.sh 120 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tail -1 $o/smoke.log
