#!/bin/bash
# round 6, last build: the C5 lines and PMC passes, the C3 steady-state line
# with its trace and PMC, the whole GPU suite and smoke()
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06_final2}; mkdir -p $o
tools/gpu_tests.sh ${1:-r06_final2} 1050 tests/ -m gpu || exit 1
tools/gpu_step.sh 120 $o/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tail -1 $o/smoke.log
