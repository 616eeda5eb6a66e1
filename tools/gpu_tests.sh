#!/bin/bash
# GPU tests of one call: pytest under its own time limit, output under
# gpurun_out/<tag>/tests.log.  usage: tools/gpu_tests.sh <tag> <seconds> <pytest args...>
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; t=$2; shift 2
mkdir -p $o
timeout -k 10 "$t" python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $o/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "passed|failed|error" $o/tests.log | tail -3
exit $rc
