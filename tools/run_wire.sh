#!/bin/bash
# GPU: the wire-path tests, then the full GPU suite.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wire
tools/gpu_step.sh 300 gpurun_out/wire/pytest_wire.log python -u -m pytest tests/test_gpu_wire.py -x -v --timeout 120 --timeout-method thread || exit 1
tail -15 gpurun_out/wire/pytest_wire.log
grep -q " passed" gpurun_out/wire/pytest_wire.log || exit 1
grep -q "failed" gpurun_out/wire/pytest_wire.log && exit 1
exit 0
