#!/bin/bash
# GPU: selected tests (pytest -k expression in $2), then optionally a
# bench line (args in $3...).  Each step under its own limit.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-q}; shift
mkdir -p "$o"
export TMPDIR=/tmp
k=$1; shift
if [ -n "$k" ]; then
  tools/gpu_step.sh 900 "$o/pytest_gpu.log" python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -k "$k" || exit 1
  tail -3 "$o/pytest_gpu.log"
  grep -E "FAILED|ERROR" "$o/pytest_gpu.log" | head -30
fi
if [ $# -gt 0 ]; then
  tools/gpu_step.sh 400 "$o/bench.log" python bench.py "$@" || exit 1
  tail -2 "$o/bench.log" | cut -c1-1500
fi
