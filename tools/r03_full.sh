#!/bin/bash
# full GPU suite, then the HEAD profile (tools/prof_steady.sh)
mkdir -p gpurun_out
tools/gpu_step.sh 1000 gpurun_out/tall.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests -m gpu || exit 1
tools/gpu_step.sh 200 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
tools/prof_steady.sh ${1:-r03_head3}
