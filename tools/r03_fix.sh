#!/bin/bash
# the tests that failed on the first full runs of round 3
mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/tfix1.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_elections.py -m gpu || exit 1
tools/gpu_step.sh 300 gpurun_out/tfix2.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_transfer.py tests/test_gpu_staging.py -m gpu || exit 1
