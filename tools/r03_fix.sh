#!/bin/bash
mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/tfix2.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_transfer.py -m gpu || exit 1
