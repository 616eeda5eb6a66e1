#!/bin/bash
mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/t7.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_elections.py -k spread -m gpu -x || exit 1
