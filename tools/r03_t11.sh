#!/bin/bash
mkdir -p gpurun_out
tools/gpu_step.sh 400 gpurun_out/t11.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_prevote.py -m gpu || exit 1
tools/gpu_step.sh 600 gpurun_out/rehearse.log bash tools/rehearse_dist.sh || exit 1
