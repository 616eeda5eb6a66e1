#!/bin/bash
mkdir -p gpurun_out
tools/gpu_step.sh 600 gpurun_out/t12.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_c4_ingest.py tests/test_gpu_wire.py \
  tests/test_gpu_fallback.py tests/test_gpu_prevote.py -m gpu || exit 1
