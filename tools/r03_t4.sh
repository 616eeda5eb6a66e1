#!/bin/bash
mkdir -p gpurun_out
tools/gpu_step.sh 600 gpurun_out/t4.log python -u -m pytest -x -v --timeout 300 \
  --timeout-method thread tests/test_gpu_elections.py tests/test_gpu_reads.py \
  tests/test_gpu_staging.py tests/test_gpu_quiesce.py -m gpu || exit 1
tools/gpu_step.sh 300 gpurun_out/b4.log python bench.py --steps 20 --warmup 5 --no-wire || exit 1
