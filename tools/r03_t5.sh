#!/bin/bash
# round 3: leader transfer + the tests not yet run on the split build
mkdir -p gpurun_out
tools/gpu_step.sh 300 gpurun_out/t5a.log python -u -m pytest -x -v --timeout 120 \
  --timeout-method thread tests/test_gpu_transfer.py -m gpu || exit 1
tools/gpu_step.sh 700 gpurun_out/t5b.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_elections.py tests/test_gpu_reads.py \
  tests/test_gpu_staging.py tests/test_gpu_quiesce.py tests/test_gpu_truncation.py -m gpu || exit 1
tools/gpu_step.sh 300 gpurun_out/b5.log python bench.py --steps 20 --warmup 5 --no-wire || exit 1
