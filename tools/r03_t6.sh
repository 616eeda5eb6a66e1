#!/bin/bash
# C4 elections + follower inbox prefetch: tests, then base vs no-prefetch
mkdir -p gpurun_out
tools/gpu_step.sh 900 gpurun_out/t6.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_elections.py tests/test_gpu_parity.py \
  tests/test_gpu_quiesce.py tests/test_gpu_fullsize.py -m gpu -x || exit 1
tools/exp_variants.sh r03_fpf base nofpf base2 nofpf2
