#!/bin/bash
# round 3: new GPU tests, then C3 at the KV fill's steady state against a
# near-empty KV and writes-only, one box
mkdir -p gpurun_out
tools/gpu_step.sh 500 gpurun_out/t3.log python -u -m pytest -x -v --timeout 300 \
  --timeout-method thread tests/test_gpu_truncation.py tests/test_gpu_reads.py \
  tests/test_gpu_staging.py -m gpu || exit 1
for a in "--kv-fill 0" "" "--no-read-index" "--kv-fill 0 --no-read-index"; do
  n=$(echo "x$a" | tr -c 'a-z0-9' '_')
  tools/gpu_step.sh 300 gpurun_out/b3$n.log python bench.py --steps 20 --warmup 5 \
    --no-cpu-baseline --no-wire --host-staged 0 $a || exit 1
done
