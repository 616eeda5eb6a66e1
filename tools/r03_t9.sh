#!/bin/bash
# wire ingest: tests, then the traced C3 bench (ingest phases)
mkdir -p gpurun_out/r03_ingest
tools/gpu_step.sh 400 gpurun_out/r03_ingest/pytest_wire.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_wire.py -m gpu -x || exit 1
DRB_INGEST_TRACE=1 tools/gpu_step.sh 300 gpurun_out/r03_ingest/bench_trace.log python bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-staged 0 --kv-fill 0 || exit 1
tools/gpu_step.sh 300 gpurun_out/r03_ingest/bench.log python bench.py --steps 10 --warmup 3 --no-cpu-baseline --host-staged 0 --kv-fill 0 || exit 1
