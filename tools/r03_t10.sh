#!/bin/bash
mkdir -p gpurun_out/r03_ingest
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/r03_ingest/trace.log rocprofv3 --kernel-trace --stats -d gpurun_out/r03_ingest/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --host-staged 0 --kv-fill 0 || exit 1
