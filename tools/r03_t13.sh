#!/bin/bash
mkdir -p gpurun_out/r03_c5prof
export TMPDIR=/tmp
tools/gpu_step.sh 400 gpurun_out/r03_c5prof/trace.log rocprofv3 --kernel-trace --stats -d gpurun_out/r03_c5prof/trace -o run --output-format csv -- python bench.py --workload c5 --payload 128 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
python tools/trace_summary.py gpurun_out/r03_c5prof/trace 20 gpurun_out/r03_c5prof/kernels_last20.csv > gpurun_out/r03_c5prof/kernels_last20.txt
