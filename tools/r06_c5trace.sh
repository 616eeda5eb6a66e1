#!/bin/bash
# C5 128 B kernel trace with the lean kernel (timed rounds: the last 20)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06_c5trace}; mkdir -p $o
shift
B="python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --no-wire --host-staged 0 $*"
tools/gpu_step.sh 400 $o/trace.log rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- $B || exit 1
python tools/trace_summary.py $o/trace 20 $o/kernels_last20.csv > $o/kernels_last20.txt
cat $o/kernels_last20.txt | head -20
