#!/bin/bash
# round 6: where a C2 round goes -- the step kernels' phases (timing
# variant) and the kernel trace of the timed rounds
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_c2; mkdir -p $o
DRB_ENGINE_LIB=dragonboat_amd/_lib/variants/phase.so DRB_PHASE=1 tools/gpu_step.sh 300 $o/c2_phase.log python bench.py --workload c2 --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
grep phase $o/c2_phase.log
tools/gpu_step.sh 300 $o/trace.log rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python bench.py --workload c2 --steps 40 --warmup 8 --no-cpu-baseline --no-wire --host-staged 0 --step-worker 0 || exit 1
python tools/trace_summary.py $o/trace 40 $o/kernels_last40.csv > $o/kernels_last40.txt
head -8 $o/kernels_last40.txt
python tools/trace_union.py $o/trace "step_kernel<3, true" 40 | head -8
