#!/bin/bash
# round 6: where C5's full-kernel time goes -- the phase profile of the
# heavy / escalated lanes (timing variant) and the SQ wave-state breakdown
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_n; mkdir -p $o
DRB_ENGINE_LIB=dragonboat_amd/_lib/variants/phase.so DRB_PHASE=1 tools/gpu_step.sh 300 $o/c5_phase.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 || exit 1
grep phase $o/c5_phase.log
WL="C5 128 B (bench.py --workload c5 --payload 128), timed rounds" tools/prof_stall.sh r06_n/stall --workload c5 --payload 128 --step-worker 0 || exit 1
cat $o/stall/stall.txt
