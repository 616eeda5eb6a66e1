#!/bin/bash
# round 6: why C5's light lanes escalate from the lean kernel (timing
# variant DRB_LEAN_WHY: per role, escalated lanes and each reason's count)
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_o; mkdir -p $o
DRB_ENGINE_LIB=dragonboat_amd/_lib/variants/leanwhy.so DRB_PHASE=1 tools/gpu_step.sh 300 $o/c5_why.log python bench.py --workload c5 --payload 128 --no-cpu-baseline --host-staged 0 --step-worker 0 || exit 1
grep phase $o/c5_why.log
