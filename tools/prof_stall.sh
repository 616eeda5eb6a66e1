#!/bin/bash
# Wave-state breakdown of the round's kernels at the C3 steady state: two
# SQ counter passes (8 SQ counters each, + GRBM), each its own run, over the
# 20 timed rounds.  usage: tools/prof_stall.sh <tag> [bench args]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/${1:-r06_stall}; shift
mkdir -p $o
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wire --host-staged 0 $*"
tools/gpu_step.sh 60 $o/list.log timeout -s KILL 50 rocprofv3 -L || exit 1
P1="SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VMEM,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_SCA"
P2="SQ_WAVES,SQ_BUSY_CYCLES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_INSTS_LDS,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE"
tools/gpu_step.sh 300 $o/p1.log timeout -s KILL 280 rocprofv3 --pmc $P1 -d $o/p1 -o run --output-format csv -- $B || exit 1
tools/gpu_step.sh 300 $o/p2.log timeout -s KILL 280 rocprofv3 --pmc $P2 -d $o/p2 -o run --output-format csv -- $B || exit 1
python tools/stall_summary.py $o/stall.json $o/p1 $o/p2 --last 20 --workload "${WL:-C3 steady state (bench.py defaults), timed rounds}" > $o/stall.txt
