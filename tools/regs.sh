#!/bin/bash
# VGPR / SGPR / spill / LDS / occupancy of the step kernels.
# usage: tools/regs.sh [R] [kinds...] [-- extra hipcc flags]
#   kinds: 0 lead, 1 lead ext, 2 follow, 3 follow ext, 4 raft launch
R=${1:-3}; shift
kinds=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do kinds+=("$1"); shift; done
[ "$1" == "--" ] && shift
[ ${#kinds[@]} -eq 0 ] && kinds=(0 2)
for k in "${kinds[@]}"; do
  ( cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC \
      -Wno-pass-failed --cuda-device-only -c -Rpass-analysis=kernel-resource-usage \
      -DDRB_INST_R=$R -DDRB_INST_KIND=$k "$@" \
      /root/repo/dragonboat_amd/csrc/drb_step_inst.hip -o /tmp/regs_$k.o 2>&1 |
    grep -A11 "Function Name: .*step_kernel" |
    grep "Function Name\|VGPRs:\|SGPRs Spill\|VGPRs Spill\|Occupancy\|LDS Size\|ScratchSize" |
    sed 's/.*remark: *//; s/ \[-Rpass.*//' ) &
done
wait
