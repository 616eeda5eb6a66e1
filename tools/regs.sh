#!/bin/bash
# VGPR / SGPR / spill / LDS / occupancy of the step kernels (R=3, R=5)
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Wno-pass-failed \
  -Rpass-analysis=kernel-resource-usage "$@" /root/repo/dragonboat_amd/csrc/drb_engine.hip -o /tmp/regs.o 2>&1 |
  grep -A11 "Function Name: .*\(step_kernelILi[35]E\|serve_reads\)" |
  grep "Function Name\|VGPRs:\|SGPRs Spill\|VGPRs Spill\|Occupancy\|LDS Size\|ScratchSize" |
  sed 's/.*remark: *//; s/ \[-Rpass.*//'
