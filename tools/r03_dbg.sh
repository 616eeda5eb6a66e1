#!/bin/bash
mkdir -p gpurun_out
DRB_ENGINE_LIB=dragonboat_amd/_lib/dbgx5.so tools/gpu_step.sh 200 gpurun_out/xfer5d.log python -u tools/dbg/xfer5.py || exit 1
