#!/bin/bash
# GPU box rehearsal of the multi-rank bench control flow (what the driver's
# 8-GPU scaling run executes with nccl): 2 ranks over gloo sharing the one
# GPU, C3 groups per rank, each step under its own limit.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-dist}
mkdir -p "$o"
export TMPDIR=/tmp
tools/gpu_step.sh 600 "$o/bench_2ranks.log" python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 3 --no-cpu-baseline --no-wire --host-staged 0 --groups 262144 || exit 1
grep '^{' "$o/bench_2ranks.log" | cut -c1-700
