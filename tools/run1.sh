set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -x -q || exit 1
tools/gpu_step.sh 300 gpurun_out/bench_small.log python bench.py --groups 65536 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh 400 gpurun_out/bench_1m.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/bench_small.log; tail -2 gpurun_out/bench_1m.log
