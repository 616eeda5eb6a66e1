set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 300 gpurun_out/bench5.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tick-every 1 || exit 1
tail -1 gpurun_out/bench5.log | cut -c1-1200
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x || exit 1
tail -3 gpurun_out/pytest_gpu.log
