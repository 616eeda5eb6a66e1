set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x || exit 1
tail -2 gpurun_out/pytest_gpu.log
tools/gpu_step.sh 400 gpurun_out/bench9.log python bench.py || exit 1
tail -1 gpurun_out/bench9.log
tools/gpu_step.sh 400 gpurun_out/prof9.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof9/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
grep -E "step_kernel|serve" gpurun_out/prof9/trace/run_kernel_stats.csv | cut -c1-160
