set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x || exit 1
for W in 1 3 4; do
  DRB_ENGINE_LIB=$PWD/dragonboat_amd/_lib/var/w$W.so tools/gpu_step.sh 300 gpurun_out/bench_w$W.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tick-every 1 || exit 1
done
tools/gpu_step.sh 400 gpurun_out/prof4_trace.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof4/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tick-every 1 || exit 1
tail -3 gpurun_out/pytest_gpu.log
for W in 1 3 4; do tail -1 gpurun_out/bench_w$W.log | cut -c1-300; done
cat gpurun_out/prof4/trace/run_kernel_stats.csv | cut -c1-200
