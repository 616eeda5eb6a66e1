set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof3
export TMPDIR=/tmp
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x || exit 1
tools/gpu_step.sh 400 gpurun_out/bench_t1.log python bench.py --steps 30 --warmup 5 --no-cpu-baseline --tick-every 1 || exit 1
tools/gpu_step.sh 400 gpurun_out/bench_auto.log python bench.py --steps 30 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh 400 gpurun_out/prof3_trace.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof3/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tick-every 1 || exit 1
tools/gpu_step.sh 400 gpurun_out/prof3_fetch.log rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof3/fetch -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --tick-every 1 || exit 1
tools/gpu_step.sh 400 gpurun_out/prof3_write.log rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof3/write -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --tick-every 1 || exit 1
tail -3 gpurun_out/pytest_gpu.log
tail -1 gpurun_out/bench_t1.log | cut -c1-600
tail -1 gpurun_out/bench_auto.log | cut -c1-600
