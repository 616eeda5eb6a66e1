set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q || exit 1
tools/gpu_step.sh 400 gpurun_out/prof_trace.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tools/gpu_step.sh 400 gpurun_out/prof_fetch.log rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline || exit 1
tools/gpu_step.sh 400 gpurun_out/prof_write.log rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline || exit 1
tail -3 gpurun_out/pytest_gpu.log
find gpurun_out/prof -name "*.csv" | head -20
