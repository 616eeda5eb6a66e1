set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x || exit 1
tail -2 gpurun_out/pytest_gpu.log
tools/gpu_step.sh 400 gpurun_out/bench10.log python bench.py --no-cpu-baseline || exit 1
tail -1 gpurun_out/bench10.log | cut -c1-400
tools/gpu_step.sh 400 gpurun_out/prof10.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof10/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
grep -E "step_kernel|serve" gpurun_out/prof10/trace/run_kernel_stats.csv | cut -c1-160
tools/gpu_step.sh 400 gpurun_out/prof10_f.log rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof10/fetch -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline || exit 1
tools/gpu_step.sh 400 gpurun_out/prof10_w.log rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof10/write -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline || exit 1
python tools/pmc_summary.py gpurun_out/prof10/fetch gpurun_out/prof10/write gpurun_out/prof10/pmc_summary.json --workload C3
