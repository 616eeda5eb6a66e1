cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c4
tools/gpu_step.sh 300 gpurun_out/c4/bench_c4_n1.log python bench.py --workload c4 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
tail -1 gpurun_out/c4/bench_c4_n1.log | cut -c1-900
tools/gpu_step.sh 300 gpurun_out/c4/bench_c3.log python bench.py --steps 30 --warmup 5 --no-cpu-baseline || exit 1
tail -1 gpurun_out/c4/bench_c3.log | cut -c1-300
