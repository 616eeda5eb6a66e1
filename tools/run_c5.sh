cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5
tools/gpu_step.sh 600 gpurun_out/c5/pytest.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c5_sparse or long_payloads or device_gen" || exit 1
tail -2 gpurun_out/c5/pytest.log
tools/gpu_step.sh 400 gpurun_out/c5/bench_128.log python bench.py --workload c5 --payload 128 --steps 30 --warmup 5 --cpu-seconds 8 || exit 1
tail -1 gpurun_out/c5/bench_128.log | cut -c1-1500
tools/gpu_step.sh 500 gpurun_out/c5/bench_1k.log python bench.py --workload c5 --payload 1024 --steps 30 --warmup 5 --no-cpu-baseline || exit 1
tail -1 gpurun_out/c5/bench_1k.log | cut -c1-1500
