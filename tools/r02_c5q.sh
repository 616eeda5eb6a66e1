#!/bin/bash
# GPU: full -m gpu suite, then C5 (128 B) with Quiesce at 1 % and 0.1 %
# activity after a warmup past the quiesce threshold (200 ticks).
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-c5q}
mkdir -p "$o"
export TMPDIR=/tmp
tools/gpu_step.sh 900 "$o/pytest_gpu.log" python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread || exit 1
tail -3 "$o/pytest_gpu.log"
grep -E "FAILED|ERROR" "$o/pytest_gpu.log" | head -30
for ppm in 10000 1000; do
  tools/gpu_step.sh 400 "$o/c5_$ppm.log" python bench.py --workload c5 --payload 128 --active-ppm $ppm --steps 50 --warmup 300 --no-cpu-baseline || exit 1
  tail -2 "$o/c5_$ppm.log" | cut -c1-300
  tail -1 "$o/c5_$ppm.log" | grep -o '"ms_per_step": [0-9.]*\|"fallbacks": [0-9]*\|"kernel_ms": [0-9.]*'
done
tools/gpu_step.sh 400 "$o/c5_noq.log" python bench.py --workload c5 --payload 128 --quiesce 0 --steps 50 --warmup 300 --no-cpu-baseline || exit 1
tail -1 "$o/c5_noq.log" | grep -o '"ms_per_step": [0-9.]*\|"fallbacks": [0-9]*\|"kernel_ms": [0-9.]*'
