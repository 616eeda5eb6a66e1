#!/bin/bash
# GPU check of a build: the whole -m gpu suite (no -x: every failure is
# listed), then short C3 and C5 bench lines.  Each step under its own limit.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-r02}
mkdir -p "$o"
export TMPDIR=/tmp
tools/gpu_step.sh 900 "$o/pytest_gpu.log" python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread || exit 1
tail -5 "$o/pytest_gpu.log"
grep -E "FAILED|ERROR" "$o/pytest_gpu.log" | head -30
tools/gpu_step.sh 300 "$o/bench_c3.log" python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wire || exit 1
tail -1 "$o/bench_c3.log" | cut -c1-600
tools/gpu_step.sh 400 "$o/bench_c5.log" python bench.py --workload c5 --payload 128 --steps 30 --warmup 5 --no-cpu-baseline || exit 1
tail -2 "$o/bench_c5.log" | cut -c1-900
