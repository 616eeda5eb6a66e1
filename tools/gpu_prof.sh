#!/bin/bash
# One GPU call: parity tests, the default bench, a rocprofv3 kernel trace
# and the two HBM PMC passes of the same bench, summarised into
# gpurun_out/<tag>/.  Every GPU step runs under its own time limit and the
# call stops at the first fault / abort / timeout (tools/gpu_step.sh).
# usage: tools/gpu_prof.sh <tag> [--no-tests] [extra bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
tests=1
if [ "$1" = "--no-tests" ]; then tests=0; shift; fi
o=gpurun_out/$tag
mkdir -p "$o"
export TMPDIR=/tmp
if [ $tests = 1 ]; then
  tools/gpu_step.sh 600 "$o/pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
  tail -3 "$o/pytest_gpu.log"
  grep -q " passed" "$o/pytest_gpu.log" || exit 1
  grep -q "failed\|error" "$o/pytest_gpu.log" && { grep -i "failed\|error" "$o/pytest_gpu.log" | head -20; }
fi
tools/gpu_step.sh 400 "$o/bench.log" python bench.py "$@" || exit 1
tail -1 "$o/bench.log" > "$o/bench.json"
cut -c1-400 "$o/bench.json"
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tick-every 1 $*"
tools/gpu_step.sh 300 "$o/trace.log" rocprofv3 --kernel-trace --stats -d "$o/trace" -o run --output-format csv -- $B || exit 1
tools/gpu_step.sh 200 "$o/fetch.log" rocprofv3 --pmc FETCH_SIZE -d "$o/fetch" -o run --output-format csv -- $B || exit 1
tools/gpu_step.sh 200 "$o/write.log" rocprofv3 --pmc WRITE_SIZE -d "$o/write" -o run --output-format csv -- $B || exit 1
f=$(ls "$o"/trace/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -z "$f" ] && f=$(find "$o/trace" -name "*kernel_stats.csv" | head -1)
cp "$f" "$o/kernel_stats.csv" && head -8 "$o/kernel_stats.csv" | cut -c1-200
python tools/pmc_summary.py "$(dirname $(find $o/fetch -name '*counter_collection.csv' | head -1))" \
  "$(dirname $(find $o/write -name '*counter_collection.csv' | head -1))" "$o/pmc_summary.json" --workload C3
