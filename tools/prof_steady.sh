#!/bin/bash
# HEAD profile at the KV steady state: the bench JSON, the kernel trace and
# the two HBM PMC passes over the timed rounds (last 20 launches of each
# kernel).  usage: tools/prof_steady.sh <tag> [bench args]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/${1:-r03_head}; shift
mkdir -p $o
tools/gpu_step.sh 400 $o/bench.log python bench.py "$@" || exit 1
tail -1 $o/bench.log > $o/bench.json
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wire --host-staged 0 $*"
tools/gpu_step.sh 300 $o/trace.log rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- $B || exit 1
python tools/trace_summary.py $o/trace 20 $o/kernels_last20.csv > $o/kernels_last20.txt
tools/gpu_step.sh 300 $o/fetch.log timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d $o/fetch -o run --output-format csv -- $B || exit 1
tools/gpu_step.sh 300 $o/write.log timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d $o/write -o run --output-format csv -- $B || exit 1
python tools/pmc_summary.py "$(dirname $(find $o/fetch -name '*counter_collection.csv' | head -1))" \
  "$(dirname $(find $o/write -name '*counter_collection.csv' | head -1))" $o/pmc_summary.json --workload "C3 at the KV steady state (bench.py --kv-fill 1536), timed rounds only (--last 20)" --last 20
