#!/bin/bash
# A round's closing measurements in one call: the default bench (C3 with
# the CPU baseline, wire, host-staged and step-worker lines), the other
# workloads' lines at N = 1, then the C3 kernel trace and the two HBM PMC
# passes of the timed rounds at the KV steady state (tools/prof_steady.sh's
# recipe).  usage: tools/final_run.sh <tag>
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/${1:-r05_final}
mkdir -p $o
tools/gpu_step.sh 400 $o/bench_c3.log python bench.py || exit 1
grep -E '^\{' $o/bench_c3.log > $o/bench_c3.json
for w in "c2" "c4" "c5 --payload 128" "c5 --payload 1024"; do
  n=$(echo $w | tr -d ' -' | sed 's/payload/_/')
  tools/gpu_step.sh 300 $o/bench_$n.log python bench.py --workload $w --no-cpu-baseline || exit 1
  grep -E '^\{' $o/bench_$n.log > $o/bench_$n.json
done
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wire --host-staged 0 --step-worker 0"
tools/gpu_step.sh 300 $o/trace.log rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- $B || exit 1
python tools/trace_summary.py $o/trace 20 $o/kernels_last20.csv > $o/kernels_last20.txt
tools/gpu_step.sh 300 $o/fetch.log timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d $o/fetch -o run --output-format csv -- $B || exit 1
tools/gpu_step.sh 300 $o/write.log timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d $o/write -o run --output-format csv -- $B || exit 1
python tools/pmc_summary.py "$(dirname $(find $o/fetch -name '*counter_collection.csv' | head -1))" \
  "$(dirname $(find $o/write -name '*counter_collection.csv' | head -1))" $o/pmc_summary.json --workload "C3 at the KV steady state (bench.py --kv-fill 1536), timed rounds only (--last 20)" --last 20
