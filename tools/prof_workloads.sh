#!/bin/bash
# The two HBM PMC passes (FETCH_SIZE, WRITE_SIZE) of the timed rounds of
# each non-C3 workload at N = 1 -> per-workload summaries that bench.py
# reads as roofline.traffic (profiles/pmc_<workload>.json).
# usage: tools/prof_workloads.sh <tag> [workload ...]
#   workloads: c2 c4 c5_128 c5_1024 (default: all four)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r05_pmc}; shift
wls=${*:-c2 c4 c5_128 c5_1024}
for wl in $wls; do
  o=gpurun_out/$tag/$wl
  mkdir -p $o
  case $wl in
    c2) a="--workload c2"; G=65536; R=3;;
    c4) a="--workload c4"; G=1048576; R=5;;
    c5_128) a="--workload c5 --payload 128"; G=4194304; R=3;;
    c5_1024) a="--workload c5 --payload 1024"; G=4194304; R=3;;
    *) echo "unknown workload $wl"; exit 1;;
  esac
  B="python bench.py $a --steps 20 --warmup 5 --no-cpu-baseline --no-wire --host-staged 0 --step-worker 0"
  tools/gpu_step.sh 300 $o/fetch.log timeout -s KILL 280 rocprofv3 --pmc FETCH_SIZE -d $o/fetch -o run --output-format csv -- $B || exit 1
  tools/gpu_step.sh 300 $o/write.log timeout -s KILL 280 rocprofv3 --pmc WRITE_SIZE -d $o/write -o run --output-format csv -- $B || exit 1
  python tools/pmc_summary.py "$(dirname $(find $o/fetch -name '*counter_collection.csv' | head -1))" \
    "$(dirname $(find $o/write -name '*counter_collection.csv' | head -1))" $o/pmc_summary.json \
    --groups $G --replicas $R --workload "$wl at N = 1 ($B), timed rounds only (--last 20)" --last 20 || exit 1
done
