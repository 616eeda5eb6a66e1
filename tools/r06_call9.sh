#!/bin/bash
# round 6: where the in-process 8-rank C4 round goes (kernel trace)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
o=gpurun_out/r06_p; mkdir -p $o
tools/gpu_step.sh 300 $o/c4l8.log python bench.py --workload c4 --local-ranks 8 --no-cpu-baseline || exit 1
grep -E '^\{' $o/c4l8.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4l8', d['ms_per_step'], d.get('exchange'))"
tools/gpu_step.sh 300 $o/trace.log rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- python bench.py --workload c4 --local-ranks 8 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
python tools/trace_summary.py $o/trace 160 $o/kernels.csv > $o/kernels.txt
head -20 $o/kernels.txt
python tools/trace_union.py $o/trace k_plane_pull 80 > $o/union.txt
cat $o/union.txt | head -20
