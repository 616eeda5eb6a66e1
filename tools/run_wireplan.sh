#!/bin/bash
# GPU suite, then the wire encode A/B: in-tree lib vs tools/_bin/oldplan.so
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/wireplan; mkdir -p $o
tools/gpu_step.sh 400 $o/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
tail -2 $o/pytest.log
grep -q " passed" $o/pytest.log && ! grep -q failed $o/pytest.log || exit 1
for n in base oldplan base2 oldplan2; do
  lib=""; [ "${n:0:7}" = oldplan ] && lib=tools/_bin/oldplan.so
  DRB_ENGINE_LIB=$lib tools/gpu_step.sh 200 $o/$n.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  echo "$n $(tail -1 $o/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d["wire"])')"
done
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline"
tools/gpu_step.sh 300 $o/trace.log rocprofv3 --kernel-trace --stats -d $o/trace -o run --output-format csv -- $B || exit 1
f=$(find $o/trace -name "*kernel_stats.csv" | head -1); cp $f $o/kernel_stats.csv; grep wire $o/kernel_stats.csv | cut -c1-60,150-260
