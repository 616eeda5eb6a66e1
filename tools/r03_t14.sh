#!/bin/bash
# C5 128 B: quiesce fields stored only when changed (base) vs always; the
# quiesce GPU tests first
mkdir -p gpurun_out/r03_c5q
tools/gpu_step.sh 400 gpurun_out/r03_c5q/tests.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_quiesce.py tests/test_gpu_elections.py -k "quiesce or quiesced" -m gpu || exit 1
for n in base qsall base2 qsall2; do
  if [ "${n:0:4}" = base ]; then lib=""; else lib=dragonboat_amd/_lib/variants/${n%2}.so; fi
  DRB_ENGINE_LIB=$lib tools/gpu_step.sh 300 gpurun_out/r03_c5q/$n.log python bench.py --workload c5 --payload 128 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  echo "$n $(tail -1 gpurun_out/r03_c5q/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d["counters"]["fallbacks"])')"
done
