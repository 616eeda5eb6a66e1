#!/bin/bash
# full suite; C5 128 B with and without the remotes' dirty-field stores; C3
mkdir -p gpurun_out/r03_c5
tools/gpu_step.sh 1000 gpurun_out/t8.log python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests -m gpu || exit 1
for n in base nodirty; do
  if [ $n = base ]; then lib=""; else lib=dragonboat_amd/_lib/variants/$n.so; fi
  DRB_ENGINE_LIB=$lib tools/gpu_step.sh 300 gpurun_out/r03_c5/$n.log python bench.py --workload c5 --payload 128 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
done
tools/gpu_step.sh 300 gpurun_out/r03_c5/c3.log python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-wire || exit 1
