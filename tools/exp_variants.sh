#!/bin/bash
# usage: tools/exp_variants.sh <outdir> name[:benchargs] ...   ("base" = in-tree lib)
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; shift
mkdir -p $o
for spec in "$@"; do
  n=${spec%%:*}; a=""; [ "$spec" != "$n" ] && a=${spec#*:}
  if [ "${n:0:4}" = base ]; then lib=""; else lib=dragonboat_amd/_lib/variants/$n.so; fi
  DRB_ENGINE_LIB=$lib tools/gpu_step.sh 200 $o/$n.log python bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-wire --host-staged 0 $a || exit 1
  echo "$spec $(tail -1 $o/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), round(d["roofline"]["kernel_ms"],4), d["counters"]["fallbacks"], d["counters"]["reads_served"])')"
done
