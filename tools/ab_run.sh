#!/bin/bash
# A/B of engine settings within ONE GPU call (box-to-box spread is ~5 %,
# same-box repeats agree to ~0.2 %): each spec is label:ENV=V,ENV2=V:args
# and runs bench.py at C3 with those environment settings and extra args.
# usage: tools/ab_run.sh <outdir> spec...
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; shift
mkdir -p "$o"
for spec in "$@"; do
  IFS=: read -r label envs args <<< "$spec"
  envl=$(echo "$envs" | tr ',' ' ')
  env $envl tools/gpu_step.sh 240 "$o/$label.log" python bench.py --steps 40 \
    --warmup 8 --no-cpu-baseline --no-wire --host-staged 0 $args || exit 1
  echo "$label $(tail -1 "$o/$label.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), round(d["roofline"]["kernel_ms"],4), d["counters"]["fallbacks"], d["counters"]["reads_served"])')"
done
