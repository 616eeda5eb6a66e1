#!/bin/bash
# A/B of wire-ingest settings within ONE GPU call: each spec is
# label:ENV=V,ENV2=V and runs bench.py's C3 wire ingest (from a pageable
# and from a pinned stream) with those settings, twice, in alternation.
# usage: tools/ab_ingest.sh <outdir> spec...
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/$1; shift
mkdir -p "$o"
for rep in 1 2; do
  for spec in "$@"; do
    IFS=: read -r label envs <<< "$spec"
    envl=$(echo "$envs" | tr ',' ' ')
    log="$o/$label.$rep.log"
    env $envl tools/gpu_step.sh 240 "$log" python bench.py \
      --steps 5 --warmup 2 --no-cpu-baseline --host-staged 0 || exit 1
    echo "$label $(tail -1 "$log" | python -c 'import json,sys; d=json.loads(sys.stdin.read())["wire"]; print(round(d["ingest"]["ms"],3), round(d["ingest_pinned"]["ms"],3), d["ingest_pinned"]["accepted"], d["ingest"]["accepted"])')"
  done
done
