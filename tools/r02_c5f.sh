#!/bin/bash
# GPU: C5 bench lines at the SURVEY 8d shape (1 % active, Quiesce on,
# listed rounds) for 128 B and 1 KB payloads, after a warmup past the
# quiesce threshold; the fallback histogram is in each JSON line.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-c5f}
mkdir -p "$o"
export TMPDIR=/tmp
for pl in 128 1024; do
  tools/gpu_step.sh 500 "$o/c5_$pl.log" python bench.py --workload c5 --payload $pl --steps 50 --warmup ${W:-300} --no-cpu-baseline || exit 1
  tail -1 "$o/c5_$pl.log" | grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.e+]*\|"fallbacks": [0-9]*\|"fallbacks_by_reason": {[^}]*}\|"replicas_stepped_per_round": [0-9.]*'
done
