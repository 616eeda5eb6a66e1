#!/bin/bash
# Times the C3 step round of older commits against HEAD in ONE GPU call
# (box-to-box spread is ~5 %).  Each _bisect/<sha> is a git
# worktree of that commit with its own in-tree build (tools/bisect_build.sh);
# its own bench.py runs there.  usage: tools/bisect_run.sh <outdir> sha...
# ("head" = this tree, "head-fill" = this tree at the default KV fill).
# Every other run is at --kv-fill 0 (round 2's benchmark had no fill; a
# commit without the flag runs as is).
R=$GRAFT_REPO_ROOT
cd "$R"
o=$R/gpurun_out/$1; shift
mkdir -p "$o"
A="--steps 40 --warmup 8 --no-cpu-baseline --no-wire --host-staged 0"
for sha in "$@"; do
  d=$R/_bisect/$sha
  fill="--kv-fill 0"
  case $sha in head) d=$R;; head-fill) d=$R; fill="";; esac
  grep -q -- "--kv-fill" "$d/bench.py" || fill=""
  extra=""
  grep -q -- "--step-worker" "$d/bench.py" && extra="--step-worker 0"
  echo "== $(date +%T) $sha" >> "$o/steps.log"
  (cd "$d" && timeout -k 10 240 python bench.py $A $fill $extra) > "$o/$sha.log" 2>&1
  rc=$?
  echo "== rc=$rc $(date +%T)" >> "$o/steps.log"
  case $rc in 0) ;; *) echo "FATAL rc=$rc in $sha"; exit 99;; esac
  echo "$sha $(tail -1 $o/$sha.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), round(d["roofline"]["kernel_ms"],4), d["counters"]["fallbacks"])')"
done
