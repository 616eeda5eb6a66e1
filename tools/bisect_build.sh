#!/bin/bash
# Builds older commits for tools/bisect_run.sh: a git worktree per commit
# under _bisect/ (git-ignored; it travels to the GPU box with the tree),
# each with its own in-tree engine build, the build objects removed after.
# usage: tools/bisect_build.sh sha...
cd "$(dirname "$0")/.."
mkdir -p _bisect
for s in "$@"; do
  [ -d "_bisect/$s" ] || git worktree add -f "_bisect/$s" "$s" > /dev/null
  t0=$(date +%s)
  (cd "_bisect/$s" && python dragonboat_amd/build.py > build.log 2>&1)
  echo "$s rc=$? $(( $(date +%s) - t0 ))s"
  rm -rf "_bisect/$s/dragonboat_amd/_lib/obj" "_bisect/$s/dragonboat_amd/_lib/obj_"*
done
