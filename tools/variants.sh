#!/bin/bash
# Builds timing variants of the engine into dragonboat_amd/_lib/variants/:
#   tools/variants.sh name "-DFOO=1 -DBAR=2" [name2 "defs2" ...]
# (the R = 3 step kernels with the defines, the rest from the in-tree
# build) and bench.py picks one with
# DRB_ENGINE_LIB=dragonboat_amd/_lib/variants/<name>.so.
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  n=$1; d=$2; shift 2
  python dragonboat_amd/build.py --variant $n $d &
done
wait
ls -la dragonboat_amd/_lib/variants
