#!/bin/bash
# Builds timing variants of the engine into tools/_bin/ (CPU side):
#   tools/variants.sh name "-DFOO=1 -DBAR=2" [name2 "defs2" ...]
# (the R = 3 step kernels with the defines, the rest from the in-tree
# build) and bench.py picks one with DRB_ENGINE_LIB=tools/_bin/<name>.so.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_bin
while [ $# -ge 2 ]; do
  n=$1; d=$2; shift 2
  python dragonboat_amd/build.py --variant $n $d &
done
wait
ls -la tools/_bin
