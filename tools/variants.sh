#!/bin/bash
# Builds timing variants of the engine into tools/_bin/ (CPU side):
#   tools/variants.sh name "-DFOO=1 -DBAR=2" [name2 "defs2" ...]
# and bench.py picks one with DRB_ENGINE_LIB=tools/_bin/<name>.so.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_bin
while [ $# -ge 2 ]; do
  n=$1; d=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-pass-failed \
    $d -o tools/_bin/$n.so dragonboat_amd/csrc/drb_engine.hip &
done
wait
ls -la tools/_bin
