#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a
# fault / abort / timeout (exit codes 124, 134, 137, 139 and their -N
# Python forms) so no further GPU work starts after one.
# usage: tools/gpu_step.sh <seconds> <logfile> <cmd...>
t=$1; shift; log=$1; shift
echo "== $(date +%T) $*" >> gpurun_out/steps.log
timeout -k 10 "$t" "$@" > "$log" 2>&1
rc=$?
echo "== rc=$rc $(date +%T)" >> gpurun_out/steps.log
case $rc in
  124|134|137|139|250|251|245|243) echo "FATAL rc=$rc in: $*"; exit 99;;
esac
exit 0
