#!/bin/bash
# gpurun with retries on infrastructure-side failures (status=transient,
# backing off, no box): usage tools/gpurun_retry.sh <out> <timeout> <cmd>
out=$1; t=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient\|backing off" "$out" || [ $rc = 3 ]; then
    sleep 150; continue
  fi
  exit $rc
done
exit 3
