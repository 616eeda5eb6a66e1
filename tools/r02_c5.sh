#!/bin/bash
# GPU: C5 128 B variants after a warmup past the quiesce threshold:
# listed / unlisted at 0.1 % and 1 % activity, and quiesce off.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-c5}; shift
mkdir -p "$o"
export TMPDIR=/tmp
for v in "1000 1 1" "1000 0 1" "10000 1 1" "10000 1 0"; do
  set -- $v
  tools/gpu_step.sh 400 "$o/c5_$1_l$2_q$3.log" python bench.py --workload c5 --payload 128 --active-ppm $1 --listed $2 --quiesce $3 --steps 50 --warmup ${W:-300} --no-cpu-baseline || exit 1
  echo "ppm=$1 listed=$2 quiesce=$3"
  tail -1 "$o/c5_$1_l$2_q$3.log" | grep -o '"ms_per_step": [0-9.]*\|"fallbacks": [0-9]*\|"replicas_stepped_per_round": [0-9.]*\|"committed_per_round": [0-9.]*'
done
