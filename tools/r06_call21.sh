#!/bin/bash
# round 6: C2 through drb_step_rounds (one chunk of every group: plain
# rounds from one C call) -- parity, then the c2 line at 1 / 8 / 16 rounds
# per call, alternated
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_c2b; mkdir -p $o
tools/gpu_tests.sh r06_c2b 600 tests/test_gpu_rounds.py || exit 1
for rep in 1 2; do
  for r in 1 8 16; do
    tools/gpu_step.sh 300 $o/c2_rpc${r}_$rep.log python bench.py --workload c2 --rounds-per-call $r --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
  done
done
tools/gpu_step.sh 300 $o/c2_default.log python bench.py --workload c2 --no-cpu-baseline || exit 1
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_c2b/c2_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); c = d["counters"]
            print(f.split("/")[-1], round(d["ms_per_step"], 4), round(d["value"]/1e6, 1), c["fallbacks"], c["committed_per_round"], d["config"].get("rounds_per_call"), round(d["roofline"]["frac"], 4))
PY
