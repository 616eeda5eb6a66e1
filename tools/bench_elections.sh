#!/bin/bash
# GPU: the elections tests, then C3 with and without elections on the GPU
# (steady state), then the 1M-group failover.  Each step under its own limit.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-elections}
mkdir -p "$o"
export TMPDIR=/tmp
tools/gpu_step.sh 600 "$o/pytest_gpu.log" python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -k "elections or census" || exit 1
tail -3 "$o/pytest_gpu.log"
B="--steps 30 --warmup 5 --no-cpu-baseline --no-wire --host-staged 0"
tools/gpu_step.sh 300 "$o/c3_plain.log" python bench.py $B || exit 1
tail -1 "$o/c3_plain.log" > "$o/c3_plain.json"
tools/gpu_step.sh 300 "$o/c3_elections.log" python bench.py $B --elections 1 --failover || exit 1
tail -1 "$o/c3_elections.log" > "$o/c3_elections.json"
python - "$o" <<'PY'
import json, sys
for n in ("c3_plain", "c3_elections"):
    d = json.load(open(sys.argv[1] + "/" + n + ".json"))
    print(n, "%.3f ms" % d["ms_per_step"], "%.1f M/s" % (d["value"] / 1e6),
          json.dumps(d.get("failover")))
PY
