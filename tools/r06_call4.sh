#!/bin/bash
# round 6: lean kernel (sequential) parity, the default bench line, C5 and
# the C5 128 B PMC passes
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_k; mkdir -p $o
tools/gpu_tests.sh r06_k 900 tests/test_gpu_lean.py tests/test_gpu_quiesce.py || exit 1
tools/gpu_step.sh 500 $o/bench_c3.log python bench.py || exit 1
grep -E '^\{' $o/bench_c3.log > $o/bench_c3.json
tools/gpu_step.sh 400 $o/bench_c5_128.log python bench.py --workload c5 --payload 128 --no-cpu-baseline || exit 1
grep -E '^\{' $o/bench_c5_128.log > $o/bench_c5_128.json
tools/prof_workloads.sh r06_k/pmc c5_128 || exit 1
python - <<'PY'
import json
for f in ("gpurun_out/r06_k/bench_c3.json", "gpurun_out/r06_k/bench_c5_128.json"):
    d = json.load(open(f)); c = d["counters"]
    print(f, round(d["ms_per_step"], 4), round(d["roofline"]["frac"], 4), c["fallbacks"], c.get("lean_stepped_per_round"),
          {k: (round(v["ms_per_step"], 3), v.get("download_bytes_per_round"), v.get("upload_bytes_per_round")) for k, v in d.items() if isinstance(v, dict) and "ms_per_step" in v})
s = json.load(open("gpurun_out/r06_k/pmc/c5_128/pmc_summary.json"))
print("c5 pmc", s["round_hbm_bytes"], s["round_hbm_bytes_lower"])
for k, v in s["kernels"].items():
    if "kernel" in k: print(k[:60], round(v["hbm_bytes"] / 1e6, 1))
PY
