#!/bin/bash
# round 6: tests of the new paths, then C5 lean vs full A/B, and the C2
# drb_step_rounds A/B
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_e; mkdir -p $o
tools/gpu_tests.sh r06_e 1000 tests/test_gpu_worker.py tests/test_gpu_staging.py \
  tests/test_gpu_propose.py::test_legacy_ingest_reports_diversion \
  tests/test_gpu_xplan.py tests/test_gpu_bench_dist.py tests/test_gpu_rounds.py \
  "tests/test_gpu_fullsize.py::test_fullsize_c4_spread_sampled" || exit 1
B="python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline"
tools/gpu_step.sh 400 $o/c5_lean.log $B || exit 1
tools/gpu_step.sh 400 $o/c5_full.log $B --no-lean || exit 1
tools/gpu_step.sh 300 $o/c2_ab.log python bench.py --workload c2 --steps 40 --warmup 8 --no-cpu-baseline --no-wire --host-staged 0 --chunk-ab 65536:8,65536:16,32768:8,16384:8,16384:16 || exit 1
for f in c5_lean c5_full c2_ab; do tail -1 $o/$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"][:30], round(d["ms_per_step"],4), d["counters"]["fallbacks"], d.get("chunk_ab"))'; done
