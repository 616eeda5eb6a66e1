#!/bin/bash
# round 6: the ADVICE fixes, the lean worker records, partitions, the
# counted plan and the full-size C4 test; then the C2 drb_step_rounds A/B
cd "$GRAFT_REPO_ROOT"
tools/gpu_tests.sh r06_c 1000 tests/test_gpu_worker.py tests/test_gpu_staging.py \
  tests/test_gpu_propose.py::test_legacy_ingest_reports_diversion \
  tests/test_gpu_xplan.py tests/test_gpu_bench_dist.py tests/test_gpu_rounds.py \
  "tests/test_gpu_fullsize.py::test_fullsize_c4_spread_sampled" || exit 1
tools/gpu_step.sh 300 gpurun_out/r06_c/c2_ab.log python bench.py --workload c2 --steps 40 --warmup 8 --no-cpu-baseline --no-wire --host-staged 0 --chunk-ab 65536:8,65536:16,32768:8,16384:8,16384:16 || exit 1
tail -1 gpurun_out/r06_c/c2_ab.log
