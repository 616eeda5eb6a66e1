#!/bin/bash
# round 6: zero-copy in-process exchange (drb_exchange_local_bind) --
# parity (small spread cases, the refusals, C4 at full size), the
# --local-ranks 8 line bound vs pull, and C3 with / without the peer reads
# compiled in (DRB_PEERS=0 variant), alternated
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/r06_q; mkdir -p $o
tools/gpu_tests.sh r06_q 1000 tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "spread or bound" || exit 1
for m in bind pull; do
  tools/gpu_step.sh 300 $o/c4l8_$m.log python bench.py --workload c4 --local-ranks 8 --local-exchange $m --no-cpu-baseline || exit 1
done
for rep in 1 2; do
  tools/gpu_step.sh 400 $o/c3_peers_$rep.log python bench.py --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
  DRB_ENGINE_LIB=dragonboat_amd/_lib/variants/nopeers.so tools/gpu_step.sh 400 $o/c3_nopeers_$rep.log python bench.py --no-cpu-baseline --host-staged 0 --step-worker 0 --no-wire || exit 1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r06_q/c*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f.split("/")[-1], round(d["ms_per_step"], 4), d["counters"]["fallbacks"] if "counters" in d else "", d.get("exchange", {}).get("bytes_per_round_per_rank", ""))
PY
