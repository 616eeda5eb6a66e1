#!/bin/bash
# GPU: the persistence outputs side by side on one box -- C3 with no saves,
# EntryBatch + CRC and tan records; C5 128 B / 1 KB with EntryBatch and tan.
# Each bench under its own limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT"
o=gpurun_out/${1:-saves}
mkdir -p "$o"
export TMPDIR=/tmp
B="--steps 30 --warmup 5 --no-cpu-baseline --no-wire --host-staged 0"
for s in none entrybatch tan tanmux; do
  tools/gpu_step.sh 300 "$o/c3_$s.log" python bench.py $B --save $s || exit 1
  tail -1 "$o/c3_$s.log" > "$o/c3_$s.json"
done
for p in 128 1024; do
  for s in entrybatch tan tanmux; do
    tools/gpu_step.sh 400 "$o/c5_${p}_$s.log" python bench.py $B --workload c5 --payload $p --save $s || exit 1
    tail -1 "$o/c5_${p}_$s.log" > "$o/c5_${p}_$s.json"
  done
done
python - "$o" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.load(open(f))
    c = d["counters"]
    print(os.path.basename(f), "%.3f ms" % d["ms_per_step"], "%.1f M/s" % (d["value"] / 1e6),
          "saved_bytes/round %.0f" % (c["saved_bytes"] / d["steps"]),
          "recs", c.get("log_records"), "syncs", c.get("log_syncs"), "fb", c["fallbacks"])
PY
