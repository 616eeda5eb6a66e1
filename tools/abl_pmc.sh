# per variant: timing + FETCH/WRITE passes -> gpurun_out/abl/<name>_{bench,fetch,write}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/abl; mkdir -p $o
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tick-every 1"
for n in "$@"; do
  if [ "${n:0:4}" = base ]; then lib=""; else lib=dragonboat_amd/_lib/variants/$n.so; fi
  export DRB_ENGINE_LIB=$lib
  tools/gpu_step.sh 200 $o/${n}_bench.log python bench.py --steps 40 --warmup 8 --no-cpu-baseline || exit 1
  tools/gpu_step.sh 200 $o/${n}_fetch.log rocprofv3 --pmc FETCH_SIZE -d $o/${n}_fetch -o run --output-format csv -- $B || exit 1
  tools/gpu_step.sh 200 $o/${n}_write.log rocprofv3 --pmc WRITE_SIZE -d $o/${n}_write -o run --output-format csv -- $B || exit 1
  python tools/pmc_summary.py $o/${n}_fetch $o/${n}_write $o/${n}_pmc.json >/dev/null
  python - $o/${n}_pmc.json $o/${n}_bench.log $n <<'PY'
import json,sys
d=json.load(open(sys.argv[1])); b=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
G=d["groups"]; ks=d["kernels"]
s=" ".join("%s F%.0f W%.0f"%("L" if "true" in k else "F", v.get("FETCH_SIZE",0)/G, v.get("WRITE_SIZE",0)/G) for k,v in ks.items() if "step_kernel" in k)
print(sys.argv[3], round(b["ms_per_step"],4), "fb", b["counters"]["fallbacks"], s)
PY
done
