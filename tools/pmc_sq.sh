cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
o=gpurun_out/sq; mkdir -p $o
B="python bench.py --steps 10 --warmup 3 --no-cpu-baseline --tick-every 1"
tools/gpu_step.sh 200 $o/sq1.log timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAIT_INST_ANY -d $o/p1 -o run --output-format csv -- $B || exit 1
tools/gpu_step.sh 200 $o/sq2.log timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d $o/p2 -o run --output-format csv -- $B || exit 1
python - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/sq/p1", "gpurun_out/sq/p2"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].split("(")[0]
        if "step_kernel" in n:
            acc[(n, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items()):
        print(k[0][-30:], k[1], round(sum(v) / len(v)))
PY
