set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 900 gpurun_out/pytest_gpu.log python -m pytest tests -m gpu -q -x || exit 1
tail -2 gpurun_out/pytest_gpu.log
for W in def 3 4; do
  if [ $W = def ]; then unset DRB_ENGINE_LIB; else export DRB_ENGINE_LIB=$PWD/dragonboat_amd/_lib/var/w$W.so; fi
  tools/gpu_step.sh 400 gpurun_out/prof6_$W.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof6/$W -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --tick-every 1 || exit 1
  echo "== $W"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/prof6_$W.log; grep step_kernel gpurun_out/prof6/$W/run_kernel_stats.csv | cut -d, -f1-4
done
