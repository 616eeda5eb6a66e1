set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export DRB_ENGINE_LIB=$PWD/dragonboat_amd/_lib/var/w3.so
tools/gpu_step.sh 400 gpurun_out/prof7_fetch.log rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof7/fetch -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --tick-every 1 || exit 1
tools/gpu_step.sh 400 gpurun_out/prof7_write.log rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof7/write -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --tick-every 1 || exit 1
tools/gpu_step.sh 400 gpurun_out/prof7_occ.log rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/prof7/occ -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --tick-every 1 || exit 1
