set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tools/gpu_step.sh 120 gpurun_out/calib.log tools/_bin/calib_hbm || exit 1
tools/gpu_step.sh 200 gpurun_out/calib_fetch.log rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib/fetch -o run --output-format csv -- tools/_bin/calib_hbm || exit 1
tools/gpu_step.sh 200 gpurun_out/calib_write.log rocprofv3 --pmc WRITE_SIZE -d gpurun_out/calib/write -o run --output-format csv -- tools/_bin/calib_hbm || exit 1
cat gpurun_out/calib.log
