cd $GRAFT_REPO_ROOT
bash tools/run_dbg.sh e2a4r1 e3a4 || exit 1
tools/gpu_step.sh 900 gpurun_out/exp10_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
tail -3 gpurun_out/exp10_pytest.log
