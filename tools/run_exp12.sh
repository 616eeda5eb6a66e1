cd $GRAFT_REPO_ROOT
tools/gpu_step.sh 900 gpurun_out/exp12_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
tail -2 gpurun_out/exp12_pytest.log
tools/exp_variants.sh exp12 "base_c5:--workload c5 --payload 128" "ext3:--workload c5 --payload 128" base head
