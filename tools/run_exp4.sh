cd $GRAFT_REPO_ROOT
tools/gpu_step.sh 600 gpurun_out/exp4_pytest.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
tail -2 gpurun_out/exp4_pytest.log
grep -q " passed" gpurun_out/exp4_pytest.log || exit 1
tools/exp_variants.sh exp4 base pre_save cur34 cur33 cur24 base_b cur34 pre_save
