cd $GRAFT_REPO_ROOT
tools/gpu_step.sh 600 gpurun_out/exp6_pytest.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "read or c3 or write_rounds_r3 or idle" || exit 1
tail -2 gpurun_out/exp6_pytest.log
grep -q "failed" gpurun_out/exp6_pytest.log && exit 1
tools/exp_variants.sh exp6 base nosplit head base_b nosplit head
