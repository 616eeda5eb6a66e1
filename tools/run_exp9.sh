cd $GRAFT_REPO_ROOT
tools/gpu_step.sh 900 gpurun_out/exp9_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
tail -3 gpurun_out/exp9_pytest.log
grep -q " passed" gpurun_out/exp9_pytest.log || exit 1
grep -q "failed" gpurun_out/exp9_pytest.log && exit 1
tools/exp_variants.sh exp9 base pw1 pw2 pw8 "base_k:--kv-slots 1024" "pw1:--kv-slots 1024" "pw2:--kv-slots 1024" base_c
