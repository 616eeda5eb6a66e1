cd $GRAFT_REPO_ROOT
tools/gpu_prof.sh r01_packed --no-tests --steps 40 --warmup 8 || exit 1
tools/exp_variants.sh exp8 base lw2 fw5 fw3 base_b head
