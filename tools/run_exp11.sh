cd $GRAFT_REPO_ROOT
tools/exp_variants.sh exp11 base w1 w2 wr1 w8 "base_k:--kv-slots 1024" "w1_k:--kv-slots 1024" "wr1_k:--kv-slots 1024" base_c head
