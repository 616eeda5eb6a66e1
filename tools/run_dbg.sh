cd $GRAFT_REPO_ROOT
for n in "$@"; do
  echo "== $n"
  DRB_ENGINE_LIB=tools/_bin/$n.so timeout -k 10 120 python tools/dbg_saves.py 2>&1 | grep round || exit 1
done
