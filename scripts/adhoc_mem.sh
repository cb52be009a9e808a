cd $GRAFT_REPO_ROOT
for c in C1 C2 C4 C5; do
  bash scripts/gpu_mem.sh mem_r03_$c $c || exit $?
done
