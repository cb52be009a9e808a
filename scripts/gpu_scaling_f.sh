#!/bin/bash
# tile_scaling.py at several frames-per-step (auto split)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in ${1:-C2 C3}; do
  for f in ${2:-8 16 32}; do
    timeout -k 10 200 python3 scripts/tile_scaling.py $c $f 0 2>&1 | grep -v amdgpu.ids | sed "s/^/F=$f /" || exit $?
  done
done 2>&1 | tee gpurun_out/scaling_f.log
