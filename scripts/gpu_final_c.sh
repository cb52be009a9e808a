#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for cfg in ${CFGS:-C2 C3}; do
  bash scripts/gpu_mem.sh ${1:-final}_$cfg $cfg || exit $?
done
exit 0
