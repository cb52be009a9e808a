#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_mem.sh ${1:-final}_C5 C5 || exit $?
bash scripts/gpu_valu.sh ${1:-final}_valu C2 || exit $?
bash scripts/gpu_rehearsal.sh ${1:-final}_reh || exit $?
exit 0
