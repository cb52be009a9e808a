#!/bin/bash
# r05m: the round's profile pass on the final library -- GPU tests, smoke,
# bench lines for every config, kernel traces and FETCH/WRITE passes
# (scripts/gpu_round.sh), then the C2 unit counters (scripts/gpu_mem.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash scripts/gpu_round.sh r05m || exit $?
bash scripts/gpu_mem.sh r05m_mem_c2 C2 || exit $?
