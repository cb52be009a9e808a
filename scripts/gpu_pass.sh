#!/bin/bash
# The round's profile pass on the production library: GPU tests, smoke, bench
# lines for every config, kernel traces and FETCH/WRITE passes
# (scripts/gpu_round.sh), then the C2 unit counters (scripts/gpu_mem.sh).
#   bash scripts/gpu_pass.sh <tag>
# then: python3 scripts/summarize_round.py gpurun_out/<tag> <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${1:-pass}
bash scripts/gpu_round.sh $TAG || exit $?
bash scripts/gpu_mem.sh ${TAG}_mem_c2 C2 || exit $?
