#!/bin/bash
# Usage on the GPU box: bash scripts/gpu_ab.sh [ab.py args...]  (variants/*.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 scripts/ab.py "$@" 2>&1 | tee gpurun_out/ab.log
