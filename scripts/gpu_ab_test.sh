#!/bin/bash
# A/B variants, then the GPU test suite of the in-tree library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 scripts/ab.py "$@" 2>&1 | tee gpurun_out/ab.log
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python3 -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; grep -h "nodes/ray\|pixels differ" gpurun_out/pytest_gpu.log
exit $rc
