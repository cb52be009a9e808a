#!/bin/bash
# Q4 check: A/B against the binary walk (same images expected), then the GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${1:-q4}; mkdir -p $OUT; export TMPDIR=/tmp
bash scripts/gpu_ab_r02.sh ${1:-q4} noq4 base || exit $?
timeout -k 10 420 python3 -u -m pytest tests -m gpu -rA -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
echo "pytest rc=$?"; tail -3 $OUT/pytest.log
exit 0
