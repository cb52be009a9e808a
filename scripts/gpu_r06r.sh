set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_service.py -x -v --timeout 200 --timeout-method thread -k "shortage or deferred_gather or session_limits" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -8
exit $rc
