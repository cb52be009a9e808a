set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 480 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_rehearsal.sh r06k
