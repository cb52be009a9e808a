set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest.log
timeout -k 10 300 python3 scripts/ab.py --cfg C2 --frames 16 --steps 10 --interactive 30 abl/libvrhip_off.so abl/libvrhip_skip.so abl/libvrhip_on.so > $O/ab_C2.txt 2>&1; echo "ab rc=$?"; cat $O/ab_C2.txt
timeout -k 10 200 python3 scripts/ab.py --cfg C2D --frames 16 --steps 10 abl/libvrhip_off.so abl/libvrhip_on.so > $O/ab_C2D.txt 2>&1; cat $O/ab_C2D.txt
