set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_service.py -x -q --timeout 200 --timeout-method thread -k "graph" > $O/pytest_graph.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_graph.log
[ $rc -ne 0 ] && exit $rc
L=vrenderer_pathtracer_amd/libvrhip.so
for cfg in C2 C3; do
timeout -k 10 300 python3 scripts/ab.py --cfg $cfg --frames 16 --steps 3 --interactive 60 $L@VRHIP_KERNEL_TIMING=0,VRHIP_GRAPH=0 $L@VRHIP_KERNEL_TIMING=0,VRHIP_GRAPH=1 $L@VRHIP_KERNEL_TIMING=0,VRHIP_GRAPH=0 $L@VRHIP_KERNEL_TIMING=0,VRHIP_GRAPH=1 > $O/ab_$cfg.txt 2>&1; echo "ab $cfg rc=$?"; cat $O/ab_$cfg.txt
done
