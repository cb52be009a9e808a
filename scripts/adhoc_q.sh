cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit $?
for c in C2 C3 C5; do
  timeout -k 10 300 python3 -u scripts/ab.py --cfg $c --frames 4 --steps 2 --interactive 30 variants/libvrhip_head.so vrenderer_pathtracer_amd/libvrhip.so 2>&1 | grep -v amdgpu.ids || exit $?
done
