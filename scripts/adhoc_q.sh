cd $GRAFT_REPO_ROOT
VRHIP_LIB=$PWD/variants/libvrhip_sp1.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread 2>&1 | tail -2 || exit $?
LIBS="variants/libvrhip_sp0.so variants/libvrhip_sp1.so variants/libvrhip_sp1w5.so"
for c in C2 C3 C5; do
timeout -k 10 300 python3 -u scripts/ab.py --cfg $c --frames 4 --steps 2 --interactive 30 $LIBS 2>&1 | grep -v amdgpu.ids || exit $?
done
