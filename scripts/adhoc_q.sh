cd $GRAFT_REPO_ROOT
LIBS="variants/libvrhip_base.so variants/libvrhip_q5.so variants/libvrhip_q7.so variants/libvrhip_q7b.so"
VRHIP_LIB=$PWD/variants/libvrhip_q7b.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread 2>&1 | tail -1 || exit $?
bash scripts/gpu_libs.sh qscan7 C2,C3 160x96,1280x720 $LIBS || exit $?
for lib in $LIBS; do
  for c in C2 C3 C5; do
    VRHIP_LIB=$PWD/$lib timeout -k 10 120 python3 -u scripts/tile_scaling.py $c 16 0 8 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $lib) |" || exit $?
  done
done
bash scripts/gpu_tl.sh tl2 "C3 16 8" variants/libvrhip_q7b.so
