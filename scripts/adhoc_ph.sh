cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ph2
for a in "C2 1 16 16" "C2 1 160 96" "C3 1 16 16" "C3 1 160 96" "C2 1" "C3 1"; do
  VRHIP_LIB=$PWD/variants/libvrhip_ph.so timeout -k 10 120 python3 -u scripts/wave_phases.py $a 2>&1 | grep -v amdgpu.ids || exit $?
done | tee gpurun_out/ph2/phases.log
