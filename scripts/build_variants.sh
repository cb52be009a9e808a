#!/bin/bash
# Build libvrhip.so variants for scripts/ab.py: each argument is NAME=FLAGS,
# e.g.  bash scripts/build_variants.sh base= w5="-DVR_PATH_BLOCK=256 -DVR_PATH_WAVES=5"
# Prints VGPRs / spills of the C2 specialisation (render_kernel<16,false,9>).
set -e
cd "$(dirname "$0")/.."
mkdir -p variants
SRC="vrenderer_pathtracer_amd/csrc/vr_kernel.hip vrenderer_pathtracer_amd/csrc/vrhip_api.cpp vrenderer_pathtracer_amd/csrc/vr_bvh.cpp vrenderer_pathtracer_amd/csrc/vr_exr.cpp -lz -lrccl"
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  ( rm -f variants/libvrhip_$name.so
    hipcc -O3 -std=c++17 -ffp-contract=off -fPIC -shared -pthread --offload-arch=gfx950 -Xclang -target-feature -Xclang -packed-fp32-ops $flags \
      -o variants/libvrhip_$name.so $SRC -Rpass-analysis=kernel-resource-usage > variants/$name.log 2>&1
    grep -E -A12 "render_wave_kernelILi16ELj2147483657ELi[0-9]+E" variants/$name.log | grep -E "VGPRs:|VGPRs Spill|Scratch" \
      | sed 's/.*remark: *//;s/ \[-Rpass.*//' | tr '\n' ' ' | sed "s/^/$name: /"; echo
    [ -f variants/libvrhip_$name.so ] || { grep -m5 error: variants/$name.log; echo "$name: BUILD FAILED"; } ) &
done
wait
