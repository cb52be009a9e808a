#!/bin/bash
# A/B of the in-tree library against variants/libvrhip_cw7.so, then the full
# GPU pass (scripts/gpu_r02.sh) with cw7 installed in-tree on the box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_ab_r02.sh ab_cw7 base cw7 || exit $?
cp variants/libvrhip_cw7.so vrenderer_pathtracer_amd/libvrhip.so && bash scripts/gpu_r02.sh ${1:-r02g}
