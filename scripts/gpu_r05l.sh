#!/bin/bash
# r05l: tests, smoke, bench C2/C3/C5, C2D service vs launch path, C2 fixed-
# cadence projection on the 7-wave Cornell service.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash scripts/gpu_quick.sh r05l C2 C3 C5 || exit $?
OUT=gpurun_out/r05l
timeout -k 10 300 python3 -u scripts/ab.py --cfg C2D --frames 16 --steps 6 variants/libvrhip_nocf.so vrenderer_pathtracer_amd/libvrhip.so variants/libvrhip_nocf.so vrenderer_pathtracer_amd/libvrhip.so > $OUT/ab_C2D.log 2>&1 || exit $?
echo "== C2D"; grep -v amdgpu.ids $OUT/ab_C2D.log | tail -5
timeout -k 10 300 python3 -u scripts/tile_scaling.py C2 16 0 1,2,4,8 > $OUT/ts_C2.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/ts_C2.log
