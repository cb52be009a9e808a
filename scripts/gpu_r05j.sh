#!/bin/bash
# C2 whole frames on the render service (VRHIP_SERVICE=1): the production
# service kernel (6 waves) and the 7-wave Cornell residency variant, against
# the production launch path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r05j; mkdir -p $OUT
P=vrenderer_pathtracer_amd/libvrhip.so; V=variants/libvrhip_svc7.so
timeout -k 10 300 python3 -u scripts/ab.py --cfg C2 --frames 16 --steps 6 $P $P > $OUT/ab_launch.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/ab_launch.log | tail -3
VRHIP_SERVICE=1 timeout -k 10 300 python3 -u scripts/ab.py --cfg C2 --frames 16 --steps 6 $P $V $P $V > $OUT/ab_svc.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/ab_svc.log | tail -5
