#!/bin/bash
# r05b: wide-node line-cost micro-benchmark, the new service tests, and the
# 5-wave service kernels (0 VGPR spills) against production on C3 / C5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r05b; mkdir -p $OUT
timeout -k 10 120 ./scripts/micro/node_wide.bin > $OUT/node_wide.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_service.py -x -v --timeout 200 --timeout-method thread > $OUT/svc_tests.log 2>&1; echo "svc tests rc=$?"; tail -3 $OUT/svc_tests.log
for cfg in C3 C5; do
  timeout -k 10 300 python3 -u scripts/ab.py --cfg $cfg --frames 16 --steps 6 vrenderer_pathtracer_amd/libvrhip.so variants/libvrhip_svc5.so vrenderer_pathtracer_amd/libvrhip.so variants/libvrhip_svc5.so > $OUT/ab_$cfg.log 2>&1 || exit $?
  grep -v amdgpu.ids $OUT/ab_$cfg.log | tail -6
done
cat $OUT/node_wide.log
