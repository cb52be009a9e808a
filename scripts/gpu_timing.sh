#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in C2 C3 C5; do
  VRHIP_LIB=variants/libvrhip_timing.so timeout -k 10 300 python3 scripts/phase_timing.py $c 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/timing.log || exit $?
done
