#!/bin/bash
# Per-wave timelines (scripts/wave_times.py) of VR_WAVE_TIMES builds: bash scripts/gpu_wt.sh "wt wtnd" "C3 16 8;C2 16 8"
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
VARS=${1:-wt}; RUNS=${2:-"C3 16 8;C2 16 8"}
IFS=';' read -ra R <<< "$RUNS"
for v in $VARS; do
  for a in "${R[@]}"; do
    VRHIP_LIB=$PWD/variants/libvrhip_$v.so timeout -k 10 120 python3 scripts/wave_times.py $a 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit $?
  done
done | tee gpurun_out/wt.log
