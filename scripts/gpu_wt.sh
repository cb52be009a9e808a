#!/bin/bash
# Drain diagnostics of the path kernel: per-wave timelines (scripts/wave_times.py)
# and per-path records (scripts/path_times.py) of a -DVR_WAVE_TIMES -DVR_PATH_TIMES
# build (scripts/build_variants.sh pt="-DVR_WAVE_TIMES -DVR_PATH_TIMES -DVR_PATH_COUNTS"; ptl: the same without -DVR_PATH_COUNTS, fewer registers).
#   bash scripts/gpu_wt.sh <variant> "C2 1;C3 1"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=${1:-pt}; RUNS=${2:-"C2 1;C3 1"}
IFS=';' read -ra R <<< "$RUNS"
for a in "${R[@]}"; do
  VRHIP_LIB=$PWD/variants/libvrhip_$V.so timeout -k 10 120 python3 -u scripts/path_times.py $a 2>&1 | grep -v amdgpu.ids || exit $?
done | tee gpurun_out/wt_$V.log
