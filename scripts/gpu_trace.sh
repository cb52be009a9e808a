#!/bin/bash
# Kernel timeline (rocprofv3 --kernel-trace) of back-to-back render steps:
#   bash scripts/gpu_trace.sh <tag> <tile_scaling.py args...>   e.g.  c3n8 C3 16 0 8
# then: python3 scripts/trace_timeline.py gpurun_out/trace_<tag>
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$TAG -o run -- python3 scripts/tile_scaling.py "$@" > gpurun_out/trace_$TAG.log 2>&1
