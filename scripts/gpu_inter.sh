#!/bin/bash
# Kernel timeline of the interactive cadence (one frame per synchronous
# render() call) for C2 / C3:  bash scripts/gpu_inter.sh <tag>
# then: python3 scripts/trace_timeline.py gpurun_out/inter_<tag>_C2 100
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1
for C in C2 C3; do
  timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/inter_${TAG}_$C -o run -- \
    python3 bench.py --config $C --steps 1 --warmup 1 --no-cpu --no-roof --interactive-frames 30 \
    > gpurun_out/inter_${TAG}_$C.log 2>&1 || exit $?
done
