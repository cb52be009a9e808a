#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r04c; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_C4 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-roof --interactive-frames 0 --strong-steps 0 --config C4 > $OUT/trace_C4.log 2>&1
rc=$?; echo "trace rc=$rc"; cut -d, -f1-4 $OUT/trace_C4/run_kernel_stats.csv | head -8
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_mem_lib.sh r04c/mem_prod C2 vrenderer_pathtracer_amd/libvrhip.so || exit $?
bash scripts/gpu_mem_lib.sh r04c/mem_pc1 C2 variants/libvrhip_pc1.so || exit $?
bash scripts/gpu_mem_lib.sh r04c/mem_pc4 C2 variants/libvrhip_pc4.so || exit $?
exit 0
