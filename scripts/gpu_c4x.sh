#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-c4x}; shift
mkdir -p $OUT
timeout -k 10 240 python3 scripts/ab.py --cfg C4 --frames 16 --steps 8 vrenderer_pathtracer_amd/libvrhip.so "$@" > $OUT/ab_C4.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab_C4.log | tail -4
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_C4 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-roof --interactive-frames 0 --strong-steps 0 --config C4 > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; cut -d, -f1-4 $OUT/trace_C4/run_kernel_stats.csv | head -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -u scripts/class_probe.py vrenderer_pathtracer_amd/libvrhip.so variants/libvrhip_head.so > $OUT/class_probe.log 2>&1
rc=$?; echo "class_probe rc=$rc"; grep -v amdgpu.ids $OUT/class_probe.log
exit 0
