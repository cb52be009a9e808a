#!/bin/bash
# HIP API + kernel traces of synchronous one-frame C2 calls with and without
# the one-frame graph (VRHIP_GRAPH), kernel timing off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-graph}; mkdir -p $O; export TMPDIR=/tmp
for g in 0 1; do
  VRHIP_GRAPH=$g VRHIP_KERNEL_TIMING=0 timeout -k 10 150 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv \
    -d $O/api_g$g -o run -- python3 scripts/inter_probe.py C2 vrenderer_pathtracer_amd/libvrhip.so > $O/api_g$g.log 2>&1
  rc=$?; echo "graph=$g rc=$rc"; tail -2 $O/api_g$g.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
