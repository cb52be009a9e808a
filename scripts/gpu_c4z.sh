#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-c4z}; mkdir -p $OUT
timeout -k 10 200 python3 -u scripts/c4_probe.py > $OUT/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids $OUT/probe.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 scripts/c4_probe.py > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"
exit 0
