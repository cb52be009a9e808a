#!/bin/bash
# A/B of library builds at the interactive cadence (one frame per synchronous
# call, scripts/ab.py --interactive) plus 16-frame steps:
#   bash scripts/gpu_abi.sh <tag> "<configs>" lib.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; CFGS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for cfg in $CFGS; do
  timeout -k 10 400 python3 -u scripts/ab.py --cfg $cfg --frames 16 --steps 4 --interactive 40 "$@" "$@" > $OUT/abi_$cfg.log 2>&1 || exit $?
  echo "== $cfg"; grep -v amdgpu.ids $OUT/abi_$cfg.log | tail -$((2 * $# + 1))
done
