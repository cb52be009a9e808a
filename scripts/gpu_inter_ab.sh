#!/bin/bash
# One-frame-per-call A/B (kernel timing off, as the Qt adapter): bash scripts/gpu_inter_ab.sh <tag> "<cfgs>" lib...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=$1; shift; CFGS=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for cfg in $CFGS; do
  args=(); for l in "$@"; do args+=("$l@VRHIP_KERNEL_TIMING=0"); done
  timeout -k 10 400 python3 scripts/ab.py --cfg $cfg --frames 16 --steps 3 --interactive 60 "${args[@]}" > $O/inter_$cfg.txt 2>&1
  rc=$?; echo "== $cfg rc=$rc"; cat $O/inter_$cfg.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
