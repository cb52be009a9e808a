#!/bin/bash
# A/B timing of abl/ variants: bash scripts/gpu_ab.sh <tag> "<cfg:frames:inter> ..." lib...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; TAG=$1; shift; CFGS=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for spec in $CFGS; do
  IFS=: read cfg fr it <<< "$spec"
  timeout -k 10 400 python3 scripts/ab.py --cfg $cfg --frames $fr --steps 10 --interactive $it "$@" > $O/ab_$cfg.txt 2>&1
  rc=$?; echo "== $cfg rc=$rc"; cat $O/ab_$cfg.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
