#!/bin/bash
# 8-rank rehearsal of one config with several library builds (VRHIP_LIB):
# bash scripts/gpu_rehearsal_ab.sh <tag> "<cfgs>" lib...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; shift; CFGS=$1; shift; mkdir -p $O
for cfg in $CFGS; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    VRHIP_LIB=$lib timeout -k 10 300 python3 scripts/rank_rehearsal.py $cfg 8 16 100 > $O/reh_${cfg}_$n.json 2> $O/reh_${cfg}_$n.err
    rc=$?; echo "$cfg $n rc=$rc"
    [ $rc -ne 0 ] && { tail -5 $O/reh_${cfg}_$n.err; exit $rc; }
    python3 -c "
import json,sys; d=json.load(open('$O/reh_${cfg}_$n.json'))
print(' '.join('%.4f' % r['step_ms'] for r in d['per_rank']), 'max %.4f' % max(r['step_ms'] for r in d['per_rank']), 'eff %.4f' % d['projected_efficiency'])"
  done
done
exit 0
