#!/bin/bash
# 8-rank projections of C2..C5 rehearsed on one GPU (scripts/rank_rehearsal.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/${1:-rehearsal}; mkdir -p $O
for cfg in C2 C3 C4 C5; do
  timeout -k 10 300 python3 scripts/rank_rehearsal.py $cfg 8 16 100 > $O/rehearsal_$cfg.json 2> $O/rehearsal_$cfg.err
  rc=$?; echo "$cfg rc=$rc"; tail -c 600 $O/rehearsal_$cfg.json
  [ $rc -ne 0 ] && { tail -5 $O/rehearsal_$cfg.err; exit $rc; }
done
exit 0
