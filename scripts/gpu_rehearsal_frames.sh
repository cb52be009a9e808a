#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06zf; mkdir -p $O
for spec in ${SPECS:-C3:16:100 C3:32:50 C3:64:25 C2:16:100 C2:64:25}; do
  IFS=: read cfg fr st <<< "$spec"
  timeout -k 10 300 python3 scripts/rank_rehearsal.py $cfg 8 $fr $st > $O/reh_${cfg}_$fr.json 2> $O/reh_${cfg}_$fr.err
  rc=$?; echo "$spec rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/reh_${cfg}_$fr.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$O/reh_${cfg}_$fr.json')); pr=d['per_rank']
m=sum(r['step_ms'] for r in pr)/len(pr)
print('one-gpu %.4f  mean-rank %.4f  max %.4f  ratio(mean*8/one) %.3f  eff %.3f' % (d['one_gpu_step_ms'], m, max(r['step_ms'] for r in pr), m*8/d['one_gpu_step_ms'], d['projected_efficiency']))"
done
