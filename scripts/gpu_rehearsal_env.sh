#!/bin/bash
# One config's 8-rank rehearsal under several library environment settings:
# bash scripts/gpu_rehearsal_env.sh <tag> <cfg> "ENV=V ENV2=V" ...   (- for none)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/$1; CFG=$2; shift 2; mkdir -p $O
i=0
for envs in "$@"; do
  i=$((i+1))
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 300 python3 scripts/rank_rehearsal.py $CFG 8 16 100 > $O/reh_${CFG}_$i.json 2> $O/reh_${CFG}_$i.err
  rc=$?; echo "[$envs] rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/reh_${CFG}_$i.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('$O/reh_${CFG}_$i.json')); pr=d['per_rank']
m=sum(r['step_ms'] for r in pr)/len(pr)
print('  one-gpu %.4f  mean-rank %.4f  max %.4f  ratio %.3f  eff %.3f' % (d['one_gpu_step_ms'], m, max(r['step_ms'] for r in pr), m*8/d['one_gpu_step_ms'], d['projected_efficiency']))"
done
