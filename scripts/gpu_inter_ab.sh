#!/bin/bash
# Interactive-cadence A/B: bench.py (batched + one frame per synchronous call)
# per variant, then the kernel timeline of the default library.
#   bash scripts/gpu_inter_ab.sh <tag> <variant names...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
for C in C2 C3 C5; do
  for v in "$@"; do
    VRHIP_LIB=$PWD/variants/libvrhip_$v.so timeout -k 10 200 python3 bench.py --config $C --steps 10 --no-cpu --no-roof \
      --interactive-frames 30 > $OUT/bench_${C}_$v.log 2>&1 || { echo "bench $C $v failed"; tail -5 $OUT/bench_${C}_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], d['value'], d['interactive']['value'], d['interactive']['ms_per_frame'])" \
      $OUT/bench_${C}_$v.log $C $v
  done
done
bash scripts/gpu_inter.sh $TAG
