#!/bin/bash
# bench.py lines for the other BASELINE configurations (C3, C5) on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/configs
for cfg in C3 C5; do
  timeout -k 10 400 python3 bench.py --config $cfg --no-cpu > gpurun_out/configs/bench_$cfg.log 2>&1 || exit $?
  grep '^{' gpurun_out/configs/bench_$cfg.log
done
