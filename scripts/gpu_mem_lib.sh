#!/bin/bash
# TD / TA busy and VALU counters of one library build (VRHIP_LIB) on one
# config: passes 1, 2 and 7 of scripts/gpu_mem.sh (summarize_mem.py reads them).
#   bash scripts/gpu_mem_lib.sh <tag> <config> <lib.so>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; CFG=$2; export VRHIP_LIB=$(readlink -f $3); OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
BENCH="bench.py --steps 3 --warmup 1 --no-cpu --no-roof --interactive-frames 0 --strong-steps 0 --config $CFG"
i=0
for PMC in "GRBM_GUI_ACTIVE TA_TA_BUSY_sum" "TD_TD_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1)); n=$i; [ $i -eq 3 ] && n=7
  timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc$n -o run -- python3 $BENCH > $OUT/pmc$n.log 2>&1
  rc=$?; echo "pmc$n ($PMC) rc=$rc"
  if [ $rc -ne 0 ]; then grep -m3 -i "error" $OUT/pmc$n.log; exit $rc; fi
done
exit 0
