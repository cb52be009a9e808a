#!/bin/bash
# Memory-pipeline / issue counters of the current production kernel, one
# counter group per rocprofv3 pass.  Usage: bash scripts/gpu_mem.sh <tag> [config]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-mem}; CFG=${2:-C2}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
BENCH="bench.py --steps 3 --warmup 1 --no-cpu --no-roof --no-verify --interactive-frames 0 --config $CFG"
i=0
for PMC in "GRBM_GUI_ACTIVE TA_TA_BUSY_sum" "TD_TD_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc$i -o run -- python3 $BENCH > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($PMC) rc=$rc"
  if [ $rc -ne 0 ]; then grep -m3 -i "error" $OUT/pmc$i.log; exit $rc; fi
done
exit 0
