#!/bin/bash
# Memory-pipeline PMC passes of bench.py's render kernel (separate passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-mem}; OUT=gpurun_out/prof_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
BENCH="bench.py --steps 3 --warmup 1 --no-cpu"
i=0
for PMC in "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_TCP_LATENCY_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCP_PENDING_STALL_CYCLES_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum" "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" "TD_TD_BUSY_sum" "TD_TC_STALL_sum" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
           "SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 90 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc$i -o run -- python3 $BENCH > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i rc=$rc"
  if [ $rc -ne 0 ]; then grep -m3 "Could not\|error" $OUT/pmc$i.log; exit $rc; fi
done
