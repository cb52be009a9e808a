#!/bin/bash
# TA/TD/SQ counters of bench.py's render kernel for two library builds.
#   bash scripts/profile_pair.sh tag variants/libA.so variants/libB.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift
for LIB in "$@"; do
  N=$(basename $LIB .so)
  OUT=gpurun_out/pair_$TAG/$N; mkdir -p $OUT
  i=0
  for PMC in "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TD_TD_BUSY_sum" "TD_TC_STALL_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY" "TCP_TOTAL_CACHE_ACCESSES_sum" "TCP_TCC_READ_REQ_sum"; do
    i=$((i+1))
    VRHIP_LIB=$LIB timeout -k 10 90 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/pmc$i.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$N pmc$i rc=$rc"; exit $rc; fi
  done
  echo "$N done"
done
