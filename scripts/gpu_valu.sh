#!/bin/bash
# VALU instruction mix of the production kernel (one counter group per
# rocprofv3 pass).  Usage: bash scripts/gpu_valu.sh <tag> [config]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-valu}; CFG=${2:-C2}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
BENCH="bench.py --steps 3 --warmup 1 --no-cpu --no-roof --no-verify --interactive-frames 0 --strong-steps 0 --config $CFG"
i=0
for PMC in "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32" \
           "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INST_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $PMC --output-format csv -d $OUT/valu$i -o run -- python3 $BENCH > $OUT/valu$i.log 2>&1
  rc=$?; echo "valu$i ($PMC) rc=$rc"
  if [ $rc -ne 0 ]; then grep -m3 -i "error" $OUT/valu$i.log; exit $rc; fi
done
exit 0
