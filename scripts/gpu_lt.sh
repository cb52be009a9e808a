#!/bin/bash
# LDS-resident tree A/B: leaf-4 trees (fit in LDS) with and without the mode, and the leaf-2 global walk.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${1:-lt}; mkdir -p $OUT
for cfg in C2 C3; do
  for leaf in 4 2; do
    timeout -k 10 300 python3 scripts/ab.py --cfg $cfg --frames 16 --leaf $leaf variants/libvrhip_nolt.so variants/libvrhip_base.so > $OUT/ab_${cfg}_$leaf.log 2>&1
    rc=$?; echo "== $cfg leaf $leaf rc=$rc"; cat $OUT/ab_${cfg}_$leaf.log; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
