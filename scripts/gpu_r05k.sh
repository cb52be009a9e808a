#!/bin/bash
# dk (polynomial constants produced at each use, single refill start in the
# service kernel) and sv7 (the same + 7-wave Cornell service kernel) against
# production: C2 on the launch path and on the service, C3, C5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r05k; mkdir -p $OUT
P=variants/libvrhip_prod.so; D=variants/libvrhip_dk.so; S=variants/libvrhip_sv7.so
timeout -k 10 300 python3 -u scripts/ab.py --cfg C2 --frames 16 --steps 6 $P $D $P $D > $OUT/ab_C2.log 2>&1 || exit $?
echo "== C2 launch path"; grep -v amdgpu.ids $OUT/ab_C2.log | tail -5
VRHIP_SERVICE=1 timeout -k 10 300 python3 -u scripts/ab.py --cfg C2 --frames 16 --steps 6 $D $S $D $S > $OUT/ab_C2svc.log 2>&1 || exit $?
echo "== C2 service"; grep -v amdgpu.ids $OUT/ab_C2svc.log | tail -5
for cfg in C3 C5; do
  timeout -k 10 300 python3 -u scripts/ab.py --cfg $cfg --frames 16 --steps 6 $P $D $P $D > $OUT/ab_$cfg.log 2>&1 || exit $?
  echo "== $cfg"; grep -v amdgpu.ids $OUT/ab_$cfg.log | tail -5
done
