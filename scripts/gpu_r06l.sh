set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06l; mkdir -p $O
for cfg in C3 C2; do
  for lib in abl/libvrhip_s32.so vrenderer_pathtracer_amd/libvrhip.so; do
    VRHIP_LIB=$lib timeout -k 10 300 python3 scripts/rank_rehearsal.py $cfg 8 16 100 > $O/reh_${cfg}_$(basename $lib .so).json 2>$O/err.txt; rc=$?
    echo "$cfg $lib rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/err.txt; exit $rc; }
    python3 -c "import json;d=json.load(open('$O/reh_${cfg}_$(basename $lib .so).json'));print(d['one_gpu_mpaths'], max(x['step_ms'] for x in d['per_rank']), d['projected_efficiency'], d['efficiency_without_gather'])"
  done
done
timeout -k 10 300 python3 scripts/ab.py --cfg C2 --frames 16 --steps 40 abl/libvrhip_s32.so vrenderer_pathtracer_amd/libvrhip.so > $O/ab_C2.txt 2>&1; cat $O/ab_C2.txt
