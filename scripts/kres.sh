#!/bin/bash
# VGPRs / spills of the production path-kernel specialisations in a
# build_variants log:  bash scripts/kres.sh variants/<name>.log
for k in "16ELj2147483657ELi256:C2-16f" "16ELj2147508233ELi256:C2-1f" "16ELj2147500041ELi256:C2-shard" \
         "16ELj2147483880ELi768:C3-16f" "16ELj2147508456ELi256:C3-1f" "16ELj2147500264ELi256:C3-shard" \
         "24ELj2147483656ELi768:C5-16f" "24ELj2147500040ELi256:C5-shard"; do
  n=${k%%:*}; lab=${k#*:}
  echo "$lab: $(grep -A14 "render_wave_kernelILi${n}EEEvNS_12RenderParamsE" $1 | grep -E "VGPRs:|VGPRs Spill|SGPRs Spill|ScratchSize" | sed 's/.*remark: *//;s/ \[-Rpass.*//' | tr '\n' ' ')"
done
