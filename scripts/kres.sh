#!/bin/bash
# VGPRs / spills / scratch of the production path-kernel instantiations in a
# build_variants log (kernel-resource-usage remarks):
#   bash scripts/kres.sh variants/<name>.log
python3 - "$1" <<'PY'
import re, sys
recs, cur = {}, None
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = recs.setdefault(m.group(1), {})
        continue
    m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur is not None and m.group(1) not in cur:
        cur[m.group(1)] = int(m.group(2))
E, INL, SML, SVC, SPA = 2147483648, 8192, 16384, 32768, 65536
C2, C3, C5 = E + 9, E + 232, E + 8
CLS_C, CLS_H = (1 << 30) + 253, (1 << 30) + 252
rows = [("C2 whole frame", "render_wave_kernel", 16, C2, 256), ("C2 one frame", "render_wave_kernel", 16, C2 + INL + SML, 256),
        ("C2 service", "render_service_kernel", 16, C2 + SVC, 256),
        ("C2 small shard", "render_wave_kernel", 16, C2 + SML, 256),
        ("C3 whole frame", "render_wave_kernel", 16, C3, 768), ("C3 shard", "render_wave_kernel", 16, C3, 256),
        ("C3 small shard", "render_wave_kernel", 16, C3 + SML, 256),
        ("C3 one frame", "render_wave_kernel", 16, C3 + INL + SML, 256), ("C3 service", "render_service_kernel", 16, C3 + SVC, 256),
        ("C3 sparse frame", "render_wave_kernel", 16, C3 + SPA, 768), ("C3 sparse service", "render_service_kernel", 16, C3 + SVC + SPA, 256),
        ("C5 whole frame", "render_wave_kernel", 24, C5, 768), ("C5 shard", "render_wave_kernel", 24, C5, 256),
        ("C5 small shard", "render_wave_kernel", 24, C5 + SML, 256),
        ("C5 one frame", "render_wave_kernel", 24, C5 + INL + SML, 256), ("C5 service", "render_service_kernel", 24, C5 + SVC, 256),
        ("C5 sparse frame", "render_wave_kernel", 24, C5 + SPA, 768), ("C5 sparse service", "render_service_kernel", 24, C5 + SVC + SPA, 256),
        ("class Cornell+mesh", "render_wave_kernel", 16, CLS_C, 768), ("class HDRI+mesh", "render_wave_kernel", 16, CLS_H, 768)]
print(f"{'kernel':22s} {'VGPRs':>5s} {'spill':>5s} {'scratch':>7s} {'waves':>5s}")
for lab, k, st, feat, bt in rows:
    name = f"_ZN2vr{len(k)}{k}ILi{st}ELj{feat}ELi{bt}EEEvNS_12RenderParamsE"
    r = recs.get(name)
    if r is None:
        print(f"{lab:22s} (not in this build)")
        continue
    print(f"{lab:22s} {r.get('VGPRs', 0):5d} {r.get('VGPRs Spill', 0):5d} {r.get('ScratchSize [bytes/lane]', 0):7d} "
          f"{r.get('Occupancy [waves/SIMD]', 0):5d}")
PY
