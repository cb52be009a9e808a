#!/usr/bin/env python3
"""Kernel + HIP API timeline of one-frame synchronous calls, from a rocprofv3
--kernel-trace --hip-runtime-trace run (csv): the last `frames` path-kernel
starts, each event in us from its frame's path-kernel start (K: kernel, A: HIP
API call), and per frame the gaps that make up the host turnaround.

  python3 scripts/api_timeline.py gpurun_out/<dir> [frames=3]
"""
import csv
import glob
import os
import sys

d = sys.argv[1]
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 3
kt = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
ap = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0])))
ev = []
for r in kt:
    name = r["Kernel_Name"].split("(")[0]
    short = name.split("::")[-1][:48]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + short, "render_wave_kernel" in name))
for r in ap:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A:" + r["Function"], False))
ev.sort()
starts = [e[0] for e in ev if e[3]]
starts = starts[-(nf + 1):]
t0 = starts[0]
for s, e, name, _ in ev:
    if s < t0 - 60_000 or s > starts[-1] + 5_000:
        continue
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {name}")
print()
for a, b in zip(starts, starts[1:]):
    fin = [e for e in ev if e[2].startswith("K:") and "finish" in e[2] and a < e[0] < b]
    k_end = max((e[1] for e in ev if e[3] and e[0] == a), default=a)
    f_end = fin[-1][1] if fin else k_end
    syncs = [e for e in ev if e[2] == "A:hipStreamSynchronize" and a < e[1] < b]
    s_end = syncs[-1][1] if syncs else f_end
    print(f"frame: path kernel {(k_end - a) / 1e3:.1f} us, finish ends +{(f_end - k_end) / 1e3:.1f}, "
          f"sync returns +{(s_end - f_end) / 1e3:.1f}, next path kernel starts +{(b - s_end) / 1e3:.1f} "
          f"(frame {(b - a) / 1e3:.1f} us)")
