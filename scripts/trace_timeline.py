#!/usr/bin/env python3
"""Print the last kernels of a rocprofv3 --kernel-trace csv as a timeline (us
from the first kernel), to see whether consecutive render launches overlap.

  python3 scripts/trace_timeline.py gpurun_out/trace_<tag> [n_last]
"""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
path = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    name = r["Kernel_Name"].split("(")[0][-32:]
    print(f'{name:32s} queue {r.get("Queue_Id", "?"):>3s}  start {s / 1e3:10.1f}  end {e / 1e3:10.1f}  dur {(e - s) / 1e3:8.1f} us')
