#!/usr/bin/env python3
"""Summarise scripts/profile_mem.sh passes (one counter group per pass) for
the bench's render kernel into profiles/<name>_mem.md.

  python scripts/summarize_mem.py gpurun_out/prof_<tag> <name>
"""
import csv
import re
import glob
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, name = sys.argv[1], sys.argv[2]
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if re.search(r"render_(wave_|block_)?kernel", k) and "true" not in k:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in vals.items()}
    cus = 256
    lines = [f"# Memory-pipeline counters, {name}", "",
             "Source: `scripts/profile_mem.sh` (one counter group per rocprofv3 pass) on bench.py's C2 step; "
             "per-dispatch means of the render kernel.", "", "| counter | per dispatch |", "|---|---|"]
    lines += [f"| {k} | {v:.4g} |" for k, v in sorted(m.items())]
    g = m.get("GRBM_GUI_ACTIVE")
    if g:
        g = g / 8.0      # GRBM_GUI_ACTIVE sums the 8 XCDs (checked against the kernel's duration)
        lines += ["", "Derived (per CU, over the kernel's cycles = GRBM_GUI_ACTIVE / 8 XCDs):", ""]
        for k, label in (("TA_TA_BUSY_sum", "TA busy"), ("TD_TD_BUSY_sum", "TD busy"),
                         ("TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA address stalled by TC"),
                         ("TA_DATA_STALLED_BY_TC_CYCLES_sum", "TA data stalled by TC"),
                         ("TCP_PENDING_STALL_CYCLES_sum", "TCP pending stall"),
                         ("TD_TC_STALL_sum", "TD stalled by TC")):
            if k in m:
                lines.append(f"- {label}: {m[k] / (cus * g):.3f}")
        if "TCP_TCC_READ_REQ_LATENCY_sum" in m and m.get("TCP_TCC_READ_REQ_sum"):
            lines.append(f"- mean TCP->TCC read latency: {m['TCP_TCC_READ_REQ_LATENCY_sum'] / m['TCP_TCC_READ_REQ_sum']:.0f} cycles")
        if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
            lines.append(f"- wave time waiting: {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_THREAD_CYCLES_VALU" in m and "SQ_ACTIVE_INST_VALU" in m:
            lines.append(f"- VALU lane utilisation: {m['SQ_THREAD_CYCLES_VALU'] / (64 * m['SQ_ACTIVE_INST_VALU']):.3f}")
        if "SQ_ACTIVE_INST_VALU" in m:
            lines.append(f"- VALU issue busy per SIMD: {m['SQ_ACTIVE_INST_VALU'] * 4 / (cus * 4 * g):.3f} "
                         "(SQ_ACTIVE_INST_VALU x 4 cycles / (4 SIMDs x CUs x cycles))")
        if "SQ_INSTS_VALU" in m and "SQ_INSTS_VMEM_RD" in m:
            lines.append(f"- VALU instructions per VMEM read: {m['SQ_INSTS_VALU'] / m['SQ_INSTS_VMEM_RD']:.1f}")
    out = os.path.join(REPO, "profiles", f"{name}_mem.md")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
