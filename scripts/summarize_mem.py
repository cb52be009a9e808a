#!/usr/bin/env python3
"""Summarise scripts/gpu_mem.sh passes into profiles/<name>_mem.md.

  python scripts/summarize_mem.py gpurun_out/<tag> <name> <config> [paths_per_launch]

Counters are means over the TIMED dispatches (the last 3 of bench.py
--steps 3) of the production render kernel (render_wave_kernel, or
render_kernel for sphere-only scenes, specialised on the scene's features;
the untimed counting kernels and primary_kernel are excluded).  Derived figures (per CU, over the kernel's cycles):
  * kernel cycles = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs);
  * TA / TD busy = TA_TA_BUSY_sum / TD_TD_BUSY_sum over 256 CUs x cycles;
  * VALU pipe busy per SIMD = SQ_INSTS_VALU x 2 cycles (a wave64 VALU
    instruction issues over 2 cycles, MI355X_MICROARCH.md "CU") over
    4 SIMDs x 256 CUs x cycles -- round 1 multiplied SQ_ACTIVE_INST_VALU
    (quad-cycles of every wave's VALU residency, overlapping across waves)
    by 4 and got 1.085, which is not a utilisation;
  * wave time waiting = SQ_WAIT_ANY / SQ_WAVE_CYCLES (both quad-cycles).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TIMED = 3
CUS = 256


def production_wave(name):
    """The scene's production render kernel: render_wave_kernel or the
    render-service kernel (mesh scenes; bench.py's timed steps of C2 / C3 /
    C5 run in one service dispatch, r05) or render_kernel<16, false, ...>
    (sphere-only scenes) specialised on the scene's exact feature set
    (F_EXACT, bit 31), not the counting copies."""
    m = re.search(r"vr::render_service_kernel<([^>]*)>", name)
    if m:
        args = [a.strip() for a in m.group(1).split(",")]
        return int(args[1].rstrip("u")) >= 2 ** 31
    m = re.search(r"vr::render_wave_kernel<([^>]*)>", name)
    if m:
        args = [a.strip() for a in m.group(1).split(",")]
        feat = int(args[1].rstrip("u"))
        return feat >= 2 ** 31 and not (feat & (1 << 10))
    m = re.search(r"vr::render_kernel<([^>]*)>", name)
    if m:
        args = [a.strip() for a in m.group(1).split(",")]
        feat = int(args[2].rstrip("u"))
        return args[1] == "false" and feat >= 2 ** 31
    return False


def main():
    src, name, cfg = sys.argv[1], sys.argv[2], sys.argv[3]
    paths = int(sys.argv[4]) if len(sys.argv) > 4 else None
    per = defaultdict(list)
    kernels = set()
    files = glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv")) + \
        glob.glob(os.path.join(src, "valu*", "*counter_collection.csv"))      # scripts/gpu_valu.sh passes
    for f in sorted(files):
        for r in csv.DictReader(open(f)):
            if production_wave(r["Kernel_Name"]):
                kernels.add(r["Kernel_Name"].split("(")[0])
                per[r["Counter_Name"]].append((int(r["Start_Timestamp"]), float(r["Counter_Value"]),
                                               int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                               "render_service_kernel" in r["Kernel_Name"]))
    m, dur = {}, {}
    svc = any("render_service_kernel" in k for k in kernels)
    for k, v in per.items():
        v.sort()
        # a service run: its timed steps are the FIRST service dispatch (one
        # session; the warmup step before it ran on the launch path, and
        # bench.py's self-check after the timed loop renders one more session
        # and launch-path steps)
        if svc:
            t = [x for x in v if x[3]][:1]
        else:
            t = [x for x in v if not x[3]][:TIMED + 1][-TIMED:]   # (warmup first, then the timed steps)
        m[k] = sum(x[1] for x in t) / len(t)
        dur[k] = sum(x[2] for x in t) / len(t)
    lines = [f"# Issue and memory-pipeline counters, {name} ({cfg})", "",
             f"Source: `scripts/gpu_mem.sh` (one counter group per rocprofv3 pass) on `bench.py --config {cfg}`; "
             f"means over the {TIMED} timed dispatches of the production kernel "
             + ", ".join(f"`{k}`" for k in sorted(kernels)) + ".", "",
             "| counter | per dispatch |", "|---|---|"]
    lines += [f"| {k} | {v:.4g} |" for k, v in sorted(m.items())]
    g = m.get("GRBM_GUI_ACTIVE")
    if g:
        cyc = g / 8.0
        ns = dur.get("GRBM_GUI_ACTIVE", 0)
        lines += ["", f"Kernel cycles (GRBM_GUI_ACTIVE / 8) = {cyc:.4g}"
                  + (f" over {ns / 1e6:.3f} ms (profiled dispatch) = {cyc / ns:.2f} GHz" if ns else ""), "",
                  "Derived (per CU, over the kernel's cycles):", ""]
        for k, label in (("TA_TA_BUSY_sum", "TA busy"), ("TD_TD_BUSY_sum", "TD busy"),
                         ("TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA address stalled by TC"),
                         ("TCP_PENDING_STALL_CYCLES_sum", "TCP pending stall"),
                         ("TD_TC_STALL_sum", "TD stalled by TC")):
            if k in m:
                lines.append(f"- {label}: {m[k] / (CUS * cyc):.3f}")
        if "SQ_INSTS_VALU" in m:
            lines.append(f"- VALU pipe busy per SIMD: {m['SQ_INSTS_VALU'] * 2 / (4 * CUS * cyc):.3f} "
                         "(SQ_INSTS_VALU x 2 cycles / (4 SIMDs x 256 CUs x cycles))")
        if "SQ_INSTS_SALU" in m:
            lines.append(f"- SALU instructions per SIMD-cycle: {m['SQ_INSTS_SALU'] / (4 * CUS * cyc):.3f}")
    if "TCP_TCC_READ_REQ_LATENCY_sum" in m and m.get("TCP_TCC_READ_REQ_sum"):
        lines.append(f"- mean TCP->TCC read latency: {m['TCP_TCC_READ_REQ_LATENCY_sum'] / m['TCP_TCC_READ_REQ_sum']:.0f} cycles")
    if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None:
        lines.append(f"- L2 hit rate: {m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.4f}")
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in m and m.get("TCP_TCC_READ_REQ_sum"):
        lines.append(f"- L1 (TCP) accesses per L2 read request: {m['TCP_TOTAL_CACHE_ACCESSES_sum'] / m['TCP_TCC_READ_REQ_sum']:.2f}")
    if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
        lines.append(f"- wave time waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES): {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
    if "SQ_THREAD_CYCLES_VALU" in m and "SQ_ACTIVE_INST_VALU" in m:
        lines.append(f"- VALU lane utilisation (SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)): "
                     f"{m['SQ_THREAD_CYCLES_VALU'] / (64 * m['SQ_ACTIVE_INST_VALU']):.3f}")
    if "SQ_INSTS_VALU" in m and "SQ_INSTS_VMEM_RD" in m:
        lines.append(f"- VALU instructions per VMEM read instruction: {m['SQ_INSTS_VALU'] / m['SQ_INSTS_VMEM_RD']:.1f}")
    if paths:
        for k, label in (("SQ_INSTS_VMEM_RD", "VMEM read"), ("SQ_INSTS_VALU", "VALU"), ("SQ_INSTS_SALU", "SALU"),
                         ("SQ_INSTS_LDS", "LDS"), ("SQ_INSTS_BRANCH", "branch")):
            if k in m:
                lines.append(f"- {label} wave-instructions per path: {m[k] / paths:.2f}")
    out = os.path.join(REPO, "profiles", f"{name}_mem.md")
    open(out, "w").write("\n".join(lines) + "\n")
    f64 = sum(m.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                        "SQ_INSTS_VALU_TRANS_F64"))
    if f64 and m.get("SQ_INSTS_VALU"):
        lines.append(f"- F64 VALU instructions (FMA + MUL + ADD + TRANS): {f64 / m['SQ_INSTS_VALU']:.3f} of all VALU")
        for k in ("SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_TRANS_F32",
                  "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT"):
            if k in m:
                lines.append(f"- {k[14:]}: {m[k] / m['SQ_INSTS_VALU']:.3f} of all VALU")
        if "SQ_INST_CYCLES_VALU" in m:
            lines.append(f"- VALU issue cycles per VALU instruction (SQ_INST_CYCLES_VALU / SQ_INSTS_VALU): "
                         f"{m['SQ_INST_CYCLES_VALU'] / m['SQ_INSTS_VALU']:.2f}")
    if g and "TD_TD_BUSY_sum" in m:   # unit busy fractions for bench.py's roofline.unit_busy
        cyc = g / 8.0
        units = {"source": os.path.relpath(out, REPO)}
        for k, key in (("TD_TD_BUSY_sum", "td"), ("TA_TA_BUSY_sum", "ta")):
            if k in m:
                units[key] = round(m[k] / (CUS * cyc), 4)
        if "SQ_INSTS_VALU" in m:
            units["valu"] = round(m["SQ_INSTS_VALU"] * 2 / (4 * CUS * cyc), 4)
        if "SQ_THREAD_CYCLES_VALU" in m and m.get("SQ_ACTIVE_INST_VALU"):
            units["valu_lane_util"] = round(m["SQ_THREAD_CYCLES_VALU"] / (64 * m["SQ_ACTIVE_INST_VALU"]), 4)
        units["kernels"] = sorted(kernels)
        json.dump(units, open(os.path.join(REPO, "profiles", f"units_{cfg.lower()}.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
