#!/usr/bin/env python3
"""Summarise a gpu_round.sh output directory into profiles/.

  python scripts/summarize_prof.py gpurun_out/round_<tag> <round-name>

Writes profiles/<round-name>_kernel_stats.csv (rocprofv3 --kernel-trace
--stats), profiles/<round-name>_pmc.json (per-dispatch PMC averages of the
render kernel), profiles/traffic_c2.json (HBM bytes per render launch, which
bench.py reports as roofline.traffic) and profiles/<round-name>_summary.md.

HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of a wide coalesced stream,
so the read side is doubled (an upper bound for this gather pattern, whose
calibration is unmeasured -- noted in the summary).
"""
import csv
import re
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = r"render_(wave_|block_)?kernel|primary_kernel"   # one render launch = primary_kernel + render_wave_kernel


def pmc_means(d):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if re.search(KERNELS, row["Kernel_Name"]) and "true" not in row["Kernel_Name"]:
                vals[(row["Kernel_Name"], row["Counter_Name"])].append(float(row["Counter_Value"]))
    return {f"{k[0]}|{k[1]}": sum(v) / len(v) for k, v in vals.items()}


def main():
    src, name = sys.argv[1], sys.argv[2]
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(src, "prof_trace", "*kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats[0]))) if stats else []
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{name}_kernel_stats.csv"))
    pmc = {}
    for sub in ("prof_fetch", "prof_write", "prof_sq"):
        pmc.update(pmc_means(os.path.join(src, sub)))
    json.dump(pmc, open(os.path.join(prof, f"{name}_pmc.json"), "w"), indent=1, sort_keys=True)
    kern = [r for r in rows if re.search(KERNELS, r["Name"]) and "true" not in r["Name"]]
    launch_ms = sum(float(r["AverageNs"]) for r in kern) / 1e6
    # per render launch: sum over its kernels (primary pass + path kernel)
    fetch = sum(v for k, v in pmc.items() if k.endswith("|FETCH_SIZE"))
    write = sum(v for k, v in pmc.items() if k.endswith("|WRITE_SIZE"))
    traffic = None
    if fetch and write:
        traffic = int((2 * fetch + write) * 1024)
        json.dump({"hbm_bytes_per_launch": traffic, "fetch_size_kib": fetch, "write_size_kib": write,
                   "source": f"profiles/{name}_pmc.json", "note": "2*FETCH_SIZE+WRITE_SIZE (KiB->B) per render "
                   "launch (primary_kernel + render_wave_kernel) of bench.py's C2 step; FETCH doubling per "
                   "MI355X_MICROARCH.md HBM section; WRITE is dominated by the 16 B/path result scratch"},
                  open(os.path.join(prof, "traffic_c2.json"), "w"), indent=1)
    bench = ""
    blog = os.path.join(src, "bench.log")
    if os.path.exists(blog):
        lines = [l for l in open(blog) if l.startswith("{")]
        bench = lines[-1].strip() if lines else ""
    with open(os.path.join(prof, f"{name}_summary.md"), "w") as f:
        fps = json.loads(bench)["config"].get("frames_per_step", "?") if bench else "?"
        f.write(f"# Profile {name}\n\nSource: `scripts/gpu_round.sh` on one MI355X, bench.py C2 (1280x720, "
                f"{fps} frames per launch).\n\n## rocprofv3 --kernel-trace --stats\n\n| kernel | calls | avg ms |\n|---|---|---|\n")
        for r in rows:
            f.write(f"| `{r['Name'][:70]}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} |\n")
        if kern:
            f.write(f"\nRender launch = {' + '.join(r['Name'].split('(')[0].split('::')[-1] for r in kern)}: "
                    f"{launch_ms:.3f} ms (sum of the averages; compare bench.py roofline.avg_launch_ms)\n")
        f.write("\n## PMC (render kernels, per dispatch)\n\n")
        for k, v in sorted(pmc.items()):
            f.write(f"- {k.split('|')[0].split('(')[0].split('::')[-1]} {k.split('|')[1]}: {v:.4g}\n")
        sq = {k.split('|')[1]: v for k, v in pmc.items() if "render_wave_kernel" in k}
        if "SQ_THREAD_CYCLES_VALU" in sq and "SQ_ACTIVE_INST_VALU" in sq:
            f.write(f"\nVALU lane utilisation = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU) = "
                    f"{sq['SQ_THREAD_CYCLES_VALU'] / (64 * sq['SQ_ACTIVE_INST_VALU']):.3f}\n")
        if "SQ_WAIT_ANY" in sq and "SQ_WAVE_CYCLES" in sq:
            f.write(f"Wave time waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES) = {sq['SQ_WAIT_ANY'] / sq['SQ_WAVE_CYCLES']:.3f}\n")
        if traffic:
            f.write(f"\nHBM traffic per launch = 2*FETCH_SIZE + WRITE_SIZE = {traffic / 1e6:.2f} MB "
                    "(FETCH doubling is calibrated for wide streams only; this kernel's reads are L2-resident gathers)\n")
        if bench:
            f.write(f"\n## bench.py line\n\n```\n{bench}\n```\n")
    print(f"wrote profiles/{name}_summary.md")


if __name__ == "__main__":
    main()
