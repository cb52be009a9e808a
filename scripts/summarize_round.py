#!/usr/bin/env python3
"""Summarise a scripts/gpu_round.sh output directory into profiles/.

  python scripts/summarize_round.py gpurun_out/<tag> <round-name>

Per config with a trace_<cfg>/ fetch_<cfg>/ write_<cfg>/ triple (bench.py
--steps 5 --warmup 1 under rocprofv3):
  * kernel durations from the per-dispatch kernel trace, averaged over the 5
    TIMED dispatches of each production kernel (the warmup dispatch and the
    untimed counting kernels excluded; production kernels are the named
    feature specialisations, template argument >= 2^31);
  * HBM bytes per render launch (primary_kernel + render_wave_kernel, or
    render_kernel) = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B) over the same timed
    dispatches (MI355X_MICROARCH.md "HBM": FETCH_SIZE reads half of a wide
    coalesced stream; WRITE_SIZE is exact for 16-B-per-lane stores) ->
    profiles/traffic_<cfg>.json, which bench.py reports as roofline.traffic;
  * the bench.py JSON line of the same profiled run, whose avg_launch_ms
    (HIP events around primary + path kernel) the trace sum must agree with.
Copies the rocprofv3 --stats CSVs to profiles/<round>_<cfg>_kernel_stats.csv
and writes profiles/<round>_summary.md (+ the unprofiled bench lines).
"""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STEPS = 5
RENDER = re.compile(r"vr::(render_wave_kernel|primary_kernel|render_kernel)<([^>]*)>")
SERVICE = re.compile(r"vr::(render_service_kernel<[^>]*>|svc_finish_kernel)")


def production(name):
    m = RENDER.search(name)
    if not m:
        return None
    args = [a.strip() for a in m.group(2).split(",")]
    if "true" in args:
        return None
    feat = int(args[1].rstrip("u")) if m.group(1) != "render_kernel" else int(args[2].rstrip("u"))
    # exact scene specialisations (F_EXACT, bit 31), not the instrumented copies (F_COUNT_EXEC, bit 10)
    return m.group(1) if feat >= 2 ** 31 and not (feat & (1 << 10)) else None


def timed_durations(trace_csv):
    per = defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        k = production(r["Kernel_Name"])
        if k:
            per[(k, r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = {}
    for key, v in per.items():
        v.sort()
        t = [d for _, d in v[-STEPS:]]
        out[key] = (sum(t) / len(t) / 1e6, len(v))
    return out


def timed_busy_ms(trace_csv):
    """Busy time per launch: the union of the timed production dispatches'
    intervals / STEPS.  Equals the sum of the averages when launches run one
    after another; with launches overlapped on several path streams (C1, C4:
    per-dispatch durations stretch while they share the GPU) it is the figure
    bench.py's events measure."""
    per = defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        k = production(r["Kernel_Name"])
        if k:
            per[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    iv = sorted(x for v in per.values() for x in sorted(v)[-STEPS:])
    busy, end = 0, None
    for a, b in iv:
        if end is None or a > end:
            busy += b - a
            end = b
        elif b > end:
            busy += b - end
            end = b
    return busy / STEPS / 1e6


def service_busy_ms(trace_csv):
    """Runs whose back-to-back launches went to a render-service session (one
    persistent render_service_kernel dispatch serving many launches, HDRI mesh
    scenes): per-dispatch averages do not apply.  Busy time per launch = the
    union of every production and service dispatch of the run / (STEPS + 1):
    the warmup launch and the 5 timed ones.  None: no service kernel ran."""
    iv, svc = [], False
    for r in csv.DictReader(open(trace_csv)):
        n = r["Kernel_Name"]
        if SERVICE.search(n):
            svc = True
        elif not production(n):
            continue
        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if not svc:
        return None
    iv.sort()
    busy, end = 0, None
    for a, b in iv:
        if end is None or a > end:
            busy += b - a
            end = b
        elif b > end:
            busy += b - end
            end = b
    return busy / (STEPS + 1) / 1e6


def timed_counter(pmc_csv, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(pmc_csv)):
        if r["Counter_Name"] != counter:
            continue
        k = production(r["Kernel_Name"])
        if k:
            per[(k, r["Kernel_Name"])].append((int(r["Start_Timestamp"]), float(r["Counter_Value"])))
    out = {}
    for key, v in per.items():
        v.sort()
        t = [x for _, x in v[-STEPS:]]
        out[key] = sum(t) / len(t)
    return out


def bench_line(log):
    if not os.path.exists(log):
        return None
    lines = [l for l in open(log) if l.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def main():
    src, name = sys.argv[1], sys.argv[2]
    prof = os.path.join(REPO, "profiles")
    md = [f"# Profile {name}\n",
          f"Source: `scripts/gpu_round.sh` on one MI355X (`{os.path.basename(src.rstrip('/'))}`); "
          "rocprofv3 runs of `bench.py --steps 5 --warmup 1 --no-cpu --no-roof --interactive-frames 0 --config <C>`; "
          f"durations and counters averaged over the {STEPS} timed dispatches of each production kernel "
          "(warmup and the untimed counting kernels excluded).\n"]
    for cfg in ("C1", "C2", "C3", "C4", "C5"):
        tdir = os.path.join(src, f"trace_{cfg}")
        traces = glob.glob(os.path.join(tdir, "*kernel_trace.csv"))
        if not traces:
            continue
        stats = glob.glob(os.path.join(tdir, "*kernel_stats.csv"))
        if stats:
            shutil.copy(stats[0], os.path.join(prof, f"{name}_{cfg.lower()}_kernel_stats.csv"))
        dur = timed_durations(traces[0])
        launch_ms = sum(ms for ms, _ in dur.values())
        fetch = write = None
        f_csv = glob.glob(os.path.join(src, f"fetch_{cfg}", "*counter_collection.csv"))
        w_csv = glob.glob(os.path.join(src, f"write_{cfg}", "*counter_collection.csv"))
        if f_csv and w_csv:
            fetch = sum(timed_counter(f_csv[0], "FETCH_SIZE").values())
            write = sum(timed_counter(w_csv[0], "WRITE_SIZE").values())
        traced_bench = bench_line(os.path.join(src, f"trace_{cfg}.log"))
        md.append(f"\n## {cfg}\n\n| kernel | dispatches | avg ms (timed) |\n|---|---|---|\n")
        for (k, full), (ms, n) in sorted(dur.items()):
            md.append(f"| `{full.replace('void ', '').split('(')[0]}` | {n} | {ms:.4f} |\n")
        busy_ms = timed_busy_ms(traces[0])
        svc_ms = service_busy_ms(traces[0])
        md.append(f"\nRender launch (sum of the production kernels) = **{launch_ms:.4f} ms** per launch")
        if svc_ms is not None:
            busy_ms = svc_ms
            md.append(f" (launches after the first ran in a render-service session, one persistent "
                      f"dispatch: busy time {svc_ms:.4f} ms per launch, the union of all production and "
                      f"service dispatches / {STEPS + 1} launches)")
        elif abs(busy_ms - launch_ms) > 0.02 * launch_ms:
            md.append(f" (dispatches overlapped on several path streams: busy time "
                      f"{busy_ms:.4f} ms per launch, the union of the timed dispatches' intervals / {STEPS})")
        if traced_bench:
            rl = traced_bench["roofline"]
            md.append(f"; bench.py's HIP events in the same profiled run: {rl['avg_launch_ms']:.4f} ms "
                      f"over {rl['launches']} launches ({traced_bench['value']:.1f} Mpaths/s under the profiler)")
        md.append(".\n")
        if fetch is not None and write is not None:
            traffic = int((2 * fetch + write) * 1024)
            paths = traced_bench["config"]["paths_per_step"] if traced_bench else None
            json.dump({"hbm_bytes_per_launch": traffic, "fetch_size_kib": fetch, "write_size_kib": write,
                       "launch_ms_trace": launch_ms, "busy_ms_trace": busy_ms, "paths_per_launch": paths,
                       "source": f"profiles/{name}_summary.md ({os.path.basename(src.rstrip('/'))}, fetch_{cfg} / write_{cfg})",
                       "note": "2*FETCH_SIZE + WRITE_SIZE (KiB -> B) per render launch (production render kernels), "
                               f"mean of the {STEPS} timed dispatches; FETCH doubling per MI355X_MICROARCH.md HBM, "
                               "checked for the kernel's 16/32/72-B gathers in profiles/r03_fetch_calibration.md "
                               "(one 128-B line request per line touched, tallied at 64 B)"},
                      open(os.path.join(prof, f"traffic_{cfg.lower()}.json"), "w"), indent=1)
            md.append(f"\nHBM per launch: FETCH_SIZE {fetch / 1024:.1f} MiB, WRITE_SIZE {write / 1024:.1f} MiB -> "
                      f"2*FETCH + WRITE = {traffic / 1e6:.1f} MB = {traffic / 1e9 / (busy_ms / 1e3):.1f} GB/s "
                      f"over the launch's busy time ({traffic / 1e9 / (busy_ms / 1e3) / 8000:.4f} of 8 TB/s)")
            if paths:
                md.append(f"; WRITE_SIZE / (12 B x {paths} path results) = {write * 1024 / (12 * paths):.3f} (12-B radiances since r02e; 16-B float4 before)")
            md.append(".\n")
        unprof = bench_line(os.path.join(src, f"bench_{cfg}.log"))
        for tag, b in (("unprofiled bench.py", unprof), ("profiled bench.py", traced_bench)):
            if b:
                md.append(f"\n{tag}:\n\n```\n{json.dumps(b)}\n```\n")
    out = os.path.join(prof, f"{name}_summary.md")
    open(out, "w").write("".join(md))
    print("wrote", out)


if __name__ == "__main__":
    main()
