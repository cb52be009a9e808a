#!/usr/bin/env python3
"""bench.py -- Mpaths/s of the MI355X path-tracing megakernel (BASELINE.json metric).

Workload (BASELINE.json configs[1], SURVEY.md 8d "C2"): Cornell box + 10k-tri
torus knot, diffuse only, 1280x720, 2 paths/pixel/frame, 4 bounces, default
camera, Fresnel 0.1/3.0.  One "step" = one progressive accumulation step of
FRAMES_PER_STEP frames over the whole image (inputs resident in HBM), ending
with the tile gather to rank 0 when N > 1.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--frames-per-step F] [--config C1..C5]

--config runs the same measurement on another BASELINE.json configuration
(C1 Cornell + example sphere 512x512, C3 HDRI + textured knot 1280x720, C4
MERL BRDF sphere under HDRI 1920x1080, C5 1M-triangle knot under HDRI
3840x2160); the default and the number of record is C2.

N > 1: one process per GPU.  Without an external launcher (WORLD_SIZE unset)
this process starts `torch.distributed.run` with N ranks as a CHILD process
(it never touches the GPU itself) and exits with the child's status.  16x16
pixel tiles are dealt round-robin; each rank renders its tiles of every frame,
then one RCCL gather (ncclGather through the library's C ABI,
vrhip_comm_gather) brings the RGBA8 tiles to rank 0 per step.  The frame size
is fixed and a step accumulates 16 frames whatever N (a fixed display cadence:
"strong" scaling, the same total work per step).  The line also carries
`samples_weak`: 16 x N frames per step (every GPU renders the equivalent of 16
full frames per gather -- SURVEY.md 8e: several frames per gather so that the
gather and each launch's drain stay small against the step); --weak makes that
the headline instead.

Prints ONE JSON line (rank 0).  value = total paths of all ranks / max-over-
ranks wall time of the K timed steps.  "interactive" = the same config one
frame per synchronous call (the reference's render() cadence,
src/vRendererCuda.cpp:107-165).  roofline = the render kernels' EXECUTED
global-load bytes per launch (counted by the instrumented copy of the
production kernels, vrhip_render_profiled, on a separate untimed step) over
their average launch time (HIP events around primary_kernel +
render_wave_kernel on the path stream they run on, inside the timed region),
against the vector-memory gather roof measured live on this GPU
(vrhip_microbench_vmem), the L2 peak and the HBM peak (physical HBM bytes
from the rocprofv3 FETCH_SIZE/WRITE_SIZE passes in profiles/).  The reference
algorithm's bytes (SURVEY.md 8d pricing) are reported separately.
cpu_baseline = the CPU oracle (oracle/, a C restatement of the reference
kernel) on a bounded sample of the same workload on this host's cores.
verified = after the timed loop its first steps are rendered again through
the render service and launch by launch; the SHA-256 digests of the two
accumulations (and RGBA8 images) must agree on every rank, else the bench
exits with status 3.  build = the library's embedded source hash
(vrhip_build_id) and whether it matches the sources on disk.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md "HBM": 8.0 TB/s spec
L2_PEAK_GBS = 34500.0      # MI355X_MICROARCH.md "L2 (per XCD)": ~34.5 TB/s aggregate
# VALU: 256 CUs x 4 SIMDs x 32 lane-ops/cycle (wave64 over 2 cycles) x 2.4 GHz
VALU_PEAK_TOPS = round(256 * 4 * 32 * 2.4e9 / 1e12, 2)
METRIC = "Mpaths/sec (+ Mrays/sec) at 1280x720 progressive; 1/2/4/8 MI355X"
WORKLOADS = {
    "C1": ("C1: Cornell box + example sphere, 512x512, 2 spp/frame, 4 bounces",
           "synthetic (procedural Cornell box + example sphere; SURVEY.md 8d C1)"),
    "C2": ("C2: Cornell box + 10k-tri torus knot, diffuse, 1280x720, 2 spp/frame, 4 bounces",
           "synthetic (procedural Cornell box + 10k-tri torus knot; SURVEY.md 8d C2)"),
    "C3": ("C3: HDRI env + 10k-tri torus knot with diffuse/normal/specular maps + Fresnel, 1280x720, "
           "2 spp/frame, 4 bounces",
           "synthetic (procedural 2048x1024 HDRI, 1024^2 maps, 10k-tri torus knot; SURVEY.md 8d C3)"),
    "C2D": ("C2D (not a BASELINE config): C2 with a 1024^2 diffuse map on the knot, 1280x720, 2 spp/frame, 4 bounces",
            "synthetic (procedural Cornell box + 10k-tri torus knot + diffuse map; feature-class kernel)"),
    "C3D": ("C3D (not a BASELINE config): C3 with only the diffuse map, 1280x720, 2 spp/frame, 4 bounces",
            "synthetic (procedural 2048x1024 HDRI, 1024^2 diffuse map, 10k-tri torus knot; feature-class kernel)"),
    "C4": ("C4: MERL BRDF on the example sphere under HDRI, 1920x1080 (rendered 1920x1072), 2 spp/frame, 4 bounces",
           "synthetic (procedural 2048x1024 HDRI, analytic lobe sampled on the MERL grid; SURVEY.md 8d C4)"),
    "C5": ("C5: 1M-tri torus knot (SBVH-depth tree) under HDRI, 3840x2160, 2 spp/frame, 4 bounces",
           "synthetic (procedural 2048x1024 HDRI, 1M-tri torus knot; SURVEY.md 8d C5)"),
}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """Start n ranks (one per GPU) under torch.distributed.run as a child
    process; this process never initialises the GPU (no exec after GPU use)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


# ---- bytes ------------------------------------------------------------------
def reference_bytes(c: dict, paths: int, pixel_frames: int) -> float:
    """SURVEY.md 8d byte costs of the REFERENCE algorithm (strict traversal, no
    primary-hit reuse): 64 B/node visit, 48 B/triangle tested (+16 B per
    terminator slot read, 0 with the device layout), hit attribute bytes,
    16 B/texture or HDRI fetch, 12 B/BRDF lookup, 92 B of pixel I/O per pixel-frame."""
    return (64 * c["node_visits"] + 16 * c["slot_reads"] + 48 * c["tri_tests"] + c["attr_bytes"]
            + 16 * c["tex_fetches"] + 16 * c["hdr_fetches"] + 12 * c["brdf_fetches"] + 92 * pixel_frames)


def executed_loads(e: dict) -> dict:
    """Per-lane global loads the production render kernels issue, by width in
    bytes, as counted at every load site by the instrumented kernels: node
    visits not served from LDS (2x16 B per conservative fp16 node), triangle
    pairs (4x16 + 8 B), primary records (2x16 B per path), hit attributes
    (uv 3x8, tangents / normals 3x16, face-normal vertices 3x12 -- those the
    scene's specialised kernel loads), texels and HDRI (16 B), BRDF entries (12 B: the device table is
    interleaved RGB, round 6)."""
    return {16: e["lane_loads_b128"], 12: e["lane_loads_b96"], 8: e["lane_loads_b64"], 4: e["lane_loads_b32"]}


def vmem_roof(device: int) -> dict:
    """Lane loads/s of the vector-memory gather path per load width: the best
    over 1..64 distinct addresses per wave-instruction (vrhip_microbench_vmem)."""
    from vrenderer_pathtracer_amd import microbench_vmem
    roof = {}
    for w in (16, 12, 8, 4):
        rates = {d: microbench_vmem(w, d, device) for d in (1, 4, 16, 64)}
        roof[w] = {"best": max(rates.values()), "by_distinct": {str(d): round(r / 1e9, 2) for d, r in rates.items()}}
    return roof


def hbm_traffic(cfg: str):
    """Physical HBM bytes per render launch of bench.py's step on this config
    (rocprofv3 2*FETCH_SIZE + WRITE_SIZE of primary_kernel + render_wave_kernel,
    profiles/traffic_<cfg>.json, MI355X_MICROARCH.md HBM corrections)."""
    path = os.path.join(REPO, "profiles", f"traffic_{cfg.lower()}.json")
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
        return d.get("hbm_bytes_per_launch"), os.path.relpath(path, REPO)
    except Exception:
        return None, None


def unit_busy(cfg: str):
    """Busy fractions of the CU units the path kernel is bound by, from the
    rocprofv3 counter passes of this config (profiles/units_<cfg>.json,
    scripts/summarize_mem_r02.py): texture address (TA) and data (TD) paths
    per CU, VALU pipe per SIMD.  Measured on the production kernel in a
    profiled run, not live; null when no pass was kept."""
    path = os.path.join(REPO, "profiles", f"units_{cfg.lower()}.json")
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return None


# ---- CPU baseline -------------------------------------------------------------
def cpu_info() -> dict:
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = aff
    why = f"sched_getaffinity = {aff} CPUs"
    if omp and omp.isdigit() and 0 < int(omp) < aff:
        threads = int(omp)
        why += f"; OMP_NUM_THREADS = {omp} (the lease's CPU share)"
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity": aff, "threads": threads, "threads_why": why}


def cpu_baseline(scene: dict, budget_s: float) -> dict:
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import pyoracle
    pyoracle.build()
    info = cpu_info()
    threads = info["threads"]
    W, H = scene["width"], scene["height"]
    hr = (H // 16) * 16
    accum = np.zeros((H, W, 4), np.float32)
    paths, frames, t0 = 0, 0, time.perf_counter()
    chunk = 16
    while time.perf_counter() - t0 < budget_s and frames < 64:
        frame = frames + 1
        for r0 in range(0, hr, chunk):
            pyoracle.render(scene, frames=1, times=[scene["time"] + frames], first_frame=frame,
                            rows=(r0, min(hr, r0 + chunk)), threads=threads, accum=accum)
            paths += (min(hr, r0 + chunk) - r0) * (W // 16) * 16 * 2
            if time.perf_counter() - t0 >= budget_s:
                break
        frames += 1
    dt = time.perf_counter() - t0
    rows = paths // (2 * (W // 16) * 16)
    out = {"value": round(paths / dt / 1e6, 4), "unit": "Mpaths/s", "cores": threads, "kind": "port",
           "sample": f"oracle/ C restatement (glibc libm, -O2, OpenMP {threads} threads), {scene['name']} "
                     f"{W}x{H}, {rows} rows over {frames} frame(s) ({paths} paths, {dt:.1f} s)"}
    out.update(info)
    return out


# ---- self-check of the timed image ---------------------------------------------
VERIFY_STEPS = 3


def self_check(r, scene: dict, F: int, svc_mode: int, world: int, red_dev) -> dict:
    """Render the timed loop's first VERIFY_STEPS steps (same frame counts and
    times) twice from a cleared accumulation: through the render service
    (vrhip_set_service(1): every launch on the session kernel the timed steps
    run on, the sessions' multi-slot finish pass) and launch by launch
    (vrhip_set_service(0)); SHA-256 of each run's accumulation (float4 bits)
    and RGBA8 image.  verified = the digests agree on every rank.  The
    renderer is left cleared, in service mode svc_mode."""
    import hashlib
    import torch
    import torch.distributed as dist
    runs = {}
    for label, mode in (("service", 1), ("launch_path", 0)):
        r.set_service(mode)
        r.clearBuffer()
        kinds = []
        for i in range(VERIFY_STEPS):
            r.render(frames=F, times=[scene["time"] + i * F + k for k in range(F)], sync=False)
            kinds.append(r.last_launch_info()["kind"])
        r.sync()
        acc, rgba = r.read_accum(), r.read_rgba8()
        runs[label] = {"accum_sha256": hashlib.sha256(acc.tobytes()).hexdigest(),
                       "rgba8_sha256": hashlib.sha256(rgba.tobytes()).hexdigest(), "kinds": kinds}
    r.set_service(svc_mode)
    r.clearBuffer()
    r.sync()
    same = int(runs["service"]["accum_sha256"] == runs["launch_path"]["accum_sha256"]
               and runs["service"]["rgba8_sha256"] == runs["launch_path"]["rgba8_sha256"])
    ok = torch.tensor([float(same)], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    return {"verified": bool(ok.item() == 1.0), "steps": VERIFY_STEPS, "frames_per_step": F,
            "service": runs["service"], "launch_path": runs["launch_path"],
            "note": "the timed loop's first steps re-rendered from a cleared accumulation through the render service "
                    "(mode 1) and launch by launch (mode 0); SHA-256 of accum and RGBA8 (this rank's; all ranks "
                    "agree when verified)"}


# ---- main ---------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames-per-step", type=int, default=None,
                    help="frames accumulated per step (= per gather); default 16 whatever N (fixed cadence)")
    ap.add_argument("--weak", action="store_true",
                    help="16 x N frames per step as the headline (every GPU renders 16 full-frame equivalents per "
                         "step: weak scaling in samples, fixed resolution)")
    ap.add_argument("--strong", action="store_true", help="(the default) 16 frames per step for any N")
    ap.add_argument("--config", default="C2", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--interactive-frames", type=int, default=60,
                    help="frames of the one-frame-per-call measurement (0: skip)")
    ap.add_argument("--interactive-warmup", type=int, default=30,
                    help="untimed one-frame calls before it (the first ~20 ms of calls after a clear run "
                         "2-3 %% slower: profiles/r06zt/README.md)")
    ap.add_argument("--strong-steps", type=int, default=20,
                    help="steps of the secondary measurement (N > 1: the 16 x N-frame steps under 'samples_weak', "
                         "and the one-GPU 16-frame reference of 'strong'; 0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-roof", action="store_true", help="skip the vector-memory roof micro-benchmark")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the self-check after the timed loop (profiling runs: the timed dispatches are then "
                         "the run's last ones, as scripts/summarize_round.py assumes)")
    ap.add_argument("--check-launch", action="store_true",
                    help="form the process group over gloo, count the ranks and exit (no GPU; tests the launcher)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist

    if args.check_launch:
        if world > 1:
            dist.init_process_group("gloo")
        n = torch.ones(1)
        if world > 1:
            dist.all_reduce(n)
            dist.destroy_process_group()
        if rank == 0:
            print(json.dumps({"check_launch": True, "n_gpus": int(n.item()), "gpus_arg": args.gpus}), flush=True)
        return

    # VRHIP_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks
    # on one GPU (host-staged gather); the measured configuration is "nccl":
    # one rank per GPU, the tile gather over RCCL (xGMI) in the C ABI
    backend = os.environ.get("VRHIP_DIST_BACKEND", "nccl")
    gpu = local_rank if backend == "nccl" else local_rank % max(1, torch.cuda.device_count())
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        formed = dist.get_world_size()
        if formed != args.gpus:
            raise SystemExit(f"bench.py: process group formed {formed} ranks, --gpus {args.gpus}")
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    from vrenderer_pathtracer_amd import VRendererHIP, build_id, build_native, scenes
    from vrenderer_pathtracer_amd.tiles import TileGather, WHAT_RGBA8
    build_native()
    CFG = args.config
    scene = scenes.make_scene(CFG)
    W, H = scene["width"], scene["height"]
    F = args.frames_per_step or (16 * world if args.weak else 16)
    scaling = "weak" if (args.weak and world > 1) else "strong"

    r = VRendererHIP(gpu)
    scenes.load_into(r, scene)
    r.set_tiling(rank, world)
    owned = r.owned_pixels()
    gather = TileGather(r, rank, world, dev, WHAT_RGBA8)
    mesh = scene.get("mesh_flat") is not None
    # N > 1: explicit render-service mode, so a step's RCCL gather is deferred
    # to the session's close and consecutive steps share one session (their
    # drains overlap); every rank closes its session (r.sync()) before any
    # host barrier, the ordering include/vrhip.h asks of explicit mode.  One
    # rank: the library default (automatic: the first call of a burst on the
    # launch path, the calls behind it on the service)
    svc_mode = 1 if (world > 1 and gather.native) else -1
    r.set_service(svc_mode)

    # untimed counting steps on this rank's share: (1) the reference
    # algorithm's events (strict traversal, no primary-hit reuse, no last-
    # bounce shortcut) for the survey's byte pricing and Mrays/s; (2) the
    # memory operations the production kernels execute, for the roofline
    r.set_strict_traversal(True)
    ref_counts = r.render_counted(frames=F, time_seed=scene["time"])
    r.set_strict_traversal(False)
    r.clearBuffer()
    exec_counts = r.render_profiled(frames=F, time_seed=scene["time"])
    r.clearBuffer()
    r.sync()

    roof = None
    if rank == 0 and not args.no_roof:
        roof = vmem_roof(gpu)

    def step(i):
        times = [scene["time"] + i * F + k for k in range(F)]
        r.render(frames=F, times=times, sync=False)
        gather.step()

    for i in range(args.warmup):
        step(i)
    r.sync()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    r.kernel_stats(reset=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    r.sync()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kms, launches = r.kernel_stats()
    launch_info = r.last_launch_info()
    t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    wr = (W // 16) * 16
    hr = (H // 16) * 16

    # self-check of the timed path: the first VERIFY_STEPS steps of the timed
    # loop rendered again from a cleared accumulation, once on the render
    # service (mode 1: every launch through the session kernel the timed
    # steps ran on) and once launch by launch (mode 0), with the same times;
    # SHA-256 of the accumulation and RGBA8 image must agree on every rank
    verify = (self_check(r, scene, F, svc_mode, world, red_dev) if not args.no_verify
              else {"verified": None, "note": "skipped (--no-verify)"})
    if rank == 0 and verify["verified"] is False:
        print(json.dumps({"metric": METRIC, "verified": False, "verify": verify}), flush=True)
    if verify["verified"] is False:
        raise SystemExit(3)

    def timed_steps(rr, frames, steps, base, with_gather=True):
        """max-over-ranks wall time of `steps` back-to-back steps of `frames`
        frames on renderer rr (+ the tile gather per step)."""
        def one(i):
            rr.render(frames=frames, times=[base + i * frames + k for k in range(frames)], sync=False)
            if with_gather:
                gather.step()
        for i in range(2):
            one(i)
        rr.sync()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for i in range(steps):
            one(2 + i)
        rr.sync()
        if world > 1:
            dist.barrier()
        tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    # fixed cadence: 16 frames per step (per gather) whatever N -- the
    # headline by default -- against the 1-GPU rate of the same 16-frame
    # step, measured on every GPU at once over the whole image
    strong = None
    if args.strong_steps > 0:
        SF = 16
        if F != SF:
            r.clearBuffer()
            ts, n_st = timed_steps(r, SF, args.strong_steps, scene["time"] + 500000), args.strong_steps
        else:
            ts, n_st = elapsed, args.steps          # the main measurement is already at 16 frames per step
        strong = {"frames_per_step": SF, "steps": n_st,
                  "value": round(wr * hr * 2 * SF * n_st / ts / 1e6, 3),
                  "ms_per_step": round(ts / n_st * 1e3, 4)}
        if world > 1:
            # a second context renders the whole image alone on every GPU at once
            r1 = VRendererHIP(gpu)
            scenes.load_into(r1, scene)
            t1 = timed_steps(r1, SF, args.strong_steps, scene["time"] + 600000, with_gather=False)
            r1.cleanUp()
            one_gpu = wr * hr * 2 * SF * args.strong_steps / t1 / 1e6
        else:
            one_gpu = strong["value"]
        strong["one_gpu_value"] = round(one_gpu, 3)
        strong["efficiency"] = round(strong["value"] / (world * one_gpu), 4)
        strong["note"] = ("16 frames per step and per RCCL gather for any N (fixed display cadence); efficiency = "
                          "value / (N x one_gpu_value), one_gpu_value = the same 16-frame step over the whole "
                          "image on one GPU, measured in this run on every GPU at once")

    # samples-weak view: 16 x N frames per step (every GPU renders 16 full-
    # frame equivalents per gather), secondary unless --weak made it the headline
    samples_weak = None
    if world > 1 and args.strong_steps > 0:
        WF = 16 * world
        if F != WF:
            r.clearBuffer()
            tw = timed_steps(r, WF, args.strong_steps, scene["time"] + 700000)
            n_w = args.strong_steps
        else:
            tw, n_w = elapsed, args.steps
        samples_weak = {"frames_per_step": WF, "steps": n_w,
                        "value": round(wr * hr * 2 * WF * n_w / tw / 1e6, 3),
                        "ms_per_step": round(tw / n_w * 1e3, 4)}
        if strong:
            samples_weak["efficiency"] = round(samples_weak["value"] / (world * strong["one_gpu_value"]), 4)
        samples_weak["note"] = ("16 x N frames per step and per RCCL gather (every GPU renders 16 full-frame "
                                "equivalents per step); efficiency against the same one_gpu_value as 'strong'")

    # interactive cadence: one frame per synchronous render() call (+ gather)
    inter = None
    if args.interactive_frames > 0:
        r.clearBuffer()
        # the Qt adapter's configuration (integration/vRendererHIP.cpp): no
        # kernel-timing events on the launch path (nothing reads them there),
        # the library's automatic service mode
        r.set_kernel_timing(False)
        r.set_service(-1)
        base = scene["time"] + 100000
        nw = max(1, args.interactive_warmup)
        for i in range(nw):
            r.render(frames=1, times=[base + i], sync=True)
            gather.step()
        r.sync()
        if world > 1:
            dist.barrier()
        ti = time.perf_counter()
        for i in range(args.interactive_frames):
            # one synchronisation per frame, as vRendererCuda::render's
            # cudaStreamSynchronize (the tile gather, N > 1, is inside it)
            r.render(frames=1, times=[base + nw + i], sync=False)
            gather.step()
            r.sync()
        if world > 1:
            dist.barrier()
        te = torch.tensor([time.perf_counter() - ti], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(te, op=dist.ReduceOp.MAX)
        te = float(te.item())
        r.set_kernel_timing(True)
        pf = (W // 16) * 16 * (H // 16) * 16 * 2
        inter = {"frames_per_step": 1, "frames": args.interactive_frames, "warmup_frames": nw,
                 "value": round(pf * args.interactive_frames / te / 1e6, 3), "unit": "Mpaths/s",
                 "ms_per_frame": round(te / args.interactive_frames * 1e3, 4),
                 "note": "one frame per synchronous render() call (src/vRendererCuda.cpp:107-165 syncs every "
                         "frame)" + (", plus the RGBA8 tile gather to rank 0 per frame" if world > 1 else "")
                 + "; kernel-timing events off, as in the Qt adapter (vrhip_set_kernel_timing)"}

    # aggregate counts over ranks
    keys = sorted(ref_counts)
    cvec = torch.tensor([ref_counts[k] for k in keys] + [owned], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(cvec)
    tot = {k: float(v) for k, v in zip(keys + ["owned_pixels"], cvec.tolist())}

    paths_per_step = wr * hr * 2 * F
    total_paths = paths_per_step * args.steps
    value = total_paths / elapsed / 1e6
    rays_per_path = tot["rays"] / paths_per_step
    mrays = value * rays_per_path
    # rays the production kernels trace (the instrumented copy's own count:
    # camera rays once per pixel per launch, shared by its paths, plus every
    # bounce ray; no material sampling after the last bounce)
    evec = torch.tensor([float(exec_counts["rays"])], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(evec)
    rays_per_path_traced = float(evec.item()) / paths_per_step

    if rank == 0:
        own_paths = owned * 2 * F
        avg_launch_s = (kms / 1e3) / max(launches, 1)
        loads = executed_loads(exec_counts)
        load_bytes = sum(w * n for w, n in loads.items())
        lds_bytes = 32 * exec_counts["node_visits_lds"]        # fp16 node rows from the LDS copy
        # stores by launch mode (vrhip_last_launch_info): through the result
        # scratch, 12-B path radiances + the 4-B depth term per pixel (+ the
        # 32-B primary records of mesh scenes) and the finish pass's accum /
        # RGBA8 / depth; in registers (sphere-only launches of one path group)
        # only the accum / RGBA8 / depth of every pixel.  A split sphere
        # launch stores one 12-B record per pixel whose camera ray escapes
        # (its paths share it: shared_miss_paths) instead of one per path
        store_bytes = 24 * owned
        if launch_info["use_scratch"]:
            shared = int(exec_counts.get("shared_miss_paths", 0))
            store_bytes += (12 * (own_paths - shared) + 12 * (shared // (2 * F)) + 4 * owned
                            + (32 * owned if mesh else 0))
        ref_b = reference_bytes(ref_counts, own_paths, owned * F)
        achieved = load_bytes / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
        roofs = {}
        if roof and load_bytes > 0:
            t_min = sum(n / roof[w]["best"] for w, n in loads.items())
            roofs["vmem"] = {"achieved": round(achieved, 1), "peak": round(load_bytes / t_min / 1e9, 1),
                             "frac": round(t_min / avg_launch_s, 4)}
        roofs["l2"] = {"achieved": round(achieved, 1), "peak": L2_PEAK_GBS, "frac": round(achieved / L2_PEAK_GBS, 4)}
        # where the kernel's gather rate sits between the micro-benchmark's
        # one-address-per-wave roof and its 64-distinct-lines rate (every lane
        # on its own line): not a roof, a position -- the texture path charges
        # per line a lane touches, so divergent rays sit near the second figure
        gpos = None
        if roof and load_bytes > 0:
            def rate(w, d):                          # lane loads per second
                return roof[w]["by_distinct"][str(d)] * 1e9
            t_div = sum(n / rate(w, 64) for w, n in loads.items() if n)
            t_one = sum(n / rate(w, 1) for w, n in loads.items() if n)
            gpos = {"launch_ms": round(avg_launch_s * 1e3, 4), "ms_at_1_address": round(t_one * 1e3, 4),
                      "ms_at_64_lines": round(t_div * 1e3, 4),
                      "lane_loads_per_ns": round(sum(loads.values()) / avg_launch_s / 1e9, 1)}
        traffic, traffic_src = hbm_traffic(CFG)
        if traffic and world == 1:
            hbm_gbs = traffic / avg_launch_s / 1e9
            roofs["hbm"] = {"achieved": round(hbm_gbs, 1), "peak": HBM_PEAK_GBS, "frac": round(hbm_gbs / HBM_PEAK_GBS, 4)}
        ub = unit_busy(CFG)
        if load_bytes == 0 and ub and "valu" in ub and "valu_lane_util" in ub:
            # VALU roof in active lane-ops: a wave64 VALU instruction issues
            # over 2 cycles (MI355X_MICROARCH.md:54, the guide's figure; not
            # measured here), so a SIMD retires at most 32 lane-ops per cycle.
            # achieved = pipe-busy fraction (SQ_INSTS_VALU x 2 cycles) x the
            # measured VALU lane utilisation, both from this config's counter
            # pass (profiles/units_<cfg>.json)
            frac = ub["valu"] * ub["valu_lane_util"]
            roofs["valu"] = {"achieved": round(frac * VALU_PEAK_TOPS, 2), "peak": VALU_PEAK_TOPS,
                             "frac": round(frac, 4), "pipe_busy": ub["valu"], "lane_util": ub["valu_lane_util"],
                             "unit": "T VALU lane-ops/s"}
        if load_bytes == 0:
            # sphere-only scenes without textures (C1): no global loads on the
            # path -- the sphere tests and libm are VALU work, priced by the
            # VALU roof above when this config's counter pass is kept
            roofs.pop("l2", None)
            roofs.setdefault("hbm", {"achieved": 0.0, "peak": HBM_PEAK_GBS, "frac": 0.0})
        bound = max(roofs, key=lambda k: roofs[k]["frac"])
        roofline = {"bound": bound, "achieved": roofs[bound]["achieved"], "peak": roofs[bound]["peak"],
                    "unit": roofs[bound].get("unit", "GB/s"),
                    "frac": roofs[bound]["frac"], "traffic": traffic if world == 1 else None,
                    "kernel": "primary_kernel+render_wave_kernel" if mesh else "render_kernel",
                    "avg_launch_ms": round(avg_launch_s * 1e3, 4), "launches": launches,
                    "executed_load_bytes_per_launch": int(load_bytes),
                    "lane_loads_per_launch": {f"b{8 * w}": int(n) for w, n in loads.items()},
                    "lds_node_bytes_per_launch": int(lds_bytes), "store_bytes_per_launch": int(store_bytes),
                    "launch": launch_info,
                    "shared_miss_paths_per_launch": int(exec_counts.get("shared_miss_paths", 0)),
                    "roofs": roofs,
                    "gather_position": gpos,
                    "traffic_source": traffic_src,
                    "unit_busy": unit_busy(CFG),
                    "vmem_roof_lane_loads_per_ns": ({f"b{8 * w}": v["by_distinct"] for w, v in roof.items()}
                                                    if roof else None),
                    "reference_algorithm": {
                        "bytes_per_path": round(ref_b / max(own_paths, 1), 1),
                        "gbs_at_this_rate": round(ref_b / avg_launch_s / 1e9, 1) if avg_launch_s > 0 else None,
                        "note": "SURVEY 8d pricing of the reference algorithm's events (strict traversal, no "
                                "primary-hit reuse); not executed bytes, so not a roofline"},
                    "note": "achieved = global-load bytes the production kernels execute (instrumented copy, "
                            "untimed step) / render-kernel launch time; vmem peak = the same lane loads at the "
                            "live-measured gather roof (vrhip_microbench_vmem, best of 1..64 addresses per "
                            "wave-instruction); bound = the roof with the largest fraction; traffic = physical "
                            "HBM bytes per launch (rocprofv3 PMC, traffic_source)"}
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": WORKLOADS[CFG][1],
            "config": {"workload": WORKLOADS[CFG][0], "width": W, "height": H, "frames_per_step": F,
                       "paths_per_step": paths_per_step, "parallelism": f"tile{world}",
                       "gather": (("RCCL ncclGather (C ABI vrhip_comm_gather)" if backend == "nccl" else
                                   backend + " gather (host-staged rehearsal)")
                                  + " of RGBA8 tiles to rank 0 per step") if world > 1 else "none"},
            "mrays_per_s": round(mrays, 3),
            "rays_per_path": round(rays_per_path, 4),
            "mrays_per_s_traced": round(value * rays_per_path_traced, 3),
            # paths whose result was their pixel's shared escape radiance
            # (sphere-only HDRI scenes: the camera ray escapes, no jitter), so
            # they made no HDRI fetch of their own (render_kernel)
            "shared_escape_path_frac": round(exec_counts.get("shared_miss_paths", 0) / max(owned * 2 * F, 1), 4),
            "rays_per_path_traced": round(rays_per_path_traced, 4),
            "mrays_note": ("mrays_per_s is reference-equivalent: intersectScene calls of the reference algorithm "
                           "(two camera rays per pixel per frame, SURVEY 8d) at this path rate; "
                           "mrays_per_s_traced counts the rays the kernels trace (a pixel's camera ray once "
                           "per launch: no camera jitter, PathTracer.cu:842-844)"),
            "strong": strong,
            "samples_weak": samples_weak,
            "interactive": inter,
            "roofline": roofline,
            "verified": verify["verified"],
            "verify": verify,
            "build": build_id(),
        }
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(scene, args.cpu_budget)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    gather.close()
    r.cleanUp()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
