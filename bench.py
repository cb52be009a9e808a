#!/usr/bin/env python3
"""bench.py -- Mpaths/s of the MI355X path-tracing megakernel (BASELINE.json metric).

Workload (BASELINE.json configs[1], SURVEY.md 8d "C2"): Cornell box + 10k-tri
torus knot, diffuse only, 1280x720, 2 paths/pixel/frame, 4 bounces, default
camera, Fresnel 0.1/3.0.  One "step" = one progressive accumulation step of
FRAMES_PER_STEP frames over the whole 1280x720 image (inputs resident in
HBM), ending with the tile gather to rank 0 when N > 1.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--frames-per-step F] [--config C2]

--config C3 / C5 runs the same measurement on another BASELINE.json
configuration (C3: HDRI + textured knot at 1280x720; C5: 1M-triangle knot
under HDRI at 3840x2160); the default and the number of record is C2.

N > 1: one process per GPU (torch.distributed.run), 16x16 pixel
tiles dealt round-robin, each rank renders its tiles of every frame, then one
RCCL gather (torch.distributed over "nccl" = RCCL) of the RGBA8 tiles to rank
0 per step.
Strong scaling: the frame size is fixed.

Prints ONE JSON line (rank 0).  value = total paths of all ranks / max-over-
ranks wall time of the K timed steps.  roofline = the render
kernels' algorithmic bytes per launch (counted by the kernel's counting
variant on a separate, untimed step; SURVEY.md 8d byte costs) / their
average launch time (HIP events around primary_kernel + render_wave_kernel
on the path stream they run on, inside the timed region).  cpu_baseline =
the CPU oracle (oracle/, a C restatement of the reference kernel) on a
bounded sample of the same workload on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
WORKLOADS = {
    "C2": ("C2: Cornell box + 10k-tri torus knot, diffuse, 1280x720, 2 spp/frame, 4 bounces",
           "synthetic (procedural Cornell box + 10k-tri torus knot; SURVEY.md 8d C2)"),
    "C3": ("C3: HDRI env + 10k-tri torus knot with diffuse/normal/specular maps + Fresnel, 1280x720, "
           "2 spp/frame, 4 bounces",
           "synthetic (procedural 2048x1024 HDRI, 1024^2 maps, 10k-tri torus knot; SURVEY.md 8d C3)"),
    "C5": ("C5: 1M-tri torus knot (SBVH-depth tree) under HDRI, 3840x2160, 2 spp/frame, 4 bounces",
           "synthetic (procedural 2048x1024 HDRI, 1M-tri torus knot; SURVEY.md 8d C5)"),
}
PROFILE_TRAFFIC = os.path.join(REPO, "profiles", "traffic_c2.json")


def algorithmic_bytes(c: dict, paths: int, pixel_frames: int) -> float:
    """SURVEY.md 8d byte costs, as the kernel executes them: 64 B/node visit,
    48 B/triangle tested (16 B per terminator slot read, 0 with the device
    layout), hit attribute bytes, 16 B/texture or HDRI fetch, 12 B/BRDF lookup,
    92 B of pixel I/O per pixel-frame."""
    return (64 * c["node_visits"] + 16 * c["slot_reads"] + 48 * c["tri_tests"] + c["attr_bytes"]
            + 16 * c["tex_fetches"] + 16 * c["hdr_fetches"] + 12 * c["brdf_fetches"] + 92 * pixel_frames)


def cpu_baseline(scene: dict, budget_s: float, threads: int) -> dict:
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import numpy as np
    import pyoracle
    pyoracle.build()
    W, H = scene["width"], scene["height"]
    accum = np.zeros((H, W, 4), np.float32)
    paths, frames, t0 = 0, 0, time.perf_counter()
    chunk = 16
    while time.perf_counter() - t0 < budget_s and frames < 64:
        frame = frames + 1
        for r0 in range(0, H, chunk):
            pyoracle.render(scene, frames=1, times=[scene["time"] + frames], first_frame=frame,
                            rows=(r0, min(H, r0 + chunk)), threads=threads, accum=accum)
            paths += (min(H, r0 + chunk) - r0) * W * 2
            if time.perf_counter() - t0 >= budget_s:
                break
        frames += 1
    dt = time.perf_counter() - t0
    rows = paths // (2 * W)
    return {"value": round(paths / dt / 1e6, 4), "unit": "Mpaths/s", "cores": threads, "kind": "port",
            "sample": f"oracle/ C restatement (glibc libm, -O2, OpenMP {threads} threads), {scene['name']} "
                      f"{W}x{H}, {rows} rows over {frames} frame(s) ({paths} paths, {dt:.1f} s)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--frames-per-step", type=int, default=16)
    ap.add_argument("--config", default="C2", choices=sorted(WORKLOADS))
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # VRHIP_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks
    # on one GPU (host-staged gather); the measured configuration is "nccl"
    # (RCCL over xGMI), one rank per GPU
    backend = os.environ.get("VRHIP_DIST_BACKEND", "nccl")
    gpu = local_rank if backend == "nccl" else local_rank % max(1, torch.cuda.device_count())
    dev = torch.device("cuda", gpu)
    if world > 1:
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    from vrenderer_pathtracer_amd import VRendererHIP, build_native, scenes
    from vrenderer_pathtracer_amd.tiles import TileGather, WHAT_RGBA8
    build_native()
    CFG = args.config
    scene = scenes.make_scene(CFG)
    W, H = scene["width"], scene["height"]
    F = args.frames_per_step

    r = VRendererHIP(gpu)
    scenes.load_into(r, scene)
    # one non-default stream shared by the renderer and torch (the collective
    # is ordered after the pack kernel by torch's stream semantics)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    r.set_stream(stream.cuda_stream)
    r.set_tiling(rank, world)
    owned = r.owned_pixels()
    gather = TileGather(r, rank, world, dev, WHAT_RGBA8)

    # counting step (untimed): exact event counts of the REFERENCE algorithm for
    # this rank's share (strict traversal; the counting variant also skips the
    # primary-hit reuse and last-bounce shortcut), i.e. the algorithmic work
    r.set_strict_traversal(True)
    counts = r.render_counted(frames=F, time_seed=scene["time"])
    r.set_strict_traversal(False)
    r.clearBuffer()

    def step(i):
        times = [scene["time"] + i * F + k for k in range(F)]
        r.render(frames=F, times=times, sync=False)
        gather.step()

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    r.kernel_stats(reset=True)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kms, launches = r.kernel_stats()
    t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # aggregate counts over ranks
    keys = sorted(counts)
    cvec = torch.tensor([counts[k] for k in keys] + [owned], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(cvec)
    tot = {k: float(v) for k, v in zip(keys + ["owned_pixels"], cvec.tolist())}

    wr = (W // 16) * 16
    hr = (H // 16) * 16
    paths_per_step = wr * hr * 2 * F
    total_paths = paths_per_step * args.steps
    value = total_paths / elapsed / 1e6
    rays_per_path = tot["rays"] / paths_per_step
    mrays = value * rays_per_path

    if rank == 0:
        # roofline of the render kernel on rank 0 (its own share per launch)
        own_paths = owned * 2 * F
        bytes_per_launch = algorithmic_bytes(counts, own_paths, owned * F)
        avg_launch_s = (kms / 1e3) / max(launches, 1)
        achieved = bytes_per_launch / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
        traffic = None
        if CFG == "C2" and os.path.exists(PROFILE_TRAFFIC):   # rocprofv3 PMC of the C2 step
            try:
                traffic = json.load(open(PROFILE_TRAFFIC)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        out = {
            "metric": "Mpaths/sec (+ Mrays/sec) at 1280x720 progressive; 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": WORKLOADS[CFG][1],
            "config": {"workload": WORKLOADS[CFG][0], "width": W, "height": H, "frames_per_step": F,
                       "paths_per_step": paths_per_step, "parallelism": f"tile{world}",
                       "gather": ("RCCL" if backend == "nccl" else backend) + " gather of RGBA8 tiles to rank 0 per step"
                       if world > 1 else "none"},
            "mrays_per_s": round(mrays, 3),
            "rays_per_path": round(rays_per_path, 4),
            "bytes_per_path": round(bytes_per_launch / max(own_paths, 1), 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "primary_kernel+render_wave_kernel", "avg_launch_ms": round(avg_launch_s * 1e3, 4),
                         "launches": launches,
                         "note": "algorithmic bytes of the reference algorithm (SURVEY 8d), served mostly from "
                                 "L2/LDS (traffic = physical HBM bytes per launch); launches of fewer than 2^24 paths "
                                 "(sharded frames) overlap on three path streams, and then avg_launch_ms includes "
                                 "time shared with the neighbouring launch"},
        }
        if not args.no_cpu and world == 1:
            threads = min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(scene, args.cpu_budget, threads)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    r.cleanUp()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
