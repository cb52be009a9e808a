#!/usr/bin/env python3
"""Projected strong scaling of the band sharding, measured on ONE GPU.

  python scripts/tile_scaling.py [C2] [frames_per_step | wF] [path_split, 0 = auto] [N list, e.g. 1,8]

frames_per_step "w16" = 16 x N frames per step (bench.py's default: per-GPU
work per step fixed); a number = that many frames for every N (strong).

For N in 1, 2, 4, 8 this renders rank 0's share of an N-way band split (rank
0 owns the most tiles) and reports the kernel time per step, the projected
whole-job Mpaths/s (full-image paths / rank-0 time, gather excluded) and the
projected efficiency vs N x the 1-GPU rate.  It isolates the per-rank
occupancy loss of strong scaling from the gather cost.

TS_SYNC=1: every render call is synchronised (the reference's cadence --
the Qt host syncs each paint, src/vRendererCuda.cpp:107-165 -- i.e. the
vRendererHIP adapter on a vrhip_create_multi context with 1 or 4 frames per
call): the projection of the one-process multi-GPU path, gather excluded.
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
from vrenderer_pathtracer_amd import VRendererHIP, scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
FARG = sys.argv[2] if len(sys.argv) > 2 else "8"
WEAK = FARG.startswith("w")
F0 = int(FARG[1:] if WEAK else FARG)
SPLIT = int(sys.argv[3]) if len(sys.argv) > 3 else 0
NS = [int(v) for v in sys.argv[4].split(",")] if len(sys.argv) > 4 else [1, 2, 4, 8]
STEPS = int(os.environ.get("TS_STEPS", "20"))      # timed back-to-back steps per N (bench.py's strong leg: 20)
sc = scenes.make_scene(cfg)
W, H = sc["width"], sc["height"]
px = (W // 16) * 16 * (H // 16) * 16
r = VRendererHIP(0)
scenes.load_into(r, sc)
r.set_path_split(SPLIT)
if os.environ.get("TS_SERVICE"):          # experiments: vrhip_set_service mode (1 always, 0 never, -1 automatic)
    r.set_service(int(os.environ["TS_SERVICE"]))
if os.environ.get("TS_OVERLAP"):          # experiments: vrhip_set_overlap mode (1 always, 0 never, -1 automatic)
    r.set_overlap(int(os.environ["TS_OVERLAP"]))
base = None
for n in NS:
    F = F0 * n if WEAK else F0
    paths = px * 2 * F
    r.set_tiling(0, n)
    r.clearBuffer()
    # warm-up: back-to-back steps, so that every path stream has run a launch
    # of this shape (kernel code loaded, scratch allocated, first-use stream
    # joins done) before the timed steps
    W0 = 6
    SYNC = os.environ.get("TS_SYNC", "") == "1"
    for i in range(W0):
        r.render(frames=F, times=[sc["time"] + i * F + k for k in range(F)], sync=SYNC)
    r.sync()
    r.kernel_stats(reset=True)
    torch.cuda.synchronize()
    steps = STEPS
    t0 = time.perf_counter()
    for i in range(steps):
        r.render(frames=F, times=[sc["time"] + (W0 + i) * F + k for k in range(F)], sync=SYNC)
    r.sync()
    dt = (time.perf_counter() - t0) / steps
    kms, launches = r.kernel_stats()
    rate = paths / dt / 1e6
    base = base or rate
    print(f"{cfg} F={F}{' sync' if SYNC else ''} split={SPLIT} N={n}: rank-0 px {r.owned_pixels():7d}  step {dt * 1e3:8.3f} ms  kernel {kms / launches:8.3f} ms  "
          f"projected {rate:9.1f} Mpaths/s  eff {rate / (n * base):.3f}", flush=True)
r.cleanUp()
