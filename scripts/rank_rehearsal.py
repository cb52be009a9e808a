#!/usr/bin/env python3
"""8-rank projection of a BASELINE configuration, rehearsed on ONE GPU at full size.

  python scripts/rank_rehearsal.py [C5] [ranks=8] [frames_per_step=16] [steps=10]

For every rank r of an N-way tile split this times `steps` back-to-back
16-frame steps of rank r's tiles (set_tiling(r, N), the library's automatic
render service, as bench.py runs a rank), then the device pack of the rank's
RGBA8 tiles (vrhip_pack_tiles, the gather's send buffer) and, for rank 0, the
unpack of all N packed buffers into the full image (vrhip_unpack_tiles, what
rank 0 does after ncclGather).  The projected 8-GPU step is

  max over ranks of (step time + pack) + gather + unpack

with the gather (not measurable on one GPU) modelled from the payload: rank
0 receives N-1 packed buffers, one per xGMI link in parallel, at
XGMI_GBS (default 50 GB/s per link and direction, below the ~64 GB/s link
rate) plus GATHER_LAT_US (default 30 us) of collective latency.  Efficiency
= projected rate / (N x the one-GPU rate of the same 16-frame step over the
whole image, measured here).  Prints one JSON line.
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
from vrenderer_pathtracer_amd import VRendererHIP, scenes  # noqa: E402
from vrenderer_pathtracer_amd.tiles import WHAT_RGBA8, max_owned_pixels  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
F = int(sys.argv[3]) if len(sys.argv) > 3 else 16
STEPS = int(sys.argv[4]) if len(sys.argv) > 4 else 100
XGMI_GBS = float(os.environ.get("XGMI_GBS", "50"))
GATHER_LAT_US = float(os.environ.get("GATHER_LAT_US", "30"))

sc = scenes.make_scene(cfg)
W, H = sc["width"], sc["height"]
px = (W // 16) * 16 * (H // 16) * 16
r = VRendererHIP(0)
scenes.load_into(r, sc)


def steps_time(tiling):
    r.set_tiling(*tiling)
    r.clearBuffer()
    for i in range(3):                                   # warm-up: scratch, sessions, code
        r.render(frames=F, times=[sc["time"] + i * F + k for k in range(F)], sync=False)
    r.sync()
    t0 = time.perf_counter()
    for i in range(STEPS):
        r.render(frames=F, times=[sc["time"] + (3 + i) * F + k for k in range(F)], sync=False)
    r.sync()
    return (time.perf_counter() - t0) / STEPS


def kernel_time(fn, reps=50):
    fn()
    r.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    r.sync()
    return (time.perf_counter() - t0) / reps


one_gpu = steps_time((0, 1))
stride = max_owned_pixels(W, H, N) * 4
buf = torch.empty(N * stride, dtype=torch.uint8, device="cuda:0")
ranks = []
for rank in range(N):
    t_step = steps_time((rank, N))
    t_pack = kernel_time(lambda: r.pack_tiles(WHAT_RGBA8, buf.data_ptr() + rank * stride))
    ranks.append({"rank": rank, "owned_pixels": r.owned_pixels(), "step_ms": round(t_step * 1e3, 4),
                  "pack_ms": round(t_pack * 1e3, 4)})
r.set_tiling(0, 1)
t_unpack = kernel_time(lambda: r.unpack_tiles(WHAT_RGBA8, buf.data_ptr(), N, stride))
gather_s = GATHER_LAT_US * 1e-6 + stride / (XGMI_GBS * 1e9)
slowest = max(x["step_ms"] + x["pack_ms"] for x in ranks) * 1e-3
proj_step = slowest + gather_s + t_unpack
paths = px * 2 * F
out = {"config": cfg, "ranks": N, "frames_per_step": F, "steps": STEPS,
       "one_gpu_step_ms": round(one_gpu * 1e3, 4), "one_gpu_mpaths": round(paths / one_gpu / 1e6, 1),
       "per_rank": ranks, "unpack_ms": round(t_unpack * 1e3, 4),
       "gather_model_ms": round(gather_s * 1e3, 4), "gather_payload_bytes_per_rank": stride,
       "projected_step_ms": round(proj_step * 1e3, 4), "projected_mpaths": round(paths / proj_step / 1e6, 1),
       "projected_efficiency": round((paths / proj_step) / (N * paths / one_gpu), 4),
       "efficiency_without_gather": round((paths / (slowest + t_unpack)) / (N * paths / one_gpu), 4),
       "note": f"each rank's 16-frame steps timed alone on one MI355X (the whole GPU per rank, as on an 8-GPU node); "
               f"gather modelled as {GATHER_LAT_US:.0f} us + payload / {XGMI_GBS:.0f} GB/s"}
print(json.dumps(out), flush=True)
r.cleanUp()
