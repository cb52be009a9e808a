#!/usr/bin/env python3
"""SIMD utilisation of the render kernel from a -DVR_LANESTATS build.

  VRHIP_LIB=variants/libvrhip_lanes.so python scripts/lane_stats.py [C2] [split]

Prints, for the node loop, the triangle loop and the shading block, the mean
number of active lanes per wave iteration (out of 64) and the iteration
counts.  Diagnostic only: the build's run time is not a performance number.
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: F401,E402
from vrenderer_pathtracer_amd import VRendererHIP, scenes  # noqa: E402
from vrenderer_pathtracer_amd import _native  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
split = int(sys.argv[2]) if len(sys.argv) > 2 else 0
sc = scenes.make_scene(cfg)
r = VRendererHIP(0)
scenes.load_into(r, sc)
r.set_path_split(split)
r.render(frames=8, time_seed=sc["time"])
out = (ctypes.c_uint64 * 16)()
_native.lib().vrhip_debug_counters(r._ctx, out, 1)
r.render(frames=8, times=[sc["time"] + k for k in range(8)])
_native.lib().vrhip_debug_counters(r._ctx, out, 0)
for i, name in enumerate(("node loop", "triangle loop", "shading")):
    lanes, iters = out[8 + 2 * i], out[9 + 2 * i]
    print(f"{cfg} split={split} {name:14s}: {lanes / max(iters, 1):5.1f} active lanes/iteration "
          f"({iters:.3e} wave iterations)")
r.cleanUp()
