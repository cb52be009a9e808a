#!/usr/bin/env python3
"""Phase breakdown of the render kernel from a -DVR_TIMING build.

  VRHIP_LIB=variants/libvrhip_timing.so python scripts/phase_timing.py [C2]

Prints the lane-weighted share of s_memtime cycles in each phase.  The
diagnostic build's run time is not a performance number (the stamps cost
cycles and serialise), only its shares are.
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
sc = scenes.make_scene(cfg)
r = VRendererHIP(0)
scenes.load_into(r, sc)
r.render(frames=8, time_seed=sc["time"])
out = (ctypes.c_uint64 * 16)()
_native.lib().vrhip_debug_counters(r._ctx, out, 1)
r.render(frames=8, times=[sc["time"] + k for k in range(8)])
_native.lib().vrhip_debug_counters(r._ctx, out, 0)
names = ["spheres", "mesh traversal", "hit materialise", "shading", "tonemap"]
total = out[13]
print(f"{cfg}: kernel lane-cycles {total:.3e}")
for i, n in enumerate(names):
    print(f"  {n:18s} {out[8 + i] / total * 100:6.1f} %")
print(f"  {'other':18s} {(total - sum(out[8 + i] for i in range(5))) / total * 100:6.1f} %")
r.cleanUp()
