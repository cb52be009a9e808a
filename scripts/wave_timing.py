#!/usr/bin/env python3
"""Wave-time split of render_wave_kernel from a -DVR_TIMING build.

  VRHIP_LIB=variants/libvrhip_timing.so python scripts/wave_timing.py [C2]

Slots (s_memtime cycles summed over lanes): 0 ray setup (sphere tests,
traversal init), 1 traversal loop, 4 shading block, 5 whole kernel -- all
wave-level intervals, recorded by every lane; 2 and 3 are lane-level
(fill_hit, material sampling, active lanes only).  Diagnostic only.
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
total = out[13]
print(f"{cfg}: wave kernel lane-cycles {total:.3e}")
for slot, name in ((8, "ray setup"), (9, "traversal loop"), (12, "shading block"),
                   (10, "  fill_hit (active lanes)"), (11, "  material (active lanes)")):
    print(f"  {name:26s} {out[slot] / total * 100:6.1f} %")
rest = total - out[8] - out[9] - out[12]
print(f"  {'refill + loop control':26s} {rest / total * 100:6.1f} %")
r.cleanUp()
