#!/usr/bin/env python3
"""Per node visit: cycles from the fetch's issue to its data, and of the slab
/ push-pop compute after it, from a -DVR_NODE_STAMPS build (diagnostic; the
stamps serialise the loop, so only the split matters).

  VRHIP_LIB=variants/libvrhip_stamps.so python scripts/node_stamps.py [C2]
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: F401,E402
from vrenderer_pathtracer_amd import VRendererHIP, scenes, _native  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
sc = scenes.make_scene(cfg)
r = VRendererHIP(0)
scenes.load_into(r, sc)
r.render(frames=4, time_seed=sc["time"])
out = (ctypes.c_uint64 * 16)()
_native.lib().vrhip_debug_counters(r._ctx, out, 1)
r.render(frames=4, times=[sc["time"] + k for k in range(4)])
_native.lib().vrhip_debug_counters(r._ctx, out, 0)
steps = max(out[10], 1)
print(f"{cfg}: {steps:.3e} lane node visits; fetch wait {out[8] / steps:.0f} cycles, "
      f"compute + push/pop {out[9] / steps:.0f} cycles per visit")
r.cleanUp()
