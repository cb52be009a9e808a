#!/usr/bin/env python3
"""Per-wave timeline of render_wave_kernel from a -DVR_WAVE_TIMES build.

  VRHIP_LIB=variants/libvrhip_wt.so python scripts/wave_times.py [C3] [frames] [N]

Renders rank 0's share of an N-way tile split, then prints when the waves
start and end relative to the first start (us, 100 MHz realtime clock), and
the spread of paths per wave: a long tail of late-ending waves means the
launch ends on a few long path chains; late starts mean dispatch ramp.
Diagnostic only.
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: F401,E402
from vrenderer_pathtracer_amd import VRendererHIP, scenes  # noqa: E402
from vrenderer_pathtracer_amd import _native  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
F = int(sys.argv[2]) if len(sys.argv) > 2 else 16
N = int(sys.argv[3]) if len(sys.argv) > 3 else 8
sc = scenes.make_scene(cfg)
r = VRendererHIP(0)
scenes.load_into(r, sc)
r.set_tiling(0, N)
lib = _native.lib()
NW = 8192
buf = (ctypes.c_uint64 * (3 * NW))()
for rep in range(3):
    r.render(frames=F, times=[sc["time"] + rep * F + k for k in range(F)])
    r.sync()
    lib.vrhip_debug_wave_times(r._ctx, buf, NW)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(NW, 3).astype(np.int64)
    a = a[a[:, 1] > 0]
    t0 = a[:, 0].min()
    st = (a[:, 0] - t0) / 100.0
    en = (a[:, 1] - t0) / 100.0
    pc = np.percentile
    print(f"{cfg} N={N} F={F} rep {rep}: waves {len(a)}  span {en.max():8.1f} us  "
          f"start p50/p99/max {pc(st, 50):6.1f}/{pc(st, 99):6.1f}/{st.max():6.1f}  "
          f"end p1/p10/p50/p90/max {pc(en, 1):7.1f}/{pc(en, 10):7.1f}/{pc(en, 50):7.1f}/{pc(en, 90):7.1f}/{en.max():7.1f}  "
          f"paths/wave p10/p50/p90 {pc(a[:, 2], 10):.0f}/{pc(a[:, 2], 50):.0f}/{pc(a[:, 2], 90):.0f}  total {a[:, 2].sum()}",
          flush=True)
r.cleanUp()
