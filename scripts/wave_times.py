#!/usr/bin/env python3
"""Per-wave timeline of render_wave_kernel from a -DVR_WAVE_TIMES build.

  VRHIP_LIB=variants/libvrhip_pt.so python scripts/wave_times.py [C3] [frames] [N] [width height]

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
sc = scenes.make_scene(cfg, int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else scenes.make_scene(cfg)
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
    raw = np.frombuffer(buf, dtype=np.uint64).reshape(NW, 3)
    a = raw.astype(np.int64)
    keep = a[:, 1] > 0
    a = a[keep]
    w2 = raw[keep, 2]
    paths = (w2 & np.uint64(0xffff)).astype(np.int64)
    steals = ((w2 >> np.uint64(16)) & np.uint64(0xffff)).astype(np.int64)
    cycles = (w2 >> np.uint64(32)).astype(np.int64)
    t0 = a[:, 0].min()
    st = (a[:, 0] - t0) / 100.0
    en = (a[:, 1] - t0) / 100.0
    pc = np.percentile
    print(f"{cfg} N={N} F={F} rep {rep}: waves {len(a)}  span {en.max():8.1f} us  "
          f"start p50/p99/max {pc(st, 50):6.1f}/{pc(st, 99):6.1f}/{st.max():6.1f}  "
          f"end p1/p10/p50/p90/max {pc(en, 1):7.1f}/{pc(en, 10):7.1f}/{pc(en, 50):7.1f}/{pc(en, 90):7.1f}/{en.max():7.1f}  "
          f"paths/wave p10/p50/p90 {pc(paths, 10):.0f}/{pc(paths, 50):.0f}/{pc(paths, 90):.0f}  total {paths.sum()}  "
          f"subtrees handed to helpers {steals.sum()}", flush=True)
    dur = (a[:, 1] - a[:, 0]) / 100.0            # us
    long_ = dur > pc(dur, 90)
    print(f"    effective shader clock of the longest 10 % of waves: {np.median(cycles[long_] / dur[long_]):.0f} MHz "
          f"(all waves {np.median(cycles / np.maximum(dur, 1e-3)):.0f} MHz)", flush=True)
r.cleanUp()
