#!/usr/bin/env python3
"""Host-side cost of one synchronous render call (the reference's cadence)
on a tiny image, where the GPU work is a few microseconds: the floor the host
adds to every interactive frame.  Times, per call (median of 200):
  python wrapper render(sync=True) end to end; vrhip_render alone (the C ABI
  host path: parameters, events, launches); vrhip_sync alone (wait + wake-up);
  the same through ctypes without the Python wrapper.

  python scripts/host_gap.py [C2] [16x16]
"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402,F401
from vrenderer_pathtracer_amd import VRendererHIP, scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
w, h = (int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "16x16").split("x"))
sc = scenes.make_scene(cfg, w, h)
r = VRendererHIP(0)
scenes.load_into(r, sc)
L, ctx = r._lib, r._ctx
for i in range(20):
    r.render(frames=1, times=[sc["time"] + i])


def med(f, n=200):
    ts = []
    for i in range(n):
        t0 = time.perf_counter()
        f(i)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e6


arr = (ctypes.c_uint32 * 1)(sc["time"])
print(f"{cfg} {w}x{h}: python render(sync=True)   {med(lambda i: r.render(frames=1, times=[sc['time'] + i])):7.1f} us")
print(f"{cfg} {w}x{h}: ctypes render + sync        {med(lambda i: (L.vrhip_render(ctx, 1, arr, 0), L.vrhip_sync(ctx))):7.1f} us")


def split(i):
    t0 = time.perf_counter()
    L.vrhip_render(ctx, 1, arr, 0)
    t1 = time.perf_counter()
    L.vrhip_sync(ctx)
    split.r.append(t1 - t0)
    split.s.append(time.perf_counter() - t1)


split.r, split.s = [], []
med(split)
split.r.sort(); split.s.sort()
print(f"{cfg} {w}x{h}: vrhip_render host path      {split.r[100] * 1e6:7.1f} us")
print(f"{cfg} {w}x{h}: vrhip_sync (wait + wake-up)  {split.s[100] * 1e6:7.1f} us")
print(f"{cfg} {w}x{h}: vrhip_sync on an idle stream {med(lambda i: L.vrhip_sync(ctx)):7.1f} us")
r.cleanUp()
