#!/usr/bin/env python3
"""Sphere-only scenes: path groups per pixel (vrhip_set_path_split) against
the step time.  split 1 accumulates in registers (no scratch, no finish
pass); larger splits store per-path results and sum them in the finish pass.

  python scripts/split_sweep.py [C4] [frames] [splits, e.g. 1,2,4,8,0]
"""
import hashlib
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from vrenderer_pathtracer_amd import VRendererHIP, scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
F = int(sys.argv[2]) if len(sys.argv) > 2 else 16
splits = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 2, 4, 8, 0]
sc = scenes.make_scene(cfg)
r = VRendererHIP(0)
scenes.load_into(r, sc)
W, H = sc["width"], sc["height"]
paths = (W // 16) * 16 * (H // 16) * 16 * 2 * F
ref = None
for sp in splits:
    r.set_path_split(sp)
    r.clearBuffer()
    r.render(frames=F, times=[sc["time"] + k for k in range(F)])
    acc = r.read_accum()
    h = hashlib.sha256(acc.tobytes()).hexdigest()
    ref = h if ref is None else ref
    for i in range(2):
        r.render(frames=F, times=[sc["time"] + (1 + i) * F + k for k in range(F)], sync=False)
    r.sync()
    r.kernel_stats(reset=True)
    steps = 20
    t0 = time.perf_counter()
    for i in range(steps):
        r.render(frames=F, times=[sc["time"] + (3 + i) * F + k for k in range(F)], sync=False)
    r.sync()
    dt = (time.perf_counter() - t0) / steps
    kms, n = r.kernel_stats()
    r.clearBuffer()
    ti = time.perf_counter()
    for i in range(20):
        r.render(frames=1, times=[sc["time"] + 9000 + i], sync=True)
    tf = (time.perf_counter() - ti) / 20
    print(f"{cfg} F={F} split={sp}: step {dt * 1e3:7.3f} ms  render kernel {kms / max(n, 1):7.3f} ms/launch  "
          f"{paths / dt / 1e6:9.1f} Mpaths/s  one frame/call {tf * 1e3:6.3f} ms  hash {'same' if h == ref else 'DIFFERENT'}",
          flush=True)
r.cleanUp()
