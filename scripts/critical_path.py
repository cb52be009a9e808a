#!/usr/bin/env python3
"""Launch time of one-frame render calls against the image size, production
library: at small sizes the GPU is nearly idle and the launch time is the
critical path of the launch's longest path chains (no load on the memory
pipeline); at full size it is throughput plus drain.

  [VRHIP_LIB=...] python scripts/critical_path.py [C2,C3] [sizes e.g. 160x96,640x360,1280x720]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402,F401
from vrenderer_pathtracer_amd import VRendererHIP, scenes  # noqa: E402

cfgs = (sys.argv[1] if len(sys.argv) > 1 else "C2,C3").split(",")
sizes = [tuple(int(v) for v in s.split("x")) for s in
         (sys.argv[2] if len(sys.argv) > 2 else "160x96,320x192,640x368,1280x720").split(",")]
for cfg in cfgs:
    base = scenes.make_scene(cfg)
    for (w, h) in sizes:
        sc = dict(base, width=w, height=h)
        r = VRendererHIP(0)
        scenes.load_into(r, sc)
        for i in range(5):
            r.render(frames=1, times=[sc["time"] + i])
        r.kernel_stats(reset=True)
        n = 30
        t0 = time.perf_counter()
        for i in range(n):
            r.render(frames=1, times=[sc["time"] + 100 + i])
        wall = (time.perf_counter() - t0) / n
        kms, launches = r.kernel_stats()
        paths = (w // 16) * 16 * (h // 16) * 16 * 2
        print(f"{cfg} {w}x{h}: paths {paths:8d}  kernel {kms / launches * 1e3:8.1f} us/launch  call {wall * 1e6:8.1f} us",
              flush=True)
        r.cleanUp()
