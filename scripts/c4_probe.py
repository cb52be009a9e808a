#!/usr/bin/env python3
"""C4 time breakdown on one GPU: the production launch at path splits 1..8,
and the same HDRI scene without the example sphere (every pixel escapes at
its camera ray), 16 frames per launch, back-to-back steps (ab.py timing)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vrenderer_pathtracer_amd import VRendererHIP, scenes

def timed(sc, split=None, F=16, steps=8):
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    if split is not None:
        r.set_path_split(split)
    r.render(frames=F, time_seed=sc["time"])
    r.sync()
    best = 1e9
    for b in range(3):
        t0 = time.perf_counter()
        for i in range(steps):
            r.render(frames=F, times=[sc["time"] + (b * steps + i) * F + k for k in range(F)], sync=False)
        r.sync()
        best = min(best, (time.perf_counter() - t0) / steps)
    r.cleanUp()
    wr, hr = (sc["width"] // 16) * 16, (sc["height"] // 16) * 16
    return best * 1e3, wr * hr * 2 * F / best / 1e6

sc = scenes.make_scene("C4")
for split in (None, 1, 2, 4, 8, 16):
    ms, rate = timed(sc, split)
    print(f"C4 split {split}: {ms:.4f} ms/step  {rate:10.1f} Mpaths/s", flush=True)
no = dict(sc); no.update(example_sphere=False, view_brdf=False, brdf=None)
for split in (None, 1, 2, 4):
    ms, rate = timed(no, split)
    print(f"C4 without the sphere (all pixels escape), split {split}: {ms:.4f} ms/step  {rate:10.1f} Mpaths/s", flush=True)
