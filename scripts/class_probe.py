#!/usr/bin/env python3
"""Rates of feature-class scenes (tests/test_gpu_classes.py class_scene) per
library: python scripts/class_probe.py lib1.so [lib2.so ...] -- each library
in its own process (VRHIP_LIB), 16 frames per launch, back-to-back steps."""
import os, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, time
sys.path.insert(0, {repo!r}); sys.path.insert(0, {tests!r}); sys.path.insert(0, {repo!r} + "/oracle")
from test_gpu_classes import class_scene
from vrenderer_pathtracer_amd import VRendererHIP, scenes
for name, w, h in {cases!r}:
    sc = class_scene(name, w, h)
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    F = 16
    r.render(frames=F, time_seed=sc["time"]); r.sync()
    best = 1e9
    for b in range(3):
        t0 = time.perf_counter()
        for i in range(6):
            r.render(frames=F, times=[sc["time"] + (b * 6 + i) * F + k for k in range(F)], sync=False)
        r.sync()
        best = min(best, (time.perf_counter() - t0) / 6)
    acc = r.read_accum()
    r.cleanUp()
    wr, hr = (w // 16) * 16, (h // 16) * 16
    print(f"{{name}} {{w}}x{{h}}: {{best * 1e3:.4f}} ms/step {{wr * hr * 2 * F / best / 1e6:10.1f}} Mpaths/s hash {{hash(acc.tobytes()) & 0xffffffff:#x}}", flush=True)
"""
cases = [("CB", 1280, 720), ("C1T", 1280, 720), ("C4D", 1920, 1080), ("C2D", 1280, 720), ("C3D", 1280, 720), ("C3B", 1280, 720)]
for lib in sys.argv[1:]:
    env = dict(os.environ, VRHIP_LIB=os.path.abspath(lib))
    print(f"== {lib}", flush=True)
    code = CHILD.format(repo=REPO, tests=os.path.join(REPO, "tests"), cases=cases)
    rc = subprocess.call([sys.executable, "-c", code], env=env)
    if rc != 0:
        sys.exit(rc)
