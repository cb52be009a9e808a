#!/usr/bin/env python3
"""One frame per synchronous render() call (bench.py's interactive leg) per
library, each in its own process (VRHIP_LIB), and an accumulation hash:
  python scripts/inter_probe.py "C3 C5" lib1.so [lib2.so ...]"""
import os, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, time, zlib
sys.path.insert(0, {repo!r})
from vrenderer_pathtracer_amd import VRendererHIP, scenes
for cfg in {cfgs!r}:
    sc = scenes.make_scene(cfg)
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    base = sc["time"] + 100000
    for i in range(3):
        r.render(frames=1, times=[base + i], sync=True)
    r.sync()
    best = 1e9
    for b in range(3):
        r.clearBuffer()
        t0 = time.perf_counter()
        for i in range(30):
            r.render(frames=1, times=[base + 3 + i], sync=True)
            r.sync()
        best = min(best, (time.perf_counter() - t0) / 30)
    h = zlib.crc32(r.read_accum().tobytes())
    r.cleanUp()
    print(f"{{cfg}}: {{best * 1e3:.4f}} ms per frame  hash {{h:#010x}}", flush=True)
"""
cfgs = sys.argv[1].split()
for lib in sys.argv[2:]:
    print(f"== {lib}", flush=True)
    rc = subprocess.call([sys.executable, "-c", CHILD.format(repo=REPO, cfgs=cfgs)],
                         env=dict(os.environ, VRHIP_LIB=os.path.abspath(lib)))
    if rc != 0:
        sys.exit(rc)
