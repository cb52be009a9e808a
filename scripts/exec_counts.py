#!/usr/bin/env python3
"""Executed-work counts of the production kernels (vrhip_render_profiled) per
library variant: python scripts/exec_counts.py --cfg C2 lib1.so lib2.so ..."""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, json
sys.path.insert(0, {repo!r})
import torch
from vrenderer_pathtracer_amd import VRendererHIP, scenes
sc = scenes.make_scene({cfg!r})
r = VRendererHIP(0)
scenes.load_into(r, sc)
e = r.render_profiled(frames={frames}, time_seed=sc["time"])
wr, hr = (sc["width"] // 16) * 16, (sc["height"] // 16) * 16
paths = wr * hr * 2 * {frames}
print(json.dumps({{k: round(v / paths, 3) for k, v in e.items()}}))
"""

ap = argparse.ArgumentParser()
ap.add_argument("--cfg", default="C2")
ap.add_argument("--frames", type=int, default=4)
ap.add_argument("libs", nargs="+")
a = ap.parse_args()
for lib in a.libs:
    env = dict(os.environ, VRHIP_LIB=os.path.abspath(lib))
    p = subprocess.run([sys.executable, "-c", CHILD.format(repo=REPO, cfg=a.cfg, frames=a.frames)], env=env,
                       capture_output=True, text=True, timeout=600)
    if p.returncode != 0:
        print(lib, "FAILED", p.stderr[-1500:]); sys.exit(1)
    print(f"{os.path.basename(lib)} per path: {p.stdout.strip().splitlines()[-1]}", flush=True)
