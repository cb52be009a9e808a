#!/usr/bin/env python3
"""Pixels that differ between traversal modes / builds on a full frame.

  python scripts/compare_modes.py C5 [frames] lib_a.so [lib_b.so ...]

For each library: renders the scene with the default (t-culled) traversal
and, for the first library, also with strict traversal (the reference's
visit order); prints how many pixels of the accumulation differ between
every culled render and the strict one.
"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, numpy as np
sys.path.insert(0, {repo!r})
import torch
from vrenderer_pathtracer_amd import VRendererHIP, scenes
sc = scenes.make_scene({cfg!r})
r = VRendererHIP(0)
scenes.load_into(r, sc)
r.set_strict_traversal({strict})
r.render(frames={frames}, times=[sc["time"] + k for k in range({frames})])
np.save({out!r}, r.read_accum())
"""


def render(lib, cfg, frames, strict, out):
    env = dict(os.environ, VRHIP_LIB=os.path.abspath(lib))
    subprocess.run([sys.executable, "-c", CHILD.format(repo=REPO, cfg=cfg, frames=frames, strict=strict, out=out)],
                   env=env, check=True, timeout=600)
    return np.load(out)


def main():
    cfg, frames, libs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    tmp = os.path.join(REPO, "gpurun_out", "cmp_{}.npy")
    ref = render(libs[0], cfg, frames, True, tmp.format("strict"))
    npx = ref.shape[0] * ref.shape[1]
    for i, lib in enumerate(libs):
        got = render(lib, cfg, frames, False, tmp.format(i))
        diff = (got.view(np.uint32) != ref.view(np.uint32)).any(-1)
        d = np.abs(got - ref).max(-1)
        print(f"{cfg} {os.path.basename(lib)} culled vs strict: {int(diff.sum())} of {npx} pixels differ "
              f"({diff.sum() / npx:.2e}); max |delta| {float(d.max()):.3g}", flush=True)


if __name__ == "__main__":
    main()
