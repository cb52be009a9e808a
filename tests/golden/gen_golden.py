#!/usr/bin/env python3
"""Generate tests/golden/golden_images.npz: small oracle renders of the
BASELINE scene families (procedural stand-ins), used to pin the
oracle against regressions and to check the GPU path against stored data.

  python tests/golden/gen_golden.py

Each entry: <cfg>_accum_glibc / <cfg>_accum_portable (float32 HxWx4, the
io_colors buffer after N frames), <cfg>_rgba_portable (uint8), and the
parameters in <cfg>_meta (json).
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

CASES = [("C1", 64, 64, 3), ("C2", 80, 48, 2), ("C3", 80, 48, 2), ("C4", 96, 64, 2)]


def times_for(frames):
    return [12345 + 101 * i for i in range(frames)]


def main():
    import pyoracle as po
    from vrenderer_pathtracer_amd import scenes
    po.build()
    out = {}
    for cfg, w, h, frames in CASES:
        sc = scenes.make_scene(cfg, w, h)
        t = times_for(frames)
        ag, _, _, _ = po.render(sc, frames=frames, times=t, libm=po.LIBM_GLIBC)
        ap, rp, dp, _ = po.render(sc, frames=frames, times=t, libm=po.LIBM_PORTABLE)
        out[f"{cfg}_accum_glibc"] = ag
        out[f"{cfg}_accum_portable"] = ap
        out[f"{cfg}_rgba_portable"] = rp
        out[f"{cfg}_depth_portable"] = dp
        out[f"{cfg}_meta"] = np.frombuffer(json.dumps(dict(cfg=cfg, width=w, height=h, frames=frames,
                                                           times=t)).encode(), np.uint8)
    path = os.path.join(HERE, "golden_images.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
