#!/usr/bin/env python3
"""Per-path timeline of render_wave_kernel from a -DVR_WAVE_TIMES -DVR_PATH_TIMES build.

  VRHIP_LIB=variants/libvrhip_pt.so python scripts/path_times.py [C2] [frames]

Renders one launch of `frames` frames and prints the path durations by the
kind of the primary hit (from the primary records: build with
-DVR_INLINE_PRIM_PATHS=0), when the launch's last paths started, and how
much of the launch's drain the paths of each kind account for.  Diagnostic only.
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

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
F = int(sys.argv[2]) if len(sys.argv) > 2 else 1
sc = scenes.make_scene(cfg)
r = VRendererHIP(0)
scenes.load_into(r, sc)
lib = _native.lib()
npaths = r.owned_pixels() * 2 * F
assert npaths <= 4 * 1024 * 1024, "the diagnostic build records at most 4M paths (kPathTimesCap)"
NW = 8192
nrec = (3 * NW + 2 * npaths + 2) // 3
buf = (ctypes.c_uint64 * (3 * nrec))()
KINDS = {0: "none", 1: "cornell", 2: "small", 3: "example", 4: "mesh", 15: "inline"}
for rep in range(2):
    r.render(frames=F, times=[sc["time"] + rep * F + k for k in range(F)])
    r.sync()
    assert lib.vrhip_debug_wave_times(r._ctx, buf, nrec) == 0
    a = np.frombuffer(buf, dtype=np.uint64)[3 * NW:3 * NW + 2 * npaths].reshape(npaths, 2)
    st = a[:, 0].astype(np.int64)
    en = (a[:, 1] & np.uint64((1 << 56) - 1)).astype(np.int64)
    kind = (a[:, 1] >> np.uint64(56)).astype(np.int64)
    ok = st > 0
    t0 = st[ok].min()
    st = (st - t0) / 100.0
    en = (en - t0) / 100.0
    dur = en - st
    pc = np.percentile
    span = en[ok].max()
    print(f"{cfg} F={F} rep {rep}: paths {ok.sum()} span {span:.1f} us  last start {st[ok].max():.1f} us", flush=True)
    for k in sorted(set(kind[ok].tolist())):
        m = ok & (kind == k)
        print(f"  {KINDS.get(k, k):8s} n {m.sum():8d}  dur p50/p90/p99/max {pc(dur[m], 50):7.1f}/{pc(dur[m], 90):7.1f}/"
              f"{pc(dur[m], 99):7.1f}/{dur[m].max():7.1f}  ending after {span - 100:.0f} us: {(m & (en > span - 100)).sum()}",
              flush=True)
r.cleanUp()
