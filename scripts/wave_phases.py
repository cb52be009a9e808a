#!/usr/bin/env python3
"""Per-wave phase cycles of render_wave_kernel from a -DVR_WAVE_TIMES
-DVR_WAVE_PHASES build: where the launch's slowest waves spend their time.

  VRHIP_LIB=variants/libvrhip_ph.so python scripts/wave_phases.py [C2] [frames] [width height]

Prints, for the 1 % of waves that end last and for all waves, the mean
wave duration and its split into loop phases (top: age priority, camera ray,
sphere tests; trav: the mesh loop less help rounds; help; shade; refill),
the loop iterations, trav_iter calls, shading / setup rounds, and the
node-loop and leaf-pair rounds of the wave's busiest lane -- hence the
cycles per node-loop round on a launch's critical path.  Diagnostic only.
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
sc = scenes.make_scene(cfg, int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else scenes.make_scene(cfg)
r = VRendererHIP(0)
scenes.load_into(r, sc)
lib = _native.lib()
NW = 8192
wt = (ctypes.c_uint64 * (3 * NW))()
ph = (ctypes.c_uint64 * (12 * NW))()
for rep in range(3):
    r.render(frames=F, times=[sc["time"] + rep * F + k for k in range(F)])
    r.sync()
    assert lib.vrhip_debug_wave_times(r._ctx, wt, NW) == 0
    assert lib.vrhip_debug_wave_phases(r._ctx, ph, NW) == 0
    w = np.frombuffer(wt, dtype=np.uint64).reshape(NW, 3)
    q = np.frombuffer(ph, dtype=np.uint64)[:8 * NW].reshape(NW, 8)
    rr = np.frombuffer(ph, dtype=np.uint64)[8 * NW:].reshape(NW, 4).astype(np.float64)
    keep = w[:, 1] > 0
    w, q, rr = w[keep].astype(np.int64), q[keep], rr[keep]
    t0 = w[:, 0].min()
    st, en = (w[:, 0] - t0) / 100.0, (w[:, 1] - t0) / 100.0      # us
    cyc = (q[:, :5]).astype(np.float64)
    wcyc = (np.frombuffer(wt, dtype=np.uint64).reshape(NW, 3)[keep, 2] >> np.uint64(32)).astype(np.float64)
    dur = en - st
    clk = np.median(wcyc / np.maximum(dur, 1e-3)) / 1e3             # GHz: shader cycles per us / 1000
    it = (q[:, 5] & np.uint64(0xffffffff)).astype(np.int64)
    tc = (q[:, 5] >> np.uint64(32)).astype(np.int64)
    ns = (q[:, 6] & np.uint64(0xffffffff)).astype(np.int64)
    npr = (q[:, 6] >> np.uint64(32)).astype(np.int64)
    shd = (q[:, 7] & np.uint64(0xffffffff)).astype(np.int64)
    sup = (q[:, 7] >> np.uint64(32)).astype(np.int64)
    print(f"{cfg} {sc['width']}x{sc['height']} F={F} rep {rep}: waves {keep.sum()} span {en.max():.1f} us  clock {clk:.2f} GHz")
    late = en >= np.percentile(en, 99)
    for lab, m in (("last-ending 1 %", late), ("all", np.ones_like(late))):
        c = cyc[m].mean(0) / clk / 1e3
        print(f"  {lab:16s} n {m.sum():5d} dur {dur[m].mean():7.1f} us = top {c[0]:6.1f} + trav {c[1]:6.1f} + help {c[2]:5.1f}"
              f" + shade {c[3]:6.1f} + refill {c[4]:5.1f}  | iters {it[m].mean():6.1f} trav_iter calls {tc[m].mean():6.1f}"
              f" shade rounds {shd[m].mean():5.1f} setup rounds {sup[m].mean():5.1f}  max-lane node rounds {ns[m].mean():6.1f}"
              f" leaf pairs {npr[m].mean():5.1f}")
        print(f"  {'':16s} per shade round {cyc[m, 3].sum() / max(shd[m].sum(), 1):7.0f} cyc, per top {cyc[m, 0].sum() / max(it[m].sum(), 1):6.0f} cyc,"
              f" per trav_iter call {cyc[m, 1].sum() / max(tc[m].sum(), 1):6.0f} cyc, per (node round + leaf pair)"
              f" {cyc[m, 1].sum() / max(ns[m].sum() + npr[m].sum(), 1):6.0f} cyc")
        print(f"  {'':16s} wave node rounds {rr[m, 0].mean():7.1f} at {rr[m, 2].sum() / max(rr[m, 0].sum(), 1):6.0f} cyc,"
              f" leaf rounds {rr[m, 1].mean():6.1f} at {rr[m, 3].sum() / max(rr[m, 1].sum(), 1):6.0f} cyc"
              f" (node loops {rr[m, 2].mean() / clk / 1e3:6.1f} us + leaf loops {rr[m, 3].mean() / clk / 1e3:6.1f} us)")
r.cleanUp()
