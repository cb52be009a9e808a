#!/usr/bin/env python3
"""Per-path timeline of render_wave_kernel from a -DVR_WAVE_TIMES -DVR_PATH_TIMES build.

  VRHIP_LIB=variants/libvrhip_pt.so python scripts/path_times.py [C2] [frames] [width height]

Renders one launch of `frames` frames and prints, per kind of primary hit,
the path durations, node visits, triangle tests and outer traversal
iterations; when the launch's last path started; the paths still running
over the last part of the launch; and what the longest paths did (are they
expensive, or slow?).  Diagnostic only.
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
if len(sys.argv) > 4:      # a small image: the same paths on a nearly idle GPU (unloaded latency)
    sc = scenes.make_scene(cfg, int(sys.argv[3]), int(sys.argv[4]))
    cfg += f"@{sys.argv[3]}x{sys.argv[4]}"
else:
    sc = scenes.make_scene(cfg)
r = VRendererHIP(0)
scenes.load_into(r, sc)
lib = _native.lib()
npaths = r.owned_pixels() * 2 * F
assert npaths <= 4 * 1024 * 1024, "the diagnostic build records at most 4M paths (kPathTimesCap)"
NW = 8192
nrec = NW + (4 * npaths + 2) // 3   # in units of 3 u64: 3 per wave, then 4 per path
buf = (ctypes.c_uint64 * (3 * nrec))()
CLK = float(os.environ.get("PT_CLK_GHZ", "2.3"))   # effective shader clock (scripts/wave_times.py)
KINDS = {0: "none", 1: "cornell", 2: "small", 3: "example", 4: "mesh", 15: "inline"}
pc = np.percentile
for rep in range(2):
    r.render(frames=F, times=[sc["time"] + rep * F + k for k in range(F)])
    r.sync()
    assert lib.vrhip_debug_wave_times(r._ctx, buf, nrec) == 0
    a = np.frombuffer(buf, dtype=np.uint64)[3 * NW:3 * NW + 4 * npaths].reshape(npaths, 4)
    st = a[:, 0].astype(np.int64)
    en = (a[:, 1] & np.uint64((1 << 56) - 1)).astype(np.int64)
    kind = (a[:, 1] >> np.uint64(56)).astype(np.int64)
    m20 = np.uint64(0xfffff)
    nodes = (a[:, 2] & m20).astype(np.int64)
    tris = ((a[:, 2] >> np.uint64(20)) & m20).astype(np.int64)
    iters = ((a[:, 2] >> np.uint64(40)) & m20).astype(np.int64)
    m16 = np.uint64(0xffff)
    # phase cycles (x16): trav_iter, help_step, own shading, others' shading -> us at CLK
    ph = np.stack([((a[:, 3] >> np.uint64(16 * j)) & m16).astype(np.float64) * 16 / CLK / 1e3 for j in range(4)], 1)
    ok = st > 0
    t0 = st[ok].min()
    st = (st - t0) / 100.0
    en = (en - t0) / 100.0
    dur = en - st
    span = en[ok].max()
    print(f"{cfg} F={F} rep {rep}: paths {ok.sum()} span {span:.1f} us  last start {st[ok].max():.1f} us", flush=True)
    for k in sorted(set(kind[ok].tolist())):
        m = ok & (kind == k)
        print(f"  {KINDS.get(k, k):8s} n {m.sum():8d}  dur p50/p90/p99/max {pc(dur[m], 50):7.1f}/{pc(dur[m], 90):7.1f}/"
              f"{pc(dur[m], 99):7.1f}/{dur[m].max():7.1f}  nodes p50/p99 {pc(nodes[m], 50):.0f}/{pc(nodes[m], 99):.0f}"
              f"  tris p50/p99 {pc(tris[m], 50):.0f}/{pc(tris[m], 99):.0f}  iters p50/p99 {pc(iters[m], 50):.0f}/"
              f"{pc(iters[m], 99):.0f}", flush=True)
    # throughput over the launch: paths completed and in flight per 25-us bin
    edges = np.arange(0, span + 25, 25)
    done, _ = np.histogram(en[ok], edges)
    started, _ = np.histogram(st[ok], edges)
    inflight = np.cumsum(started) - np.cumsum(done)
    print("  t(us)  completed  started  in-flight(end of bin)")
    for i in range(len(done)):
        print(f"  {edges[i]:5.0f} {done[i]:9d} {started[i]:8d} {inflight[i]:9d}")
    # the paths that end last: what they did
    late = ok & (en > span - 100)
    for lab, m in (("ending in the last 100 us", late), ("all", ok)):
        if m.sum() == 0:
            continue
        print(f"  {lab}: n {m.sum()}  start p50 {pc(st[m], 50):.0f}  dur p50 {pc(dur[m], 50):.0f}  nodes p50 "
              f"{pc(nodes[m], 50):.0f}  tris p50 {pc(tris[m], 50):.0f}  iters p50 {pc(iters[m], 50):.0f}  "
              f"us/iter p50 {pc(dur[m] / np.maximum(iters[m], 1), 50):.1f}")
    top = np.argsort(-np.where(ok, dur, -1))[:10]
    print(f"  longest: start dur nodes tris iters kind | us in trav_iter help own-shade other-shade rest (at {CLK} GHz)")
    for i in top:
        rest = dur[i] - ph[i].sum()
        print(f"    {st[i]:6.0f} {dur[i]:6.0f} {nodes[i]:5d} {tris[i]:5d} {iters[i]:4d} {KINDS.get(int(kind[i]), kind[i]):8s}"
              f" | {ph[i, 0]:6.1f} {ph[i, 1]:6.1f} {ph[i, 2]:6.1f} {ph[i, 3]:6.1f} {rest:6.1f}")
    for lab, m in (("ending in the last 100 us", late), ("all", ok)):
        if m.sum():
            mp = ph[m].mean(0)
            print(f"  phases, mean over {lab}: dur {dur[m].mean():.1f} us = trav_iter {mp[0]:.1f} + help {mp[1]:.1f} + "
                  f"own shade {mp[2]:.1f} + other shade {mp[3]:.1f} + rest {dur[m].mean() - mp.sum():.1f}")
    # correlation of duration with work
    w = nodes[ok] + 2 * tris[ok]
    print(f"  corr(dur, nodes+2*tris) {np.corrcoef(dur[ok], w)[0, 1]:.3f}  corr(dur, iters) "
          f"{np.corrcoef(dur[ok], iters[ok])[0, 1]:.3f}", flush=True)
r.cleanUp()
