#!/usr/bin/env python3
"""A/B timing of libvrhip.so build variants on one GPU (each in its own process).

  python scripts/ab.py [--cfg C2] [--frames 8] [--steps 4] lib1.so lib2.so ...

Prints Mpaths/s per variant (median of 3 batches of back-to-back steps) and checks every variant's
accumulation buffer bit-equals the first one's (SHA-256 of the
float4 bytes; one-frame calls too with --interactive).
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, time, json, hashlib, numpy as np
sys.path.insert(0, {repo!r})
import torch
from vrenderer_pathtracer_amd import VRendererHIP, scenes
sc = scenes.make_scene({cfg!r})
r = VRendererHIP(0)
scenes.load_into(r, sc)
r.set_strict_traversal({strict})
if {overlap!r} != "": r.set_overlap(int({overlap!r}))
F = {frames}
r.render(frames=F, time_seed=sc["time"])     # warm-up
r.clearBuffer()
ts = []
for b in range(3):     # batches of back-to-back steps (as bench.py issues them), synced at the end
    t0 = time.perf_counter()
    for i in range({steps}):
        j = b * {steps} + i
        r.render(frames=F, times=[sc["time"] + j * F + k for k in range(F)], sync=False)
    r.sync()
    ts.append((time.perf_counter() - t0) / {steps})
acc = r.read_accum()
wr, hr = (sc["width"] // 16) * 16, (sc["height"] // 16) * 16
paths = wr * hr * 2 * F
ts.sort()
med = ts[len(ts) // 2]
inter = None
if {inter} > 0:      # one frame per synchronous call (the reference's render() cadence)
    r.clearBuffer()
    for i in range(3):
        r.render(frames=1, times=[sc["time"] + 50000 + i])
    ti = []
    for b in range(3):
        t0 = time.perf_counter()
        for i in range({inter}):
            r.render(frames=1, times=[sc["time"] + 60000 + b * 1000 + i])
        ti.append((time.perf_counter() - t0) / {inter})
    ti.sort()
    inter = ti[1] * 1e3
    iacc = r.read_accum()
    ihash = hashlib.sha256(iacc.tobytes()).hexdigest()
else:
    ihash = ""
print(json.dumps({{"mpaths": paths / med / 1e6, "best": paths / ts[0] / 1e6, "inter_ms": inter,
                   "hash": hashlib.sha256(acc.tobytes()).hexdigest(), "ihash": ihash}}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="C2")
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--strict", action="store_true")
    ap.add_argument("--leaf", type=int, default=None, help="max triangles per leaf of the scene's BVH")
    ap.add_argument("--node-cost", type=float, default=None, help="SAH node cost of the scene's BVH")
    ap.add_argument("--interactive", type=int, default=0, help="also time N one-frame synchronous calls (median of 3)")
    ap.add_argument("--overlap", default="", help="comma-separated vrhip_set_overlap modes to run per library (1, 0, -1)")
    ap.add_argument("libs", nargs="+", help="lib.so or lib.so@VAR=value,VAR2=value (environment of that run)")
    a = ap.parse_args()
    results = {}
    runs = [(lib, ov) for lib in a.libs for ov in (a.overlap.split(",") if a.overlap else [""])]
    for spec, ov in runs:
        lib, _, envs = spec.partition("@")
        env = dict(os.environ, VRHIP_LIB=os.path.abspath(lib))
        env.update(kv.split("=", 1) for kv in envs.split(",") if kv)
        if a.leaf:
            env["VRHIP_MAX_LEAF"] = str(a.leaf)
        if a.node_cost is not None:
            env["VRHIP_SAH_NODE_COST"] = str(a.node_cost)
        code = CHILD.format(repo=REPO, cfg=a.cfg, frames=a.frames, steps=a.steps, strict=a.strict, overlap=ov,
                            inter=a.interactive)
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            print(f"{lib}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
            if p.returncode < 0 or p.returncode > 1:
                sys.exit(p.returncode if p.returncode > 0 else 1)
            continue
        res = json.loads(p.stdout.strip().splitlines()[-1])
        name = os.path.basename(lib) + (f"@{envs}" if envs else "") + (f" overlap={ov}" if ov else "")
        results[name] = res
        it = f"  one frame/call {res['inter_ms']:.4f} ms" if res.get("inter_ms") else ""
        print(f"{name:40s} {res['mpaths']:9.1f} Mpaths/s (best {res['best']:.1f}){it}  sha256 {res['hash'][:16]}",
              flush=True)
    hashes = {(v["hash"], v.get("ihash", "")) for v in results.values()}
    print("all results identical" if len(hashes) == 1 else f"RESULTS DIFFER: {len(hashes)} distinct hashes")


if __name__ == "__main__":
    main()
