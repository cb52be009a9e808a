#!/usr/bin/env python3
"""Mesh upload cost of a scene: host+device time of vrhip_upload_mesh_flat
(initMesh) and the device bytes it leaves allocated.

  [VRHIP_LIB=variants/libvrhip_X.so] python scripts/upload_cost.py [C5] [reps]

Prints one JSON line: upload seconds (median of reps, each into a fresh
context), device bytes (free-memory drop across the upload), triangles and
nodes.  Used to compare libraries (e.g. before / after a layout change).
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
from vrenderer_pathtracer_amd import VRendererHIP, scenes  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
sc = scenes.make_scene(cfg)
ts, dbytes = [], []
for _ in range(reps):
    r = VRendererHIP(0)
    r.init(64, 64)
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info(0)
    t0 = time.perf_counter()
    r.initMesh(sc["mesh_flat"])
    r.sync()
    ts.append(time.perf_counter() - t0)
    free1, _ = torch.cuda.mem_get_info(0)
    dbytes.append(free0 - free1)
    depth, nodes, slots = r.bvh_info()
    r.cleanUp()
ts.sort()
print(json.dumps({"config": cfg, "lib": os.path.basename(os.environ.get("VRHIP_LIB", "libvrhip.so")),
                  "upload_s": round(ts[len(ts) // 2], 4), "upload_s_all": [round(t, 4) for t in ts],
                  "device_bytes": int(sorted(dbytes)[len(dbytes) // 2]), "bvh_depth": depth, "bvh_nodes": nodes,
                  "slots": slots}), flush=True)
