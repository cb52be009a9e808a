"""Multi-rank tile sharding on CPU: torch.distributed over gloo, world_size 2
and 3.  Each rank renders only its 16x16 tiles, dealt round-robin (tile t
belongs to rank t % N; the oracle on CPU stands in for the per-GPU kernel),
the packed tiles are gathered to rank 0 with one collective per step as
bench.py / tiles.TileGather do (over RCCL on GPUs, through the library's
vrhip_comm_gather), and rank 0's reassembled image must equal the
single-process render bit for bit (seeds depend only on global pixel
coordinates, PathTracer.cu:817-818).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import pyoracle as po
    from vrenderer_pathtracer_amd import scenes
    from vrenderer_pathtracer_amd.tiles import max_owned_pixels, owned_pixels, pack_host, unpack_host
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = scenes.make_scene("C2", 64, 112)
    W, H = sc["width"], sc["height"]
    accum = np.zeros((H, W, 4), np.float32)
    pix = owned_pixels(W, H, rank, world)
    bands = sorted(set((pix // W // 16).tolist()))   # the oracle renders whole rows: the bands holding our tiles
    cap = max_owned_pixels(W, H, world)
    for step in range(2):                       # two accumulation steps of 2 frames
        for f in range(2):
            frame = 1 + 2 * step + f
            for b in bands:
                po.render(sc, frames=1, times=[12345 + frame], first_frame=frame, rows=(16 * b, 16 * b + 16),
                          accum=accum)
        send = torch.zeros((cap, 4), dtype=torch.float32)
        send[:len(pix)] = torch.from_numpy(pack_host(accum, rank, world))
        gather = [torch.zeros_like(send) for _ in range(world)] if rank == 0 else None
        dist.gather(send, gather, dst=0)
    if rank == 0:
        full = np.zeros_like(accum)
        unpack_host([g.numpy() for g in gather], full)
        np.save(out_path, full)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_tile_sharded_render_equals_single_process(oracle, world):
    import pyoracle as po
    from vrenderer_pathtracer_amd import scenes
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "full.npy")
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        got = np.load(out)
    sc = scenes.make_scene("C2", 64, 112)
    ref, _, _, _ = po.render(sc, frames=4, times=[12345 + f for f in range(1, 5)])
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2` with no external launcher starts two ranks
    (torch.distributed.run as a child process) that form one process group;
    --check-launch stops before any GPU work, so this runs on CPU."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    res = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--check-launch"],
                         cwd=repo, env=env, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["gpus_arg"] == 2
