"""Multi-rank path on one GPU: two ranks (processes) share cuda:0 and talk
over gloo, standing in for one rank per GPU over RCCL.  Covers the device
pack/unpack kernels and tiles.TileGather end to end, and a bench.py run with
--gpus 2 through torch.distributed.run.
"""
import json
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, backend="gloo"):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from vrenderer_pathtracer_amd import VRendererHIP, scenes
    from vrenderer_pathtracer_amd.tiles import WHAT_ACCUM, WHAT_RGBA8, TileGather
    gpu = rank if backend == "nccl" else 0          # RCCL: one rank per GPU
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(gpu)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = scenes.make_scene("C2", 160, 112)
    r = VRendererHIP(gpu)
    scenes.load_into(r, sc)
    r.set_tiling(rank, world)
    g_rgba = TileGather(r, rank, world, dev, WHAT_RGBA8)
    g_acc = TileGather(r, rank, world, dev, WHAT_ACCUM)
    for step in range(2):
        r.render(frames=2, times=[sc["time"] + 2 * step + k for k in range(2)])
        g_rgba.step()
        g_acc.step()
    if rank == 0:
        r.sync()
        np.save(os.path.join(out_dir, "accum.npy"), r.read_accum())
        np.save(os.path.join(out_dir, "rgba.npy"), r.read_rgba8())
    r.cleanUp()
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_tile_gather_equals_single_rank(native):
    """The measured configuration: one rank per GPU, the tile gather through the
    library's own RCCL communicator (vrhip_comm_init / vrhip_comm_gather:
    pack, ncclGather over xGMI, unpack on rank 0).  Rank 0's image must equal
    the single-GPU render bit for bit.  Needs two GPUs (RCCL refuses two ranks
    on one device); the one-GPU boxes run the gloo rehearsal below instead."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs 2 GPUs: RCCL refuses two ranks on one device")
    from vrenderer_pathtracer_amd import VRendererHIP, scenes
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(2, _free_port(), td, "nccl"), nprocs=2, join=True)
        acc = np.load(os.path.join(td, "accum.npy"))
        rgba = np.load(os.path.join(td, "rgba.npy"))
    sc = scenes.make_scene("C2", 160, 112)
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    for step in range(2):
        r.render(frames=2, times=[sc["time"] + 2 * step + k for k in range(2)])
    ref_acc, ref_rgba = r.read_accum(), r.read_rgba8()
    r.cleanUp()
    assert np.array_equal(acc.view(np.uint32), ref_acc.view(np.uint32))
    assert np.array_equal(rgba, ref_rgba)


@pytest.mark.parametrize("world", [2, 3])
def test_tile_gather_equals_single_rank(native, world):
    from vrenderer_pathtracer_amd import VRendererHIP, scenes
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(world, _free_port(), td), nprocs=world, join=True)
        acc = np.load(os.path.join(td, "accum.npy"))
        rgba = np.load(os.path.join(td, "rgba.npy"))
    sc = scenes.make_scene("C2", 160, 112)
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    for step in range(2):
        r.render(frames=2, times=[sc["time"] + 2 * step + k for k in range(2)])
    ref_acc, ref_rgba = r.read_accum(), r.read_rgba8()
    r.cleanUp()
    assert np.array_equal(acc.view(np.uint32), ref_acc.view(np.uint32))
    assert np.array_equal(rgba, ref_rgba)


def test_bench_two_ranks_gloo_rehearsal(native):
    """`python bench.py --gpus 2` with no external launcher: bench.py starts
    the two ranks itself (they share cuda:0 over gloo here)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(VRHIP_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--frames-per-step", "2", "--no-cpu", "--no-roof", "--interactive-frames", "2", "--strong-steps", "2"]
    res = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["scaling"] == "strong"
    assert out["config"]["parallelism"] == "tile2" and out["interactive"]["frames_per_step"] == 1
    # rays: reference-equivalent and traced, side by side (the camera ray is traced once per pixel per launch)
    assert out["mrays_per_s"] > 0 and 0 < out["mrays_per_s_traced"] <= out["mrays_per_s"]
    assert 0 < out["rays_per_path_traced"] <= out["rays_per_path"]
    # the fixed-cadence view: 16 frames per step for this N, against a 1-GPU rate measured in the same run
    st = out["strong"]
    assert st["frames_per_step"] == 16 and st["value"] > 0 and st["one_gpu_value"] > 0
    assert abs(st["efficiency"] - st["value"] / (2 * st["one_gpu_value"])) < 1e-3
    # the samples-weak view (16 x N frames per step) as a secondary field
    sw = out["samples_weak"]
    assert sw["frames_per_step"] == 32 and sw["value"] > 0
    assert abs(sw["efficiency"] - sw["value"] / (2 * st["one_gpu_value"])) < 1e-3
    # kernel time is the union of overlapping launch spans: never more than the step
    assert out["roofline"]["avg_launch_ms"] <= out["ms_per_step"] * 1.001


def _single(sc, frames, times):
    from vrenderer_pathtracer_amd import VRendererHIP, scenes
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    r.render(frames=frames, times=times)
    out = r.read_accum(), r.read_rgba8(), r.read_depth8()
    r.cleanUp()
    return out


def _multi(sc, devices, calls, t0, service=None, sync=True):
    from vrenderer_pathtracer_amd import VRendererHIP, scenes
    r = VRendererHIP(list(devices))
    scenes.load_into(r, sc)
    if service is not None:
        r.set_service(service)
    assert r.device_group() == list(devices)
    t = t0
    kinds = []
    for n in calls:
        r.render(frames=n, times=[t + k for k in range(n)], sync=sync)
        kinds.append(r.last_launch_info()["kind"])
        t += n
    out = r.read_accum(), r.read_rgba8(), r.read_depth8(), r.getFrameCount()
    r.cleanUp()
    if service is not None:
        return out, kinds
    return out


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_multi_context_one_device_bitexact(native, oracle, cfg):
    """vrhip_create_multi with one device runs the multi-GPU code (fan-out of
    every setting and upload, per-device render, grouped RCCL gathers of
    RGBA8 / depth / accum to the lead over a one-rank communicator): equal to
    the plain context and to the oracle bit for bit."""
    import pyoracle as po
    from vrenderer_pathtracer_amd import scenes
    sc = scenes.make_scene(cfg, 96, 64)
    t = sc["time"]
    ga, gr, gd, nf = _multi(sc, [0], [2, 1], t)
    assert nf == 3
    sa, sr, sd = _single(sc, 3, [t, t + 1, t + 2])
    assert np.array_equal(ga.view(np.uint32), sa.view(np.uint32))
    assert np.array_equal(gr, sr) and np.array_equal(gd, sd)
    oa, orgba, _, _ = po.render(sc, frames=3, times=[t, t + 1, t + 2], libm=po.LIBM_PORTABLE)
    H, W = 64, 96
    assert np.array_equal(ga[:H, :W].view(np.uint32), oa[:H, :W].view(np.uint32))
    assert np.array_equal(gr[:H, :W], orgba[:H, :W])


def test_multi_context_refuses_per_rank_calls(native):
    """Tiling, streams, communicators and the service test hooks belong to
    the multi-device context itself: setting them on it is refused (the
    service mode fans out to the members)."""
    from vrenderer_pathtracer_amd import VRendererHIP, scenes
    from vrenderer_pathtracer_amd._native import VRHIPError
    sc = scenes.make_scene("C2", 64, 64)
    r = VRendererHIP([0])
    scenes.load_into(r, sc)
    for call in (lambda: r.set_tiling(0, 2), lambda: r.set_service_timing(1000, 0, 0),
                 lambda: r.set_service_budget(1 << 30)):
        with pytest.raises(VRHIPError):
            call()
    r.set_service(1)
    r.cleanUp()


@pytest.mark.parametrize("cfg,service", [("C2", 1), ("C3", -1)])
def test_multi_context_service_burst_bitexact(native, cfg, service):
    """A burst of unsynchronised render calls on a one-device multi context:
    the member renders on its render service (one session across the calls:
    the colour / depth gather waits for the read-back), and the lead's images
    equal the plain context's bit for bit."""
    from vrenderer_pathtracer_amd import scenes
    sc = scenes.make_scene(cfg, 160, 96) if cfg == "C2" else scenes.make_scene(cfg)
    t = sc["time"]
    calls = [2, 1, 3, 2, 4]
    (ga, gr, gd, nf), kinds = _multi(sc, [0], calls, t, service=service, sync=False)
    assert nf == sum(calls)
    assert "service" in kinds, kinds
    sa, sr, sd = _single(sc, sum(calls), [t + k for k in range(sum(calls))])
    assert np.array_equal(ga.view(np.uint32), sa.view(np.uint32))
    assert np.array_equal(gr, sr) and np.array_equal(gd, sd)


@pytest.mark.parametrize("cfg", ["C4", "C5"])
def test_eight_tile_ranks_full_size_reassemble_bitexact(native, cfg):
    """The driver's 8-GPU configurations rehearsed on one GPU at full size:
    C4 (1920x1080, MERL sphere) and C5 (3840x2160, 1M-triangle knot) rendered
    as 8 tile ranks (set_tiling(r, 8), r = 0..7, each from a cleared
    accumulation), every rank's RGBA8 / float4 accumulation / depth tiles
    packed on the device (vrhip_pack_tiles) into one rank-major gather buffer
    -- the layout ncclGather hands rank 0 -- then scattered back
    (vrhip_unpack_tiles): accum, RGBA8 and depth equal the single-context
    render of the whole image bit for bit."""
    import torch
    from vrenderer_pathtracer_amd import VRendererHIP, scenes
    from vrenderer_pathtracer_amd.tiles import WHAT_ACCUM, WHAT_DEPTH8, WHAT_RGBA8, max_owned_pixels
    sc = scenes.make_scene(cfg)
    W, H = sc["width"], sc["height"]
    n, frames = 8, 2
    times = [sc["time"] + 3, sc["time"] + 4]
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    r.render(frames=frames, times=times)
    ref = r.read_accum(), r.read_rgba8(), r.read_depth8()
    whats = (WHAT_RGBA8, WHAT_ACCUM, WHAT_DEPTH8)
    esz = {WHAT_RGBA8: 4, WHAT_ACCUM: 16, WHAT_DEPTH8: 4}
    stride = {w: max_owned_pixels(W, H, n) * esz[w] for w in whats}
    bufs = {w: torch.empty(n * stride[w], dtype=torch.uint8, device="cuda:0") for w in whats}
    owned = []
    for rank in range(n):
        r.set_tiling(rank, n)
        r.clearBuffer()
        r.render(frames=frames, times=times)
        owned.append(r.owned_pixels())
        for w in whats:
            r.pack_tiles(w, bufs[w].data_ptr() + rank * stride[w])
        r.sync()
    assert sum(owned) == (W // 16) * (H // 16) * 256
    r.set_tiling(0, 1)
    r.clearBuffer()                            # the gathering rank's images hold nothing of their own
    for w in whats:
        r.unpack_tiles(w, bufs[w].data_ptr(), n, stride[w])
    got = r.read_accum(), r.read_rgba8(), r.read_depth8()
    r.cleanUp()
    hr = (H // 16) * 16
    for g, e, what in zip(got, ref, ("accum", "rgba8", "depth8")):
        g, e = g[:hr], e[:hr]
        if g.dtype == np.float32:
            g, e = g.view(np.uint32), e.view(np.uint32)
        assert np.any(e != 0), what
        assert np.array_equal(g, e), f"{cfg} {what}: {int((g != e).any(-1).sum())} pixels differ"


def test_multi_context_two_devices_bitexact(native):
    """Two GPUs behind one context: each renders half the tiles, RCCL gathers
    them to the first; the images equal the one-GPU render bit for bit."""
    from vrenderer_pathtracer_amd import device_count
    if device_count() < 2:
        pytest.skip("needs 2 GPUs (one process drives both)")
    from vrenderer_pathtracer_amd import scenes
    sc = scenes.make_scene("C3", 160, 96)
    t = sc["time"]
    ga, gr, gd, _ = _multi(sc, [0, 1], [2, 2], t)
    sa, sr, sd = _single(sc, 4, [t + k for k in range(4)])
    assert np.array_equal(ga.view(np.uint32), sa.view(np.uint32))
    assert np.array_equal(gr, sr) and np.array_equal(gd, sd)
