"""Render service sessions (vrhip_set_service): consecutive render calls run
on ONE persistent kernel fed from a descriptor ring, their results summed in
path order by one finish pass when the session closes.  Bar: bit-identical
to launch-by-launch rendering (vrhip_set_service(0)) and to the oracle
(portable libm), whatever the session boundaries."""
import time

import numpy as np
import pytest

import pyoracle as po
from vrenderer_pathtracer_amd import VRendererHIP, scenes

pytestmark = pytest.mark.gpu


def _run(sc, calls, service, tiling=None, overlap=None, sleeps=None):
    """calls: list of frame counts per render call (async); returns accum,
    rgba, depth, frame count and the last launch's kind."""
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    r.set_service(service)
    if overlap is not None:
        r.set_overlap(overlap)
    if tiling:
        r.set_tiling(*tiling)
    t = sc["time"]
    kinds = []
    for i, n in enumerate(calls):
        r.render(frames=n, times=[t + k for k in range(n)], sync=False)
        kinds.append(r.last_launch_info()["kind"])
        t += n
        if sleeps and i in sleeps:
            time.sleep(sleeps[i])
    out = r.read_accum(), r.read_rgba8(), r.read_depth8(), r.getFrameCount()
    r.cleanUp()
    return out, kinds


def _eq(a, b, what):
    if a.dtype == np.float32:
        d = (a.view(np.uint32) != b.view(np.uint32)).any(-1)
    else:
        d = (a != b).any(-1)
    assert int(d.sum()) == 0, f"{what}: {int(d.sum())} pixels differ"


@pytest.mark.parametrize("cfg,w,h", [("C2", 96, 64), ("C3", 96, 64), ("C5", 96, 64)])
def test_service_session_equals_launch_by_launch_and_oracle(native, oracle, cfg, w, h):
    """Seven async calls of 1-4 frames in one session (the first opens it:
    service mode 1) equal the same calls without the service and the oracle's
    frame-by-frame loop, bit for bit (accum, RGBA8, depth)."""
    sc = scenes.make_scene(cfg, w, h)
    calls = [2, 1, 4, 1, 3, 2, 1]
    (a1, r1, d1, n1), k1 = _run(sc, calls, 1)
    (a0, r0, d0, n0), k0 = _run(sc, calls, 0)
    assert set(k1) == {"service"} and "service" not in k0
    assert n1 == n0 == sum(calls)
    _eq(a1, a0, "accum"); _eq(r1, r0, "rgba8"); _eq(d1, d0, "depth8")
    times = [sc["time"] + k for k in range(sum(calls))]
    oa, orgba, od, _ = po.render(sc, frames=sum(calls), times=times, libm=po.LIBM_PORTABLE)
    H, W = (h // 16) * 16, (w // 16) * 16
    _eq(a1[:H, :W], oa[:H, :W], "accum vs oracle")
    _eq(r1[:H, :W], orgba[:H, :W], "rgba8 vs oracle")
    _eq(d1[:H, :W], od[:H, :W], "depth8 vs oracle")


def test_service_session_limits(native, oracle):
    """Sessions close and reopen on their own: 140 one-frame calls (more than
    the 128 launch slots), a call of more frames than the session's slots hold
    (4 after 1-frame launches), a 70-frame call (two launches of 64 + 6).
    Bit-identical to launch-by-launch rendering."""
    sc = scenes.make_scene("C3", 64, 48)
    calls = [1] * 140 + [4, 1, 70, 2]
    (a1, r1, _, n1), _ = _run(sc, calls, 1)
    (a0, r0, _, n0), _ = _run(sc, calls, 0)
    assert n1 == n0 == sum(calls)
    _eq(a1, a0, "accum"); _eq(r1, r0, "rgba8")


def test_service_automatic_mode_and_tiling(native):
    """Automatic mode on a tiled rank: the first call of a burst runs as
    usual, the calls behind it (launch in flight) join a session; scene changes
    (Fresnel) and host pauses longer than the post window (5 ms) and than the
    kernel's idle limit (20 ms) start new sessions.  Bit-identical to
    launch-by-launch rendering."""
    sc = scenes.make_scene("C3")              # 1280x720: a 2-frame shard launch outlasts the host's next call
    calls = [2] * 6
    (a1, r1, d1, _), k1 = _run(sc, calls, -1, tiling=(1, 3), sleeps={2: 0.008, 4: 0.05})
    (a0, r0, d0, _), _ = _run(sc, calls, 0, tiling=(1, 3))
    assert "service" in k1, k1
    _eq(a1, a0, "accum"); _eq(r1, r0, "rgba8"); _eq(d1, d0, "depth8")

    def with_changes(service):
        r = VRendererHIP(0)
        scenes.load_into(r, sc)
        r.set_service(service)
        t = sc["time"]
        for i in range(3):
            r.render(frames=2, times=[t + 2 * i, t + 2 * i + 1], sync=False)
        r.setFresnelCoef(0.35)                 # another launch parameter: a new session
        for i in range(3, 6):
            r.render(frames=2, times=[t + 2 * i, t + 2 * i + 1], sync=False)
        r.set_tiling(0, 2)
        r.render(frames=1, times=[t + 12], sync=False)
        r.render(frames=1, times=[t + 13], sync=False)
        out = r.read_accum(), r.read_rgba8()
        r.cleanUp()
        return out
    (ca, cr), (ba, br) = with_changes(1), with_changes(0)
    _eq(ca, ba, "accum with scene changes"); _eq(cr, br, "rgba8 with scene changes")


def test_service_deferred_gather_single_rank(native):
    """vrhip_comm_gather inside a session (one-rank RCCL communicator,
    explicit service mode 1): the gathers are deferred to the session's close;
    the gathered image and the accumulation equal the launch-by-launch render.
    280 two-frame steps with a gather each: three sessions (128 launch slots
    each), so the next session's kernel runs while the previous session's
    deferred gathers are still queued (Session::summed)."""
    from vrenderer_pathtracer_amd.renderer import comm_unique_id
    from vrenderer_pathtracer_amd.tiles import WHAT_ACCUM, WHAT_RGBA8
    sc = scenes.make_scene("C2", 96, 64)

    def run(service):
        r = VRendererHIP(0)
        scenes.load_into(r, sc)
        r.set_service(service)
        r.comm_init(0, 1, comm_unique_id())
        t = sc["time"]
        for i in range(280):
            r.render(frames=2, times=[t + 2 * i, t + 2 * i + 1], sync=False)
            r.comm_gather(WHAT_RGBA8)
            if i % 50 == 3:
                r.comm_gather(WHAT_ACCUM)
        r.sync()
        out = r.read_accum(), r.read_rgba8(), r.read_depth8()
        info = r.service_info()
        r.comm_destroy()
        r.cleanUp()
        return out, info
    (got, gi), (base, _) = run(1), run(0)
    assert gi["sessions"] >= 3 and gi["deferred_gathers"] >= 280, gi
    for g, b, what in zip(got, base, ("accum", "rgba8", "depth8")):
        _eq(g, b, what)


def test_service_kernel_stats_count_every_launch(native):
    """The session's kernel span is accounted once for all its launches."""
    sc = scenes.make_scene("C2", 64, 64)
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    r.set_service(1)
    r.kernel_stats(reset=True)
    for i in range(5):
        r.render(frames=1, times=[sc["time"] + i], sync=False)
    ms, n = r.kernel_stats()
    r.cleanUp()
    assert n == 5 and ms > 0.0


@pytest.mark.parametrize("cfg,calls,frames", [
    ("C2", 4, 16),      # THE HEADLINE PATH: 1280x720 Cornell + knot on the 7-wave Cornell service kernel, bench cadence
    ("C3", 4, 16),      # 1280x720: 4 back-to-back 16-frame launches, 32 paths per slot, pixel list beyond 1,024 runs
    ("C5", 2, 16),      # 3840x2160 1M-triangle knot: 2 launches of 66 M paths, 64 queue heads
])
def test_service_session_full_size_equals_launch_by_launch(native, oracle, cfg, calls, frames):
    """The render-service path that produces the bench numbers, at the
    BASELINE size and cadence: `calls` back-to-back async 16-frame calls in
    ONE session (service mode 1: one session, every launch taken by it) equal
    the same calls launch by launch (service mode 0) bit for bit -- accum,
    RGBA8, depth -- so the session's 16-frame slots (32 paths per slot), its
    multi-slot finish pass, the XCD queue bands beyond the first (3,600
    sub-tiles at 720p against 128 per band) and the listed-pixel runs are
    exercised at full scale.  C2 (bench.py's workload, on the kernel the
    bench times) is also compared with the portable-libm oracle over the
    whole frame and all 64 frames, bit for bit.  C5 checks the session's image
    against the glibc oracle over a 48-row band of the 4K frame (the tolerance
    of test_gpu_parity's baseline-size test, over all the session's frames)."""
    sc = scenes.make_scene(cfg)

    def run(service):
        r = VRendererHIP(0)
        scenes.load_into(r, sc)
        r.set_service(service)
        t = sc["time"]
        kinds = []
        for i in range(calls):
            r.render(frames=frames, times=[t + frames * i + k for k in range(frames)], sync=False)
            kinds.append(r.last_launch_info()["kind"])
        out = r.read_accum(), r.read_rgba8(), r.read_depth8(), r.getFrameCount()
        info = r.service_info()
        r.cleanUp()
        return out, kinds, info
    (a1, r1, d1, n1), k1, i1 = run(1)
    (a0, r0, d0, n0), k0, i0 = run(0)
    assert set(k1) == {"service"} and "service" not in k0, (k1, k0)
    assert i1["sessions"] == 1 and i1["served"] == calls and i1["refused"] == 0, i1
    assert i0["sessions"] == 0, i0
    assert n1 == n0 == calls * frames
    _eq(a1, a0, "accum"); _eq(r1, r0, "rgba8"); _eq(d1, d0, "depth8")
    if cfg == "C2":
        nf = calls * frames
        t0 = time.perf_counter()
        oa, orgba, od, _ = po.render(sc, frames=nf, times=[sc["time"] + k for k in range(nf)],
                                     libm=po.LIBM_PORTABLE)
        print(f"C2 oracle, whole 1280x720 frame x {nf} frames: {time.perf_counter() - t0:.1f} s")
        H, W = (sc["height"] // 16) * 16, (sc["width"] // 16) * 16
        assert np.any(oa[:H, :W, :3] != 0)
        _eq(a1[:H, :W], oa[:H, :W], "C2 session accum vs oracle")
        _eq(r1[:H, :W], orgba[:H, :W], "C2 session rgba8 vs oracle")
        _eq(d1[:H, :W], od[:H, :W], "C2 session depth8 vs oracle")
    if cfg == "C5":
        TOL_RMSE, TOL_PIX_FRAC = 1e-3, 0.995      # test_gpu_parity.py's north-star tolerance
        r0_, r1_ = 1056, 1104
        nf = calls * frames
        times = [sc["time"] + k for k in range(nf)]
        oa, _, _, _ = po.render(sc, frames=nf, times=times, libm=po.LIBM_GLIBC, rows=(r0_, r1_))
        g = a1[r0_:r1_, :(sc["width"] // 16) * 16, :3] / nf
        o = oa[r0_:r1_, :(sc["width"] // 16) * 16, :3] / nf
        assert np.any(o != 0)
        d = np.abs(g - o).max(-1)
        rmse = float(np.sqrt(((g - o) ** 2).mean()))
        frac = float((d <= 1e-3).mean())
        print(f"C5 session rows {r0_}-{r1_} {nf} frames vs glibc oracle: RMSE {rmse:.3e}, {frac:.6f} within 1e-3")
        assert rmse < TOL_RMSE, rmse
        assert frac >= TOL_PIX_FRAC, frac


def test_service_retire_race_forced(native):
    """The lost-launch race, forced: the session kernel retires after 1 ms
    without a launch, the host's post window is 50 ms and the host sleeps 3 ms
    between that window check and every post after a session's first, so
    each session serves its first launch and the next post meets a retiring
    kernel.  The store-fence-load hand-shake must hand each such launch to the
    launch path (counted by vrhip_service_stats), the consumed-count check at
    sync must pass, and the image must equal launch-by-launch rendering --
    with launches served by sessions and others refused, in one run."""
    sc = scenes.make_scene("C3", 96, 64)
    calls = [2, 1, 3, 2, 1, 2]

    def run(service, timing):
        r = VRendererHIP(0)
        scenes.load_into(r, sc)
        r.set_service(service)
        if timing:
            r.set_service_timing(*timing)
        t = sc["time"]
        for n in calls:
            r.render(frames=n, times=[t + k for k in range(n)], sync=False)
            t += n
        r.sync()
        out = r.read_accum(), r.read_rgba8(), r.read_depth8(), r.getFrameCount()
        refused = r.service_refused()
        info = r.service_info()
        r.cleanUp()
        return out, refused, info
    (a1, r1, d1, n1), refused, info = run(1, (1000, 50000, 3000))
    (a0, r0, d0, n0), none, _ = run(0, None)
    assert refused >= 1 and none == 0, (refused, none)
    assert info["refused"] == refused and info["served"] >= 1, info
    assert info["served"] + info["refused"] == len(calls), info
    assert n1 == n0 == sum(calls)
    _eq(a1, a0, "accum"); _eq(r1, r0, "rgba8"); _eq(d1, d0, "depth8")


def test_service_gather_not_deferred_in_automatic_mode(native):
    """The deferred-gather foot-gun is gone from the default mode: in
    automatic service mode a vrhip_comm_gather inside a session closes the
    session and is enqueued at once (vrhip_service_info: no deferred gather),
    while explicit mode 1 still defers; both give the launch-by-launch image.
    One-rank RCCL communicator, back-to-back 16-frame C3 calls (each behind a
    launch in flight, so automatic mode opens sessions)."""
    from vrenderer_pathtracer_amd.renderer import comm_unique_id
    from vrenderer_pathtracer_amd.tiles import WHAT_RGBA8
    sc = scenes.make_scene("C3")

    def run(service):
        r = VRendererHIP(0)
        scenes.load_into(r, sc)
        r.set_service(service)
        r.comm_init(0, 1, comm_unique_id())
        t = sc["time"]
        for i in range(4):
            r.render(frames=16, times=[t + 16 * i + k for k in range(16)], sync=False)
            r.comm_gather(WHAT_RGBA8)
        r.sync()
        out = r.read_accum(), r.read_rgba8()
        info = r.service_info()
        r.comm_destroy()
        r.cleanUp()
        return out, info
    (aa, ar), ia = run(-1)
    (ea, er), ie = run(1)
    (ba, br), _ = run(0)
    assert ia["sessions"] >= 1 and ia["deferred_gathers"] == 0, ia
    assert ie["deferred_gathers"] >= 1, ie
    for g in ((aa, ar), (ea, er)):
        _eq(g[0], ba, "accum"); _eq(g[1], br, "rgba8")


@pytest.mark.parametrize("mode", [-1, 1])
def test_service_budget_falls_back_to_launch_path(native, mode):
    """Launches whose result slot the service's scratch budget cannot hold
    twice take the ordinary launch path in every mode instead of failing
    (round 4 returned VRHIP_ERR_NOMEM): C3 1280x720 calls of 64 frames (1.4 GB
    per slot) behind a launch in flight, with a 1 GiB budget.  The image
    equals launch-by-launch rendering."""
    sc = scenes.make_scene("C3")

    def run(service, budget):
        r = VRendererHIP(0)
        scenes.load_into(r, sc)
        r.set_service(service)
        r.set_service_budget(budget)
        t = sc["time"]
        kinds = []
        for i in range(3):
            r.render(frames=64, times=[t + 64 * i + k for k in range(64)], sync=False)
            kinds.append(r.last_launch_info()["kind"])
        out = r.read_accum(), r.read_rgba8()
        r.cleanUp()
        return out, kinds
    (a1, r1), k1 = run(mode, 1 << 30)
    (a0, r0), _ = run(0, 0)
    assert "service" not in k1, k1
    _eq(a1, a0, "accum"); _eq(r1, r0, "rgba8")


def test_service_4k_hdri_mesh_64_frame_calls(native):
    """The advisor's case: back-to-back 64-frame calls of the 4K HDRI-mesh
    scene in automatic mode (two launch slots of 12.8 GB fit the default
    24 GiB budget, so they join a session) render without error and equal
    launch-by-launch rendering."""
    sc = scenes.make_scene("C5")

    def run(service):
        r = VRendererHIP(0)
        scenes.load_into(r, sc)
        r.set_service(service)
        t = sc["time"]
        for i in range(2):
            r.render(frames=64, times=[t + 64 * i + k for k in range(64)], sync=False)
        out = r.read_accum(), r.read_rgba8()
        r.cleanUp()
        return out
    (a1, r1), (a0, r0) = run(-1), run(0)
    _eq(a1, a0, "accum"); _eq(r1, r0, "rgba8")


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_one_frame_graph_equals_launches(native, oracle, cfg):
    """VRHIP_GRAPH=1: synchronous one-frame calls (kernel timing off, the Qt
    adapter's configuration) launch the path kernel + finish pass as one HIP
    graph, captured per longest-first order slot and re-captured when the
    launch changes (here: a Fresnel change and a clear mid-run).  Images equal
    plain launches bit for bit and, for the first frames, the oracle."""
    import os
    sc = scenes.make_scene(cfg, 96, 64)

    def run(graph):
        old = os.environ.get("VRHIP_GRAPH")
        os.environ["VRHIP_GRAPH"] = "1" if graph else "0"
        try:
            r = VRendererHIP(0)
            scenes.load_into(r, sc)            # (init() creates the context, which reads VRHIP_GRAPH)
        finally:
            if old is None:
                del os.environ["VRHIP_GRAPH"]
            else:
                os.environ["VRHIP_GRAPH"] = old
        r.set_kernel_timing(False)
        t = sc["time"]
        kinds, snaps = [], []
        for i in range(12):
            if i == 6:
                snaps.append(r.read_accum())
                r.setFresnelCoef(0.3)          # another launch parameter (and a clear): a new capture
            r.render(frames=1, times=[t + i], sync=True)
            kinds.append(r.last_launch_info()["kind"])
        out = r.read_accum(), r.read_rgba8(), r.read_depth8()
        r.cleanUp()
        return snaps + list(out), kinds
    g, gk = run(True)
    b, bk = run(False)
    assert "path_pool_graph" in gk and "path_pool_graph" not in bk, (gk, bk)
    for x, y, what in zip(g, b, ("accum@6", "accum", "rgba8", "depth8")):
        _eq(x, y, what)
    oa, _, _, _ = po.render(sc, frames=6, times=[sc["time"] + k for k in range(6)], libm=po.LIBM_PORTABLE)
    H, W = (64 // 16) * 16, (96 // 16) * 16
    _eq(g[0][:H, :W], oa[:H, :W], "graph accum@6 vs oracle")


def test_service_scratch_shortage_takes_the_launch_path(native):
    """A session whose launch slots do not fit in half of the device memory
    free when it opens is not opened: its launches take the launch path
    (vrhip_service_info counts the fallback) and the image equals
    launch-by-launch rendering.  Forced by holding all but ~1.2 GB of the
    device memory in a torch tensor after a first (launch-path) call has
    allocated its scratch; two 376-MB C3 slots then exceed the half.
    (Automatic mode: the first two calls of the burst take the launch path,
    the later ones would open a session.)"""
    import torch
    sc = scenes.make_scene("C3")

    def run(service, hog):
        r = VRendererHIP(0)
        scenes.load_into(r, sc)
        r.set_service(service)
        r.set_service_budget(1 << 40)          # the budget allows the slots: the free-memory cap decides
        t = sc["time"]
        r.render(frames=16, times=[t + k for k in range(16)], sync=True)
        hold = None
        if hog:
            free, _ = torch.cuda.mem_get_info(0)
            hold = torch.empty(max(0, free - (1200 << 20)), dtype=torch.uint8, device="cuda:0")
        kinds = []
        for i in range(1, 4):
            r.render(frames=16, times=[t + 16 * i + k for k in range(16)], sync=False)
            kinds.append(r.last_launch_info()["kind"])
        out = r.read_accum(), r.read_rgba8()
        info = r.service_info()
        r.cleanUp()
        del hold
        torch.cuda.empty_cache()
        return out, kinds, info
    (a1, r1), k1, i1 = run(-1, True)       # automatic: calls 3-4 are behind a launch in flight
    (a0, r0), _, _ = run(0, False)
    assert i1["alloc_fallbacks"] >= 1 and "service" not in k1, (i1, k1)
    _eq(a1, a0, "accum"); _eq(r1, r0, "rgba8")


def _one_frame_calls(sc, n, flag, shared=None):
    """n synchronous one-frame calls (render + vrhip_sync, the reference's
    cadence) with the completion flag on or off; `shared`: hand the stream or
    the buffers out first.  Returns the images, the sync counts and the
    accumulation read between calls."""
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    r.set_sync_flag(flag)
    if shared == "stream":
        r.get_stream()
    mid = None
    for i in range(n):
        r.render(frames=1, times=[sc["time"] + i], sync=True)
        if shared == "buffers" and i == 0:
            r.device_buffers()
        if i == n // 2:
            mid = r.read_accum()
    out = r.read_accum(), r.read_rgba8(), r.read_depth8(), r.getFrameCount(), r.sync_info(), mid
    r.cleanUp()
    return out


@pytest.mark.parametrize("cfg,w,h", [("C2", 160, 96), ("C3", 160, 96), ("C2", 1280, 720)])
def test_sync_flag_one_frame_calls_equal_stream_sync(native, oracle, cfg, w, h):
    """vrhip_sync ended by the finish pass's completion flag (the default
    after a call of one launch): every synchronous call's images equal those
    of stream-synchronised calls bit for bit, read-backs between calls
    included, and the 160x96 ones equal the oracle; the flag ends every
    synchronisation of the flagged context and none of the other."""
    sc = scenes.make_scene(cfg, w, h)
    n = 6
    a1, r1, d1, f1, s1, m1 = _one_frame_calls(sc, n, True)
    a0, r0, d0, f0, s0, m0 = _one_frame_calls(sc, n, False)
    assert f1 == f0 == n
    assert s1["flag"] == n and s0["flag"] == 0 and s0["stream"] >= n
    _eq(a1, a0, "accum"); _eq(r1, r0, "rgba8"); _eq(d1, d0, "depth8"); _eq(m1, m0, "mid-run accum")
    if w * h <= 160 * 96:
        times = [sc["time"] + k for k in range(n)]
        oa, orgba, od, _ = po.render(sc, frames=n, times=times, libm=po.LIBM_PORTABLE)
        H, W = (h // 16) * 16, (w // 16) * 16
        _eq(a1[:H, :W], oa[:H, :W], "accum vs oracle")
        _eq(r1[:H, :W], orgba[:H, :W], "rgba8 vs oracle")


@pytest.mark.parametrize("shared", ["stream", "buffers"])
def test_sync_flag_off_when_stream_or_buffers_handed_out(native, shared):
    """A context whose stream or device buffers the caller holds (it may read
    the images from its own streams) waits for the stream at every sync."""
    sc = scenes.make_scene("C2", 96, 64)
    a1, r1, d1, f1, s1, _ = _one_frame_calls(sc, 4, True, shared)
    a0, r0, d0, f0, s0, _ = _one_frame_calls(sc, 4, False)
    if shared == "stream":
        assert s1["flag"] == 0
    else:
        assert s1["flag"] <= 1          # the first call's sync precedes the hand-out
    _eq(a1, a0, "accum"); _eq(r1, r0, "rgba8")


def test_sync_flag_multi_frame_and_async_calls(native):
    """Multi-frame calls, async bursts (the second call overlaps the first on
    a path stream or the render service), clears and camera moves between
    synchronisations: images equal the stream-synchronised context's."""
    sc = scenes.make_scene("C2", 160, 96)

    def run(flag):
        r = VRendererHIP(0)
        scenes.load_into(r, sc)
        r.set_sync_flag(flag)
        t = sc["time"]
        outs = []
        for calls in ([3], [1, 1, 1], [2], [1]):
            for n in calls:
                r.render(frames=n, times=[t + k for k in range(n)], sync=False)
                t += n
            r.sync()
            outs.append(r.read_accum())
        r.clearBuffer()
        r.render(frames=1, times=[t], sync=True)
        outs.append(r.read_rgba8())
        info = r.sync_info()
        r.cleanUp()
        return outs, info

    o1, i1 = run(True)
    o0, _ = run(False)
    assert i1["flag"] >= 2             # the single-launch calls
    for k, (x, y) in enumerate(zip(o1, o0)):
        _eq(x, y, f"step {k}")
