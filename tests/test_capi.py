"""CPU tests of the C ABI (include/vrhip.h) and the host-side BVH / layout code.

No compute call needs a GPU here: the library must load, export every
declared symbol, fail loudly (status codes, no exit) without a device, and
its host helpers (BVH build, flattening, validation, tiling) must be right.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import pyoracle as po
from vrenderer_pathtracer_amd import _native, build_flat, scenes, validate_flat
from vrenderer_pathtracer_amd.build import LIB_PATH
from vrenderer_pathtracer_amd.tiles import owned_pixels, pack_host, unpack_host

_f = ctypes.POINTER(ctypes.c_float)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol(native):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (vrhip_\w+)", out))
    declared = set(_native.header_symbols())
    assert declared, "no symbols parsed from include/vrhip.h"
    assert declared <= exported, sorted(declared - exported)
    assert native.vrhip_abi_version() == 6


def test_build_id_ties_library_to_sources(native):
    """The library embeds the SHA-256 of the sources, include/vrhip.h and the
    compile flags (vrhip_build_id); it equals the hash of the files on disk,
    and the loader's staleness check reads it from the file itself."""
    from vrenderer_pathtracer_amd import build
    bid = native.vrhip_build_id().decode()
    assert re.fullmatch(r"[0-9a-f]{64}", bid), bid
    assert bid == build.source_id() == build.lib_build_id(LIB_PATH)
    assert not build.needs_build()
    assert _native.build_id()["matches_sources"]
    # any change to a source or flag changes the id
    assert build.source_id(["-DVR_SOMETHING=1"]) != bid


def _has_gpu(native):
    n = ctypes.c_int(0)
    return native.vrhip_device_count(ctypes.byref(n)) == 0 and n.value > 0


def test_create_without_device_fails_loudly(native):
    if _has_gpu(native):
        pytest.skip("a GPU is visible")
    ctx = ctypes.c_void_p()
    rc = native.vrhip_create(0, 64, 64, ctypes.byref(ctx))
    assert rc == -5 and not ctx.value
    assert b"device" in native.vrhip_last_error().lower()


def test_create_rejects_bad_sizes(native):
    """Sizes are checked before any device call: 0 and > 65535 pixels per side
    (path-kernel pixel coordinates are 16-bit) are VRHIP_ERR_INVALID."""
    for w, h in ((0, 64), (64, 0), (65536, 64), (64, 70000)):
        ctx = ctypes.c_void_p()
        assert native.vrhip_create(0, w, h, ctypes.byref(ctx)) == -1 and not ctx.value
        assert b"create" in native.vrhip_last_error().lower()


def test_null_context_is_invalid(native):
    assert native.vrhip_clear(None) == -1
    assert native.vrhip_render(None, 1, None, 0) == -1
    assert native.vrhip_set_fresnel(None, 0.1, 3.0) == -1
    assert native.vrhip_set_overlap(None, -1) == -1
    assert native.vrhip_set_path_split(None, 0) == -1
    assert native.vrhip_selftest_rcp(0, 0, 1, None, None) == -1
    assert native.vrhip_selftest_sqrt(0, 0, 1, None, None) == -1
    assert native.vrhip_destroy(None) == 0
    assert native.vrhip_build_flat(None, None, None, None, 0, None, 0, 4, None, None, None, None, None, None,
                                   None) == -1


def _mesh_arrays(m):
    return m["positions"], m["tris"]


def test_build_flat_references_every_triangle_once(native):
    m = scenes.torus_knot(40, 20)
    flat = build_flat(m)
    verts = flat["verts"]
    term = verts[:, 0].view(np.uint32) == 0x80000000
    tri_slots = verts[~term]
    assert tri_slots.shape[0] == 3 * m["tris"].shape[0]
    # each original triangle appears exactly once (object-split builder)
    P = m["positions"]
    key = lambda a: tuple(np.round(a, 5).reshape(-1))
    want = sorted(key(P[t]) for t in m["tris"])
    got = sorted(key(tri_slots[i:i + 3, :3]) for i in range(0, tri_slots.shape[0], 3))
    assert want == got


def test_build_flat_node_bounds_contain_children(native):
    flat = build_flat(scenes.torus_knot(30, 12))
    bvh, verts = flat["bvh"], flat["verts"]
    depth, n_nodes = validate_flat(flat)
    assert n_nodes == bvh.shape[0] // 4 and 1 <= depth <= 30

    def tri_run(idx):
        s = ~idx
        pts = []
        while verts[s, 0].view(np.uint32) != 0x80000000:
            pts.append(verts[s:s + 3, :3])
            s += 3
        return np.concatenate(pts) if pts else np.zeros((0, 3), np.float32)

    def subtree_points(idx):
        if idx < 0:
            return tri_run(idx)
        n = bvh[idx:idx + 4]
        kids = n[3, :2].view(np.int32)
        return np.concatenate([subtree_points(int(kids[0])), subtree_points(int(kids[1]))])

    for off in range(0, bvh.shape[0], 4):
        n = bvh[off:off + 4]
        kids = n[3, :2].view(np.int32)
        for c in range(2):
            lo = np.array([n[c, 0], n[c, 2], n[2, 2 * c]])
            hi = np.array([n[c, 1], n[c, 3], n[2, 2 * c + 1]])
            pts = subtree_points(int(kids[c]))
            assert pts.size and (pts >= lo).all() and (pts <= hi).all()


def test_build_flat_single_triangle_has_inner_root(native):
    m = dict(positions=np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32), tris=np.array([[0, 1, 2]], np.uint32))
    flat = build_flat(m)
    assert flat["bvh"].shape == (4, 4)
    kids = flat["bvh"][3, :2].view(np.int32)
    assert (kids < 0).all()
    assert validate_flat(flat)[0] == 1


def test_validate_flat_rejects_corruption(native):
    flat = build_flat(scenes.torus_knot(20, 10))
    bad = {k: v.copy() for k, v in flat.items()}
    bad["bvh"][3, 0] = np.array([10 ** 6], np.int32).view(np.float32)[0]        # child out of range
    with pytest.raises(_native.VRHIPError):
        validate_flat(bad)
    bad = {k: v.copy() for k, v in flat.items()}
    bad["bvh"][3, 0] = np.array([0], np.int32).view(np.float32)[0]              # cycle back to the root
    with pytest.raises(_native.VRHIPError):
        validate_flat(bad)
    bad = {k: v.copy() for k, v in flat.items()}
    term = np.where(bad["verts"][:, 0].view(np.uint32) == 0x80000000)[0]
    bad["verts"][term[-1], 0] = 1.0                                              # lost terminator
    with pytest.raises(_native.VRHIPError):
        validate_flat(bad)


def test_validate_flat_rejects_shared_nodes_and_leaves(native):
    """The device layout keys the equal-t tie-break on each triangle's unique
    root path (vrhip_api.cpp tri_paths), so the flattened BVH must be a tree
    (the reference's LIFO flatten always is, src/vRendererCuda.cpp:204-279):
    an inner node or a leaf run reached from two parents is rejected before
    upload (vrhip_upload_mesh_flat validates first)."""
    flat = build_flat(scenes.torus_knot(20, 10))
    kids = flat["bvh"][3::4, :2].view(np.int32)            # child indices of every node
    inner = [(n, c, int(kids[n, c])) for n in range(kids.shape[0]) for c in range(2) if kids[n, c] > 0]
    leaves = [(n, c, int(kids[n, c])) for n in range(kids.shape[0]) for c in range(2) if kids[n, c] < 0]
    assert len(inner) >= 2 and len(leaves) >= 2
    bad = {k: v.copy() for k, v in flat.items()}
    (n0, c0, i0), (n1, c1, _) = inner[0], inner[-1]
    bad["bvh"][4 * n1 + 3, c1] = np.array([i0], np.int32).view(np.float32)[0]   # a second parent of node i0
    with pytest.raises(_native.VRHIPError):
        validate_flat(bad)
    bad = {k: v.copy() for k, v in flat.items()}
    (n0, c0, l0), (n1, c1, _) = leaves[0], leaves[-1]
    bad["bvh"][4 * n1 + 3, c1] = np.array([l0], np.int32).view(np.float32)[0]   # one leaf run, two parents
    with pytest.raises(_native.VRHIPError):
        validate_flat(bad)


@pytest.mark.parametrize("cfg", ["C2", "C3"])
def test_bvh_traversal_equals_brute_force(oracle, cfg):
    """The closest hit does not depend on the tree (no t-culling in the
    reference traversal): BVH traversal == testing every triangle."""
    sc = scenes.make_scene(cfg, 64, 48)
    a, _, _, _ = po.render(sc, frames=1)
    b, _, _, _ = po.render(sc, frames=1, brute_force=True)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_random_soup_bvh_equals_brute_force(oracle):
    rng = np.random.default_rng(5)
    n = 300
    c = rng.uniform(-30, 30, (n, 1, 3))
    P = (c + rng.normal(0, 4, (n, 3, 3))).reshape(-1, 3).astype(np.float32)
    m = dict(positions=P, normals=np.tile([0, 0, 1], (3 * n, 1)).astype(np.float32),
             tangents=np.tile([1, 0, 0], (3 * n, 1)).astype(np.float32),
             uvs=rng.uniform(0, 1, (3 * n, 2)).astype(np.float32),
             tris=np.arange(3 * n, dtype=np.uint32).reshape(-1, 3))
    sc = scenes.make_scene("C2", 48, 32)
    sc["mesh_flat"] = build_flat(m, max_leaf_tris=3)
    a, _, _, _ = po.render(sc, frames=1)
    b, _, _, _ = po.render(sc, frames=1, brute_force=True)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_spatial_split_bvh_equals_brute_force(oracle, monkeypatch):
    """The opt-in spatial-split builder (VRHIP_SBVH_ALPHA, vr_bvh.cpp
    SpatialBuilder): a triangle split across leaves is still found wherever a
    ray meets it -- traversal == testing every triangle, on a soup of large
    overlapping triangles where splits do happen."""
    rng = np.random.default_rng(11)
    n = 200
    c = rng.uniform(-30, 30, (n, 1, 3))
    P = (c + rng.normal(0, 12, (n, 3, 3))).reshape(-1, 3).astype(np.float32)
    m = dict(positions=P, normals=np.tile([0, 0, 1], (3 * n, 1)).astype(np.float32),
             tangents=np.tile([1, 0, 0], (3 * n, 1)).astype(np.float32),
             uvs=rng.uniform(0, 1, (3 * n, 2)).astype(np.float32),
             tris=np.arange(3 * n, dtype=np.uint32).reshape(-1, 3))
    plain = build_flat(m, max_leaf_tris=2)
    monkeypatch.setenv("VRHIP_SBVH_ALPHA", "1e-5")
    split = build_flat(m, max_leaf_tris=2)
    validate_flat(split)
    assert len(split["verts"]) > len(plain["verts"])          # references were split
    sc = scenes.make_scene("C2", 48, 32)
    sc["mesh_flat"] = split
    a, _, _, _ = po.render(sc, frames=1)
    b, _, _, _ = po.render(sc, frames=1, brute_force=True)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("W,H,n", [(1280, 720, 1), (1280, 720, 2), (1280, 720, 8), (1920, 1080, 8), (64, 40, 3),
                                   (40, 15, 2), (48, 48, 16)])
def test_tile_pixels_partition(native, W, H, n):
    """Tiles dealt round-robin along the row-rotated dealing sequence: a disjoint
    cover of the rendered region, equal counts +-1 tile, diagonals per rank."""
    parts = [owned_pixels(W, H, r, n) for r in range(n)]
    allp = np.sort(np.concatenate(parts))
    wr, hr = (W // 16) * 16, (H // 16) * 16
    expect = (np.arange(hr)[:, None] * W + np.arange(wr)[None, :]).ravel()
    assert np.array_equal(allp, np.sort(expect))
    tiles_x = W // 16
    for r, pix in enumerate(parts):
        y, x = pix // W, pix % W
        ty, tx = (y // 16).astype(np.int64), (x // 16).astype(np.int64)
        s = ty * tiles_x + ((tx - ty) % tiles_x if n > 1 else tx)   # the tile's position in the dealing sequence
        assert (s % n == r).all()
    sizes = [len(p) // 256 for p in parts]
    assert max(sizes) - min(sizes) <= 1


def test_pack_unpack_host_roundtrip(native):
    img = np.random.default_rng(0).random((720, 64, 4)).astype(np.float32)
    packed = [pack_host(img, r, 3) for r in range(3)]
    out = np.zeros_like(img)
    unpack_host(packed, out)
    assert np.array_equal(out, img)


def test_parallel_builder_is_deterministic(native):
    """The multi-threaded SAH builder (vr_bvh.cpp) gives the same flattened tree
    for any thread count (min/max boxes and counts are order-independent)."""
    import subprocess
    import sys
    code = ("import hashlib, sys; sys.path.insert(0, %r)\n"
            "from vrenderer_pathtracer_amd import scenes, renderer\n"
            "f = renderer.build_flat(scenes.torus_knot(400, 200))\n"
            "print(hashlib.sha1(b''.join(f[k].tobytes() for k in sorted(f))).hexdigest())\n") % REPO
    hashes = set()
    for threads in ("1", "3", "8"):
        env = dict(os.environ, VRHIP_BUILD_THREADS=threads)
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr[-2000:]
        hashes.add(out.stdout.strip())
    assert len(hashes) == 1


def test_load_merl_matches_reference_layout(native, tmp_path):
    """vrhip_load_merl == vBRDFLoader::loadBinary: dims header, doubles -> floats, same order."""
    from vrenderer_pathtracer_amd.renderer import load_merl
    n = 90 * 90 * 180
    vals = np.random.default_rng(3).random(3 * n) * 3.0
    f = tmp_path / "test.binary"
    with open(f, "wb") as fh:
        fh.write(np.array([90, 90, 180], np.int32).tobytes())
        fh.write(vals.astype(np.float64).tobytes())
    got = load_merl(f)
    assert np.array_equal(got, vals.astype(np.float32))
    bad = tmp_path / "bad.binary"
    with open(bad, "wb") as fh:
        fh.write(np.array([90, 90, 90], np.int32).tobytes())
        fh.write(vals[: 3 * 90 * 90 * 90].astype(np.float64).tobytes())
    with pytest.raises(_native.VRHIPError):
        load_merl(bad)
    short = tmp_path / "short.binary"
    with open(short, "wb") as fh:
        fh.write(np.array([90, 90, 180], np.int32).tobytes())
        fh.write(vals[:1000].astype(np.float64).tobytes())
    with pytest.raises(_native.VRHIPError):
        load_merl(short)


@pytest.mark.parametrize("compression,ptype,channels,origin", [
    (0, 1, "RGBA", (0, 0)), (3, 2, "RGB", (0, 0)), (2, 1, "RGBA", (3, 5)), (1, 1, "RGBA", (0, 0)),
    (3, 1, "BGR", (-2, 7)), (1, 2, "A", (0, 0))])
def test_load_exr_roundtrip(native, tmp_path, compression, ptype, channels, origin):
    """vrhip_load_exr (vr_exr.cpp) against tests/exr_writer.py: half RGBA over the
    data window, FLOAT samples rounded to half, missing R/G/B = 0 and A = 1."""
    from exr_writer import write_exr
    from vrenderer_pathtracer_amd.renderer import load_exr
    rng = np.random.default_rng(compression * 10 + ptype)
    h, w = 37, 53
    img = (rng.random((h, w, 4)) * 8.0).astype(np.float32)
    img[5:20, 10:30] = 2.5                                   # flat region: RLE runs
    f = tmp_path / "t.exr"
    write_exr(f, img, channels=channels, pixel_type=ptype, compression=compression, origin=origin)
    got = load_exr(f)
    assert got.shape == (h, w, 4) and got.dtype == np.float16
    exp = np.zeros((h, w, 4), np.float16)
    exp[..., 3] = 1.0
    for c in channels:
        exp[..., "RGBA".index(c)] = img[..., "RGBA".index(c)].astype(np.float16)
    assert np.array_equal(got.view(np.uint16), exp.view(np.uint16))


def test_load_exr_rejects_unsupported(native, tmp_path):
    from exr_writer import write_exr
    from vrenderer_pathtracer_amd.renderer import load_exr
    img = np.ones((8, 8, 4), np.float32)
    f = tmp_path / "piz.exr"
    write_exr(f, img, compression=0)
    data = bytearray(open(f, "rb").read())
    i = data.find(b"compression\0compression\0") + len(b"compression\0compression\0") + 4
    data[i] = 4                                              # PIZ
    open(f, "wb").write(bytes(data))
    with pytest.raises(_native.VRHIPError):
        load_exr(f)
    with pytest.raises(_native.VRHIPError):
        load_exr(tmp_path / "missing.exr")
    (tmp_path / "junk.exr").write_bytes(b"not an exr file at all")
    with pytest.raises(_native.VRHIPError):
        load_exr(tmp_path / "junk.exr")


def test_create_multi_rejects_bad_device_lists(native):
    """vrhip_create_multi checks its device list before touching a GPU: no
    devices, a NULL list, a repeated device, more than 64 are refused."""
    import ctypes
    ctx = ctypes.c_void_p(None)
    for devs in ([], [0, 0], [1, 2, 1]):
        arr = (ctypes.c_int * max(len(devs), 1))(*devs)
        assert native.vrhip_create_multi(arr, len(devs), 64, 64, ctypes.byref(ctx)) == -1
        assert not ctx.value
    assert native.vrhip_create_multi(None, 2, 64, 64, ctypes.byref(ctx)) == -1
    arr = (ctypes.c_int * 65)(*range(65))
    assert native.vrhip_create_multi(arr, 65, 64, 64, ctypes.byref(ctx)) == -1
