"""GPU parity of the feature-class kernels (vr_cls_*.hip): every flag
combination the Qt UI produces outside the five exact BASELINE feature sets
(vr_kernel.hpp feature_class) -- texture maps and the BRDF view tested at run
time, Cornell / HDRI and mesh / spheres fixed at compile time -- bit-exact
against the portable-libm oracle (oracle/vro.c, the line-cited restatement of
PathTracer.cu:597-770), on multi-frame, one-frame (inline camera ray), tiled
(shard) and render-service launches.
"""
import numpy as np
import pytest

import pyoracle as po
from vrenderer_pathtracer_amd import VRendererHIP, scenes

pytestmark = pytest.mark.gpu


def class_scene(name, w, h):
    """Scenes outside the exact specialisations C1..C5."""
    tex = scenes.procedural_textures(n=256)
    if name == "C2D":                  # Cornell + mesh + diffuse map
        sc = scenes.make_scene("C2D", w, h)
    elif name == "C3D":                # HDRI + mesh + diffuse map only
        sc = scenes.make_scene("C3D", w, h)
    elif name == "C2N":                # Cornell + mesh + normal and specular maps (Fresnel)
        sc = scenes.make_scene("C2", w, h)
        sc.update(tex_normal=tex["tex_normal"], tex_specular=tex["tex_specular"])
    elif name == "C3B":                # HDRI + mesh shaded by the MERL BRDF (kViewBRDF)
        sc = scenes.make_scene("C3", w, h)
        sc.update(view_brdf=True, brdf=scenes.synthetic_merl())
    elif name == "C5T":                # HDRI + 1M-tri knot (24-entry stacks) + all maps
        sc = scenes.make_scene("C5", w, h)
        sc.update(tex)
    elif name == "C1T":                # Cornell + example sphere with all maps
        sc = scenes.make_scene("C1", w, h)
        sc.update(tex)
    elif name == "C4D":                # HDRI + example sphere, diffuse map, no BRDF view
        sc = scenes.make_scene("C4", w, h)
        sc.update(view_brdf=False, brdf=None, tex_diffuse=tex["tex_diffuse"])
    elif name == "CB":                 # the empty Cornell box (no mesh, no example sphere)
        sc = scenes.make_scene("C1", w, h)
        sc.update(example_sphere=False)
    elif name == "C3X":                # mesh loaded AND the example sphere on: the reference ignores the mesh
        sc = scenes.make_scene("C3", w, h)
        sc.update(example_sphere=True)
    else:
        raise ValueError(name)
    sc["name"] = name
    return sc


CASES = [("C2D", 160, 96), ("C3D", 160, 96), ("C2N", 160, 96), ("C3B", 160, 96), ("C5T", 96, 64),
         ("C1T", 128, 96), ("C4D", 128, 96), ("CB", 96, 64), ("C3X", 128, 96)]


def run(sc, times, one_frame=False, tiling=None, service=None):
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    if tiling:
        r.set_tiling(*tiling)
    if service is not None:
        r.set_service(service)
    if one_frame:
        for t in times:
            r.render(frames=1, times=[t], sync=False)
        r.sync()
    else:
        r.render(frames=len(times), times=times)
    out = r.read_accum(), r.read_rgba8(), r.read_depth8(), r.getFrameCount()
    r.cleanUp()
    return out


def bitexact(g, o, sc, what):
    h, w = (sc["height"] // 16) * 16, (sc["width"] // 16) * 16
    g, o = g[:h, :w], o[:h, :w]
    diff = (g.view(np.uint32) != o.view(np.uint32)) if g.dtype == np.float32 else (g != o)
    n = int(diff.any(-1).sum())
    assert n == 0, f"{what}: {n} pixels differ (first at {np.argwhere(diff.any(-1))[:3].tolist()})"


@pytest.mark.parametrize("name,w,h", CASES)
def test_feature_class_bitexact_vs_portable_oracle(native, oracle, name, w, h):
    sc = class_scene(name, w, h)
    times = [12345 + 7 * i for i in range(3)]
    ga, gr, gd, nf = run(sc, times)
    oa, orgba, od, _ = po.render(sc, frames=len(times), times=times, libm=po.LIBM_PORTABLE)
    assert nf == len(times)
    bitexact(ga, oa, sc, f"{name} accum")
    bitexact(gr, orgba, sc, f"{name} rgba8")
    bitexact(gd, od, sc, f"{name} depth8")
    assert np.any(oa[..., :3] != 0)


@pytest.mark.parametrize("name,mode", [("C2D", "one_frame"), ("C3D", "one_frame"), ("C2D", "tiled"),
                                       ("C3B", "tiled"), ("C3D", "service"), ("C2N", "service")])
def test_feature_class_launch_kinds_bitexact(native, oracle, name, mode):
    """The class kernels' one-frame (F_INLINE_PRIM), shard and render-service
    instantiations against the oracle; a tiled rank renders only its tiles, so
    rank 0 of 2 is compared on the tiles it owns."""
    sc = class_scene(name, 96, 64)
    times = [777 + 5 * i for i in range(4)]
    oa, _, _, _ = po.render(sc, frames=len(times), times=times, libm=po.LIBM_PORTABLE)
    if mode == "one_frame":
        ga, _, _, nf = run(sc, times, one_frame=True)
        assert nf == len(times)
        bitexact(ga, oa, sc, f"{name} one-frame calls")
    elif mode == "service":
        ga, _, _, nf = run(sc, times, one_frame=True, service=1)
        assert nf == len(times)
        bitexact(ga, oa, sc, f"{name} service session")
    else:
        ga, _, _, _ = run(sc, times, tiling=(0, 2))
        tiles_x = (sc["width"] // 16)
        own = np.zeros(ga.shape[:2], bool)
        for t in range(0, tiles_x * (sc["height"] // 16), 2):
            ty = t // tiles_x
            tx = (t % tiles_x + ty) % tiles_x               # row-rotated dealing (include/vrhip.h)
            own[ty * 16:(ty + 1) * 16, tx * 16:(tx + 1) * 16] = True
        assert (ga[own].view(np.uint32) == oa[own].view(np.uint32)).all()
        assert not ga[~own].any()


@pytest.mark.parametrize("view,service", [("away", None), ("away", 1), ("close", None)])
def test_escaped_ray_skipping_extremes_bitexact(native, oracle, view, service):
    """HDRI mesh launches skip the pixels whose camera ray escapes (F_SPARSE):
    with the camera turned away from the knot no pixel is listed (the path
    kernel gets no work, every pixel takes its shared result), close to the
    knot nearly every pixel is; both, in launches and in a render-service
    session, equal the oracle bit for bit."""
    sc = scenes.make_scene("C3", 96, 64)
    if view == "away":        # looking down +z, away from the knot at the origin
        sc["camera"] = dict(sc["camera"], dir=(0.0, 0.0, 1.0), right=(-1.0, 0.0, 0.0))
    else:                     # 30 units from the knot's centre
        sc["camera"] = dict(sc["camera"], origin=(0.0, 0.0, 30.0))
    times = [4321 + 3 * i for i in range(5)]
    ga, gr, gd, nf = run(sc, times, one_frame=service is not None, service=service)
    oa, orgba, od, _ = po.render(sc, frames=len(times), times=times, libm=po.LIBM_PORTABLE)
    assert nf == len(times)
    bitexact(ga, oa, sc, f"{view} accum")
    bitexact(gr, orgba, sc, f"{view} rgba8")
    bitexact(gd, od, sc, f"{view} depth8")
