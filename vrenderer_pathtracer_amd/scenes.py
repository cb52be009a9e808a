"""Procedural, deterministic scenes for the BASELINE.json configurations.

The reference loads assets from disk (Assimp meshes, OpenEXR environments,
QImage textures, MERL .binary tables: src/MeshLoader.cpp, src/NGLScene.cpp:
205-231, src/BRDFLoader.cpp) and none ship with it (.gitignore:8-11), so the
benchmark and the tests use synthetic stand-ins of the same shape (SURVEY.md
section 8d):

  C1  Cornell box + example sphere, 512x512
  C2  Cornell box + 10k-tri torus knot, diffuse only, 1280x720
  C3  HDRI + knot + diffuse/normal/specular maps + Fresnel, 1280x720
  C4  example sphere + MERL BRDF (synthetic table) under HDRI, 1920x1080
  C5  1M-tri torus knot under HDRI, 3840x2160

Determinism: every transcendental goes through Python's `math` (glibc) on 1-D
parameter vectors; numpy only combines them with + - * / (IEEE, identical on
any x86-64 host), so the same scene arrays are produced in this container and
on the GPU box.
"""
from __future__ import annotations

import math
import os

import numpy as np

from .renderer import BRDF_TABLE_FLOATS, build_flat, default_fov_scale

DEFAULT_TIME = 12345


def default_camera() -> dict:
    """Reference default Camera (src/Camera.cpp:11-24): origin (0,0,150), looking down -z."""
    return dict(origin=(0.0, 0.0, 150.0), dir=(0.0, 0.0, -1.0), up=(0.0, 1.0, 0.0), right=(1.0, 0.0, 0.0),
                fov_scale=default_fov_scale())


def _vec_math(fn, xs):
    return np.array([fn(float(x)) for x in xs], dtype=np.float64)


def _normalize(v):
    n = np.sqrt((v * v).sum(-1, keepdims=True))
    return v / n


def torus_knot(nu: int = 100, nv: int = 50, p: int = 2, q: int = 3, tube: float = 5.0,
               scale: float = 15.0) -> dict:
    """(p,q) torus knot tube: nu*nv*2 triangles, CCW winding seen from outside,
    per-vertex normal, tangent (along the knot) and uv; centred at the vertex
    centroid like vMeshLoader::loadMesh (src/MeshLoader.cpp:60-76)."""
    u = np.arange(nu, dtype=np.float64) * (2.0 * math.pi / nu)
    v = np.arange(nv, dtype=np.float64) * (2.0 * math.pi / nv)
    cpu, spu = _vec_math(math.cos, p * u), _vec_math(math.sin, p * u)
    cqu, squ = _vec_math(math.cos, q * u), _vec_math(math.sin, q * u)
    r = cqu + 2.0
    C = np.stack([r * cpu, r * spu, -squ], -1) * scale
    dr = -q * squ
    T = np.stack([dr * cpu - p * r * spu, dr * spu + p * r * cpu, -q * cqu], -1) * scale
    T = _normalize(T)
    radial = _normalize(np.stack([cpu, spu, np.zeros_like(cpu)], -1))
    B = _normalize(np.cross(T, radial))
    N = np.cross(B, T)
    cv, sv = _vec_math(math.cos, v), _vec_math(math.sin, v)
    nrm = cv[None, :, None] * N[:, None, :] + sv[None, :, None] * B[:, None, :]       # (nu, nv, 3)
    pos = C[:, None, :] + tube * nrm
    tan = np.broadcast_to(T[:, None, :], nrm.shape)
    uu = (np.arange(nu, dtype=np.float64) / nu)[:, None] * np.ones((1, nv))
    vv = np.ones((nu, 1)) * (np.arange(nv, dtype=np.float64) / nv)[None, :]
    uvs = np.stack([uu, vv], -1)
    pos = pos.reshape(-1, 3)
    pos = pos - pos.mean(0, keepdims=True)
    idx = lambda i, j: (i % nu) * nv + (j % nv)
    I, J = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    a, b, c, d = idx(I, J), idx(I + 1, J), idx(I + 1, J + 1), idx(I, J + 1)
    tris = np.stack([np.stack([a, b, c], -1), np.stack([a, c, d], -1)], 2).reshape(-1, 3)
    # orient CCW-outward: face normal = cross(v1-v0, v2-v0) along the vertex normal
    P = pos
    fn = np.cross(P[tris[:, 1]] - P[tris[:, 0]], P[tris[:, 2]] - P[tris[:, 0]])
    nflat = nrm.reshape(-1, 3)
    if (fn * nflat[tris[:, 0]]).sum() < 0:
        tris = tris[:, [0, 2, 1]]
    return dict(positions=pos.astype(np.float32), normals=nflat.astype(np.float32),
                tangents=tan.reshape(-1, 3).astype(np.float32), uvs=uvs.reshape(-1, 2).astype(np.float32),
                tris=tris.astype(np.uint32))


def procedural_hdr(w: int = 2048, h: int = 1024, seed: int = 7) -> np.ndarray:
    """Equirect environment (rows = acos(dir.y)/pi, cols = atan2(x,z)/2pi as
    sampled at PathTracer.cu:636-643): sky gradient, ground, a sun disc and
    seeded noise; quantised to half like an OpenEXR Imf::Rgba and returned as
    float32 (H,W,4) (what vRendererCuda::loadHDR uploads)."""
    theta = (np.arange(h, dtype=np.float64) + 0.5) * (math.pi / h)
    phi = (np.arange(w, dtype=np.float64) + 0.5) * (2.0 * math.pi / w)
    cy, sy = _vec_math(math.cos, theta), _vec_math(math.sin, theta)
    cp, sp = _vec_math(math.cos, phi), _vec_math(math.sin, phi)
    up = np.clip(cy, 0.0, 1.0)[:, None]
    sky = np.array([0.85, 0.9, 1.0]) * (1.0 - up[..., None]) + np.array([0.25, 0.45, 1.1]) * up[..., None]
    ground = np.array([0.35, 0.3, 0.25])
    img = np.where((cy >= 0.0)[:, None, None], sky * np.ones((1, w, 1)), ground * np.ones((h, w, 1)))
    # sun: direction at theta0 = 50 deg from +y, phi0 = 40 deg
    th0, ph0 = math.radians(50.0), math.radians(40.0)
    sd = np.array([math.sin(th0) * math.sin(ph0), math.cos(th0), math.sin(th0) * math.cos(ph0)])
    dx = sy[:, None] * sp[None, :]
    dz = sy[:, None] * cp[None, :]
    dy = cy[:, None] * np.ones((1, w))
    cosang = dx * sd[0] + dy * sd[1] + dz * sd[2]
    cos_r = math.cos(math.radians(2.5))
    sun = np.where(cosang > cos_r, 40.0, 0.0)
    img = img + sun[..., None] * np.array([1.0, 0.95, 0.85])
    rng = np.random.default_rng(seed)
    img = img * (1.0 + 0.05 * rng.standard_normal((h, w, 1)))
    out = np.ones((h, w, 4), dtype=np.float64)
    out[..., :3] = np.maximum(img, 0.0)
    return out.astype(np.float16).astype(np.float32)


def procedural_textures(n: int = 1024, seed: int = 11) -> dict:
    """Seeded diffuse / normal / specular maps as uint8 RGBA (QImage pixels),
    converted to float4 as vRendererCuda::loadTexture does (src/vRendererCuda.cpp:
    344-368: /255, inverse gamma 2.2 on DIFFUSE only)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    checker = (((xx // (n // 16)) + (yy // (n // 16))) % 2).astype(np.float64)
    diff = np.stack([0.25 + 0.6 * checker, 0.3 + 0.4 * (1 - checker), 0.2 + 0.3 * checker], -1)
    diff = diff + 0.05 * rng.standard_normal((n, n, 3))
    diffuse8 = np.clip(np.round(diff * 255), 0, 255).astype(np.uint8)
    bump = rng.standard_normal((n // 8, n // 8, 2)) * 0.35
    bump = np.repeat(np.repeat(bump, 8, 0), 8, 1)
    nz = np.sqrt(np.maximum(1.0 - (bump ** 2).sum(-1), 0.05))
    nm = np.concatenate([bump, nz[..., None]], -1)
    nm = nm / np.sqrt((nm * nm).sum(-1, keepdims=True))
    normal8 = np.clip(np.round((nm * 0.5 + 0.5) * 255), 0, 255).astype(np.uint8)
    spec = 0.15 + 0.7 * checker + 0.1 * rng.standard_normal((n, n))
    spec8 = np.clip(np.round(spec * 255), 0, 255).astype(np.uint8)
    alpha = np.full((n, n, 1), 255, np.uint8)
    d8 = np.concatenate([diffuse8, alpha], -1)
    n8 = np.concatenate([normal8, alpha], -1)
    s8 = np.concatenate([np.repeat(spec8[..., None], 3, -1), alpha], -1)
    inv_gamma = np.float32(2.2)
    tex_d = d8.astype(np.float32) / np.float32(255.0)
    tex_d[..., :3] = tex_d[..., :3] ** inv_gamma
    return dict(tex_diffuse=tex_d.astype(np.float32),
                tex_normal=(n8.astype(np.float32) / np.float32(255.0)),
                tex_specular=(s8.astype(np.float32) / np.float32(255.0)))


def synthetic_merl() -> np.ndarray:
    """Analytic isotropic BRDF sampled on the MERL grid (90 theta_h x 90
    theta_d x 180 phi_d, planar R,G,B; src/BRDFLoader.cpp:20-43) in raw MERL
    units (value * {1,1.15,1.66}/1500 = BRDF, PathTracer.cu:20-22)."""
    th = (np.arange(90, dtype=np.float64) / 90.0) ** 2 * (math.pi / 2)   # inverse of the sqrt index map
    td = np.arange(90, dtype=np.float64) * (math.pi / 2 / 90.0)
    pd = np.arange(180, dtype=np.float64) * (math.pi / 180.0)
    lobe = _vec_math(lambda a: math.exp(-(a / 0.12) ** 2), th)
    fres = _vec_math(lambda a: 0.04 + 0.96 * (1.0 - math.cos(a)) ** 5, td)
    aniso = 1.0 + 0.1 * _vec_math(math.cos, 2.0 * pd)
    spec = lobe[:, None, None] * fres[None, :, None] * aniso[None, None, :]
    kd = np.array([0.55, 0.35, 0.2]) / math.pi
    ks = np.array([6.0, 6.0, 6.0])
    scales = np.array([1.0, 1.15, 1.66]) / 1500.0
    chans = [(kd[c] + ks[c] * spec) / scales[c] for c in range(3)]
    table = np.concatenate([ch.reshape(-1) for ch in chans]).astype(np.float32)
    assert table.size == BRDF_TABLE_FLOATS
    return table


_MESH_CACHE: dict = {}


def knot_flat(nu: int, nv: int, max_leaf_tris: int = None) -> dict:
    # leaves of <= 2 triangles (one paired load per leaf) for the 10k knot:
    # C2 +4 % over 4 with the fp16-node kernel, C3 within noise; the 1M knot
    # (C5, triangles streamed from HBM) keeps 4 (2: -2 %) (scripts/gpu_bvh_sweep.sh).
    # VRHIP_MAX_LEAF overrides it for builder experiments (scripts/ab.py --leaf)
    if max_leaf_tris is None:
        max_leaf_tris = int(os.environ.get("VRHIP_MAX_LEAF", "2" if nu * nv * 2 <= 100000 else "4"))
    key = (nu, nv, max_leaf_tris)
    if key not in _MESH_CACHE:
        _MESH_CACHE[key] = build_flat(torus_knot(nu, nv), max_leaf_tris=max_leaf_tris)
    return _MESH_CACHE[key]


def make_scene(config: str, width: int = None, height: int = None, knot=None) -> dict:
    """Scene dict for C1..C5, C2D / C3D (optionally at another resolution)."""
    cfg = config.upper()
    sc = dict(camera=default_camera(), fresnel_coef=0.1, fresnel_pow=3.0, time=DEFAULT_TIME,
              cornell=False, example_sphere=False, view_brdf=False, name=cfg)
    if cfg == "C1":
        sc.update(width=512, height=512, cornell=True, example_sphere=True)
    elif cfg == "C2":
        sc.update(width=1280, height=720, cornell=True, mesh_flat=knot_flat(*(knot or (100, 50))))
    elif cfg == "C3":
        sc.update(width=1280, height=720, hdr=procedural_hdr(), mesh_flat=knot_flat(*(knot or (100, 50))))
        sc.update(procedural_textures())
    elif cfg == "C2D":
        # not a BASELINE config: C2 with a diffuse map on the knot (a feature
        # set outside the five exact specialisations: the Cornell-mesh class kernel)
        sc.update(width=1280, height=720, cornell=True, mesh_flat=knot_flat(*(knot or (100, 50))))
        sc.update(tex_diffuse=procedural_textures()["tex_diffuse"])
    elif cfg == "C3D":
        # not a BASELINE config: C3 with only the diffuse map (the HDRI-mesh class kernel)
        sc.update(width=1280, height=720, hdr=procedural_hdr(), mesh_flat=knot_flat(*(knot or (100, 50))))
        sc.update(tex_diffuse=procedural_textures()["tex_diffuse"])
    elif cfg == "C4":
        sc.update(width=1920, height=1080, hdr=procedural_hdr(), example_sphere=True, view_brdf=True,
                  brdf=synthetic_merl())
    elif cfg == "C5":
        sc.update(width=3840, height=2160, hdr=procedural_hdr(), mesh_flat=knot_flat(*(knot or (1000, 500))))
    else:
        raise ValueError(f"unknown config {config}")
    if width is not None:
        sc["width"] = width
    if height is not None:
        sc["height"] = height
    return sc


def load_into(renderer, scene: dict) -> None:
    """Drive a VRendererHIP the way NGLScene drives vRendererCuda."""
    from .renderer import Camera
    renderer.init(scene["width"], scene["height"])
    cam = scene["camera"]
    renderer.setCamera(Camera(cam["origin"], cam["dir"], cam["up"], cam["right"], cam["fov_scale"]))
    renderer.useCornellBox(scene.get("cornell", False))
    renderer.useExampleSphere(scene.get("example_sphere", False))
    renderer.useBRDF(scene.get("view_brdf", False))
    renderer.m_fresnelCoef = scene.get("fresnel_coef", 0.1)
    renderer.setFresnelPower(scene.get("fresnel_pow", 3.0))
    if scene.get("mesh_flat") is not None:
        renderer.initMesh(scene["mesh_flat"])
    if scene.get("hdr") is not None:
        renderer.loadHDR(scene["hdr"])
    for key, t in (("tex_diffuse", 0), ("tex_normal", 1), ("tex_specular", 2)):
        if scene.get(key) is not None:
            renderer.loadTexture(scene[key], 1.0, t)
    if scene.get("brdf") is not None:
        renderer.loadBRDF(scene["brdf"])
    renderer.default_time = scene.get("time", DEFAULT_TIME)
    renderer.clearBuffer()
