"""ORACLE / TEST INFRASTRUCTURE ONLY -- ctypes binding of oracle/liboracle_vro.so.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker.  The product (vrenderer_pathtracer_amd) never imports it.
The C restatement it binds follows /root/reference/cuda/src/PathTracer.cu
(see oracle/vro.c for per-function citations).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_vro.so")

LIBM_GLIBC = 0
LIBM_PORTABLE = 1

_f = ctypes.POINTER(ctypes.c_float)


class VroScene(ctypes.Structure):
    _fields_ = [
        ("cam_origin", ctypes.c_float * 4), ("cam_dir", ctypes.c_float * 4),
        ("cam_up", ctypes.c_float * 4), ("cam_right", ctypes.c_float * 4),
        ("fov_scale", ctypes.c_float),
        ("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
        ("fresnel_coef", ctypes.c_float), ("fresnel_pow", ctypes.c_float),
        ("use_cornell", ctypes.c_int), ("use_example_sphere", ctypes.c_int),
        ("view_brdf", ctypes.c_int), ("mesh_initialised", ctypes.c_int),
        ("bvh", _f), ("n_bvh_f4", ctypes.c_size_t),
        ("verts", _f), ("normals", _f), ("tangents", _f), ("uvs", _f),
        ("n_slots", ctypes.c_size_t),
        ("hdr", _f), ("hdr_w", ctypes.c_uint32), ("hdr_h", ctypes.c_uint32),
        ("tex", _f * 3), ("tex_w", ctypes.c_uint32 * 3), ("tex_h", ctypes.c_uint32 * 3),
        ("brdf", _f),
        ("libm", ctypes.c_int), ("brute_force", ctypes.c_int),
    ]


COUNTER_FIELDS = ["paths", "rays", "node_visits", "slot_reads", "tri_tests", "hits",
                  "attr_bytes", "tex_fetches", "hdr_fetches", "brdf_fetches",
                  "pixel_io_bytes", "max_stack"]


class VroCounters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in COUNTER_FIELDS]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n in COUNTER_FIELDS}


_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with its own Makefile (gcc, -ffp-contract=off)."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.vro_render.restype = ctypes.c_int
        L.vro_render.argtypes = [ctypes.POINTER(VroScene), _f, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                 ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                 ctypes.POINTER(VroCounters)]
        L.vro_hash.restype = ctypes.c_uint32
        L.vro_hash.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
        L.vro_rng_uniforms.argtypes = [ctypes.c_uint32, ctypes.c_int, _f]
        L.vro_intersect_triangle.argtypes = [_f] * 6
        L.vro_sphere_intersect.restype = ctypes.c_float
        L.vro_sphere_intersect.argtypes = [ctypes.c_int, _f, _f]
        L.vro_brdf_index.restype = ctypes.c_int
        L.vro_brdf_index.argtypes = [_f, _f, _f, _f, ctypes.c_int]
        L.vro_span.argtypes = [_f, _f]
        L.vro_primary_ray.argtypes = [ctypes.POINTER(VroScene), ctypes.c_uint32, ctypes.c_uint32, _f, _f]
        L.vro_trace_sample.argtypes = [ctypes.POINTER(VroScene), ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, _f]
        for n in ["vro_p_sinf", "vro_p_cosf", "vro_p_atanf", "vro_p_acosf"]:
            getattr(L, n).restype = ctypes.c_float
            getattr(L, n).argtypes = [ctypes.c_float]
        for n in ["vro_p_atan2f", "vro_p_powf"]:
            getattr(L, n).restype = ctypes.c_float
            getattr(L, n).argtypes = [ctypes.c_float, ctypes.c_float]
        _lib = L
    return _lib


def _fp(a):
    if a is None:
        return None
    return a.ctypes.data_as(_f)


class OracleScene:
    """Holds numpy arrays alive and a VroScene pointing at them."""

    def __init__(self, scene: dict, libm: int = LIBM_GLIBC, brute_force: bool = False):
        self._keep = []
        s = VroScene()
        cam = scene["camera"]
        for name in ("origin", "dir", "up", "right"):
            v = np.asarray(cam[name], dtype=np.float32)
            arr = getattr(s, "cam_" + name)
            for i in range(3):
                arr[i] = float(v[i])
            arr[3] = 0.0
        s.fov_scale = float(np.float32(cam["fov_scale"]))
        s.width, s.height = int(scene["width"]), int(scene["height"])
        s.fresnel_coef = float(np.float32(scene.get("fresnel_coef", 0.1)))
        s.fresnel_pow = float(np.float32(scene.get("fresnel_pow", 3.0)))
        s.use_cornell = int(bool(scene.get("cornell", False)))
        s.use_example_sphere = int(bool(scene.get("example_sphere", False)))
        s.view_brdf = int(bool(scene.get("view_brdf", False)))
        mesh = scene.get("mesh_flat")
        if mesh is not None:
            arrs = {k: np.ascontiguousarray(mesh[k], dtype=np.float32)
                    for k in ("bvh", "verts", "normals", "tangents", "uvs")}
            self._keep.append(arrs)
            s.bvh = _fp(arrs["bvh"]); s.n_bvh_f4 = arrs["bvh"].size // 4
            s.verts = _fp(arrs["verts"]); s.normals = _fp(arrs["normals"])
            s.tangents = _fp(arrs["tangents"]); s.uvs = _fp(arrs["uvs"])
            s.n_slots = arrs["verts"].size // 4
            s.mesh_initialised = 1
        hdr = scene.get("hdr")
        if hdr is not None:
            h = np.ascontiguousarray(hdr, dtype=np.float32)
            self._keep.append(h)
            s.hdr = _fp(h); s.hdr_h, s.hdr_w = h.shape[0], h.shape[1]
        for i, key in enumerate(("tex_diffuse", "tex_normal", "tex_specular")):
            t = scene.get(key)
            if t is not None:
                t = np.ascontiguousarray(t, dtype=np.float32)
                self._keep.append(t)
                s.tex[i] = _fp(t); s.tex_h[i], s.tex_w[i] = t.shape[0], t.shape[1]
        brdf = scene.get("brdf")
        if brdf is not None:
            b = np.ascontiguousarray(brdf, dtype=np.float32)
            assert b.size == 3 * 1458000
            self._keep.append(b)
            s.brdf = _fp(b)
        s.libm = libm
        s.brute_force = int(brute_force)
        self.s = s
        self.width, self.height = s.width, s.height


def render(scene: dict, frames: int = 1, times=None, first_frame: int = 1, libm: int = LIBM_GLIBC,
           rows=None, threads: int = 0, accum=None, count: bool = False, brute_force: bool = False):
    """Render frames first_frame..first_frame+frames-1 with the oracle.

    Returns (accum float32[H,W,4], rgba uint8[H,W,4], depth uint8[H,W,4], counters|None).
    """
    L = lib()
    os_ = OracleScene(scene, libm=libm, brute_force=brute_force)
    W, H = os_.width, os_.height
    if accum is None:
        accum = np.zeros((H, W, 4), dtype=np.float32)
    rgba = np.zeros((H, W, 4), dtype=np.uint8)
    depth = np.zeros((H, W, 4), dtype=np.uint8)
    if times is None:
        times = [scene.get("time", 12345)] * frames
    t = (ctypes.c_uint32 * frames)(*[int(v) & 0xFFFFFFFF for v in times])
    r0, r1 = (0, H) if rows is None else rows
    cnt = VroCounters() if count else None
    rc = L.vro_render(ctypes.byref(os_.s), _fp(accum), rgba.ctypes.data, depth.ctypes.data,
                      first_frame, frames, t, r0, r1, threads,
                      ctypes.byref(cnt) if cnt is not None else None)
    if rc != 0:
        raise RuntimeError(f"vro_render failed: {rc}")
    return accum, rgba, depth, (cnt.as_dict() if cnt is not None else None)
