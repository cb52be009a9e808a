"""Python host mirror of the reference's renderer interface, over the C ABI.

`VRendererHIP` has the method names, argument meanings and error behaviour of
the reference's abstract `vRenderer` (include/vRenderer.h:30-168) as
implemented by `vRendererCuda` (src/vRendererCuda.cpp), so tests read like
code driving the reference.  Differences, all deliberate:
  * errors raise VRHIPError instead of printing, writing errorlog.txt and
    calling exit(0) (src/vRendererCuda.cpp:454-467);
  * GL interop (registerTextureBuffer / registerDepthBuffer) is replaced by
    device RGBA8 buffers plus read-back (headless);
  * render(frames=K) renders K progressive frames in one device pass;
  * the RNG `_time` seed is explicit (the reference uses wall-clock ms,
    src/vRendererCuda.cpp:114,153).
"""
from __future__ import annotations

import ctypes
import time as _time

import numpy as np

from . import _native
from ._native import VRHIPError, check, fptr

BRDF_SAMPLING_RES_THETA_H = 90      # include/vRenderer.h:23-25
BRDF_SAMPLING_RES_THETA_D = 90
BRDF_SAMPLING_RES_PHI_D = 360
BRDF_TABLE_FLOATS = 3 * BRDF_SAMPLING_RES_THETA_H * BRDF_SAMPLING_RES_THETA_D * BRDF_SAMPLING_RES_PHI_D // 2

DIFFUSE, NORMAL, SPECULAR = 0, 1, 2     # vTextureType (cuda/include/PathTracer.cuh:86)


def _f32(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if shape is not None:
        a = a.reshape(shape)
    return a


def build_flat(mesh: dict, max_leaf_tris: int = 2) -> dict:
    """Native BVH build + reference flattening (src/vRendererCuda.cpp:204-279).

    mesh: positions (N,3), normals (N,3), tangents (N,3), uvs (N,2), tris (M,3) uint32.
    Returns dict bvh (n,4), verts/normals/tangents (s,4), uvs (s,2) float32 arrays.
    """
    L = _native.lib()
    pos = _f32(mesh["positions"])
    nrm = _f32(mesh["normals"]) if mesh.get("normals") is not None else None
    tan = _f32(mesh["tangents"]) if mesh.get("tangents") is not None else None
    uvs = _f32(mesh["uvs"]) if mesh.get("uvs") is not None else None
    tris = np.ascontiguousarray(mesh["tris"], dtype=np.uint32)
    nv, nt = pos.shape[0], tris.shape[0]
    n_bvh = ctypes.c_size_t(0)
    n_slots = ctypes.c_size_t(0)
    tp = tris.ctypes.data_as(_native._u32)
    check(L.vrhip_build_flat(fptr(pos), fptr(nrm), fptr(tan), fptr(uvs), nv, tp, nt, max_leaf_tris,
                             None, ctypes.byref(n_bvh), None, None, None, None, ctypes.byref(n_slots)),
          "vrhip_build_flat(size)")
    out = {"bvh": np.zeros((n_bvh.value, 4), np.float32),
           "verts": np.zeros((n_slots.value, 4), np.float32),
           "normals": np.zeros((n_slots.value, 4), np.float32),
           "tangents": np.zeros((n_slots.value, 4), np.float32),
           "uvs": np.zeros((n_slots.value, 2), np.float32)}
    check(L.vrhip_build_flat(fptr(pos), fptr(nrm), fptr(tan), fptr(uvs), nv, tp, nt, max_leaf_tris,
                             fptr(out["bvh"]), ctypes.byref(n_bvh), fptr(out["verts"]), fptr(out["normals"]),
                             fptr(out["tangents"]), fptr(out["uvs"]), ctypes.byref(n_slots)),
          "vrhip_build_flat")
    return out


def validate_flat(flat: dict) -> tuple[int, int]:
    """Returns (depth, inner node count) of a flattened tree, raising if malformed."""
    L = _native.lib()
    d = ctypes.c_uint32(0)
    n = ctypes.c_uint32(0)
    bvh = _f32(flat["bvh"])
    verts = _f32(flat["verts"])
    check(L.vrhip_validate_flat(fptr(bvh), bvh.size // 4, fptr(verts), verts.size // 4, ctypes.byref(d),
                                ctypes.byref(n)), "vrhip_validate_flat")
    return d.value, n.value


_POWF_LUTS = {}


def texture_to_float4(rgba8: np.ndarray, gamma: float, tex_type: int) -> np.ndarray:
    """QImage pixels (uint8 (H,W,4), RGBA) -> the float4 texels
    vRendererCuda::loadTexture uploads (src/vRendererCuda.cpp:344-368):
    channel / 255.f; on DIFFUSE maps the colour channels raised to
    1.f / gamma with std::pow(float, float) -- libm's powf, applied here
    through a 256-entry table of its own results, so every texel rounds as
    the C++ host's does (numpy's float32 power may differ by an ulp)."""
    corr = np.float32(1.0) / np.float32(gamma) if gamma > 0.001 else np.float32(1.0)
    lin = np.arange(256, dtype=np.float32) / np.float32(255.0)
    if tex_type == DIFFUSE:
        key = float(corr)
        lut = _POWF_LUTS.get(key)
        if lut is None:
            libm = ctypes.CDLL("libm.so.6")
            libm.powf.restype = ctypes.c_float
            libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
            lut = np.array([libm.powf(float(v), key) for v in lin], np.float32)
            _POWF_LUTS[key] = lut
    else:
        lut = lin
    t = np.asarray(rgba8, np.uint8)
    return np.stack([lut[t[..., 0]], lut[t[..., 1]], lut[t[..., 2]], lin[t[..., 3]]], -1).astype(np.float32)


def load_merl(path: str) -> np.ndarray:
    """vBRDFLoader::loadBinary (src/BRDFLoader.cpp:15-50) through the C ABI:
    a MERL .binary file as float32[3*90*90*180] (planar R, G, B), ready for loadBRDF."""
    L = _native.lib()
    out = np.zeros(BRDF_TABLE_FLOATS, np.float32)
    check(L.vrhip_load_merl(str(path).encode(), fptr(out), out.size), "vrhip_load_merl")
    return out


def load_exr(path: str) -> np.ndarray:
    """The HDRI read of NGLScene::loadHDRMap (src/NGLScene.cpp:205-231,
    Imf::RgbaInputFile) through the C ABI: float16 (H, W, 4) RGBA over the data
    window, ready for VRendererHIP.loadHDR."""
    L = _native.lib()
    w = ctypes.c_uint32(0)
    h = ctypes.c_uint32(0)
    p = str(path).encode()
    check(L.vrhip_load_exr(p, None, 0, ctypes.byref(w), ctypes.byref(h)), "vrhip_load_exr")
    out = np.zeros((h.value, w.value, 4), np.uint16)
    check(L.vrhip_load_exr(p, out.ctypes.data_as(_native._u16), out.size, ctypes.byref(w), ctypes.byref(h)),
          "vrhip_load_exr")
    return out.view(np.float16)


class Camera:
    """Host camera state, the reference's Camera (src/Camera.cpp) reduced to
    what the renderer consumes: origin, dir, up, right, fovScale."""

    def __init__(self, origin=(0.0, 0.0, 150.0), dir=(0.0, 0.0, -1.0), up=(0.0, 1.0, 0.0),
                 right=(1.0, 0.0, 0.0), fov_scale=None):
        self.origin = np.asarray(origin, np.float32)
        self.dir = np.asarray(dir, np.float32)
        self.up = np.asarray(up, np.float32)
        self.right = np.asarray(right, np.float32)
        self.fov_scale = np.float32(default_fov_scale() if fov_scale is None else fov_scale)
        self.dirty = False

    def is_dirty(self) -> bool:
        return self.dirty


def default_fov_scale() -> float:
    """Camera::getFovScale for the default 75 degree FOV (src/Camera.cpp:4,119-123), in fp32 + tanf."""
    libm = ctypes.CDLL("libm.so.6")
    libm.tanf.restype = ctypes.c_float
    libm.tanf.argtypes = [ctypes.c_float]
    k_deg_in_rad = np.float32(np.pi / np.float64(np.float32(180.0)))
    fov_rad = np.float32(np.float32(75.0) * k_deg_in_rad)
    return float(libm.tanf(float(np.float32(fov_rad / np.float32(2.0)))))


class VRendererHIP:
    """MI355X peer of vRendererCuda behind the vRenderer interface."""

    def __init__(self, device=0):
        """device: a GPU index, or a sequence of them for one renderer over
        several GPUs of this process (vrhip_create_multi: the tiles are dealt
        over the devices, the images gathered to the first)."""
        self._lib = _native.lib()
        self._ctx = ctypes.c_void_p(None)
        self._device = device
        self._camera = None
        self.m_fresnelCoef = 0.1     # src/vRendererCuda.cpp:27-28
        self.m_fresnelPow = 3.0
        self.width = self.height = 0
        self.default_time = None

    # -- vRenderer pure virtuals (include/vRenderer.h:48-133) ------------
    def init(self, w: int, h: int) -> None:
        assert w != 0 and h != 0
        if self._ctx:
            self.cleanUp()
        if isinstance(self._device, (list, tuple)):
            devs = (ctypes.c_int * len(self._device))(*[int(d) for d in self._device])
            check(self._lib.vrhip_create_multi(devs, len(self._device), w, h, ctypes.byref(self._ctx)),
                  "vrhip_create_multi")
        else:
            check(self._lib.vrhip_create(self._device, w, h, ctypes.byref(self._ctx)), "vrhip_create")
        self.width, self.height = w, h
        check(self._lib.vrhip_set_fresnel(self._ctx, self.m_fresnelCoef, self.m_fresnelPow), "vrhip_set_fresnel")

    def registerTextureBuffer(self, texture=None) -> None:
        """GL interop is replaced by the device RGBA8 buffer (read with read_rgba8)."""

    def registerDepthBuffer(self, depth_texture=None) -> None:
        """GL interop is replaced by the device depth buffer (read with read_depth8)."""

    def render(self, frames: int = 1, times=None, time_seed=None, sync: bool = True) -> None:
        self._need_ctx()
        if self._camera is not None and self._camera.is_dirty():
            self.updateCamera()
        arr = None
        if times is not None:
            arr = (ctypes.c_uint32 * frames)(*[int(t) & 0xFFFFFFFF for t in times])
        if time_seed is None:
            time_seed = self.default_time if self.default_time is not None else int(_time.time() * 1000)
        check(self._lib.vrhip_render(self._ctx, frames, arr, int(time_seed) & 0xFFFFFFFF), "vrhip_render")
        if sync:
            check(self._lib.vrhip_sync(self._ctx), "vrhip_sync")

    def cleanUp(self) -> None:
        if self._ctx:
            self._lib.vrhip_destroy(self._ctx)
            self._ctx = ctypes.c_void_p(None)

    def updateCamera(self) -> None:
        self._need_ctx()
        cam = self._camera or Camera()
        check(self._lib.vrhip_set_camera(self._ctx, fptr(_f32(cam.origin)), fptr(_f32(cam.dir)),
                                         fptr(_f32(cam.up)), fptr(_f32(cam.right)), float(cam.fov_scale)),
              "vrhip_set_camera")
        cam.dirty = False

    def initMesh(self, mesh: dict) -> None:
        """mesh: either a flattened dict (bvh/verts/normals/tangents/uvs, the
        layout vRendererCuda::initMesh produces) or an indexed triangle mesh
        (positions/normals/tangents/uvs/tris) that is built here."""
        self._need_ctx()
        flat = mesh if "bvh" in mesh else build_flat(mesh)
        arrs = {k: _f32(flat[k]) for k in ("bvh", "verts", "normals", "tangents", "uvs")}
        check(self._lib.vrhip_upload_mesh_flat(self._ctx, fptr(arrs["bvh"]), arrs["bvh"].size // 4,
                                               fptr(arrs["verts"]), fptr(arrs["normals"]),
                                               fptr(arrs["tangents"]), fptr(arrs["uvs"]),
                                               arrs["verts"].size // 4), "vrhip_upload_mesh_flat")

    def loadHDR(self, pixels, w: int = None, h: int = None) -> None:
        """pixels: float32 (H,W,4) or float16 (H,W,4) (Imf::Rgba layout)."""
        self._need_ctx()
        a = np.ascontiguousarray(pixels)
        h = a.shape[0] if h is None else h
        w = a.shape[1] if w is None else w
        if a.dtype == np.float16:
            check(self._lib.vrhip_upload_hdr_half(self._ctx, a.view(np.uint16).ctypes.data_as(_native._u16), w, h),
                  "vrhip_upload_hdr_half")
        else:
            a = _f32(a)
            check(self._lib.vrhip_upload_hdr(self._ctx, fptr(a), w, h), "vrhip_upload_hdr")

    def loadTexture(self, texture, gamma: float = 1.0, type: int = DIFFUSE) -> None:
        """texture: uint8 (H,W,4) image (QImage pixels) -> float4 as
        vRendererCuda::loadTexture does (inverse gamma on DIFFUSE only,
        src/vRendererCuda.cpp:344-368); or a float32 (H,W,4) array used as is."""
        self._need_ctx()
        t = np.asarray(texture)
        if t.dtype == np.uint8:
            t = texture_to_float4(t, gamma, type)
        t = _f32(t)
        check(self._lib.vrhip_upload_texture(self._ctx, int(type), fptr(t), t.shape[1], t.shape[0]),
              "vrhip_upload_texture")

    def useBRDF(self, v: bool) -> None:
        self._need_ctx()
        check(self._lib.vrhip_use_brdf(self._ctx, int(bool(v))), "vrhip_use_brdf")

    def useExampleSphere(self, v: bool) -> None:
        self._need_ctx()
        check(self._lib.vrhip_use_example_sphere(self._ctx, int(bool(v))), "vrhip_use_example_sphere")

    def useCornellBox(self, v: bool) -> None:
        self._need_ctx()
        check(self._lib.vrhip_use_cornell_box(self._ctx, int(bool(v))), "vrhip_use_cornell_box")

    def set_strict_traversal(self, strict: bool) -> None:
        """True: visit every box the ray pierces, exactly like the reference."""
        check(self._lib.vrhip_set_strict_traversal(self._need_ctx(), int(bool(strict))), "vrhip_set_strict_traversal")

    def clearBuffer(self) -> None:
        self._need_ctx()
        check(self._lib.vrhip_clear(self._ctx), "vrhip_clear")

    def loadBRDF(self, brdf) -> bool:
        """Returns False for None, like vRendererCuda::loadBRDF (src/vRendererCuda.cpp:413-437)."""
        if brdf is None:
            return False
        self._need_ctx()
        b = _f32(brdf).reshape(-1)
        check(self._lib.vrhip_upload_brdf(self._ctx, fptr(b), b.size), "vrhip_upload_brdf")
        return True

    def getFrameCount(self) -> int:
        self._need_ctx()
        n = ctypes.c_uint32(0)
        check(self._lib.vrhip_frame_count(self._ctx, ctypes.byref(n)), "vrhip_frame_count")
        return n.value

    # -- non-virtual vRenderer members (include/vRenderer.h:139-151) -----
    def setFresnelCoef(self, v: float) -> None:
        self.m_fresnelCoef = float(v)
        self._need_ctx()
        check(self._lib.vrhip_set_fresnel(self._ctx, self.m_fresnelCoef, self.m_fresnelPow), "vrhip_set_fresnel")
        self.clearBuffer()

    def setFresnelPower(self, v: float) -> None:
        self.m_fresnelPow = float(v)
        self._need_ctx()
        check(self._lib.vrhip_set_fresnel(self._ctx, self.m_fresnelCoef, self.m_fresnelPow), "vrhip_set_fresnel")
        self.clearBuffer()

    def setCamera(self, cam: Camera) -> None:
        self._camera = cam
        self.updateCamera()

    # -- read-back / multi-GPU helpers ------------------------------------
    def read_accum(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), np.float32)
        check(self._lib.vrhip_read_accum(self._need_ctx(), fptr(out)), "vrhip_read_accum")
        return out

    def read_rgba8(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), np.uint8)
        check(self._lib.vrhip_read_rgba8(self._need_ctx(), out.ctypes.data_as(_native._u8)), "vrhip_read_rgba8")
        return out

    def read_depth8(self) -> np.ndarray:
        out = np.zeros((self.height, self.width, 4), np.uint8)
        check(self._lib.vrhip_read_depth8(self._need_ctx(), out.ctypes.data_as(_native._u8)), "vrhip_read_depth8")
        return out

    def set_stream(self, stream_handle) -> None:
        check(self._lib.vrhip_set_stream(self._need_ctx(), ctypes.c_void_p(stream_handle)), "vrhip_set_stream")

    def get_stream(self) -> int:
        """hipStream_t the context enqueues on (as an integer handle)."""
        return int(self._lib.vrhip_get_stream(self._need_ctx()) or 0)

    def sync(self) -> None:
        check(self._lib.vrhip_sync(self._need_ctx()), "vrhip_sync")

    def set_tiling(self, rank: int, n_ranks: int) -> None:
        check(self._lib.vrhip_set_tiling(self._need_ctx(), rank, n_ranks), "vrhip_set_tiling")

    def set_path_split(self, groups: int) -> None:
        """Path groups per pixel per launch (0 = automatic, 1 = off); results are unchanged."""
        check(self._lib.vrhip_set_path_split(self._need_ctx(), groups), "vrhip_set_path_split")

    def set_overlap(self, mode: int) -> None:
        """Overlap of consecutive render launches: 1 always, 0 never, -1 automatic (vrhip_set_overlap)."""
        check(self._lib.vrhip_set_overlap(self._need_ctx(), int(mode)), "vrhip_set_overlap")

    def device_group(self) -> list:
        """The devices this renderer runs on (lead first; vrhip_device_group)."""
        n = ctypes.c_uint32(0)
        check(self._lib.vrhip_device_group(self._need_ctx(), ctypes.byref(n), None), "vrhip_device_group")
        devs = (ctypes.c_int * n.value)()
        check(self._lib.vrhip_device_group(self._ctx, ctypes.byref(n), devs), "vrhip_device_group")
        return list(devs)

    def set_service(self, mode: int) -> None:
        """Render service sessions (consecutive launches on one persistent
        kernel): 1 always, 0 never, -1 automatic (vrhip_set_service)."""
        check(self._lib.vrhip_set_service(self._need_ctx(), int(mode)), "vrhip_set_service")

    def set_kernel_timing(self, on: bool) -> None:
        """HIP events around calls and launches for kernel_stats /
        last_kernel_ms (vrhip_set_kernel_timing; off saves ~8 us per
        synchronous one-frame call)."""
        check(self._lib.vrhip_set_kernel_timing(self._need_ctx(), int(bool(on))), "vrhip_set_kernel_timing")

    def set_sync_flag(self, on: bool) -> None:
        """vrhip_sync by the finish pass's completion flag after one-launch
        calls (vrhip_set_sync_flag; on by default)."""
        check(self._lib.vrhip_set_sync_flag(self._need_ctx(), int(bool(on))), "vrhip_set_sync_flag")

    def sync_info(self) -> dict:
        """Synchronisations since creation, by how they ended (vrhip_sync_info)."""
        c = (ctypes.c_uint64 * 2)()
        check(self._lib.vrhip_sync_info(self._need_ctx(), c), "vrhip_sync_info")
        return {"flag": int(c[0]), "stream": int(c[1])}

    def set_service_timing(self, idle_us: int = 0, post_window_us: int = 0, post_delay_us: int = 0) -> None:
        """Test hook (vrhip_set_service_timing): the session kernel's idle
        limit, the host's post window and a host delay before each post
        (0 = default)."""
        check(self._lib.vrhip_set_service_timing(self._need_ctx(), int(idle_us), int(post_window_us),
                                                 int(post_delay_us)), "vrhip_set_service_timing")

    def set_service_budget(self, nbytes: int = 0) -> None:
        """Scratch budget of the render service's launch slots (0: default)."""
        check(self._lib.vrhip_set_service_budget(self._need_ctx(), int(nbytes)), "vrhip_set_service_budget")

    def service_refused(self) -> int:
        """Launches that met a retiring session kernel and took the launch path."""
        n = ctypes.c_uint64(0)
        check(self._lib.vrhip_service_stats(self._need_ctx(), ctypes.byref(n)), "vrhip_service_stats")
        return int(n.value)

    def service_info(self) -> dict:
        """Render-service counts since creation (vrhip_service_info)."""
        c = (ctypes.c_uint64 * 5)()
        check(self._lib.vrhip_service_info(self._need_ctx(), c), "vrhip_service_info")
        return {"refused": int(c[0]), "sessions": int(c[1]), "served": int(c[2]), "deferred_gathers": int(c[3]),
                "alloc_fallbacks": int(c[4])}

    def owned_pixels(self) -> int:
        """Pixels this rank renders (256 per owned 16x16 tile)."""
        n = ctypes.c_uint32(0)
        check(self._lib.vrhip_owned_pixels(self._need_ctx(), ctypes.byref(n)), "vrhip_owned_pixels")
        return n.value

    def pack_tiles(self, what: int, dst_ptr: int) -> None:
        check(self._lib.vrhip_pack_tiles(self._need_ctx(), what, ctypes.c_void_p(dst_ptr)), "vrhip_pack_tiles")

    def unpack_tiles(self, what: int, src_ptr: int, n_ranks: int, stride_bytes: int = 0) -> None:
        check(self._lib.vrhip_unpack_tiles(self._need_ctx(), what, ctypes.c_void_p(src_ptr), n_ranks, stride_bytes),
              "vrhip_unpack_tiles")

    # -- multi-GPU tile gather over RCCL (vrhip_comm_*) --------------------
    def comm_init(self, rank: int, n_ranks: int, unique_id: bytes) -> None:
        """Join the n_ranks RCCL communicator named by unique_id (from
        comm_unique_id() on rank 0) and take tiles rank, rank+n, ... ."""
        if len(unique_id) != COMM_ID_BYTES:
            raise ValueError(f"unique id must be {COMM_ID_BYTES} bytes")
        buf = (ctypes.c_uint8 * COMM_ID_BYTES).from_buffer_copy(unique_id)
        check(self._lib.vrhip_comm_init(self._need_ctx(), rank, n_ranks, buf), "vrhip_comm_init")

    def comm_gather(self, what: int) -> None:
        """Pack, ncclGather to rank 0, unpack on rank 0 (enqueued on the context stream)."""
        check(self._lib.vrhip_comm_gather(self._need_ctx(), int(what)), "vrhip_comm_gather")

    def comm_destroy(self) -> None:
        check(self._lib.vrhip_comm_destroy(self._need_ctx()), "vrhip_comm_destroy")

    def render_counted(self, frames: int = 1, times=None, time_seed=None) -> dict:
        """Render through the counting kernel variant; returns the event counts."""
        arr = None
        if times is not None:
            arr = (ctypes.c_uint32 * frames)(*[int(t) & 0xFFFFFFFF for t in times])
        if time_seed is None:
            time_seed = self.default_time if self.default_time is not None else int(_time.time() * 1000)
        c = (ctypes.c_uint64 * 8)()
        check(self._lib.vrhip_render_counted(self._need_ctx(), frames, arr, int(time_seed) & 0xFFFFFFFF, c),
              "vrhip_render_counted")
        names = ["rays", "node_visits", "slot_reads", "tri_tests", "attr_bytes", "tex_fetches", "hdr_fetches",
                 "brdf_fetches"]
        return {n: int(v) for n, v in zip(names, c)}

    def render_profiled(self, frames: int = 1, times=None, time_seed=None) -> dict:
        """Render through the instrumented production kernels (vrhip_render_profiled):
        the same work as render(), plus counts of the memory operations it issues."""
        arr = None
        if times is not None:
            arr = (ctypes.c_uint32 * frames)(*[int(t) & 0xFFFFFFFF for t in times])
        if time_seed is None:
            time_seed = self.default_time if self.default_time is not None else int(_time.time() * 1000)
        c = (ctypes.c_uint64 * 17)()
        check(self._lib.vrhip_render_profiled(self._need_ctx(), frames, arr, int(time_seed) & 0xFFFFFFFF, c),
              "vrhip_render_profiled")
        names = ["rays", "node_visits", "slot_reads", "tri_tests", "attr_bytes", "tex_fetches", "hdr_fetches",
                 "brdf_fetches", "node_visits_lds", "tri_loads", "mesh_hits", "nmap_hits", "lane_loads_b128",
                 "lane_loads_b96", "lane_loads_b64", "lane_loads_b32", "shared_miss_paths"]
        return {n: int(v) for n, v in zip(names, c)}

    def kernel_stats(self, reset: bool = False):
        ms = ctypes.c_double(0)
        n = ctypes.c_uint64(0)
        check(self._lib.vrhip_kernel_stats(self._need_ctx(), ctypes.byref(ms), ctypes.byref(n), int(reset)),
              "vrhip_kernel_stats")
        return float(ms.value), int(n.value)

    def last_launch_info(self) -> dict:
        """Shape of the last production launch (vrhip_last_launch_info)."""
        sp, us, kd = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        check(self._lib.vrhip_last_launch_info(self._need_ctx(), ctypes.byref(sp), ctypes.byref(us), ctypes.byref(kd)),
              "vrhip_last_launch_info")
        return {"split": int(sp.value), "use_scratch": int(us.value),
                "kind": ("render_kernel", "path_pool", "service", "path_pool_graph")[min(int(kd.value), 3)]}

    def device_buffers(self):
        a, r, d = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        check(self._lib.vrhip_device_buffers(self._need_ctx(), ctypes.byref(a), ctypes.byref(r), ctypes.byref(d)),
              "vrhip_device_buffers")
        return a.value, r.value, d.value

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_float(0)
        check(self._lib.vrhip_last_kernel_ms(self._need_ctx(), ctypes.byref(ms)), "vrhip_last_kernel_ms")
        return float(ms.value)

    def bvh_info(self):
        d, n, s = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        check(self._lib.vrhip_bvh_info(self._need_ctx(), ctypes.byref(d), ctypes.byref(n), ctypes.byref(s)),
              "vrhip_bvh_info")
        return d.value, n.value, s.value

    def _need_ctx(self):
        if not self._ctx:
            raise VRHIPError(-1, "VRendererHIP", "init() has not been called")
        return self._ctx

    def __del__(self):
        try:
            self.cleanUp()
        except Exception:
            pass


def selftest_math(fn: int, a, b=None, device: int = 0) -> np.ndarray:
    """Evaluate the device libm (0 sin, 1 cos, 2 acos, 3 atan2, 4 pow, 5 fmin, 6 fmax, 7 f2i)."""
    a = _f32(a).reshape(-1)
    b = _f32(np.zeros_like(a) if b is None else b).reshape(-1)
    out = np.zeros_like(a)
    check(_native.lib().vrhip_selftest_math(device, fn, fptr(a), fptr(b), fptr(out), a.size), "vrhip_selftest_math")
    return out


def selftest_rcp(lo_bits: int, hi_bits: int, device: int = 0):
    """Exhaustively compare the kernels' reciprocal with IEEE 1/x over the float
    bit patterns [lo_bits, hi_bits) and their negations: (mismatches, first_bad)."""
    n = ctypes.c_uint64(0)
    first = ctypes.c_uint32(0)
    check(_native.lib().vrhip_selftest_rcp(device, lo_bits, hi_bits, ctypes.byref(n), ctypes.byref(first)),
          "vrhip_selftest_rcp")
    return int(n.value), int(first.value)


def selftest_tonemap(lo_bits: int = 0, hi_bits: int = 0x3F800001, device: int = 0):
    """Exhaustively compare the kernels' table tonemap byte with the f64
    pow byte over the float bit patterns [lo_bits, hi_bits) (+ -0.0):
    (mismatches, first_bad)."""
    n = ctypes.c_uint64(0)
    first = ctypes.c_uint32(0)
    check(_native.lib().vrhip_selftest_tonemap(device, lo_bits, hi_bits, ctypes.byref(n), ctypes.byref(first)),
          "vrhip_selftest_tonemap")
    return int(n.value), int(first.value)


def selftest_sqrt(lo_bits: int, hi_bits: int, device: int = 0):
    """Exhaustively compare the kernels' square root with sqrtf over the float
    bit patterns [lo_bits, hi_bits): (mismatches, first_bad)."""
    n = ctypes.c_uint64(0)
    first = ctypes.c_uint32(0)
    check(_native.lib().vrhip_selftest_sqrt(device, lo_bits, hi_bits, ctypes.byref(n), ctypes.byref(first)),
          "vrhip_selftest_sqrt")
    return int(n.value), int(first.value)


def microbench_vmem(width_bytes: int, distinct: int, device: int = 0) -> float:
    """Lane loads per second of the device's vector-memory gather path (vrhip_microbench_vmem)."""
    r = ctypes.c_double(0)
    check(_native.lib().vrhip_microbench_vmem(device, width_bytes, distinct, ctypes.byref(r)), "vrhip_microbench_vmem")
    return float(r.value)


COMM_ID_BYTES = 128    # VRHIP_COMM_ID_BYTES


def comm_unique_id() -> bytes:
    """A fresh RCCL communicator id (vrhip_comm_unique_id), to hand to every rank."""
    buf = (ctypes.c_uint8 * COMM_ID_BYTES)()
    check(_native.lib().vrhip_comm_unique_id(buf), "vrhip_comm_unique_id")
    return bytes(buf)


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = _native.lib().vrhip_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0
