"""ctypes binding of libvrhip.so (the C ABI in include/vrhip.h).

There is no fallback: if the HIP library is missing or fails to load, every
entry point raises.  torch is imported first when available so that the
process shares ONE HIP runtime (torch ships its own libamdhip64 with the same
soname; loading ours first would pull in a second copy).
"""
from __future__ import annotations

import ctypes
import os
import re

from . import build as _build

try:  # share torch's HIP runtime if torch is in use
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the C ABI
    torch = None

_f = ctypes.POINTER(ctypes.c_float)
_u8 = ctypes.POINTER(ctypes.c_uint8)
_u16 = ctypes.POINTER(ctypes.c_uint16)
_u32 = ctypes.POINTER(ctypes.c_uint32)
_sz = ctypes.POINTER(ctypes.c_size_t)
_vp = ctypes.c_void_p
_ctx = ctypes.c_void_p

VRHIP_OK = 0
ERRORS = {-1: "VRHIP_ERR_INVALID", -2: "VRHIP_ERR_HIP", -3: "VRHIP_ERR_NO_ENV", -4: "VRHIP_ERR_BVH",
          -5: "VRHIP_ERR_NO_DEVICE", -6: "VRHIP_ERR_NOMEM",
          -7: "VRHIP_ERR_COMM"}

_SIGNATURES = {
    "vrhip_last_error": (ctypes.c_char_p, []),
    "vrhip_abi_version": (ctypes.c_int, []),
    "vrhip_build_id": (ctypes.c_char_p, []),
    "vrhip_service_info": (ctypes.c_int, [_ctx, ctypes.POINTER(ctypes.c_uint64)]),
    "vrhip_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "vrhip_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(_ctx)]),
    "vrhip_destroy": (ctypes.c_int, [_ctx]),
    "vrhip_create_multi": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.POINTER(_ctx)]),
    "vrhip_device_group": (ctypes.c_int, [_ctx, _u32, ctypes.POINTER(ctypes.c_int)]),
    "vrhip_set_stream": (ctypes.c_int, [_ctx, _vp]),
    "vrhip_get_stream": (_vp, [_ctx]),
    "vrhip_set_camera": (ctypes.c_int, [_ctx, _f, _f, _f, _f, ctypes.c_float]),
    "vrhip_clear": (ctypes.c_int, [_ctx]),
    "vrhip_set_fresnel": (ctypes.c_int, [_ctx, ctypes.c_float, ctypes.c_float]),
    "vrhip_use_cornell_box": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "vrhip_use_example_sphere": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "vrhip_use_brdf": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "vrhip_set_strict_traversal": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "vrhip_upload_mesh_flat": (ctypes.c_int, [_ctx, _f, ctypes.c_size_t, _f, _f, _f, _f, ctypes.c_size_t]),
    "vrhip_upload_mesh_indexed": (ctypes.c_int, [_ctx, _f, _f, _f, _f, ctypes.c_uint32, _u32, ctypes.c_uint32,
                                                 ctypes.c_uint32]),
    "vrhip_upload_hdr": (ctypes.c_int, [_ctx, _f, ctypes.c_uint32, ctypes.c_uint32]),
    "vrhip_upload_hdr_half": (ctypes.c_int, [_ctx, _u16, ctypes.c_uint32, ctypes.c_uint32]),
    "vrhip_upload_texture": (ctypes.c_int, [_ctx, ctypes.c_int, _f, ctypes.c_uint32, ctypes.c_uint32]),
    "vrhip_upload_brdf": (ctypes.c_int, [_ctx, _f, ctypes.c_size_t]),
    "vrhip_load_merl": (ctypes.c_int, [ctypes.c_char_p, _f, ctypes.c_size_t]),
    "vrhip_load_exr": (ctypes.c_int, [ctypes.c_char_p, _u16, ctypes.c_size_t, _u32, _u32]),
    "vrhip_gl_register_image": (ctypes.c_int, [_ctx, ctypes.c_int, ctypes.c_uint, ctypes.c_uint]),
    "vrhip_gl_present": (ctypes.c_int, [_ctx]),
    "vrhip_render": (ctypes.c_int, [_ctx, ctypes.c_uint32, _u32, ctypes.c_uint32]),
    "vrhip_render_counted": (ctypes.c_int, [_ctx, ctypes.c_uint32, _u32, ctypes.c_uint32,
                                            ctypes.POINTER(ctypes.c_uint64)]),
    "vrhip_render_profiled": (ctypes.c_int, [_ctx, ctypes.c_uint32, _u32, ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint64)]),
    "vrhip_microbench_vmem": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_double)]),
    "vrhip_kernel_stats": (ctypes.c_int, [_ctx, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64),
                                          ctypes.c_int]),
    "vrhip_debug_counters": (ctypes.c_int, [_ctx, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "vrhip_sync": (ctypes.c_int, [_ctx]),
    "vrhip_set_path_split": (ctypes.c_int, [_ctx, ctypes.c_uint32]),
    "vrhip_set_overlap": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "vrhip_frame_count": (ctypes.c_int, [_ctx, _u32]),
    "vrhip_read_accum": (ctypes.c_int, [_ctx, _f]),
    "vrhip_read_rgba8": (ctypes.c_int, [_ctx, _u8]),
    "vrhip_read_depth8": (ctypes.c_int, [_ctx, _u8]),
    "vrhip_device_buffers": (ctypes.c_int, [_ctx, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp)]),
    "vrhip_set_tiling": (ctypes.c_int, [_ctx, ctypes.c_uint32, ctypes.c_uint32]),
    "vrhip_owned_pixels": (ctypes.c_int, [_ctx, _u32]),
    "vrhip_tile_pixels": (ctypes.c_int, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _u32,
                                         _u32]),
    "vrhip_pack_tiles": (ctypes.c_int, [_ctx, ctypes.c_int, _vp]),
    "vrhip_unpack_tiles": (ctypes.c_int, [_ctx, ctypes.c_int, _vp, ctypes.c_uint32, ctypes.c_size_t]),
    "vrhip_comm_unique_id": (ctypes.c_int, [_u8]),
    "vrhip_comm_init": (ctypes.c_int, [_ctx, ctypes.c_uint32, ctypes.c_uint32, _u8]),
    "vrhip_comm_gather": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "vrhip_comm_destroy": (ctypes.c_int, [_ctx]),
    "vrhip_last_kernel_ms": (ctypes.c_int, [_ctx, _f]),
    "vrhip_last_launch_info": (ctypes.c_int, [_ctx, _u32, _u32, _u32]),
    "vrhip_set_service": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "vrhip_set_kernel_timing": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "vrhip_set_sync_flag": (ctypes.c_int, [_ctx, ctypes.c_int]),
    "vrhip_sync_info": (ctypes.c_int, [_ctx, ctypes.POINTER(ctypes.c_uint64)]),
    "vrhip_set_service_timing": (ctypes.c_int, [_ctx, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "vrhip_service_stats": (ctypes.c_int, [_ctx, ctypes.POINTER(ctypes.c_uint64)]),
    "vrhip_set_service_budget": (ctypes.c_int, [_ctx, ctypes.c_size_t]),
    "vrhip_bvh_info": (ctypes.c_int, [_ctx, _u32, _u32, _u32]),
    "vrhip_selftest_math": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _f, _f, _f, ctypes.c_size_t]),
    "vrhip_selftest_rcp": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.POINTER(ctypes.c_uint64), _u32]),
    "vrhip_selftest_tonemap": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.POINTER(ctypes.c_uint64), _u32]),
    "vrhip_selftest_sqrt": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.POINTER(ctypes.c_uint64), _u32]),
    "vrhip_build_flat": (ctypes.c_int, [_f, _f, _f, _f, ctypes.c_uint32, _u32, ctypes.c_uint32, ctypes.c_uint32,
                                        _f, _sz, _f, _f, _f, _f, _sz]),
    "vrhip_validate_flat": (ctypes.c_int, [_f, ctypes.c_size_t, _f, ctypes.c_size_t, _u32, _u32]),
}

_lib = None


class VRHIPError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: {ERRORS.get(code, code)}: {msg}")
        self.code = code


def header_symbols() -> list[str]:
    """Function names declared in include/vrhip.h."""
    hdr = os.path.join(_build.REPO_DIR, "include", "vrhip.h")
    text = open(hdr).read()
    return sorted(set(re.findall(r"\b(vrhip_[a-z0-9_]+)\s*\(", text)))


def lib():
    global _lib
    if _lib is None:
        path = os.environ.get("VRHIP_LIB", _build.LIB_PATH)   # VRHIP_LIB: A/B builds of the same ABI
        if path == _build.LIB_PATH and os.path.exists(path) and _build.needs_build():
            # built from other sources than those on disk (its embedded
            # vrhip_build_id differs): rebuild so what runs is what is checked in
            _build.build()
        if not os.path.exists(path):
            raise RuntimeError(f"libvrhip.so not built ({path}); run vrenderer_pathtracer_amd.build.build()")
        L = ctypes.CDLL(path)
        for name, (res, args) in _SIGNATURES.items():
            if path != _build.LIB_PATH and not hasattr(L, name):
                continue   # an older A/B build may predate a diagnostics entry point
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def build_id() -> dict:
    """The loaded library's embedded build id (vrhip_build_id) and whether it
    equals the SHA-256 of the sources and flags on disk."""
    got = lib().vrhip_build_id().decode()
    path = os.environ.get("VRHIP_LIB", _build.LIB_PATH)
    return {"build_id": got, "matches_sources": got == _build.source_id(),
            "lib": os.path.relpath(path, _build.REPO_DIR)}


def check(code: int, where: str) -> None:
    if code != VRHIP_OK:
        msg = lib().vrhip_last_error()
        raise VRHIPError(code, where, msg.decode() if msg else "")


def fptr(a):
    return None if a is None else a.ctypes.data_as(_f)
