"""vrenderer_pathtracer_amd -- MI355X-native progressive path-tracing backend.

The product is libvrhip.so (HIP for gfx950 behind the C ABI in
include/vrhip.h).  This package is the thin Python host mirror of the
reference's vRenderer interface (renderer.VRendererHIP), the procedural
scenes used by the benchmark and tests, and the build script.
"""
from .build import build as build_native, LIB_PATH  # noqa: F401
from .renderer import (VRendererHIP, Camera, build_flat, validate_flat, selftest_math, selftest_rcp, selftest_sqrt, selftest_tonemap, load_merl, load_exr,  # noqa: F401
                       device_count, microbench_vmem, DIFFUSE, NORMAL, SPECULAR)
from ._native import VRHIPError, build_id  # noqa: F401

__all__ = ["VRendererHIP", "Camera", "build_flat", "validate_flat", "selftest_math", "selftest_rcp", "selftest_sqrt", "selftest_tonemap", "device_count", "microbench_vmem",
           "build_native", "VRHIPError", "DIFFUSE", "NORMAL", "SPECULAR", "LIB_PATH"]
