"""Build the native backend in-tree: libvrhip.so (HIP, gfx950) via hipcc.

The product is a C-ABI shared library (include/vrhip.h); Python only loads it
with ctypes.  Built in-tree so it travels with the repository snapshot.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libvrhip.so")
# the path kernels' scene specialisations are separate translation units
# (vr_spec_*.hip) so that they compile in parallel
SOURCES = ["vr_spec_generic.hip", "vr_cls_cornell_mesh.hip", "vr_cls_hdri_mesh.hip", "vr_spec_c2.hip", "vr_spec_c3.hip", "vr_spec_c5.hip", "vr_spec_c1.hip",
           "vr_spec_c4.hip", "vr_cls_sphere.hip", "vr_kernel.hip", "vrhip_api.cpp", "vr_bvh.cpp", "vr_exr.cpp",
           "vr_merl.cpp"]
HEADERS = ["vr_params.hpp", "vr_math.hpp", "vr_bvh.hpp", "vr_exr.hpp", "vr_merl.hpp", "vr_kernel.hpp"]
ARCH = os.environ.get("VRHIP_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: results are defined without FMA contraction (parity
# with the CPU oracle); division and sqrt stay IEEE (hipcc default).
# -packed-fp32-ops: no v_pk_{add,mul,fma}_f32.  The path kernel's float math
# comes in 3-component vectors, and pairing it costs more v_mov_b32 operand
# shuffles (and registers: C2 path kernel 111 -> 89 VGPRs) than the packed
# ops save; the kernel is VALU-issue heavy, so C2 +10 %, C3 +2.7 %, C5 +0.9 %
# (identical results: packed and scalar f32 ops round the same).
HIPCC_FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-Wall", "-pthread",
               f"--offload-arch={ARCH}", "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: cannot build libvrhip.so")


BUILD_ID_TAG = b"vrhip-build-id:"


def source_id(extra_flags=None) -> str:
    """SHA-256 of everything the library is compiled from: every source and
    header (by name and content), include/vrhip.h, and the compile flags.
    Embedded in the library (vrhip_build_id) so that a loaded or timed
    library can be tied to the sources on disk."""
    h = hashlib.sha256()
    for name in sorted(SOURCES + HEADERS):
        h.update(name.encode() + b"\0")
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(f.read())
    with open(os.path.join(REPO_DIR, "include", "vrhip.h"), "rb") as f:
        h.update(b"vrhip.h\0" + f.read())
    h.update(" ".join(HIPCC_FLAGS + list(extra_flags or [])).encode())
    return h.hexdigest()


def lib_build_id(path: str = LIB_PATH):
    """The build id embedded in a built library file (without loading it), or None."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(BUILD_ID_TAG)
    if i < 0:
        return None
    hexid = data[i + len(BUILD_ID_TAG):i + len(BUILD_ID_TAG) + 64]
    return hexid.decode("ascii", "replace")


def needs_build() -> bool:
    """The library is missing or was built from other sources / flags than
    those on disk (content hash, not modification times)."""
    return lib_build_id(LIB_PATH) != source_id()


def _jobs() -> int:
    for var in ("MAX_JOBS", "OMP_NUM_THREADS"):
        v = os.environ.get(var, "")
        if v.isdigit() and int(v) > 0:
            return min(int(v), 16)
    return max(1, min(os.cpu_count() or 1, 16))


def build(force: bool = False, verbose: bool = False, extra_flags=None, out_path: str = None) -> str:
    """Compile every source to an object in parallel (hipcc -c), then link
    libvrhip.so.  extra_flags / out_path: variant builds (scripts/build_variants.sh)."""
    out = os.path.abspath(out_path or LIB_PATH)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    if not force and out_path is None and not needs_build():
        return LIB_PATH
    import concurrent.futures
    import tempfile
    hipcc = _hipcc()
    bid = source_id(extra_flags)
    compile_flags = ([f for f in HIPCC_FLAGS if f != "-shared"] + list(extra_flags or [])
                     + [f'-DVRHIP_BUILD_ID="{BUILD_ID_TAG.decode()}{bid}"'])
    with tempfile.TemporaryDirectory(prefix="vrhip_build_") as tmpd:
        objs = [os.path.join(tmpd, os.path.splitext(s)[0] + ".o") for s in SOURCES]

        def compile_one(i):
            cmd = [hipcc] + compile_flags + ["-c", "-o", objs[i], os.path.join(CSRC, SOURCES[i])]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            return subprocess.run(cmd, capture_output=True, text=True)

        with concurrent.futures.ThreadPoolExecutor(max_workers=_jobs()) as ex:
            results = list(ex.map(compile_one, range(len(SOURCES))))
        for src, res in zip(SOURCES, results):
            if verbose and res.stderr.strip():
                print(res.stderr, file=sys.stderr)
            if res.returncode != 0:
                raise RuntimeError(f"hipcc failed on {src}:\n" + res.stdout + res.stderr)
        tmp = f"{out}.tmp{os.getpid()}"      # ranks that build at once each link their own file
        cmd = [hipcc] + HIPCC_FLAGS + list(extra_flags or []) + ["-o", tmp] + objs + ["-lz", "-lrccl"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError("hipcc link failed:\n" + res.stdout + res.stderr)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
