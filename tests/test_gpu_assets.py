"""Assets through their loaders into a GPU render (the reference's ingestion
paths, then the kernel), and the display-interop entry points without a GL
context.

  * HDRI: an OpenEXR half-RGBA file (NGLScene::loadHDRMap, src/NGLScene.cpp:
    205-231) -> vrhip_load_exr -> loadHDR (half, converted on the device) ->
    C3 render == the render of the same environment uploaded as float4.
  * MERL: a .binary file (vBRDFLoader::loadBinary, src/BRDFLoader.cpp:15-50)
    -> vrhip_load_merl -> loadBRDF -> C4 render == the in-memory table's.
  * GL interop (src/vRendererCuda.cpp:57-67): no GL context exists on the
    GPU box (no EGL / X server in the image), so registering a texture must
    fail with a status code and leave the context rendering exactly as before.
No OpenEXR sample or MERL measurement exists in this environment (the
reference's assets are git-ignored), so the files are written here: by
tests/exr_writer.py (an independent writer of the published EXR layout, ZIP
compression) and in the MERL layout (3 int32 dims, then doubles).
"""
import numpy as np
import pytest

from vrenderer_pathtracer_amd import VRendererHIP, load_exr, load_merl, scenes, VRHIPError

pytestmark = pytest.mark.gpu


def _render(sc, frames=2):
    r = VRendererHIP(0)
    scenes.load_into(r, sc)
    r.render(frames=frames, times=[sc["time"] + i for i in range(frames)])
    out = r.read_accum(), r.read_rgba8()
    r.cleanUp()
    return out


def test_exr_file_to_render(native, tmp_path):
    from exr_writer import write_exr
    sc = scenes.make_scene("C3", 128, 96)
    f = tmp_path / "env.exr"
    write_exr(f, sc["hdr"], channels="RGBA", pixel_type=1, compression=3)   # ZIP, half
    half = load_exr(f)
    assert half.shape == sc["hdr"].shape
    assert np.array_equal(half.astype(np.float32), sc["hdr"])              # the procedural map is half-exact
    base = _render(sc)
    sc2 = dict(sc, hdr=half)                                               # uploaded as half, widened on the GPU
    got = _render(sc2)
    assert np.array_equal(got[0].view(np.uint32), base[0].view(np.uint32))
    assert np.array_equal(got[1], base[1])


def test_merl_file_to_render(native, tmp_path):
    sc = scenes.make_scene("C4", 96, 64)
    table = sc["brdf"]
    f = tmp_path / "synthetic.binary"
    with open(f, "wb") as fh:
        fh.write(np.array([90, 90, 180], np.int32).tobytes())
        fh.write(table.astype(np.float64).tobytes())
    loaded = load_merl(f)
    assert np.array_equal(loaded, table)
    base = _render(sc)
    got = _render(dict(sc, brdf=loaded))
    assert np.array_equal(got[0].view(np.uint32), base[0].view(np.uint32))


_GL_CHILD = r"""
import sys, json, hashlib, numpy as np
sys.path.insert(0, {repo!r})
import torch
from vrenderer_pathtracer_amd import VRendererHIP, scenes, _native
sc = scenes.make_scene("C2", 64, 48)
r = VRendererHIP(0)
scenes.load_into(r, sc)
L = _native.lib()
rc = L.vrhip_gl_register_image(r._ctx, 0, 1, 0x0DE1)     # GL_TEXTURE_2D, texture 1, no current context
rc_bad = L.vrhip_gl_register_image(r._ctx, 2, 1, 0x0DE1)  # bad `which`
rc_present = L.vrhip_gl_present(r._ctx)                  # nothing registered: a no-op
r.render(frames=2, times=[sc["time"], sc["time"] + 1])
acc = r.read_accum()
r.cleanUp()
print(json.dumps(dict(rc=rc, rc_bad=rc_bad, rc_present=rc_present,
                      h=hashlib.sha256(acc.tobytes()).hexdigest())))
"""


def test_gl_register_without_context_fails_cleanly(native):
    """In a child process (the HIP runtime's GL path must not take the test
    run down if it misbehaves): registration fails with a status code, present
    is a no-op, and the context then renders the same bits as one that never
    tried."""
    import json
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, "-c", _GL_CHILD.format(repo=repo)], capture_output=True, text=True,
                         timeout=180)
    assert res.returncode == 0, res.stderr[-2000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out["rc"] != 0 and out["rc_bad"] == -1 and out["rc_present"] == 0
    sc = scenes.make_scene("C2", 64, 48)
    base = _render(sc)
    import hashlib
    assert out["h"] == hashlib.sha256(np.ascontiguousarray(base[0]).tobytes()).hexdigest()
