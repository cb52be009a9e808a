"""The C++ vRendererHIP adapter (integration/) against the vRenderer interface.

CPU: compiles and links against libvrhip.so with stand-ins for the Qt/GL/EXR
types (tests/stubs).  GPU: a driver renders 3 frames through the interface
(init, register*, setCamera, useCornellBox, useExampleSphere, setFresnel*,
render, getFrameCount) and its colour texture must equal the oracle's RGBA8.
"""
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "vrenderer_pathtracer_amd")


def _build_driver(tmp_path):
    exe = str(tmp_path / "adapter_driver")
    cmd = ["g++", "-std=c++14", "-O1", "-Wall", "-I", os.path.join(REPO, "tests", "stubs"),
           "-I", os.path.join(REPO, "include"), "-I", os.path.join(REPO, "integration"),
           os.path.join(REPO, "tests", "adapter_driver.cpp"), os.path.join(REPO, "integration", "vRendererHIP.cpp"),
           "-L", PKG, "-lvrhip", f"-Wl,-rpath,{PKG}", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_adapter_compiles_and_links(native, tmp_path):
    exe = _build_driver(tmp_path)
    assert os.path.exists(exe)


@pytest.mark.gpu
def test_adapter_renders_like_oracle(native, oracle, tmp_path):
    exe = _build_driver(tmp_path)
    out = str(tmp_path / "out.bin")
    env = dict(os.environ, VRHIP_FIXED_TIME="12345")
    subprocess.run([exe, out], check=True, env=env, timeout=120)
    raw = open(out, "rb").read()
    frames = int(np.frombuffer(raw[:4], np.uint32)[0])
    rgba = np.frombuffer(raw[4:], np.uint8).reshape(64, 64, 4)
    from vrenderer_pathtracer_amd import scenes
    sc = scenes.make_scene("C1", 64, 64)
    _, ref, _, _ = oracle.render(sc, frames=3, times=[12345] * 3, libm=oracle.LIBM_PORTABLE)
    assert frames == 3
    assert np.array_equal(rgba, ref)
