"""CPU AddressSanitizer + UndefinedBehaviorSanitizer run over the host code
of libvrhip.so that parses untrusted input (SURVEY.md §5 names ASan for
exactly this): the OpenEXR reader (vrhip_load_exr, vr_exr.cpp), the MERL
reader (vrhip_load_merl, vr_merl.cpp; the reference's loader is
src/BRDFLoader.cpp:15-50), the BVH builder and the flattened-tree validator
(vrhip_build_flat / vrhip_validate_flat, vr_bvh.cpp; the reference flattens in
src/vRendererCuda.cpp:204-279 and uploads in :282-317).

tests/sanitize_driver.cpp is compiled with g++ -fsanitize=address,undefined
-fno-sanitize-recover=all together with those sources (no HIP) and fed valid
files, every truncation of them, byte-flipped copies, hostile headers,
degenerate meshes and corrupted flat arrays.  Every input must be accepted or
rejected with an error -- no sanitizer report, no crash."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from exr_writer import write_exr

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "vrenderer_pathtracer_amd", "csrc")
SAN_ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("san") / "sanitize_driver")
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-pthread", "-I", CSRC, os.path.join(REPO, "tests", "sanitize_driver.cpp"),
           os.path.join(CSRC, "vr_bvh.cpp"), os.path.join(CSRC, "vr_exr.cpp"), os.path.join(CSRC, "vr_merl.cpp"),
           "-lz", "-o", out]
    res = subprocess.run(cmd, capture_output=True, text=True)
    assert res.returncode == 0, res.stderr[-3000:]
    return out


def _run(driver, *args):
    res = subprocess.run([driver, *args], capture_output=True, text=True, env=SAN_ENV, timeout=600)
    report = res.stderr
    assert "AddressSanitizer" not in report and "runtime error" not in report and "LeakSanitizer" not in report, \
        report[-4000:]
    assert res.returncode == 0, (res.returncode, report[-4000:])
    line = res.stdout.strip().splitlines()[-1]
    mode, ok, rej = line.split()
    return int(ok.split("=")[1]), int(rej.split("=")[1])


def _exr_corpus(d):
    """Valid files of every supported compression and sample type, every
    truncation of two of them, byte-flipped copies and hostile headers."""
    rng = np.random.default_rng(5)
    img = rng.random((19, 23, 4)).astype(np.float32) * 4
    valid = []
    for comp in (0, 1, 2, 3):
        for ptype in (1, 2):
            p = os.path.join(d, f"ok_c{comp}_t{ptype}.exr")
            write_exr(p, img, pixel_type=ptype, compression=comp, origin=(-3, 5))
            valid.append(p)
    p = os.path.join(d, "ok_rgb.exr")
    write_exr(p, img, channels="RGB", compression=3)
    valid.append(p)
    files = list(valid)
    for src in (valid[2], valid[7]):                       # RLE half, ZIP float: every truncation length
        data = open(src, "rb").read()
        for n in range(0, len(data), max(1, len(data) // 400)):
            q = os.path.join(d, f"trunc_{os.path.basename(src)}_{n}.exr")
            open(q, "wb").write(data[:n])
            files.append(q)
    for i in range(300):                                   # random byte flips
        data = bytearray(open(valid[i % len(valid)], "rb").read())
        for _ in range(1 + i % 4):
            data[int(rng.integers(0, len(data)))] = int(rng.integers(0, 256))
        q = os.path.join(d, f"flip_{i}.exr")
        open(q, "wb").write(bytes(data))
        files.append(q)

    def attr(name, typ, data):
        return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data
    chl = b"R\0" + struct.pack("<iBBBBii", 1, 0, 0, 0, 0, 1, 1) + b"\0"
    head = struct.pack("<II", 20000630, 2)
    hostile = {
        "huge_window": head + attr("channels", "chlist", chl) + attr("compression", "compression", b"\0")
        + attr("dataWindow", "box2i", struct.pack("<iiii", -2**31, -2**31, 2**31 - 1, 2**31 - 1)) + b"\0",
        "big_window": head + attr("channels", "chlist", chl) + attr("compression", "compression", b"\0")
        + attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, 60000, 60000)) + b"\0",
        "empty_compression": head + attr("channels", "chlist", chl) + attr("compression", "compression", b"") + b"\0",
        "short_window": head + attr("channels", "chlist", chl) + attr("compression", "compression", b"\0")
        + attr("dataWindow", "box2i", b"\1\0\0\0") + b"\0",
        "negative_attr": head + b"channels\0chlist\0" + struct.pack("<i", -5) + b"\0" * 16,
        "huge_attr": head + b"channels\0chlist\0" + struct.pack("<i", 2**31 - 1) + b"\0" * 16,
        "bad_offsets": head + attr("channels", "chlist", chl) + attr("compression", "compression", b"\0")
        + attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, 3, 1)) + b"\0"
        + struct.pack("<QQ", 2**63, 2**64 - 1),
        "chunk_outside": head + attr("channels", "chlist", chl) + attr("compression", "compression", b"\0")
        + attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, 3, 0)) + b"\0",
        "bad_chlist": head + attr("channels", "chlist", b"R\0" + b"\1\0") + b"\0",
        "subsampled": head + attr("channels", "chlist", b"R\0" + struct.pack("<iBBBBii", 1, 0, 0, 0, 0, 2, 2) + b"\0")
        + b"\0",
        "bad_magic": b"\x76\x2f\x31\x02" + b"\0" * 32,
        "tiled": struct.pack("<II", 20000630, 2 | 0x200) + b"\0" * 16,
        "empty": b"",
    }
    # a chunk whose y lies outside the window and whose size is negative
    base = hostile["chunk_outside"]
    off = len(base) + 8
    hostile["chunk_outside"] = base + struct.pack("<Q", off) + struct.pack("<ii", 2**31 - 1, 8) + b"\0" * 8
    hostile["chunk_negative"] = base + struct.pack("<Q", off) + struct.pack("<ii", 0, -8) + b"\0" * 8
    many = b"".join(f"c{i}".encode() + b"\0" + struct.pack("<iBBBBii", 1, 0, 0, 0, 0, 1, 1) for i in range(70)) + b"\0"
    hostile["many_channels"] = head + attr("channels", "chlist", many) + attr("compression", "compression", b"\0") \
        + attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, 1, 1)) + b"\0" + struct.pack("<QQ", 0, 0)
    for name, data in hostile.items():
        q = os.path.join(d, f"hostile_{name}.exr")
        open(q, "wb").write(data)
        files.append(q)
    return valid, files


def test_exr_reader_under_sanitizers(driver, tmp_path):
    valid, files = _exr_corpus(str(tmp_path))
    ok, rejected = _run(driver, "exr", *files)
    assert ok + rejected == len(files)
    assert ok >= len(valid), (ok, len(valid))
    assert rejected > len(files) // 2, (ok, rejected)


def test_merl_reader_under_sanitizers(driver, tmp_path):
    n = 90 * 90 * 180
    rng = np.random.default_rng(3)
    body = rng.random(3 * n).astype(np.float64)
    good = os.path.join(tmp_path, "good.binary")
    with open(good, "wb") as f:
        f.write(struct.pack("<iii", 90, 90, 180) + body.tobytes())
    full = open(good, "rb").read()
    files = [good]
    for i, cut in enumerate((0, 3, 11, 12, 13, 8 * n, len(full) - 1)):
        q = os.path.join(tmp_path, f"trunc_{i}.binary")
        open(q, "wb").write(full[:cut])
        files.append(q)
    for i, dims in enumerate(((90, 90, 181), (-90, -90, 180), (0, 0, 0), (2**16, 2**16, 2**16),
                              (-1, -1458000, 1), (1458000, 1, 1), (2**31 - 1, 2**31 - 1, 2))):
        q = os.path.join(tmp_path, f"dims_{i}.binary")
        open(q, "wb").write(struct.pack("<iii", *dims) + full[12:12 + 4096])
        files.append(q)
    big = os.path.join(tmp_path, "oversized.binary")            # trailing bytes are ignored, like the reference
    with open(big, "wb") as f:
        f.write(full + b"\0" * 4096)
    files.append(big)
    ok, rejected = _run(driver, "merl", *files)
    assert ok == 2 and rejected == len(files) - 2, (ok, rejected)


def test_bvh_builder_under_sanitizers(driver):
    ok, rejected = _run(driver, "bvh")
    assert ok >= 4 and rejected >= 8, (ok, rejected)


def test_flat_validator_under_sanitizers(driver):
    ok, rejected = _run(driver, "flat", "3000")
    assert ok + rejected == 3000 and rejected > 1000, (ok, rejected)
