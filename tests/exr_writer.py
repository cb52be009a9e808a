"""Test helper: writes single-part scanline OpenEXR files (NONE, RLE, ZIPS,
ZIP) following the OpenEXR file layout, for the vrhip_load_exr tests.  No
OpenEXR library or sample .exr exists in this environment (the reference's
hdr/ assets are git-ignored), so the reader is pinned only against this
independent writer of the published format."""
import struct
import zlib

import numpy as np

_LINES = {0: 1, 1: 1, 2: 1, 3: 16}


def _attr(name, typ, data):
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data


def _predict_interleave(raw: bytes) -> bytes:
    b = np.frombuffer(raw, np.uint8)
    t = np.concatenate([b[0::2], b[1::2]])                 # even bytes first, then odd
    d = t.astype(np.int16).copy()
    d[1:] = (t[1:].astype(np.int16) - t[:-1].astype(np.int16) + 128 + 256) % 256
    return d.astype(np.uint8).tobytes()


def _rle(data: bytes) -> bytes:
    out = bytearray()
    i, n = 0, len(data)
    while i < n:
        run = 1
        while i + run < n and data[i + run] == data[i] and run < 128:
            run += 1
        if run >= 3:
            out += struct.pack("<b", run - 1) + data[i:i + 1]
            i += run
        else:
            j = i
            while j < n and j - i < 127:
                if j + 2 < n and data[j] == data[j + 1] == data[j + 2]:
                    break
                j += 1
            out += struct.pack("<b", -(j - i)) + data[i:j]
            i = j
    return bytes(out)


def write_exr(path, rgba, channels="RGBA", pixel_type=1, compression=0, origin=(0, 0)):
    """rgba: float array (H, W, 4); writes the named channels of it."""
    h, w = rgba.shape[:2]
    names = sorted(channels)
    chl = b""
    for c in names:
        chl += c.encode() + b"\0" + struct.pack("<iBBBBii", pixel_type, 0, 0, 0, 0, 1, 1)
    chl += b"\0"
    x0, y0 = origin
    box = struct.pack("<iiii", x0, y0, x0 + w - 1, y0 + h - 1)
    head = struct.pack("<II", 20000630, 2)
    head += _attr("channels", "chlist", chl)
    head += _attr("compression", "compression", bytes([compression]))
    head += _attr("dataWindow", "box2i", box)
    head += _attr("displayWindow", "box2i", box)
    head += _attr("lineOrder", "lineOrder", b"\0")
    head += _attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
    head += _attr("screenWindowCenter", "v2f", struct.pack("<ff", 0.0, 0.0))
    head += _attr("screenWindowWidth", "float", struct.pack("<f", 1.0))
    head += b"\0"
    lpb = _LINES[compression]
    n_chunks = (h + lpb - 1) // lpb
    dt = np.float16 if pixel_type == 1 else np.float32
    chunks = []
    for c in range(n_chunks):
        lines = range(c * lpb, min(h, (c + 1) * lpb))
        raw = b""
        for y in lines:
            for name in names:
                raw += rgba[y, :, "RGBA".index(name)].astype(dt).tobytes()
        if compression == 0:
            data = raw
        elif compression == 1:
            data = _rle(_predict_interleave(raw))
        else:
            data = zlib.compress(_predict_interleave(raw))
        if len(data) >= len(raw):
            data = raw                                   # OpenEXR stores a chunk raw when packing does not help
        chunks.append(struct.pack("<ii", y0 + c * lpb, len(data)) + data)
    off = len(head) + 8 * n_chunks
    table = b""
    for ch in chunks:
        table += struct.pack("<Q", off)
        off += len(ch)
    with open(path, "wb") as f:
        f.write(head + table + b"".join(chunks))
