"""Image-tile sharding across the GPUs of one node.

The reference is single-GPU; its RNG seeds depend only on global pixel
coordinates, frame and time (cuda/src/PathTracer.cu:817-818), so any
partition of the pixels renders the same image bit for bit.  Partition:
16x16 tiles (the reference's block, PathTracer.cu:887) dealt round-robin to
ranks in row-major tile order, so ranks own equal tile counts (+-1) spread
over the whole image (sky vs mesh load balance).  Each rank keeps its own
float4 accumulation resident; after every accumulation step the ranks' RGBA8
tiles (or float4 accumulation, for parity read-out) are gathered to rank 0
with ONE collective (torch.distributed "nccl" = RCCL over xGMI, or gloo on
CPU) and scattered back into image order on the device.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native
from ._native import check

WHAT_RGBA8, WHAT_ACCUM, WHAT_DEPTH8 = 0, 1, 2
_ELEM_BYTES = {WHAT_RGBA8: 4, WHAT_ACCUM: 16, WHAT_DEPTH8: 4}


def owned_pixels(width: int, height: int, rank: int, n_ranks: int) -> np.ndarray:
    """Linear pixel indices (y*W + x) owned by `rank`, in packed order (C ABI vrhip_tile_pixels)."""
    L = _native.lib()
    n = ctypes.c_uint32(0)
    check(L.vrhip_tile_pixels(width, height, rank, n_ranks, None, ctypes.byref(n)), "vrhip_tile_pixels")
    out = np.zeros(n.value, np.uint32)
    check(L.vrhip_tile_pixels(width, height, rank, n_ranks, out.ctypes.data_as(_native._u32), ctypes.byref(n)),
          "vrhip_tile_pixels")
    return out


def max_owned_pixels(width: int, height: int, n_ranks: int) -> int:
    tiles = (width // 16) * (height // 16)
    return ((tiles + n_ranks - 1) // n_ranks) * 256


def pack_host(image: np.ndarray, rank: int, n_ranks: int) -> np.ndarray:
    """Host-side packing of a rank's tiles (the device does this with vrhip_pack_tiles).
    image: [H, W, ...] -> [n_owned_pixels, ...]."""
    H, W = image.shape[:2]
    flat = image.reshape(H * W, *image.shape[2:])
    return np.ascontiguousarray(flat[owned_pixels(W, H, rank, n_ranks)])


def unpack_host(packed: list, out: np.ndarray) -> np.ndarray:
    """Scatter per-rank packed pixels back into image order (device: vrhip_unpack_tiles).
    out: [H, W, ...] image, updated in place."""
    n = len(packed)
    H, W = out.shape[:2]
    flat = out.reshape(H * W, *out.shape[2:])
    for r, buf in enumerate(packed):
        pix = owned_pixels(W, H, r, n)
        flat[pix] = buf[:len(pix)]
    return out


class TileGather:
    """Per-step gather of every rank's tiles to rank 0 with one collective.

    renderer: VRendererHIP with set_tiling(rank, world) applied; torch tensors
    hold the send/receive buffers on the renderer's device so the collective
    runs over RCCL (backend "nccl"); rank 0's renderer receives the full
    image.  With the gloo backend (CPU rehearsal of the multi-rank path on one
    GPU) the buffers are staged through host memory.
    """

    def __init__(self, renderer, rank: int, world: int, device, what: int = WHAT_RGBA8):
        import torch
        import torch.distributed as dist
        self.r, self.rank, self.world, self.what = renderer, rank, world, what
        self.device = device
        H, W = renderer.height, renderer.width
        self.stride = max_owned_pixels(W, H, world) * _ELEM_BYTES[what]
        self.send = torch.empty(self.stride, dtype=torch.uint8, device=device)
        self.recv = None
        self.host = world > 1 and dist.get_backend() == "gloo"
        if rank == 0 and world > 1:
            self.recv = torch.empty(world * self.stride, dtype=torch.uint8, device=device)
            views = self.recv.cpu() if self.host else self.recv
            self.recv_stage = views
            self.views = list(views.view(world, self.stride).unbind(0))

    def step(self) -> None:
        import torch
        import torch.distributed as dist
        if self.world == 1:
            return
        own_stream = self.r.get_stream() != torch.cuda.current_stream(self.device).cuda_stream
        if own_stream:
            torch.cuda.current_stream(self.device).synchronize()   # the last collective has read `send`
        self.r.pack_tiles(self.what, self.send.data_ptr())
        if own_stream or self.host:
            self.r.sync()                     # the collective reads `send` on torch's stream
        send = self.send.cpu() if self.host else self.send
        dist.gather(send, self.views if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            if self.host:
                self.recv.copy_(self.recv_stage)
            if own_stream or self.host:
                torch.cuda.current_stream(self.device).synchronize()
            self.r.unpack_tiles(self.what, self.recv.data_ptr(), self.world, self.stride)
