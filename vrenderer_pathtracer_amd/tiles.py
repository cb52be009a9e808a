"""Image-tile sharding across the GPUs of one node.

The reference is single-GPU; its RNG seeds depend only on global pixel
coordinates, frame and time (cuda/src/PathTracer.cu:817-818), so any
partition of the pixels renders the same image bit for bit.  Partition:
16x16 tiles (the reference's block, PathTracer.cu:887) dealt round-robin to
ranks along a row-rotated tile order (row y's tiles start at column y mod
tiles_x; include/vrhip.h vrhip_set_tiling), so ranks own equal tile counts
(+-1) in diagonals spread over the whole image (sky vs mesh load balance).  Each rank keeps its own
float4 accumulation resident; after every accumulation step the ranks' RGBA8
tiles (or float4 accumulation, for parity read-out) are gathered to rank 0
with ONE collective (ncclGather over xGMI inside libvrhip.so,
vrhip_comm_gather; gloo through host memory for one-GPU rehearsals) and
scattered back into image order on the device.
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

    backend "nccl" (the measured configuration, one rank per GPU): the
    library's own RCCL communicator -- rank 0 draws the id
    (vrhip_comm_unique_id), torch.distributed only hands it to the other
    ranks, and every step is vrhip_comm_gather (pack, ncclGather, unpack on
    rank 0, enqueued on the renderer's stream -- or, in explicit service mode
    (renderer.set_service(1)) while a render-service session is open,
    deferred to the session's close, i.e. to the next call that closes it
    (include/vrhip.h lists them): call renderer.sync() before any host-side
    barrier with the other ranks, as bench.py does, or a rank whose gather is
    still deferred never joins the collective; the automatic mode never
    defers).  backend "gloo" (a CPU/one-GPU
    rehearsal of the multi-rank path with several ranks sharing a device,
    which RCCL refuses): packed buffers staged through host memory and
    gathered by torch.distributed.
    """

    def __init__(self, renderer, rank: int, world: int, device, what: int = WHAT_RGBA8):
        self.r, self.rank, self.world, self.what = renderer, rank, world, what
        self.device = device
        self.native = False
        if world == 1:
            return
        import torch
        import torch.distributed as dist
        if dist.get_backend() != "gloo":
            from .renderer import COMM_ID_BYTES, comm_unique_id
            uid = torch.zeros(COMM_ID_BYTES, dtype=torch.uint8, device=device)
            if rank == 0:
                uid.copy_(torch.frombuffer(bytearray(comm_unique_id()), dtype=torch.uint8))
            dist.broadcast(uid, src=0)
            renderer.comm_init(rank, world, bytes(uid.cpu().numpy().tobytes()))
            self.native = True
            return
        H, W = renderer.height, renderer.width
        self.stride = max_owned_pixels(W, H, world) * _ELEM_BYTES[what]
        self.send = torch.empty(self.stride, dtype=torch.uint8, device=device)
        self.recv = None
        if rank == 0:
            self.recv = torch.empty(world * self.stride, dtype=torch.uint8, device=device)
            self.recv_stage = self.recv.cpu()
            self.views = list(self.recv_stage.view(world, self.stride).unbind(0))

    def step(self) -> None:
        if self.world == 1:
            return
        if self.native:
            self.r.comm_gather(self.what)
            return
        import torch
        import torch.distributed as dist
        torch.cuda.current_stream(self.device).synchronize()
        self.r.pack_tiles(self.what, self.send.data_ptr())
        self.r.sync()                          # the packed tiles are complete before the host copy
        dist.gather(self.send.cpu(), self.views if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            self.recv.copy_(self.recv_stage)
            torch.cuda.current_stream(self.device).synchronize()
            self.r.unpack_tiles(self.what, self.recv.data_ptr(), self.world, self.stride)

    def close(self) -> None:
        if self.native:
            self.r.comm_destroy()
            self.native = False
