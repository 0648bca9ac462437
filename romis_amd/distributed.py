"""Multi-GPU frames with a reservoir halo exchange over torch.distributed.

One process per GPU, each rank owning one screen tile of a tiles_x x tiles_y split.  Primary rays, RIS and
temporal reuse are pixel-local; before every spatial pass the reservoirs within r of a tile border move to the
adjacent ranks (restir_halo_plan).  With the "nccl" backend (RCCL over xGMI on MI355X) the halo buffers are
device tensors and the exchange is one batched send/recv group per pass; with "gloo" (CPU tests, one GPU
shared by several ranks) the library stages the bytes through host tensors.  Frames are bit-identical to the
same pixels of a single-GPU restir_render frame, temporal reuse included -- the ghost-zone path
(restir_render with a tile) cannot carry the predecessor's ghost zone and refuses temporal reuse on tiles.
"""
from __future__ import annotations

from . import restir


class HaloFrames:
    """Renders this rank's tile of successive frames (restir_halo_begin .. restir_halo_end)."""

    def __init__(self, renderer: "restir.Renderer", width: int, height: int, tiles: tuple, rank: int, features,
                 group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.r = renderer
        self.W, self.H, self.tiles, self.rank, self.f = width, height, tuple(tiles), rank, features
        self.group = group
        self.passes = features.spatial_resampling_passes if features.spatial_reuse else 0
        radius = features.spatial_resample_radius
        self.tile = restir.tile_plan(width, height, tiles[0], tiles[1], rank, radius if self.passes else 0)
        self.send, self.recv = restir.halo_plan(width, height, tiles[0], tiles[1], rank, radius,
                                                features.num_samples_in_reservoir)
        self.on_device = dist.get_backend(group) == "nccl"
        dev = torch.device("cuda", torch.cuda.current_device()) if self.on_device else torch.device("cpu")
        sb = sum(s.bytes for s in self.send)
        rb = sum(s.bytes for s in self.recv)
        self.sendbuf = torch.empty(max(sb, 1), dtype=torch.uint8, device=dev)
        self.recvbuf = torch.empty(max(rb, 1), dtype=torch.uint8, device=dev)

    def _exchange(self):
        dist = self.dist
        ops = []
        for s, r in zip(self.send, self.recv):
            ops.append(dist.P2POp(dist.isend, self.sendbuf[s.offset:s.offset + s.bytes], s.rank, self.group))
            ops.append(dist.P2POp(dist.irecv, self.recvbuf[r.offset:r.offset + r.bytes], r.rank, self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        if self.on_device:
            self.torch.cuda.synchronize()   # the received bytes are complete before the library's stream reads them

    def render(self, prev, camera, want_rgb: bool = True, want_grid: bool = True):
        """One frame: (rgb of the owned tile [h][w][3], row 0 = top, or None; ReservoirGrid for temporal reuse)."""
        sb, rb = self.r.halo_begin(prev, camera, self.W, self.H, self.f, self.tiles, self.rank)
        host = not self.on_device
        for _ in range(self.passes):
            self.r.halo_pack(self.sendbuf.data_ptr(), sb, host)
            self._exchange()
            self.r.halo_unpack(self.recvbuf.data_ptr(), rb, host)
            self.r.halo_spatial()
        return self.r.halo_end(self.tile, want_rgb, want_grid)
