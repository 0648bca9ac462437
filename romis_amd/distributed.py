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
    """Renders this rank's tile of successive frames (restir_halo_begin .. restir_halo_end).

    transport "torch" (default): torch.distributed batch_isend_irecv on device tensors (nccl) or host tensors
    (gloo, the CPU / single-GPU tests); the pass's interior is issued before the exchange and runs on the GPU while
    the host drives it, the border strips after the unpack.  transport "native" (opt-in, nccl backend): the
    library's own RCCL communicator moves the halo on a communication stream while the pass's interior runs
    (restir_halo_pass) -- no host round trip, no device synchronisation; the library checks that the
    communicator's rank and size match the tile plan.  bench.py --mode halo --halo-transport native selects it."""

    def __init__(self, renderer: "restir.Renderer", width: int, height: int, tiles: tuple, rank: int, features,
                 group=None, transport: str | None = None, layout=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.r = renderer
        self.W, self.H, self.tiles, self.rank, self.f = width, height, tuple(tiles), rank, features
        self.group = group
        # layout: an uneven tile layout (restir.layout_balanced; every rank must pass the same one), else the even split
        if layout is not None and (layout.tiles_x, layout.tiles_y) != self.tiles:
            raise ValueError(f"HaloFrames: a {layout.tiles_x}x{layout.tiles_y} layout for {tiles[0]}x{tiles[1]} tiles")
        self.layout = layout
        self.passes = features.spatial_resampling_passes if features.spatial_reuse else 0
        radius = features.spatial_resample_radius
        self.tile = restir.tile_plan(width, height, tiles[0], tiles[1], rank, radius if self.passes else 0, layout=layout)
        self.send, self.recv = restir.halo_plan(width, height, tiles[0], tiles[1], rank, radius,
                                                features.num_samples_in_reservoir, layout=layout)
        if dist.get_rank(group) != rank or dist.get_world_size(group) != tiles[0] * tiles[1]:
            raise ValueError(f"HaloFrames: rank {rank} of a {tiles[0]}x{tiles[1]} tile plan, but the group's rank is "
                             f"{dist.get_rank(group)} of {dist.get_world_size(group)}: the halo peers are tile ranks")
        self.on_device = dist.get_backend(group) == "nccl"
        self.transport = transport or "torch"
        if self.transport not in ("torch", "native", "record"):
            raise ValueError(f"HaloFrames: unknown transport {self.transport!r}")
        if self.transport == "record":
            # the native pass without RCCL (restir_halo_record): every step it would issue is logged, nothing moves
            # (zeroed receive buffers) -- the plumbing check of tests/test_gpu_halo.py, not a valid frame
            self.r.halo_record(True)
            return
        # any other transport renders real frames: leave a record-only mode an earlier HaloFrames("record") set on this
        # renderer (the native attach below also clears it in the library)
        self.r.halo_record(False)
        if self.transport == "native":
            # one rank draws the communicator id, every rank receives it over the torch group; its last byte says
            # whether rank 0 could draw one, so that every rank fails together (never some ranks waiting inside a
            # collective the others left)
            n_id = restir._abi.RESTIR_RCCL_ID_BYTES
            idt = torch.zeros(n_id + 1, dtype=torch.uint8)
            if dist.get_rank(group) == 0:
                try:
                    idt[:n_id] = torch.frombuffer(bytearray(restir.rccl_unique_id()), dtype=torch.uint8)
                    idt[n_id] = 1
                except restir._abi.RestirError:
                    pass
            dev = torch.device("cuda", torch.cuda.current_device()) if self.on_device else torch.device("cpu")
            idt = idt.to(dev)
            dist.broadcast(idt, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
            host = idt.cpu()
            if int(host[n_id]) != 1:
                raise restir._abi.RestirError("HaloFrames: RCCL unavailable on rank 0 (native transport)")
            err = None
            try:   # ncclCommInitRank: every rank joins the same communicator
                self.r.halo_attach_rccl(bytes(host[:n_id].numpy().tobytes()), dist.get_world_size(group),
                                        dist.get_rank(group))
            except restir._abi.RestirError as e:
                err = e
            ok = torch.tensor([0 if err else 1], dtype=torch.int32, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)
            if int(ok.item()) != 1:
                raise err or restir._abi.RestirError("HaloFrames: the RCCL communicator failed on another rank")
            return
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
            # the received bytes are complete before the library's stream reads them: wait for torch's current
            # stream only (req.wait() ordered it behind the transfer), not the whole device -- the pass's interior
            # launch on the library's stream keeps running
            self.torch.cuda.current_stream().synchronize()

    def render(self, prev, camera, want_rgb: bool = True, want_grid: bool = True):
        """One frame: (rgb of the owned tile [h][w][3], row 0 = top, or None; ReservoirGrid for temporal reuse)."""
        sb, rb = self.r.halo_begin(prev, camera, self.W, self.H, self.f, self.tiles, self.rank, layout=self.layout)
        if self.transport in ("native", "record"):
            for _ in range(self.passes):
                self.r.halo_pass()
            return self.r.halo_end(self.tile, want_rgb, want_grid)
        host = not self.on_device
        for _ in range(self.passes):
            self.r.halo_pack(self.sendbuf.data_ptr(), sb, host)
            self.r.halo_spatial_interior()   # runs on the GPU while the exchange below is in flight
            self._exchange()
            self.r.halo_unpack(self.recvbuf.data_ptr(), rb, host)
            self.r.halo_spatial_border()
        return self.r.halo_end(self.tile, want_rgb, want_grid)


def tile_mismatches(mine, other, group=None) -> int:
    """Bit-for-bit comparison of two renderings of this rank's tile (float32 arrays of one shape), summed over the
    group's ranks: the number of 32-bit words that differ anywhere (a shape mismatch counts every word)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    a = np.ascontiguousarray(mine, dtype=np.float32)
    b = np.ascontiguousarray(other, dtype=np.float32)
    n = int((a.view(np.uint32) != b.view(np.uint32)).sum()) if a.shape == b.shape else max(a.size, b.size, 1)
    if not dist.is_initialized():
        return n
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    t = torch.tensor([n], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return int(t.item())


def exchange_probe(send, recv, group=None, iters: int = 20) -> float:
    """Microseconds of one halo exchange -- the plan's segments (restir_halo_plan: the bytes and peers a spatial pass
    moves) as one batch of torch.distributed point-to-point transfers on device buffers (nccl = RCCL over xGMI;
    host buffers under gloo) -- median of `iters`, max over the group's ranks.  The pass itself overlaps this with
    the interior launch; this is the transfer alone."""
    import statistics
    import time

    import torch
    import torch.distributed as dist
    on_dev = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_dev else torch.device("cpu")
    sb = torch.zeros(max(1, sum(s.bytes for s in send)), dtype=torch.uint8, device=dev)
    rb = torch.zeros(max(1, sum(r.bytes for r in recv)), dtype=torch.uint8, device=dev)

    def once():
        ops = []
        for s, r in zip(send, recv):
            ops.append(dist.P2POp(dist.isend, sb[s.offset:s.offset + s.bytes], s.rank, group))
            ops.append(dist.P2POp(dist.irecv, rb[r.offset:r.offset + r.bytes], r.rank, group))
        if ops:
            for q in dist.batch_isend_irecv(ops):
                q.wait()
        if on_dev:
            torch.cuda.current_stream().synchronize()

    once()
    times = []
    for _ in range(iters):
        dist.barrier(group=group)
        t0 = time.perf_counter()
        once()
        times.append(time.perf_counter() - t0)
    us = statistics.median(times) * 1e6
    t = torch.tensor([us], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())
