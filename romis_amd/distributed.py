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


# Cost-balanced screen tiles.  A frame's time on a rank follows its geometry pixels (a background
# pixel misses the scene: its RIS, spatial and shading work is a shortcut); the weight of a background pixel relative
# to a geometry pixel in halo-mode frames is measured in profiles/r6/balance.json (scripts/balance_measure.py).
COST_GRID = (480, 270)       # cost cells over the image (4K: 8 x 8 px, 8K: 16 x 16 px)
BACKGROUND_WEIGHT = 0.1      # cost of a background pixel / a geometry pixel (profiles/r6/balance.json fit)
LAYOUT_ALIGN = (32, 8)       # cut granularity: whole 32-px tile columns, 8-px tile rows


def geometry_cost(renderer: "restir.Renderer", camera_fn, width: int, height: int, grid=COST_GRID,
                  background=BACKGROUND_WEIGHT):
    """The cost grid [rows (row 0 = bottom)][cols] of a width x height frame: one primary ray per cell through the
    library's own primary-ray kernel (restir_stage_primary over a grid-sized image with the same camera framing,
    camera_fn(w, h)), 1 where it hits the scene, `background` where it misses."""
    import numpy as np
    gw, gh = min(grid[0], width), min(grid[1], height)
    renderer.stage_configure(gw, gh, 1)
    renderer.stage_primary(camera_fn(gw, gh))
    n_t = renderer.download(restir._abi.BUF_GBUF_N_T)
    hit = (n_t[:, 3] < 1e30).reshape(gh, gw)   # t = FLT_MAX on a miss
    return np.where(hit, np.float32(1.0), np.float32(background)).astype(np.float32)


def cell_owners(layout, cost_shape):
    """[rows][cols] rank owning each cost cell's centre under `layout` (cell (i, j) as restir_layout_balanced maps it)."""
    import numpy as np
    ch, cw = cost_shape
    W, H = layout.global_width, layout.global_height
    cx = ((np.arange(cw) + 0.5) * W / cw).astype(np.int64)
    cy = ((np.arange(ch) + 0.5) * H / ch).astype(np.int64)
    xc = np.asarray(list(layout.x_cuts[:layout.tiles_x + 1]))
    col = np.clip(np.searchsorted(xc, cx, side="right") - 1, 0, layout.tiles_x - 1)
    own = np.zeros((ch, cw), np.int64)
    for i in range(cw):
        yc = np.asarray(list(layout.y_cuts[col[i]][:layout.tiles_y + 1]))
        row = np.clip(np.searchsorted(yc, cy, side="right") - 1, 0, layout.tiles_y - 1)
        own[:, i] = row * layout.tiles_x + col[i]
    return own


def refine_cost(cost, layout, rank_seconds):
    """The cost grid corrected by measured per-rank frame times under `layout`: every cell a rank owns is scaled by
    (the rank's share of the measured time) / (its share of the modelled cost), so that a rank whose pixels proved
    dearer than the model (specular materials, occluded lights, the visibility pass's rays) weighs more in the next
    cut.  Results do not depend on the layout (any layout is bit-identical); only the balance does."""
    import numpy as np
    t = np.asarray(rank_seconds, np.float64)
    share_t = t / t.sum()
    share_c = restir.layout_shares(layout, cost)
    scale = np.where(share_c > 0, share_t / np.maximum(share_c, 1e-12), 1.0)
    out = cost.astype(np.float64) * scale[cell_owners(layout, cost.shape)]
    return (out / out.mean()).astype(np.float32)


def _layout_buf(L, eff):
    import numpy as np
    nx, ny = restir._abi.RESTIR_MAX_TILES_X + 1, restir._abi.RESTIR_MAX_TILES_Y + 1
    buf = np.zeros(nx + restir._abi.RESTIR_MAX_TILES_X * ny + 1, np.int64)
    buf[:nx] = list(L.x_cuts)
    buf[nx:-1] = np.asarray([list(r) for r in L.y_cuts], np.int64).reshape(-1)
    buf[-1] = int(round(eff * 1e6))
    return buf


def _layout_from_buf(buf, width, height, tiles):
    nx, ny = restir._abi.RESTIR_MAX_TILES_X + 1, restir._abi.RESTIR_MAX_TILES_Y + 1
    L = restir._abi.TileLayout()
    L.global_width, L.global_height, L.tiles_x, L.tiles_y = width, height, tiles[0], tiles[1]
    for i in range(nx):
        L.x_cuts[i] = int(buf[i])
    yc = buf[nx:-1].reshape(restir._abi.RESTIR_MAX_TILES_X, ny)
    for c in range(restir._abi.RESTIR_MAX_TILES_X):
        for i in range(ny):
            L.y_cuts[c][i] = int(yc[c, i])
    return L, float(buf[-1]) / 1e6


def balanced_layout(renderer: "restir.Renderer", camera_fn, width: int, height: int, tiles: tuple, group=None,
                    align=LAYOUT_ALIGN, time_tile=None, rounds: int = 3):
    """(layout, record): rank 0 of the group measures the geometry (geometry_cost) and cuts the tiles
    (restir_layout_balanced); the cuts are broadcast, so every rank holds the same layout (once per camera).
    time_tile(layout) -> this rank's frame seconds on its tile of `layout`: then the layout and `rounds` refinements of it
    (refine_cost on rank 0 from the gathered times, new cuts broadcast) are each measured, and the layout with the best
    measured balance (mean / max of the ranks' times) is returned -- noisy or contended timings can make one refinement
    worse than the one before, and every rank sees the same gathered times, so all choose alike."""
    import numpy as np
    import torch
    import torch.distributed as dist
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    dev = torch.device("cuda", torch.cuda.current_device()) if multi and dist.get_backend(group) == "nccl" else "cpu"
    src = (dist.get_global_rank(group, 0) if group is not None else 0) if multi else 0

    def share(buf):   # rank 0's cuts to every rank: (layout, model efficiency, the buffer every rank now holds)
        if multi:
            t = torch.from_numpy(buf).to(dev)
            dist.broadcast(t, src=src, group=group)
            buf = t.cpu().numpy()
        return _layout_from_buf(buf, width, height, tiles) + (buf,)

    cost = None
    buf = np.zeros(restir._abi.RESTIR_MAX_TILES_X + 1 + restir._abi.RESTIR_MAX_TILES_X * (restir._abi.RESTIR_MAX_TILES_Y + 1)
                   + 1, np.int64)
    if rank == 0:
        cost = geometry_cost(renderer, camera_fn, width, height)
        buf = _layout_buf(*restir.layout_balanced(width, height, tiles[0], tiles[1], cost, align))
    L, eff, held = share(buf)
    rec = {"kind": "cost-balanced (restir_layout_balanced)", "model_efficiency": round(eff, 4),
           "cost_grid": list(COST_GRID), "background_weight": BACKGROUND_WEIGHT, "align": list(align), "refinement": []}
    best = None   # (measured efficiency, round, the layout's buffer)
    n = rounds + 1 if time_tile is not None else 0
    for i in range(n):
        mine = float(time_tile(L))
        times = [mine]
        if multi:
            t = torch.tensor([mine], dtype=torch.float64, device=dev)
            outs = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
            dist.all_gather(outs, t, group=group)
            times = [float(o.item()) for o in outs]
        measured = float(np.mean(times) / max(times))
        rec["refinement"].append({"cuts": L.cuts(), "rank_ms": [round(v * 1e3, 4) for v in times],
                                  "measured_efficiency": round(measured, 4)})
        if best is None or measured > best[0]:
            best = (measured, i, held.copy())
        if i + 1 < n:
            if rank == 0:
                cost = refine_cost(cost, L, times)
                buf = _layout_buf(*restir.layout_balanced(width, height, tiles[0], tiles[1], cost, align))
            L, eff, held = share(buf)
    if best is not None:
        L, _ = _layout_from_buf(best[2], width, height, tiles)
        rec["chosen_round"] = best[1]
    rec["cuts"] = L.cuts()
    return L, rec


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
