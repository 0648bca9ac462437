"""Multi-GPU decomposition on CPU: world_size-2 (and 4) gloo process groups.

Each rank takes its screen tile from the product's host tile planner (restir_tile_plan in libromis_amd.so --
the same call bench.py and restir_render use), renders tile + ghost zone with the oracle, and the tiles are
gathered to rank 0, which checks that the stitched image equals a single-process frame bit-for-bit.  This
pins the ghost-zone width (passes * r) and the global-coordinate RNG / clamping the GPU tiles rely on.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

W, H = 72, 40


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# an uneven layout of the 72 x 40 test frame: per-column row cuts, columns 8-28 px wide
UNEVEN_4X2 = {"x": [0, 28, 44, 56, 72], "y": [[0, 12, 40], [0, 25, 40], [0, 31, 40], [0, 18, 40]]}
UNEVEN_2X4 = {"x": [0, 40, 72], "y": [[0, 6, 17, 30, 40], [0, 12, 20, 26, 40]]}


def _layout(cuts):
    from romis_amd import _abi
    return None if cuts is None else _abi.TileLayout.from_cuts(W, H, cuts)


def _worker(rank, world, port, tiles, passes, result_path, cuts=None):
    import ctypes as C
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import pyoracle
    from romis_amd import _abi, scene

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    lib = _abi.load_library()
    f = _abi.default_features(num_samples_in_reservoir=1, spatial_resampling_passes=passes, temporal_reuse=0)
    t = _abi.Tile()
    if cuts is None:
        assert lib.restir_tile_plan(W, H, tiles[0], tiles[1], rank, passes * f.spatial_resample_radius, C.byref(t)) == 0
    else:
        L = _layout(cuts)
        assert lib.restir_layout_tile(C.byref(L), rank, passes * f.spatial_resample_radius, C.byref(t)) == 0
    name = "nightclub_128pt"
    sc = scene.bench_scene(name)
    cam = scene.camera_for(name, W, H)
    osc = pyoracle.OracleScene(sc)
    view = pyoracle.Rect(t.gx0, t.gy0, t.gwidth, t.gheight)
    rect = pyoracle.Rect(t.x0, t.y0, t.width, t.height)
    rgb, _, _ = pyoracle.render_frame(osc, cam, f, W, H, view=view, rect=rect, threads=1)
    # rows of rgb: row 0 = top of the tile; place into a full image (row 0 = top = global y H-1)
    full = np.zeros((H, W, 3), np.float32)
    r0 = H - (t.y0 + t.height)
    full[r0:r0 + t.height, t.x0:t.x0 + t.width] = rgb
    mask = np.zeros((H, W), np.int32)
    mask[r0:r0 + t.height, t.x0:t.x0 + t.width] = 1
    ft = torch.from_numpy(full.view(np.int32).copy())
    mt = torch.from_numpy(mask)
    dist.all_reduce(ft, op=dist.ReduceOp.SUM)    # tiles are disjoint: the sum of bit patterns is a stitch
    dist.all_reduce(mt, op=dist.ReduceOp.SUM)
    if rank == 0:
        ref, _, _ = pyoracle.render_frame(osc, cam, f, W, H, threads=1)
        ok = bool((mt.numpy() == 1).all()) and np.array_equal(ft.numpy().view(np.float32).view(np.uint32),
                                                              ref.view(np.uint32))
        with open(result_path, "w") as fh:
            fh.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,tiles,passes,cuts", [(2, (2, 1), 1, None), (2, (1, 2), 2, None), (4, (2, 2), 1, None),
                                                     (8, (4, 2), 1, None), (8, (4, 2), 2, UNEVEN_4X2),
                                                     (8, (2, 4), 1, UNEVEN_2X4)])
def test_tiles_over_gloo_ranks_match_single_frame(tmp_path, world, tiles, passes, cuts, abi_lib, oracle):
    """Ghost-zone tiles of the even split and of uneven layouts (restir_layout_tile) stitch to the single frame."""
    result = str(tmp_path / "result.txt")
    mp.spawn(_worker, args=(world, _free_port(), tiles, passes, result, cuts), nprocs=world, join=True)
    with open(result) as fh:
        assert fh.read() == "ok"


# ---- halo-exchange mode (restir_halo_plan) with temporal reuse ------------------------------------------------
def _halo_worker(rank, world, port, tiles, passes, frames, result_path, name="nightclub_128pt", cuts=None):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import pyoracle
    from romis_amd import _abi, restir, scene

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    N = 1
    f = _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=passes, temporal_reuse=1)
    R = f.spatial_resample_radius
    layout = _layout(cuts)
    t = restir.tile_plan(W, H, tiles[0], tiles[1], rank, R, layout=layout)
    send, recv = restir.halo_plan(W, H, tiles[0], tiles[1], rank, R, N, layout=layout)
    sc = scene.bench_scene(name)
    cam = scene.camera_for(name, W, H)
    osc = pyoracle.OracleScene(sc)
    origin = np.asarray(list(pyoracle.camera_frame(cam).origin), np.float32)
    view = pyoracle.Rect(t.gx0, t.gy0, t.gwidth, t.gheight)
    own = pyoracle.Rect(t.x0, t.y0, t.width, t.height)
    lib = pyoracle.lib()

    def key(stage, p, fr):
        return lib.or_rng_key(_abi.RESTIR_DEFAULT_SEED, fr, stage, p)

    def idx(x, y):
        return (y - t.gy0) * t.gwidth + (x - t.gx0)

    def rect_ids(g):
        return np.array([idx(x, y) for y in range(g.y0, g.y0 + g.height) for x in range(g.x0, g.x0 + g.width)], np.int64)

    owned_mask = np.zeros(t.gwidth * t.gheight, bool)
    owned_mask[rect_ids(_abi.HaloSegment(0, t.x0, t.y0, t.width, t.height, 0, 0))] = True

    def poison(a, b):   # ring pixels must be refilled by the exchange before every pass
        a[:, ~owned_mask] = np.nan
        b[:, ~owned_mask] = np.nan

    n_t, p_mat = pyoracle.gbuffer(osc, cam, W, H, view=view)
    prev = None
    stitched = []
    for fr in range(frames):
        a, b, _ = pyoracle.ris(osc, f, key(_abi.RESTIR_STAGE_RIS, 0, fr), origin, W, H, n_t, p_mat, view=view)
        if prev is not None:
            a, b, _ = pyoracle.temporal(osc, f, key(_abi.RESTIR_STAGE_TEMPORAL, 0, fr), origin, W, H, n_t, p_mat,
                                        (a, b), prev, view=view)
        for p in range(passes):
            poison(a, b)
            reqs, bufs = [], []
            for s, r in zip(send, recv):
                ids = rect_ids(s)
                payload = np.concatenate([a[0, ids], b[0, ids]], axis=1).copy()   # [pixel][res_a, res_b]
                reqs.append(dist.isend(torch.from_numpy(payload), s.rank))
                rbuf = torch.empty((r.width * r.height, 8), dtype=torch.float32)
                reqs.append(dist.irecv(rbuf, r.rank))
                bufs.append((r, rbuf))
            for q in reqs:
                q.wait()
            for r, rbuf in bufs:
                ids = rect_ids(r)
                a[0, ids] = rbuf.numpy()[:, :4]
                b[0, ids] = rbuf.numpy()[:, 4:]
            a, b, _ = pyoracle.spatial_pass(osc, f, key(_abi.RESTIR_STAGE_SPATIAL, p, fr), origin, W, H, n_t, p_mat,
                                            (a, b), view=view, rect=own)
        rgb = pyoracle.final(osc, f, origin, W, H, n_t, p_mat, (a, b), view=view, rect=own)
        prev = (a, b)
        full = np.zeros((H, W, 3), np.float32)
        r0 = H - (t.y0 + t.height)
        full[r0:r0 + t.height, t.x0:t.x0 + t.width] = rgb
        ft = torch.from_numpy(full.view(np.int32).copy())
        dist.all_reduce(ft, op=dist.ReduceOp.SUM)
        stitched.append(ft.numpy().view(np.float32))
    if rank == 0:
        ok = True
        prev_full = None
        for fr in range(frames):
            ref, grid, _ = pyoracle.render_frame(osc, cam, f, W, H, frame=fr, prev=prev_full, threads=1)
            prev_full = grid
            ok = ok and np.array_equal(stitched[fr].view(np.uint32), ref.view(np.uint32))
        with open(result_path, "w") as fh:
            fh.write("ok" if ok else "mismatch")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,tiles,passes,name,cuts", [(2, (2, 1), 2, "nightclub_128pt", None),
                                                         (4, (2, 2), 1, "nightclub_128pt", None),
                                                         (4, (2, 2), 2, "nightclub_128pt", None),
                                                         (8, (4, 2), 2, "nightclub_128pt", None),
                                                         (8, (4, 2), 1, "cornell_1024", None),
                                                         (8, (4, 2), 2, "nightclub_128pt", UNEVEN_4X2),
                                                         (8, (2, 4), 1, "cornell_1024", UNEVEN_2X4)])
def test_halo_exchange_with_temporal_matches_single_frames(tmp_path, world, tiles, passes, name, cuts, abi_lib, oracle):
    """The halo protocol (restir_halo_plan segments, pack order [pixel][res_a, res_b], ring refilled before every
    pass) reproduces a 3-frame temporal sequence of single-process frames bit-for-bit -- on the even split and on
    uneven layouts (restir_layout_halo_plan: a rank's partners across per-column row cuts)."""
    result = str(tmp_path / "result.txt")
    mp.spawn(_halo_worker, args=(world, _free_port(), tiles, passes, 3, result, name, cuts), nprocs=world, join=True)
    with open(result) as fh:
        assert fh.read() == "ok"


# ---- bench.py's N > 1 halo self-check (romis_amd.distributed.tile_mismatches / exchange_probe) -----------------
def _selfcheck_worker(rank, world, port, tiles, result_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import pyoracle
    from romis_amd import _abi, distributed, restir, scene

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    f = _abi.default_features(num_samples_in_reservoir=1, spatial_resampling_passes=2, temporal_reuse=0)
    R, P = f.spatial_resample_radius, f.spatial_resampling_passes
    name = "nightclub_128pt"
    osc = pyoracle.OracleScene(scene.bench_scene(name))
    cam = scene.camera_for(name, W, H)
    # the two decompositions bench.py compares, here on the oracle: ghost zone (tile + P * r) and the tile owned
    # with an r-ring that an exchange fills (the halo protocol itself is pinned by the halo tests above; its
    # frame on the owned tile equals the full frame's, so the ghost tile's)
    tg = restir.tile_plan(W, H, tiles[0], tiles[1], rank, P * R)
    ghost, _, _ = pyoracle.render_frame(osc, cam, f, W, H, view=pyoracle.Rect(tg.gx0, tg.gy0, tg.gwidth, tg.gheight),
                                        rect=pyoracle.Rect(tg.x0, tg.y0, tg.width, tg.height), threads=1)
    full, _, _ = pyoracle.render_frame(osc, cam, f, W, H, threads=1)
    r0 = H - (tg.y0 + tg.height)
    owned = np.ascontiguousarray(full[r0:r0 + tg.height, tg.x0:tg.x0 + tg.width])
    same = distributed.tile_mismatches(owned, ghost)
    flipped = ghost.copy()
    if rank == world - 1:               # one flipped bit on the last rank must reach every rank's count
        flipped.view(np.uint32)[0, 0, 0] ^= 1
    diff = distributed.tile_mismatches(owned, flipped)
    shape = distributed.tile_mismatches(owned, ghost[:-1] if rank == 0 else ghost)
    send, recv = restir.halo_plan(W, H, tiles[0], tiles[1], rank, R, 1)
    us = distributed.exchange_probe(send, recv, iters=3)
    with open(f"{result_path}.{rank}", "w") as fh:
        fh.write(f"{same} {diff} {int(shape >= ghost.size // 3)} {int(us > 0)}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,tiles", [(2, (2, 1)), (8, (4, 2))])
def test_bench_halo_self_check_over_gloo(tmp_path, world, tiles, abi_lib, oracle):
    """bench.py --gpus N's self-check: equal tiles count 0 mismatches on every rank, a single flipped bit on one
    rank is seen by all, a shape mismatch counts the whole tile; the exchange probe moves the plan's segments."""
    result = str(tmp_path / "r")
    mp.spawn(_selfcheck_worker, args=(world, _free_port(), tiles, result), nprocs=world, join=True)
    for rank in range(world):
        with open(f"{result}.{rank}") as fh:
            assert fh.read().split() == ["0", "1", "1", "1"], rank


# ---- the native RCCL halo transport's operations, moved over gloo ------------------------------------------
# restir_halo_pass posts, per spatial pass, the list restir_halo_ops returns (one ncclSend then one ncclRecv per
# plan segment, inside one group).  Here every rank takes that list from the library, fills its send buffer from
# its owned reservoirs exactly as k_halo_pack lays them out ([sub-reservoir][pixel row-major][res_a, res_b]; the
# reservoirs are synthetic, a function of global pixel, sub-reservoir and field), posts the same sends / receives
# (peer, offset, bytes) over gloo, and checks that every received byte is the reservoir k_halo_unpack would
# write at that ring pixel.  Every rank's sends must also equal its peers' receives (gathered and paired), and the
# list must be the segments the torch transport moves (HaloFrames: restir_halo_plan).
def _synthetic_reservoirs(x0, y0, w, h, N):
    """[N][h*w][8] float32 words (res_a xyzw, res_b xyzw) of the global rectangle, bit patterns from the pixel id."""
    ys, xs = np.mgrid[y0:y0 + h, x0:x0 + w]
    g = (ys.astype(np.uint64) * 100003 + xs.astype(np.uint64)).reshape(-1)
    out = np.zeros((N, w * h, 8), np.uint32)
    for j in range(N):
        for k in range(8):
            out[j, :, k] = ((g * 8 + k) * 2654435761 + j * 40503 + 1) & 0x7F7FFFFF   # finite float bit patterns
    return out.view(np.float32)


def _native_ops_worker(rank, world, port, tiles, Wimg, Himg, R, N, result_dir, cuts=None):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from romis_amd import _abi, restir

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    errs = []
    layout = None if cuts is None else _abi.TileLayout.from_cuts(Wimg, Himg, cuts)
    ops = restir.halo_ops(Wimg, Himg, tiles[0], tiles[1], rank, R, N, layout=layout)
    send, recv = restir.halo_plan(Wimg, Himg, tiles[0], tiles[1], rank, R, N, layout=layout)
    # the posting order and the torch transport's segments
    if len(ops) != 2 * len(send):
        errs.append(f"{len(ops)} operations for {len(send)} segments")
    for i, (s, r) in enumerate(zip(send, recv)):
        o, p = ops[2 * i], ops[2 * i + 1]
        for op, seg, kind in ((o, s, _abi.RESTIR_HALO_OP_SEND), (p, r, _abi.RESTIR_HALO_OP_RECV)):
            want = (kind, seg.rank, seg.offset, seg.bytes, seg.x0, seg.y0, seg.width, seg.height)
            got = (op.kind, op.peer, op.offset, op.bytes, op.x0, op.y0, op.width, op.height)
            if got != want:
                errs.append(f"op {2 * i + (kind == _abi.RESTIR_HALO_OP_RECV)}: {got} != segment {want}")
    # pack as k_halo_pack does, then post exactly the listed operations
    sb = sum(o.bytes for o in ops if o.kind == _abi.RESTIR_HALO_OP_SEND)
    rb = sum(o.bytes for o in ops if o.kind == _abi.RESTIR_HALO_OP_RECV)
    sendbuf = torch.zeros(max(1, sb), dtype=torch.uint8)
    recvbuf = torch.full((max(1, rb),), 0xAB, dtype=torch.uint8)
    t = restir.tile_plan(Wimg, Himg, tiles[0], tiles[1], rank, 0, layout=layout)
    for o in ops:
        if o.kind != _abi.RESTIR_HALO_OP_SEND:
            continue
        inside = t.x0 <= o.x0 and o.x0 + o.width <= t.x0 + t.width and t.y0 <= o.y0 and o.y0 + o.height <= t.y0 + t.height
        if not inside:
            errs.append(f"send to {o.peer}: rectangle outside the owned tile")
        if o.bytes != o.width * o.height * N * 32:
            errs.append(f"send to {o.peer}: {o.bytes} bytes for a {o.width}x{o.height} rectangle")
        blob = _synthetic_reservoirs(o.x0, o.y0, o.width, o.height, N).tobytes()
        sendbuf[o.offset:o.offset + o.bytes] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    p2p = []
    for o in ops:
        if o.kind == _abi.RESTIR_HALO_OP_SEND:
            p2p.append(dist.P2POp(dist.isend, sendbuf[o.offset:o.offset + o.bytes], o.peer))
        else:
            p2p.append(dist.P2POp(dist.irecv, recvbuf[o.offset:o.offset + o.bytes], o.peer))
    if p2p:
        for q in dist.batch_isend_irecv(p2p):
            q.wait()
    got = recvbuf.numpy()
    ring = 0
    for o in ops:
        if o.kind != _abi.RESTIR_HALO_OP_RECV:
            continue
        want = _synthetic_reservoirs(o.x0, o.y0, o.width, o.height, N).view(np.uint8).reshape(-1)
        if not np.array_equal(got[o.offset:o.offset + o.bytes], want):
            errs.append(f"recv from {o.peer}: bytes differ from that rank's reservoirs at {o.x0},{o.y0} {o.width}x{o.height}")
        # the received rectangle lies in this rank's ring: outside the owned tile, within R of it
        for yy in (o.y0, o.y0 + o.height - 1):
            for xx in (o.x0, o.x0 + o.width - 1):
                owned = t.x0 <= xx < t.x0 + t.width and t.y0 <= yy < t.y0 + t.height
                near = t.x0 - R <= xx < t.x0 + t.width + R and t.y0 - R <= yy < t.y0 + t.height + R
                if owned or not near:
                    errs.append(f"recv from {o.peer}: pixel {xx},{yy} not in the ring")
        ring += o.width * o.height
    # sends pair with the peers' receives: same rectangle, same bytes, one each
    allops = [None] * world
    dist.all_gather_object(allops, [(o.kind, o.peer, o.x0, o.y0, o.width, o.height, o.bytes) for o in ops])
    for k, p, x0, y0, w, h, b in allops[rank]:
        if k == _abi.RESTIR_HALO_OP_SEND:
            match = [q for q in allops[p] if q == (_abi.RESTIR_HALO_OP_RECV, rank, x0, y0, w, h, b)]
            if len(match) != 1:
                errs.append(f"send {rank}->{p} {x0},{y0} {w}x{h}: {len(match)} matching receives")
    # every ring pixel a spatial pass may read (+-R around the tile, clamped to the image) is received exactly once
    need = sum(1 for yy in range(max(0, t.y0 - R), min(Himg, t.y0 + t.height + R))
               for xx in range(max(0, t.x0 - R), min(Wimg, t.x0 + t.width + R))
               if not (t.x0 <= xx < t.x0 + t.width and t.y0 <= yy < t.y0 + t.height))
    if ring != need:
        errs.append(f"{ring} ring pixels received, {need} needed")
    with open(os.path.join(result_dir, f"rank{rank}.txt"), "w") as fh:
        fh.write("\n".join(errs) if errs else "ok")
    dist.barrier()
    dist.destroy_process_group()


# C4's balanced 4 x 2 cuts (profiles/r6/balance.json) scaled to 3840 / 16 x 2160 / 16
C4_BALANCED_16 = {"x": [0, 92, 118, 142, 240], "y": [[0, 71, 135], [0, 70, 135], [0, 68, 135], [0, 72, 135]]}


@pytest.mark.parametrize("world,tiles,Wimg,Himg,R,N,cuts", [(2, (2, 1), 96, 40, 10, 1, None), (4, (2, 2), 101, 67, 7, 2, None),
                                                            (8, (4, 2), 3840 // 16, 2160 // 16, 10, 1, None),
                                                            (8, (4, 2), 90, 33, 12, 3, None),
                                                            (8, (4, 2), 3840 // 16, 2160 // 16, 10, 1, C4_BALANCED_16),
                                                            (8, (4, 2), 72, 40, 10, 2, UNEVEN_4X2)])
def test_native_halo_operations_over_gloo(tmp_path, world, tiles, Wimg, Himg, R, N, cuts, abi_lib):
    mp.spawn(_native_ops_worker, args=(world, _free_port(), tiles, Wimg, Himg, R, N, str(tmp_path), cuts), nprocs=world,
             join=True)
    for r in range(world):
        msg = open(tmp_path / f"rank{r}.txt").read()
        assert msg == "ok", f"rank {r}: {msg}"


# ---- bench.py's halo transport choice ------------------------------------
# select_halo builds the run's one HaloFrames, checks it against the ghost-zone tile and falls back to the torch
# transport on a construction failure (every rank together) or a native mismatch; the instance it returns is the one
# the halo-mode loop times, so the record's transport is the timed transport.  Stand-ins replace HaloFrames and the
# tile comparison: a "native" transport whose tile differs (a corrupted segment), one whose attach fails on one rank,
# and a torch transport that differs too (the run must fail).
class _StandInHalo:
    def __init__(self, transport):
        self.transport = transport


def _select_worker(rank, world, port, case, result):
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from romis_amd import _abi

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    made = []

    def make(tr):
        if case == "attach_fails" and tr == "native" and rank == world - 1:
            raise _abi.RestirError("stand-in: ncclCommInitRank failed")
        made.append(tr)
        return _StandInHalo(tr)

    def check(hf):
        # a corrupted segment on rank 0 over the native transport (every case), and over torch too in "torch_bad";
        # summed over ranks as distributed.tile_mismatches does
        bad = 1 if rank == 0 and (hf.transport == "native" or case == "torch_bad") else 0
        t = torch.tensor([bad], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return int(t.item())

    hf, rec, bad = bench.select_halo(torch, world, 0, "gloo", "native", make, check)
    with open(f"{result}.{rank}", "w") as fh:
        json.dump({"timed": hf.transport, "rec": rec, "bad": bad, "made": made}, fh)
    dist.destroy_process_group()


@pytest.mark.parametrize("case", ["native_mismatch", "attach_fails", "torch_bad"])
def test_bench_times_the_checked_halo_transport(tmp_path, case):
    """The transport bench.py times is the one its record names and the one that passed the check: a native mismatch
    or a failed native attach on any rank moves every rank to torch (recorded as native_check / native_error), and a
    torch mismatch is reported (mismatches != 0: bench exits 3)."""
    import json
    world = 2
    result = str(tmp_path / "r")
    mp.spawn(_select_worker, args=(world, _free_port(), case, result), nprocs=world, join=True)
    for rank in range(world):
        with open(f"{result}.{rank}") as fh:
            out = json.load(fh)
        assert out["timed"] == out["rec"]["transport"] == "torch", (rank, out)
        if case == "native_mismatch":
            assert out["rec"]["native_check"] == "1 mismatching values" and out["bad"] == 0
            assert out["made"] == ["native", "torch"]
        elif case == "attach_fails":
            assert out["bad"] == 0 and "native_check" not in out["rec"]
            assert ("native_error" in out["rec"]) == (rank == world - 1)
        else:
            assert out["bad"] == 1 and out["rec"]["native_check"] == "1 mismatching values"
