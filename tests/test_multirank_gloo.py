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


def _worker(rank, world, port, tiles, passes, result_path):
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
    assert lib.restir_tile_plan(W, H, tiles[0], tiles[1], rank, passes * f.spatial_resample_radius, C.byref(t)) == 0
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


@pytest.mark.parametrize("world,tiles,passes", [(2, (2, 1), 1), (2, (1, 2), 2), (4, (2, 2), 1), (8, (4, 2), 1)])
def test_tiles_over_gloo_ranks_match_single_frame(tmp_path, world, tiles, passes, abi_lib, oracle):
    result = str(tmp_path / "result.txt")
    mp.spawn(_worker, args=(world, _free_port(), tiles, passes, result), nprocs=world, join=True)
    with open(result) as fh:
        assert fh.read() == "ok"


# ---- halo-exchange mode (restir_halo_plan) with temporal reuse ------------------------------------------------
def _halo_worker(rank, world, port, tiles, passes, frames, result_path, name="nightclub_128pt"):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    from oracle import pyoracle
    from romis_amd import _abi, restir, scene

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    N = 1
    f = _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=passes, temporal_reuse=1)
    R = f.spatial_resample_radius
    t = restir.tile_plan(W, H, tiles[0], tiles[1], rank, R)
    send, recv = restir.halo_plan(W, H, tiles[0], tiles[1], rank, R, N)
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


@pytest.mark.parametrize("world,tiles,passes,name", [(2, (2, 1), 2, "nightclub_128pt"), (4, (2, 2), 1, "nightclub_128pt"),
                                                    (4, (2, 2), 2, "nightclub_128pt"), (8, (4, 2), 2, "nightclub_128pt"),
                                                    (8, (4, 2), 1, "cornell_1024")])
def test_halo_exchange_with_temporal_matches_single_frames(tmp_path, world, tiles, passes, name, abi_lib, oracle):
    """The halo protocol (restir_halo_plan segments, pack order [pixel][res_a, res_b], ring refilled before every
    pass) reproduces a 3-frame temporal sequence of single-process frames bit-for-bit."""
    result = str(tmp_path / "result.txt")
    mp.spawn(_halo_worker, args=(world, _free_port(), tiles, passes, 3, result, name), nprocs=world, join=True)
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
