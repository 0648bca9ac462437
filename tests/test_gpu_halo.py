"""Halo-exchange frames on the GPU (romis_amd/distributed.py over restir_halo_*): 2 and 4 ranks, each its
own process and restir context on the one GPU of the box, exchanging reservoir halos over gloo (host-staged;
the nccl backend moves the same device buffers over RCCL on a multi-GPU node).  A 3-frame temporal sequence
with two spatial passes must stitch to the single-GPU restir_render frames bit-for-bit."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

W, H = 96, 64
FRAMES = 3
_DEFAULT_SCENE = "nightclub_128pt"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _features(passes, N, unbiased=0, vis=0):
    from romis_amd import _abi
    return _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=passes, temporal_reuse=1,
                                 unbiased_combination=unbiased, spatial_reuse_visibility_check=vis)


# uneven layouts of the 96 x 64 frame (restir_tile_layout); "balanced": distributed.balanced_layout
# -- the cost grid from the library's primary-ray kernel on rank 0, the cuts broadcast over the group
UNEVEN = {(4, 2): {"x": [0, 36, 52, 68, 96], "y": [[0, 20, 64], [0, 36, 64], [0, 28, 64], [0, 44, 64]]},
          (2, 4): {"x": [0, 56, 96], "y": [[0, 10, 30, 44, 64], [0, 18, 32, 50, 64]]}}


def _worker(rank, world, port, tiles, passes, N, out_dir, name="nightclub_128pt", records=0, backend="gloo",
            width=W, height=H, unbiased=0, vis=0, layout_kind=None, frames=FRAMES):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from romis_amd import _abi, distributed, restir, scene

    W, H = width, height
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    r = restir.Renderer(0)
    r.set_tuning("layout.records", records)
    sc = scene.bench_scene(name)
    r.set_scene(sc)
    r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
    cam = scene.camera_for(name, W, H)
    layout = None
    if layout_kind == "uneven":
        layout = _abi.TileLayout.from_cuts(W, H, UNEVEN[tuple(tiles)])
    elif layout_kind == "balanced":
        layout, _ = distributed.balanced_layout(r, lambda w, h: scene.camera_for(name, w, h), W, H, tiles, align=(8, 8))
    hf = distributed.HaloFrames(r, W, H, tiles, rank, _features(passes, N, unbiased, vis), layout=layout)
    prev = None
    for fr in range(frames):
        rgb, prev = hf.render(prev, cam)
        t = hf.tile
        full = np.zeros((H, W, 3), np.float32)
        r0 = H - (t.y0 + t.height)
        full[r0:r0 + t.height, t.x0:t.x0 + t.width] = rgb
        ft = torch.from_numpy(full.view(np.int32).copy())
        dist.all_reduce(ft, op=dist.ReduceOp.SUM)    # disjoint tiles: the sum of bit patterns stitches them
        if rank == 0:
            np.save(os.path.join(out_dir, f"frame{fr}.npy"), ft.numpy().view(np.float32))
    dist.barrier()
    prev = None
    r.close()
    dist.destroy_process_group()


def _single_gpu_check(tmp_path, passes, N, name=_DEFAULT_SCENE, records=0, width=W, height=H, unbiased=0, vis=0,
                      frames=FRAMES):
    from romis_amd import _abi, restir, scene
    W, H = width, height
    r = restir.Renderer(0)
    try:
        r.set_tuning("layout.records", records)
        r.set_scene(scene.bench_scene(name))
        r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
        cam = scene.camera_for(name, W, H)
        f = _features(passes, N, unbiased, vis)
        prev = None
        for fr in range(frames):
            want, prev = r.render_restir(prev, cam, W, H, f)
            got = np.load(str(tmp_path / f"frame{fr}.npy"))
            bad = np.flatnonzero(got.view(np.uint32) != want.view(np.uint32))
            assert bad.size == 0, f"frame {fr}: {bad.size} words differ"
        prev = None
    finally:
        r.close()


# Each rank is its own process and restir context on the box's one GPU; the pass runs as interior (issued
# before the exchange) + border strips (after the unpack).  (8, (4, 2)): the C4 / C5 split; (8, (8, 1)): tiles
# 12 px wide, narrower than 2R, so the interior is empty and the border strips cover the tile.  The unbiased cases
# run the lean N = 1 unbiased pass (k_spatial1u[_vis]), whose Z term reads the pdf cache at neighbour pixels: in a
# border strip those may lie in the exchanged ring, which carries no cache (restir.cpp halo_spatial_part).
@pytest.mark.gpu
@pytest.mark.parametrize("world,tiles,passes,N,name,records,unbiased,vis,layout_kind", [
    (2, (2, 1), 2, 1, _DEFAULT_SCENE, 0, 0, 0, None), (4, (2, 2), 2, 1, _DEFAULT_SCENE, 0, 0, 0, None),
    (4, (2, 2), 1, 2, _DEFAULT_SCENE, 0, 0, 0, None),
    (2, (2, 1), 2, 1, _DEFAULT_SCENE, 1, 0, 0, None), (4, (2, 2), 1, 2, _DEFAULT_SCENE, 1, 0, 0, None),
    (8, (4, 2), 2, 1, "cornell_1024", 0, 0, 0, None), (8, (8, 1), 1, 1, _DEFAULT_SCENE, 0, 0, 0, None),
    (2, (2, 1), 2, 1, _DEFAULT_SCENE, 0, 1, 0, None), (4, (2, 2), 1, 1, "cornell_1024", 0, 1, 1, None),
    (8, (4, 2), 2, 1, "cornell_4096", 0, 1, 1, None), (4, (2, 2), 1, 2, _DEFAULT_SCENE, 0, 1, 1, None),
    (8, (4, 2), 2, 1, _DEFAULT_SCENE, 0, 0, 0, "uneven"), (8, (2, 4), 1, 2, "cornell_1024", 0, 0, 0, "uneven"),
    (8, (4, 2), 1, 1, "cornell_4096", 0, 1, 1, "balanced"), (8, (4, 2), 2, 1, "cornell_1024", 0, 0, 0, "balanced")])
def test_halo_frames_match_single_gpu_sequence(tmp_path, world, tiles, passes, N, name, records, unbiased, vis,
                                               layout_kind):
    mp.spawn(_worker, args=(world, _free_port(), tiles, passes, N, str(tmp_path), name, records, "gloo", W, H,
                            unbiased, vis, layout_kind), nprocs=world, join=True)
    _single_gpu_check(tmp_path, passes, N, name, records, unbiased=unbiased, vis=vis)


# The C4 / C5 strong-scaling split at full size: 8 processes on the box's GPU, each rendering its
# rect of the 4K / 8K frame (the TOML camera: 87 % background) through the halo passes of a cost-balanced 4 x 2 layout
# (distributed.balanced_layout: uneven per-column row cuts), halos over gloo; the stitched frame against restir_render's
# single-GPU frame, which the full-size band tests pin to the oracle (test_full_size_frames_c4_c5_band_parity).
@pytest.mark.gpu
@pytest.mark.parametrize("name,width,height,unbiased,vis", [("cornell_1024", 3840, 2160, 0, 0),
                                                          ("cornell_4096", 7680, 4320, 1, 1)])
def test_halo_full_size_balanced_split(tmp_path, name, width, height, unbiased, vis):
    mp.spawn(_worker, args=(8, _free_port(), (4, 2), 1, 1, str(tmp_path), name, 0, "gloo", width, height, unbiased, vis,
                            "balanced", 1), nprocs=8, join=True)
    _single_gpu_check(tmp_path, 1, 1, name, 0, width, height, unbiased, vis, frames=1)


# The native transport (restir_halo_pass: the library's own RCCL communicator, grouped ncclSend / ncclRecv on a
# communication stream overlapped with the interior).  The box has one GPU; RCCL may refuse two ranks on one
# device -- then this test skips, and the path runs only on a multi-GPU node.
def _native_worker(rank, world, port, out_dir, tiles=(2, 1)):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from romis_amd import _abi, distributed, restir, scene
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    r = restir.Renderer(0)
    try:
        r.set_scene(scene.bench_scene(_DEFAULT_SCENE))
        r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
        cam = scene.camera_for(_DEFAULT_SCENE, W, H)
        try:
            hf = distributed.HaloFrames(r, W, H, tiles, rank, _features(2, 1), transport="native")
        except _abi.RestirError as e:
            with open(os.path.join(out_dir, f"skip{rank}.txt"), "w") as fh:
                fh.write(str(e))
            return
        prev = None
        for fr in range(FRAMES):
            rgb, prev = hf.render(prev, cam)
            t = hf.tile
            full = np.zeros((H, W, 3), np.float32)
            r0 = H - (t.y0 + t.height)
            full[r0:r0 + t.height, t.x0:t.x0 + t.width] = rgb
            ft = torch.from_numpy(full.view(np.int32).copy())
            dist.all_reduce(ft, op=dist.ReduceOp.SUM)
            if rank == 0:
                np.save(os.path.join(out_dir, f"frame{fr}.npy"), ft.numpy().view(np.float32))
        prev = None
    finally:
        r.close()
        dist.destroy_process_group()


@pytest.mark.gpu
def test_native_rccl_halo_frames(tmp_path):
    mp.spawn(_native_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    skips = sorted(p for p in os.listdir(tmp_path) if p.startswith("skip"))
    if skips:
        pytest.skip("RCCL with two ranks on one GPU: " + open(os.path.join(tmp_path, skips[0])).read()[:200])
    _single_gpu_check(tmp_path, 2, 1)


@pytest.mark.gpu
def test_ghost_tiles_refuse_temporal_reuse():
    from romis_amd import _abi, restir, scene
    r = restir.Renderer(0)
    try:
        r.set_scene(scene.bench_scene("nightclub_128pt"))
        cam = scene.camera_for("nightclub_128pt", W, H)
        f = _features(1, 1)
        t = restir.tile_plan(W, H, 2, 1, 0, f.spatial_resample_radius)
        _, g = r.render_restir(None, cam, W, H, f, tile=t)
        with pytest.raises(_abi.RestirError, match="UNSUPPORTED"):
            r.render_restir(g, cam, W, H, f, tile=t)
    finally:
        r.close()


@pytest.mark.gpu
def test_native_rccl_halo_single_rank(tmp_path):
    """One rank, one tile: restir_halo_pass's stream / event plumbing (pack, communication-stream wait, interior,
    unpack, border) with an RCCL communicator of size 1 and no segments, against restir_render."""
    mp.spawn(_native_worker, args=(1, _free_port(), str(tmp_path), (1, 1)), nprocs=1, join=True)
    skips = sorted(p for p in os.listdir(tmp_path) if p.startswith("skip"))
    assert not skips, open(os.path.join(tmp_path, skips[0])).read()
    _single_gpu_check(tmp_path, 2, 1)


# Record-only restir_halo_pass (restir_halo_record): the native transport's plumbing on the box's one GPU.  For
# every rank of a split, one context runs a frame's passes through restir_halo_pass without a communicator; its log
# must show, per pass, the pack and its event on the context stream, the communication stream's wait for that
# event, the group of sends / receives -- exactly restir_halo_ops' list (peer, offset, bytes), the list the CPU
# suite moves over gloo (tests/test_multirank_gloo.py) -- and its completion event, then the interior launch, the
# context stream's wait for the transfer, the unpack and the border launches; and every rank's sends must pair
# with its peers' receives.
@pytest.mark.gpu
@pytest.mark.parametrize("world,tiles,N", [(2, (2, 1), 1), (4, (2, 2), 2), (8, (4, 2), 1)])
def test_native_halo_pass_record_only(world, tiles, N):
    from romis_amd import _abi, restir, scene
    passes = 2
    f = _features(passes, N)
    R = f.spatial_resample_radius
    E = _abi
    logs = {}
    r = restir.Renderer(0)
    try:
        r.set_scene(scene.bench_scene(_DEFAULT_SCENE))
        cam = scene.camera_for(_DEFAULT_SCENE, W, H)
        r.halo_record(True)
        for rank in range(world):
            t = restir.tile_plan(W, H, tiles[0], tiles[1], rank, R)
            sb, rb = r.halo_begin(None, cam, W, H, f, tiles, rank)
            for _ in range(passes):
                r.halo_pass()
            r.halo_end(t, False, False)
            r.synchronize()
            logs[rank] = [(e.what, e.stream, e.peer, e.pass_, e.offset, e.bytes) for e in r.halo_log()]
            ops = restir.halo_ops(W, H, tiles[0], tiles[1], rank, R, N)
            assert sb == sum(o.bytes for o in ops if o.kind == E.RESTIR_HALO_OP_SEND)
            assert rb == sum(o.bytes for o in ops if o.kind == E.RESTIR_HALO_OP_RECV)
            want = []
            for p in range(passes):
                want += [(E.RESTIR_HALO_EV_PACK, 0, 0, p, 0, sb), (E.RESTIR_HALO_EV_RECORD, 0, 0, p, 0, 0),
                         (E.RESTIR_HALO_EV_WAIT, 1, 0, p, 0, 0), (E.RESTIR_HALO_EV_GROUP_START, 1, 0, p, 0, 0)]
                want += [(E.RESTIR_HALO_EV_SEND if o.kind == E.RESTIR_HALO_OP_SEND else E.RESTIR_HALO_EV_RECV, 1, o.peer,
                          p, o.offset, o.bytes) for o in ops]
                want += [(E.RESTIR_HALO_EV_GROUP_END, 1, 0, p, 0, 0), (E.RESTIR_HALO_EV_RECORD, 1, 1, p, 0, 0),
                         (E.RESTIR_HALO_EV_INTERIOR, 0, 0, p, 0, 0), (E.RESTIR_HALO_EV_WAIT, 0, 1, p, 0, 0),
                         (E.RESTIR_HALO_EV_UNPACK, 0, 0, p, 0, rb), (E.RESTIR_HALO_EV_BORDER, 0, 0, p, 0, 0)]
            assert logs[rank] == want, f"rank {rank}"
            for o in ops:   # the rectangle each send carries is one of the peer's receives, byte count included
                if o.kind == E.RESTIR_HALO_OP_SEND:
                    peer = restir.halo_ops(W, H, tiles[0], tiles[1], o.peer, R, N)
                    m = [q for q in peer if q.kind == E.RESTIR_HALO_OP_RECV and q.peer == rank and
                         (q.x0, q.y0, q.width, q.height, q.bytes) == (o.x0, o.y0, o.width, o.height, o.bytes)]
                    assert len(m) == 1, f"send {rank}->{o.peer}"
        r.halo_record(False)
        with pytest.raises(_abi.RestirError, match="STATE"):   # no communicator outside record mode
            r.halo_begin(None, cam, W, H, f, tiles, 0)
            r.halo_pass()
    finally:
        r.close()
