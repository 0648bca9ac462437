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


def _features(passes, N):
    from romis_amd import _abi
    return _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=passes, temporal_reuse=1)


def _worker(rank, world, port, tiles, passes, N, out_dir, name="nightclub_128pt", records=0, backend="gloo",
            width=W, height=H):
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
    hf = distributed.HaloFrames(r, W, H, tiles, rank, _features(passes, N))
    prev = None
    for fr in range(FRAMES):
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


def _single_gpu_check(tmp_path, passes, N, name=_DEFAULT_SCENE, records=0, width=W, height=H):
    from romis_amd import _abi, restir, scene
    W, H = width, height
    r = restir.Renderer(0)
    try:
        r.set_tuning("layout.records", records)
        r.set_scene(scene.bench_scene(name))
        r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
        cam = scene.camera_for(name, W, H)
        f = _features(passes, N)
        prev = None
        for fr in range(FRAMES):
            want, prev = r.render_restir(prev, cam, W, H, f)
            got = np.load(str(tmp_path / f"frame{fr}.npy"))
            bad = np.flatnonzero(got.view(np.uint32) != want.view(np.uint32))
            assert bad.size == 0, f"frame {fr}: {bad.size} words differ"
        prev = None
    finally:
        r.close()


# Each rank is its own process and restir context on the box's one GPU; the pass runs as interior (issued
# before the exchange) + border strips (after the unpack).  (8, (4, 2)): the C4 / C5 split; (8, (8, 1)): tiles
# 12 px wide, narrower than 2R, so the interior is empty and the border strips cover the tile.
@pytest.mark.gpu
@pytest.mark.parametrize("world,tiles,passes,N,name,records", [
    (2, (2, 1), 2, 1, _DEFAULT_SCENE, 0), (4, (2, 2), 2, 1, _DEFAULT_SCENE, 0), (4, (2, 2), 1, 2, _DEFAULT_SCENE, 0),
    (2, (2, 1), 2, 1, _DEFAULT_SCENE, 1), (4, (2, 2), 1, 2, _DEFAULT_SCENE, 1),
    (8, (4, 2), 2, 1, "cornell_1024", 0), (8, (8, 1), 1, 1, _DEFAULT_SCENE, 0)])
def test_halo_frames_match_single_gpu_sequence(tmp_path, world, tiles, passes, N, name, records):
    mp.spawn(_worker, args=(world, _free_port(), tiles, passes, N, str(tmp_path), name, records), nprocs=world,
             join=True)
    _single_gpu_check(tmp_path, passes, N, name, records)


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
