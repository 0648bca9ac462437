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


@pytest.mark.parametrize("world,tiles,passes", [(2, (2, 1), 1), (2, (1, 2), 2), (4, (2, 2), 1)])
def test_tiles_over_gloo_ranks_match_single_frame(tmp_path, world, tiles, passes, abi_lib, oracle):
    result = str(tmp_path / "result.txt")
    mp.spawn(_worker, args=(world, _free_port(), tiles, passes, result), nprocs=world, join=True)
    with open(result) as fh:
        assert fh.read() == "ok"
