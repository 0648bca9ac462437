"""Screen-tile layouts (include/restir_c.h "Uneven screen tiles"): pure host logic of libromis_amd.so, no GPU.

restir_layout_even is restir_tile_plan's split; restir_layout_balanced cuts the columns at equal shares of a cost grid
and each column's rows at equal shares of its own cost, so that a frame whose geometry fills only the middle of the image
(C4 / C5's TOML camera) still gives every rank the same work.  Any layout is a partition of the image into
one rectangle per rank, and its halo plan pairs every send with the partner's receive.
"""
import ctypes as C

import numpy as np
import pytest

from romis_amd import _abi, restir

RESTIR_ERR_INVALID = 1   # include/restir_c.h restir_status


def rects(L):
    return [restir.tile_plan(0, 0, 0, 0, q, 0, layout=L) for q in range(L.tiles_x * L.tiles_y)]


def assert_partition(L):
    W, H = L.global_width, L.global_height
    own = np.zeros((H, W), np.int32)
    for t in rects(L):
        own[t.y0:t.y0 + t.height, t.x0:t.x0 + t.width] += 1
    assert (own == 1).all()


@pytest.mark.parametrize("W,H,tx,ty", [(1920, 1080, 2, 1), (3840, 2160, 4, 2), (101, 67, 2, 2), (7, 5, 7, 5),
                                       (7680, 4320, 2, 4), (33, 90, 1, 8)])
def test_even_layout_is_tile_plan(W, H, tx, ty, abi_lib):
    L = restir.layout_even(W, H, tx, ty)
    assert_partition(L)
    for q in range(tx * ty):
        for ghost in (0, 10, 20):
            a = restir.tile_plan(W, H, tx, ty, q, ghost)
            b = restir.tile_plan(W, H, tx, ty, q, ghost, layout=L)
            assert bytes(a) == bytes(b)
        if W >= 2 * tx * 10 and H >= 2 * ty * 10:
            sa, ra = restir.halo_plan(W, H, tx, ty, q, 10, 1)
            sb, rb = restir.halo_plan(W, H, tx, ty, q, 10, 1, layout=L)
            assert [bytes(x) for x in sa + ra] == [bytes(x) for x in sb + rb]


def _blob_cost(cw=480, ch=270, seed=0, bg=0.1):
    """A concentrated cost grid: geometry in an off-centre ellipse, background elsewhere."""
    y, x = np.mgrid[0:ch, 0:cw]
    hit = ((x - 0.55 * cw) / (0.18 * cw)) ** 2 + ((y - 0.45 * ch) / (0.3 * ch)) ** 2 < 1.0
    rng = np.random.default_rng(seed)
    return np.where(hit, 1.0 + 0.2 * rng.random((ch, cw)), bg).astype(np.float32)


@pytest.mark.parametrize("W,H,tiles", [(3840, 2160, (4, 2)), (7680, 4320, (4, 2)), (3840, 2160, (2, 4)),
                                       (3840, 2160, (8, 1)), (1920, 1080, (2, 2))])
def test_balanced_layout_partitions_and_balances(W, H, tiles, abi_lib):
    cost = _blob_cost()
    L, eff = restir.layout_balanced(W, H, tiles[0], tiles[1], cost, align=(32, 8))
    assert_partition(L)
    for c in range(1, tiles[0]):
        assert L.x_cuts[c] % 32 == 0
    for c in range(tiles[0]):
        for r in range(1, tiles[1]):
            assert L.y_cuts[c][r] % 8 == 0
    sh = restir.layout_shares(L, cost)
    assert abs(sh.sum() - 1.0) < 1e-9
    assert eff == pytest.approx(sh.mean() / sh.max())
    even = restir.layout_shares(restir.layout_even(W, H, *tiles), cost)
    assert eff >= 0.9 > even.mean() / even.max()


def test_uniform_cost_gives_the_even_split(abi_lib):
    cost = np.ones((270, 480), np.float32)
    L, eff = restir.layout_balanced(3840, 2160, 4, 2, cost, align=(32, 8))
    assert L.cuts() == restir.layout_even(3840, 2160, 4, 2).cuts()
    assert eff == pytest.approx(1.0)


@pytest.mark.parametrize("tiles", [(4, 2), (2, 4)])
def test_balanced_halo_plans_pair_up_and_cover_the_ring(tiles, abi_lib):
    W, H, R = 3840 // 8, 2160 // 8, 10
    L, _ = restir.layout_balanced(W, H, tiles[0], tiles[1], _blob_cost(W // 2, H // 2), align=(8, 8))
    n = tiles[0] * tiles[1]
    plans = [restir.halo_plan(W, H, *tiles, q, R, 2, layout=L) for q in range(n)]
    ts = rects(L)
    for q, (send, recv) in enumerate(plans):
        assert len(send) <= 8
        for s in send:   # rank q's send to p is p's receive from q: same rectangle and bytes
            match = [r for r in plans[s.rank][1] if r.rank == q]
            assert len(match) == 1 and (match[0].x0, match[0].y0, match[0].width, match[0].height, match[0].bytes) == \
                (s.x0, s.y0, s.width, s.height, s.bytes)
        t = ts[q]
        ring = np.zeros((H, W), np.int32)
        for r in recv:
            ring[r.y0:r.y0 + r.height, r.x0:r.x0 + r.width] += 1
        want = np.zeros((H, W), np.int32)
        want[max(0, t.y0 - R):t.y0 + t.height + R, max(0, t.x0 - R):t.x0 + t.width + R] = 1
        want[t.y0:t.y0 + t.height, t.x0:t.x0 + t.width] = 0
        assert np.array_equal(ring, want), q


def test_malformed_layouts_are_refused(abi_lib):
    lib = _abi.load_library()
    L = restir.layout_even(64, 32, 2, 2)
    t = _abi.Tile()
    L.x_cuts[1] = 0   # not increasing
    assert lib.restir_layout_tile(C.byref(L), 0, 0, C.byref(t)) == RESTIR_ERR_INVALID
    L = restir.layout_even(64, 32, 2, 2)
    L.y_cuts[1][2] = 31   # does not reach the height
    assert lib.restir_layout_tile(C.byref(L), 0, 0, C.byref(t)) == RESTIR_ERR_INVALID
    L = restir.layout_even(64, 32, 2, 2)
    L.tiles_x = 17
    assert lib.restir_layout_tile(C.byref(L), 0, 0, C.byref(t)) == RESTIR_ERR_INVALID
    cost = np.full((4, 4), -1.0, np.float32)
    with pytest.raises(_abi.RestirError):
        restir.layout_balanced(64, 32, 2, 2, cost)
    with pytest.raises(_abi.RestirError):   # 4 tiles of at least 32 px do not fit 64 px
        restir.layout_balanced(64, 32, 4, 1, np.ones((4, 4), np.float32), align=(32, 8))


@pytest.mark.parametrize("cfg", ["c4", "c5"])
def test_c4_c5_balanced_layouts_from_the_oracle_geometry(cfg, abi_lib, oracle):
    """C4 / C5's TOML camera at the cost grid's resolution (the oracle's primary rays -- on the GPU the library's own
    kernel makes the grid, distributed.geometry_cost): the balanced 4 x 2 layout reaches >= 0.9 of perfect balance under
    the cost model, the even one ~0.56 (4 of 8 ranks without geometry)."""
    import bench
    from romis_amd import distributed, scene
    c = bench.CONFIGS[cfg]
    W, H = c["image"]
    gw, gh = distributed.COST_GRID
    osc = oracle.OracleScene(scene.bench_scene(c["scene"]))
    _, p_mat = oracle.gbuffer(osc, scene.camera_for(c["scene"], gw, gh), gw, gh)
    hit = (p_mat[:, 3].view(np.uint32) != osc.miss_material).reshape(gh, gw)
    cost = np.where(hit, 1.0, distributed.BACKGROUND_WEIGHT).astype(np.float32)
    L, eff = restir.layout_balanced(W, H, 4, 2, cost, distributed.LAYOUT_ALIGN)
    even = restir.layout_shares(restir.layout_even(W, H, 4, 2), cost)
    assert eff >= 0.9 and even.mean() / even.max() < 0.6


def test_measured_refinement_converges_on_the_true_cost(abi_lib):
    """distributed.refine_cost: a model that misjudges per-pixel cost (here: one quadrant of the geometry 3x dearer)
    is corrected by the ranks' measured times -- three rounds of re-cutting (bench.py's default) reach >= 0.93 of the
    true cost's balance."""
    from romis_amd import distributed
    W, H = 3840, 2160
    model = _blob_cost(bg=0.1)
    true = model.copy()
    ch, cw = true.shape
    true[: ch // 2, cw // 2:] *= np.where(true[: ch // 2, cw // 2:] > 0.5, 3.0, 1.0)
    L, _ = restir.layout_balanced(W, H, 4, 2, model)
    eff0 = (lambda s: s.mean() / s.max())(restir.layout_shares(L, true))
    cost = model
    for _ in range(3):
        times = restir.layout_shares(L, true)   # measured rank times follow the true cost
        cost = distributed.refine_cost(cost, L, times)
        L, _ = restir.layout_balanced(W, H, 4, 2, cost)
    eff = (lambda s: s.mean() / s.max())(restir.layout_shares(L, true))
    assert eff0 < 0.85 and eff >= 0.93, (eff0, eff)
    own = distributed.cell_owners(L, cost.shape)
    assert own.min() == 0 and own.max() == 7



def _true_share_time(L, rank, calls, inflate_call):
    """A stand-in frame time: this rank's share of a "true" cost whose top-right quadrant is 3x dearer than the model,
    inflated 5x on rank 1 at one measurement (contention)."""
    true = _blob_cost()
    ch, cw = true.shape
    true[: ch // 2, cw // 2:] *= 3.0
    calls.append(L.cuts())
    t = float(restir.layout_shares(L, true)[rank])
    return t * (5.0 if rank == 1 and len(calls) == inflate_call else 1.0)


def _best_round_worker(rank, world, port, result):
    import json
    import torch.distributed as dist
    from romis_amd import distributed
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    distributed.geometry_cost = lambda *a, **k: _blob_cost()
    calls = []
    L, rec = distributed.balanced_layout(None, None, 3840, 2160, (2, 1), time_tile=lambda L: _true_share_time(
        L, rank, calls, 2), rounds=3)
    with open(f"{result}.{rank}", "w") as fh:
        json.dump({"cuts": L.cuts(), "rec": rec}, fh)
    dist.destroy_process_group()


def test_balanced_layout_keeps_the_best_measured_round(tmp_path, abi_lib):
    """distributed.balanced_layout with time_tile over 2 gloo ranks: the model layout and each of its refinements are
    measured, and every rank returns the same layout -- the best measured one, not the last refinement (a contended
    measurement, here the first refinement's on rank 1, must not be what the bench times)."""
    import json
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    result = str(tmp_path / "r")
    mp.spawn(_best_round_worker, args=(2, port, result), nprocs=2, join=True)
    outs = []
    for rank in range(2):
        with open(f"{result}.{rank}") as fh:
            outs.append(json.load(fh))
    assert outs[0] == outs[1]
    rec = outs[0]["rec"]
    eff = [r["measured_efficiency"] for r in rec["refinement"]]
    assert len(eff) == 4 and rec["chosen_round"] == int(np.argmax(eff))
    assert rec["chosen_round"] != 1 and eff[1] < min(eff[0], eff[2], eff[3])
    assert outs[0]["cuts"] == rec["refinement"][rec["chosen_round"]]["cuts"]
    assert max(eff) > eff[0]   # refinement from measured times beats the model's cuts
