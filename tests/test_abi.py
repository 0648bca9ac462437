"""CPU tests of the C-ABI library: it loads, exports every symbol include/restir_c.h declares, and its pure
host logic (keyed RNG, camera derivation, tile plan, Features defaults) agrees with the oracle.  No GPU calls."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from romis_amd import _abi, scene

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    with open(os.path.join(ROOT, "include", "restir_c.h")) as fh:
        text = fh.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s+(restir_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_declared_symbol(abi_lib):
    names = declared_functions()
    assert len(names) >= 29
    for n in names:
        assert hasattr(abi_lib, n), n
    assert set(names) == set(_abi.SIGNATURES), "romis_amd/_abi.py must bind exactly the header's functions"
    assert abi_lib.restir_abi_version() == _abi.RESTIR_ABI_VERSION == 5


def test_rng_matches_oracle(abi_lib, oracle):
    ol = oracle.lib()
    for seed, frame, stage, p in [(0x5EED0001, 0, 1, 0), (7, 3, 3, 1), (0, 0, 2, 0), (0xFFFFFFFF, 123, 3, 4)]:
        k = abi_lib.restir_rng_key(seed, frame, stage, p)
        assert k == ol.or_rng_key(seed, frame, stage, p)
        for g in (0, 5, 99999, 33177599):
            for s in (0, 1, 2, 3, 130, 1023):
                assert abi_lib.restir_rng_draw(k, g, s) == ol.or_rng_draw(k, g, s)


@pytest.mark.parametrize("which", ["nightclub", "cornell", "odd"])
def test_camera_derive_matches_oracle(abi_lib, oracle, which):
    cam = {"nightclub": scene.nightclub_camera(1920, 1080), "cornell": scene.cornell_camera(512, 512),
           "odd": scene.make_camera(73.0, 0.5, (1, -2, 3), (-95.0, 400.0, 12.5), 7, 3)}[which]
    a, b = _abi.CameraFrame(), _abi.CameraFrame()
    abi_lib.restir_camera_derive(C.byref(cam), C.byref(a))
    oracle.lib().or_camera_derive(C.byref(cam), C.byref(b))
    fa = np.frombuffer(bytes(a), np.uint32)
    fb = np.frombuffer(bytes(b), np.uint32)
    assert np.array_equal(fa, fb)


@pytest.mark.parametrize("W,H,tx,ty,ghost", [(1920, 1080, 1, 1, 10), (3840, 1080, 2, 1, 10), (3840, 2160, 2, 2, 20),
                                             (7680, 2160, 4, 2, 10), (101, 37, 4, 2, 3), (5, 5, 5, 5, 0)])
def test_tile_plan_partitions_image(abi_lib, W, H, tx, ty, ghost):
    owner = np.full((H, W), -1, np.int32)
    for r in range(tx * ty):
        t = _abi.Tile()
        assert abi_lib.restir_tile_plan(W, H, tx, ty, r, ghost, C.byref(t)) == 0
        assert (t.global_width, t.global_height) == (W, H)
        assert (owner[t.y0:t.y0 + t.height, t.x0:t.x0 + t.width] == -1).all()
        owner[t.y0:t.y0 + t.height, t.x0:t.x0 + t.width] = r
        assert t.gx0 == max(0, t.x0 - ghost) and t.gy0 == max(0, t.y0 - ghost)
        assert t.gx0 + t.gwidth == min(W, t.x0 + t.width + ghost)
        assert t.gy0 + t.gheight == min(H, t.y0 + t.height + ghost)
    assert (owner >= 0).all()


def test_tile_plan_rejects_bad_arguments(abi_lib):
    t = _abi.Tile()
    assert abi_lib.restir_tile_plan(10, 10, 2, 2, 4, 0, C.byref(t)) == 1
    assert abi_lib.restir_tile_plan(0, 10, 1, 1, 0, 0, C.byref(t)) == 1
    assert abi_lib.restir_tile_plan(3, 10, 4, 1, 0, 0, C.byref(t)) == 1
    assert b"restir_tile_plan" in abi_lib.restir_last_error()


def test_features_default_matches_reference_struct(abi_lib):
    f = _abi.Features()
    abi_lib.restir_features_default(C.byref(f))
    assert bytes(f) == bytes(_abi.default_features())
    assert f.num_samples_in_reservoir == 2 and f.initial_light_samples == 32 and f.spatial_resample_radius == 10
    assert f.spatial_resampling_passes == 2 and f.temporal_clamp_m == 20 and abs(f.exposure - 1.5) < 1e-7


def test_context_calls_fail_cleanly_on_null(abi_lib):
    assert abi_lib.restir_set_seed(None, 1, 2) == 1
    assert abi_lib.restir_set_renders_dir(None, b"/tmp") == 1
    assert abi_lib.restir_synchronize(None) == 1
    assert abi_lib.restir_render(None, None, None, 1, 1, None, None, None, None) == 1


@pytest.mark.parametrize("W,H,tx,ty,R,N", [(72, 40, 2, 1, 10, 1), (97, 61, 2, 2, 10, 2), (3840, 2160, 4, 2, 10, 1),
                                          (50, 30, 4, 2, 7, 1)])
def test_halo_plan_is_symmetric_and_covers_the_ring(abi_lib, W, H, tx, ty, R, N):
    from romis_amd import restir
    plans = {q: restir.halo_plan(W, H, tx, ty, q, R, N) for q in range(tx * ty)}
    for q, (send, recv) in plans.items():
        assert [s.rank for s in send] == [r.rank for r in recv] == sorted(s.rank for s in send)
        off = 0
        for s in send:
            assert s.offset == off and s.bytes == s.width * s.height * N * 32
            off += s.bytes
        # what q sends to p is exactly what p expects from q
        for s in send:
            peer_recv = {r.rank: r for r in plans[s.rank][1]}[q]
            assert (peer_recv.x0, peer_recv.y0, peer_recv.width, peer_recv.height) == (s.x0, s.y0, s.width, s.height)
        # the received rectangles tile the ring: (owned grown by R, clipped) minus owned
        t = restir.tile_plan(W, H, tx, ty, q, R)
        cover = np.zeros((H, W), np.int32)
        for r in recv:
            cover[r.y0:r.y0 + r.height, r.x0:r.x0 + r.width] += 1
        want = np.zeros((H, W), np.int32)
        want[t.gy0:t.gy0 + t.gheight, t.gx0:t.gx0 + t.gwidth] = 1
        want[t.y0:t.y0 + t.height, t.x0:t.x0 + t.width] = 0
        assert np.array_equal(cover, want)
