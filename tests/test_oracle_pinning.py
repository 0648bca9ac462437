"""Pin the oracle (oracle/restir_oracle.c) against what the reference's OWN code computes.

Fixtures come from oracle/_ref/dump_ref -- the reference's scene.cpp / mesh.cpp / tone_mapping.cpp and its
vendored glm 0.9.9.9 compiled unmodified (tests/golden/make_ref_fixtures.py).  The reservoir arithmetic
itself cannot be pinned this way (those translation units need Embree / <format> / GL, absent here): see
DESIGN.md "Oracle".
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

from romis_amd import _abi, scene

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "ref_fixtures.json")


@pytest.fixture(scope="module")
def fx():
    with open(FIX) as fh:
        return json.load(fh)


_libm = C.CDLL("libm.so.6")
_libm.powf.restype = C.c_float
_libm.powf.argtypes = [C.c_float, C.c_float]
_libm.expf.restype = C.c_float
_libm.expf.argtypes = [C.c_float]


def glibc_powf(x, y):
    return _libm.powf(x, y)


def f32(bits):
    return np.asarray(bits, dtype=np.uint32).view(np.float32)


def farr(a):
    a = np.ascontiguousarray(a, np.float32)
    return a, a.ctypes.data_as(C.POINTER(C.c_float))


def test_glm_primitives_bit_exact(oracle, fx):
    """normalize / dot / length / distance / cross / mix / quat(euler) / quat * v in the oracle = vendored glm."""
    lib = oracle.lib()
    for rec in fx["glm"]:
        a, pa = farr(f32(rec["a"]))
        b, pb = farr(f32(rec["b"]))
        e, pe = farr(f32(rec["e"]))
        t = float(f32([rec["t"]])[0])
        out, po = farr(np.zeros(24, np.float32))
        lib.or_glm_probe(pa, pb, t, pe, po)
        got = out.view(np.uint32)
        assert list(got[0:4]) == rec["q"], "glm::quat(euler)"
        assert list(got[4:7]) == rec["normalize"]
        assert int(got[7]) == rec["dot"]
        assert int(got[8]) == rec["length"]
        assert int(got[9]) == rec["distance"]
        assert list(got[10:13]) == rec["cross"]
        assert list(got[13:16]) == rec["mix"]
        assert list(got[16:19]) == rec["rotate"], "quat * vec3"


def test_tonemap_matches_reference_build(oracle, fx):
    """exposureToneMapping: the oracle's glibc-restated expf / powf vs the reference's own tone_mapping.cpp
    (compiled unmodified, calling this image's libm): bit-identical on every fixture."""
    lib = oracle.lib()
    for rec in fx["tonemap"]:
        exposure, gamma = (float(x) for x in f32(rec[:2]))
        c, pc = farr(f32(rec[2]))
        want = f32(rec[3])
        out, po = farr(np.zeros(3, np.float32))
        lib.or_tonemap(pc, exposure, gamma, po)
        assert out.view(np.uint32).tolist() == want.view(np.uint32).tolist(), (exposure, gamma, c)


def test_regular_light_grid_bit_exact(fx):
    """romis_amd.scene.regular_light_grid == regularLightGrid (scene.cpp:5-28)."""
    g = fx["light_grid"]
    args = g["args"]
    lights = scene.regular_light_grid(f32(args["start"]), tuple(args["counts"]), f32(args["e01"]), f32(args["e02"]),
                                      f32(args["color"]), f32([args["free"]])[0])
    assert len(lights) == len(g["lights"])
    for l, rec in zip(lights, g["lights"]):
        for field, bits in zip(("p0", "p1", "p2"), rec):
            assert list(np.asarray(list(getattr(l, field)), np.float32).view(np.uint32)) == bits


def test_nightclub_lights_bit_exact():
    """nightclub_wall_grids() restates constructNightClubLights (scene.cpp:30-66) bit-exactly."""
    ref = scene.load_prebuilt("CornellNightClub").lights
    mine = scene.nightclub_wall_grids()
    assert len(ref) == len(mine) == 512
    for a, b in zip(ref, mine):
        assert a.type == b.type == _abi.LIGHT_PARALLELOGRAM
        for field in ("p0", "p1", "p2", "c0", "c1", "c2", "c3"):
            assert list(np.asarray(list(getattr(a, field)), np.float32).view(np.uint32)) == \
                list(np.asarray(list(getattr(b, field)), np.float32).view(np.uint32)), field


def test_prebuilt_scene_sizes():
    expect = {"SingleTriangle": (1, 1), "Cube": (12, 1), "CornellBox": (32, 1),
              "CornellBoxParallelogramLight": (32, 1), "CornellNightClub": (166, 512), "Monkey": (968, 2)}
    for name, (tris, lights) in expect.items():
        s = scene.load_prebuilt(name)
        assert s.num_triangles == tris and len(s.lights) == lights, name


def _glibc_vec(fn, *args):
    return np.array([fn(*map(float, a)) for a in zip(*args)], np.float32)


def test_portable_powf_matches_glibc(oracle):
    """or_powf (glibc 2.35's __powf_fma restated; the device runs the same sequence) vs this image's powf --
    what std::pow(float, float) calls in the reference (shading.cpp:26): bit-identical, random bases and
    exponents, every bit pattern class (the exhaustive sweep is oracle/check_libm.c, profiles/r2/libm_check.jsonl)."""
    lib = oracle.lib()
    rng = np.random.default_rng(7)
    n = 20000
    x = np.concatenate([rng.uniform(-1, 1, n), rng.uniform(0, 4, n), rng.uniform(0.99, 1.0, n),
                        rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)]).astype(np.float32)
    y = np.concatenate([np.full(n, 250.0), rng.uniform(-30, 30, n), np.full(n, 1 / 2.2),
                        rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)]).astype(np.float32)
    got = np.empty_like(x)
    lib.or_powf_n(x.ctypes.data, y.ctypes.data, got.ctypes.data, x.size)
    want = _glibc_vec(glibc_powf, x, y)
    assert got.view(np.uint32).tolist() == want.view(np.uint32).tolist()


def test_portable_expf_matches_glibc(oracle):
    lib = oracle.lib()
    rng = np.random.default_rng(8)
    x = np.concatenate([rng.uniform(-110, 90, 40000), -rng.exponential(2.0, 20000),
                        rng.integers(0, 2**32, 20000, dtype=np.uint64).astype(np.uint32).view(np.float32)]).astype(np.float32)
    got = np.empty_like(x)
    lib.or_expf_n(x.ctypes.data, got.ctypes.data, x.size)
    want = _glibc_vec(_libm.expf, x)
    assert got.view(np.uint32).tolist() == want.view(np.uint32).tolist()


def test_check_libm_strided_sweep():
    """oracle/check_libm.c over every 251st 32-bit pattern (17 M bases per exponent, and expf): 0 mismatches."""
    import subprocess
    root = os.path.dirname(HERE)
    subprocess.check_call(["make", "-s", "-C", os.path.join(root, "oracle"), "check_libm"])
    out = subprocess.run([os.path.join(root, "oracle", "_build", "check_libm"), "8", "251"], capture_output=True,
                         text=True, timeout=300)
    recs = [json.loads(l) for l in out.stdout.splitlines() if l.strip()]
    assert len(recs) == 7 and out.returncode == 0, out.stdout + out.stderr
    assert all(r["mismatches"] == 0 for r in recs)


@pytest.mark.parametrize("x,y", [(0.0, 2.0), (-0.0, 3.0), (0.0, -1.0), (-0.0, -3.0), (1.0, float("nan")),
                                 (float("nan"), 0.0), (-2.0, 3.0), (-2.0, 0.5), (float("inf"), -1.0),
                                 (-float("inf"), 3.0), (-float("inf"), 2.0), (0.5, float("inf")), (2.0, -float("inf")),
                                 (-1.0, float("inf")), (-0.7, 250.0), (-0.7, 251.0), (1e-30, 5.0), (3.0, 200.0)])
def test_portable_powf_special_cases(oracle, x, y):
    got = np.float32(oracle.lib().or_powf(x, y))
    want = np.float32(glibc_powf(x, y))
    if np.isnan(want):
        assert np.isnan(got)
    else:
        assert got == want and np.signbit(got) == np.signbit(want), (x, y, got, want)


def test_rng_golden_values(oracle):
    """The keyed RNG contract (include/restir_c.h) pinned to fixed values."""
    lib = oracle.lib()
    key = lib.or_rng_key(0x5EED0001, 0, 1, 0)
    got = [lib.or_rng_draw(key, g, s) for g in (0, 1, 1920 * 1080 - 1) for s in (0, 1, 127)]
    with open(os.path.join(HERE, "golden", "rng_golden.json")) as fh:
        want = json.load(fh)
    assert key == want["key"]
    assert got == want["draws"]


def test_cube_textured_scene_carries_its_image():
    """loadScenePrebuilt(CubeTextured) (scene.cpp:91-95): one mesh with map_Kd default.png -- a 128 x 128 Image
    whose texels are the stb bytes / 255.0f (the harness checked every texel against the reference's pixels)
    -- and per-vertex texture coordinates from the OBJ's vt records."""
    s = scene.load_prebuilt("CubeTextured")
    assert len(s.meshes) == 1 and len(s.lights) == 1
    m = s.meshes[0]
    assert m.texture is not None and m.texture.rgb.shape == (128, 128, 3)
    assert m.texcoords is not None and m.texcoords.shape == (len(m.positions), 2)
    assert 0.0 <= m.texcoords.min() and m.texcoords.max() <= 1.0
    assert len(np.unique(m.texture.rgb.reshape(-1, 3), axis=0)) >= 2


def test_acquire_texel_matches_reference_build(oracle, fx):
    """acquireTexel (texture.cpp:4-9), compiled unmodified into oracle/_ref: the oracle's restatement returns
    the reference's texel bit for bit on random, edge and texel-boundary coordinates."""
    s = scene.load_prebuilt(fx["texel"]["scene"])
    osc = oracle.OracleScene(s)
    for tc_bits, want_bits in fx["texel"]["cases"]:
        got = oracle.acquire_texel(osc, 0, f32(tc_bits))
        assert got.view(np.uint32).tolist() == want_bits, f32(tc_bits)
