"""GPU parity: every HIP kernel of libromis_amd.so against the CPU oracle (oracle/restir_oracle.c), through
the C ABI.  Stage-isolated: each pass gets the ORACLE's inputs (G-buffer, reservoirs) uploaded, so a
mismatch points at one kernel.  Bar: selected samples, M and every float bit-exact (the device reproduces
the reference's float operation order; DESIGN.md "Floating point"); RGB within 1e-5 relative as north_star
allows, checked bit-exact too where it holds.
"""
import numpy as np
import pytest

from romis_amd import _abi, scene

pytestmark = pytest.mark.gpu

W, H = 96, 64
SEED = _abi.RESTIR_DEFAULT_SEED
DEFAULT_GATHER = 1   # the library's spatial.gather default (restir_types.h Tuning::spatial_gather)


@pytest.fixture(scope="module")
def gpu():
    from romis_amd import build, restir
    build.build()
    r = restir.Renderer(0)
    yield r
    r.close()


_scenes = {}


def get_scene(name):
    if name not in _scenes:
        if name == "cornell_1024_shuffled":   # a light grid whose order is not regularLightGrid's (no kLtRegular form)
            base = scene.bench_scene("cornell_1024")
            perm = np.random.default_rng(7).permutation(len(base.lights))
            _scenes[name] = scene.Scene(base.meshes, [base.lights[i] for i in perm], name)
        else:
            _scenes[name] = scene.bench_scene(name) if name not in ("Cube", "CubeTextured") else scene.load_prebuilt(name)
    return _scenes[name]


def setup(gpu, oracle, name, N, w=W, h=H):
    s = get_scene(name)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.camera_for(name, w, h)
    gpu.stage_configure(w, h, N)
    return s, osc, cam


def origin(oracle, cam):
    return np.asarray(list(oracle.camera_frame(cam).origin), np.float32)


def key(stage, p=0, frame=0):
    from oracle import pyoracle
    return pyoracle.lib().or_rng_key(SEED, frame, stage, p)


def assert_bits(got, want, what):
    g = np.ascontiguousarray(got, np.float32).reshape(-1)
    w_ = np.ascontiguousarray(want, np.float32).reshape(-1)
    assert g.shape == w_.shape, f"{what}: shape {g.shape} != {w_.shape}"
    bad = np.flatnonzero(g.view(np.uint32) != w_.view(np.uint32))
    assert bad.size == 0, f"{what}: {bad.size}/{g.size} words differ; first idx {bad[:4].tolist()} " \
                          f"got {g[bad[:4]].tolist()} want {w_[bad[:4]].tolist()}"


def oracle_ris(oracle, osc, f, cam, n_t, p_mat, frame=0, w=W, h=H):
    return oracle.ris(osc, f, key(_abi.RESTIR_STAGE_RIS, 0, frame), origin(oracle, cam), w, h, n_t, p_mat)


SCENES = ["nightclub_128pt", "nightclub_512", "cornell_parallelogram", "Cube"]


@pytest.mark.parametrize("name", SCENES)
def test_primary_gbuffer_bit_exact(gpu, oracle, name):
    _, osc, cam = setup(gpu, oracle, name, 1)
    gpu.stage_primary(cam)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    assert_bits(gpu.download(_abi.BUF_GBUF_N_T), n_t, "n_t")
    assert_bits(gpu.download(_abi.BUF_GBUF_P_MAT), p_mat, "p_mat")
    assert (n_t[:, 3] < 1e30).mean() > 0.05   # the camera sees geometry


@pytest.mark.parametrize("name", SCENES)
@pytest.mark.parametrize("N", [1, 2, 3])
def test_ris_bit_exact(gpu, oracle, name, N):
    _, osc, cam = setup(gpu, oracle, name, N)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    gpu.upload(_abi.BUF_GBUF_N_T, n_t)
    gpu.upload(_abi.BUF_GBUF_P_MAT, p_mat)
    f = _abi.default_features(num_samples_in_reservoir=N)
    gpu.stage_ris(cam, f, key(_abi.RESTIR_STAGE_RIS))
    a, b, d = oracle_ris(oracle, osc, f, cam, n_t, p_mat)
    assert_bits(gpu.download(_abi.BUF_RES_A), a, "res_a")
    assert_bits(gpu.download(_abi.BUF_RES_B), b, "res_b")
    assert_bits(gpu.download(_abi.BUF_RES_DBG), d, "wSum/chosen")


@pytest.mark.parametrize("variant", ["visibility", "no_shading", "M1", "M64"])
def test_ris_variants_bit_exact(gpu, oracle, variant):
    N = 2
    _, osc, cam = setup(gpu, oracle, "nightclub_512", N)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    gpu.upload(_abi.BUF_GBUF_N_T, n_t)
    gpu.upload(_abi.BUF_GBUF_P_MAT, p_mat)
    kw = {"visibility": dict(initial_samples_visibility_check=1), "no_shading": dict(enable_shading=0),
          "M1": dict(initial_light_samples=1), "M64": dict(initial_light_samples=64)}[variant]
    f = _abi.default_features(num_samples_in_reservoir=N, **kw)
    gpu.stage_ris(cam, f, key(_abi.RESTIR_STAGE_RIS))
    a, b, d = oracle_ris(oracle, osc, f, cam, n_t, p_mat)
    assert_bits(gpu.download(_abi.BUF_RES_A), a, "res_a")
    assert_bits(gpu.download(_abi.BUF_RES_B), b, "res_b")


def _extreme_scene(variant):
    """Scenes that push shade() off its fast forms: colour x reflectance products past 2^120 (per-component NaN
    tests, overflowing sums), lights so far that |L|^2 overflows (sqrt / reciprocal guards), and per-mesh
    shininess mixing integer exponents (non-uniform pow chains) with non-integer ones (general pow)."""
    import copy
    base = get_scene("nightclub_128pt")
    meshes = [copy.copy(m) for m in base.meshes]
    lights = [copy.copy(l) for l in base.lights]
    if variant == "huge_colour":
        for i, l in enumerate(lights):
            for a in range(3):
                l.c0[a] = 3.0e38 if i % 3 == 0 else l.c0[a] * 1e30
    elif variant == "far_lights":
        for i, l in enumerate(lights):
            if i % 2 == 0:
                for a in range(3):
                    l.p0[a] = l.p0[a] * (1e19 if i % 4 == 0 else 1e-19)
    elif variant == "mixed_shininess":
        shin = [250.0, 37.0, 1.0, 2.5, 1048576.0, 3.0, 64.0, 0.5, 17.0, 250.0]
        for i, m in enumerate(meshes):
            m.shininess = np.float32(shin[i % len(shin)])
            m.ks = np.asarray([0.5, 0.25, 0.125], np.float32)
    return scene.Scene(meshes, lights, "extreme_" + variant)


@pytest.mark.parametrize("variant", ["huge_colour", "far_lights", "mixed_shininess"])
def test_ris_and_spatial_extreme_scenes_bit_exact(gpu, oracle, variant):
    s = _extreme_scene(variant)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.nightclub_camera(W, H)
    N = 1
    gpu.stage_configure(W, H, N)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    gpu.upload(_abi.BUF_GBUF_N_T, n_t)
    gpu.upload(_abi.BUF_GBUF_P_MAT, p_mat)
    f = _abi.default_features(num_samples_in_reservoir=N)
    gpu.stage_ris(cam, f, key(_abi.RESTIR_STAGE_RIS))
    a, b, d = oracle_ris(oracle, osc, f, cam, n_t, p_mat)
    assert_bits(gpu.download(_abi.BUF_RES_A), a, "res_a")
    assert_bits(gpu.download(_abi.BUF_RES_B), b, "res_b")
    assert_bits(gpu.download(_abi.BUF_RES_DBG), d, "wSum/chosen")
    gpu.stage_spatial(cam, f, key(_abi.RESTIR_STAGE_SPATIAL, 0))
    a2, b2, d2 = oracle.spatial_pass(osc, f, key(_abi.RESTIR_STAGE_SPATIAL, 0), origin(oracle, cam), W, H, n_t, p_mat,
                                     (a, b))
    assert_bits(gpu.download(_abi.BUF_RES_A), a2, "spatial res_a")
    assert_bits(gpu.download(_abi.BUF_RES_B), b2, "spatial res_b")


def test_ris_no_lights(gpu, oracle):
    s = get_scene("nightclub_128pt")
    empty = scene.Scene(s.meshes, [], "dark")
    gpu.set_scene(empty)
    osc = oracle.OracleScene(empty)
    cam = scene.nightclub_camera(W, H)
    gpu.stage_configure(W, H, 2)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    gpu.upload(_abi.BUF_GBUF_N_T, n_t)
    gpu.upload(_abi.BUF_GBUF_P_MAT, p_mat)
    f = _abi.default_features()
    gpu.stage_ris(cam, f, key(_abi.RESTIR_STAGE_RIS))
    b = gpu.download(_abi.BUF_RES_B)
    assert (b[..., 3].view(np.uint32) == 1).all()   # Reservoir(N) ctor M = 1 survives (light.cpp:46)
    a, b2, _ = oracle_ris(oracle, osc, f, cam, n_t, p_mat)
    assert_bits(b, b2, "res_b")


@pytest.mark.parametrize("N", [1, 2])
@pytest.mark.parametrize("clamp", [20, 1])
def test_temporal_bit_exact(gpu, oracle, N, clamp):
    _, osc, cam = setup(gpu, oracle, "nightclub_128pt", N)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    f = _abi.default_features(num_samples_in_reservoir=N, temporal_clamp_m=clamp)
    # predecessor = frame 0 after one spatial pass (so its M exceeds the clamp for clamp=1), current = frame 1 RIS
    a0, b0, _ = oracle_ris(oracle, osc, f, cam, n_t, p_mat, frame=0)
    pa, pb, _ = oracle.spatial_pass(osc, f, key(_abi.RESTIR_STAGE_SPATIAL, 0, 0), origin(oracle, cam), W, H, n_t,
                                    p_mat, (a0, b0))
    ca, cb, _ = oracle_ris(oracle, osc, f, cam, n_t, p_mat, frame=1)
    for which, arr in [(_abi.BUF_GBUF_N_T, n_t), (_abi.BUF_GBUF_P_MAT, p_mat), (_abi.BUF_RES_A, ca),
                       (_abi.BUF_RES_B, cb), (_abi.BUF_PREV_A, pa), (_abi.BUF_PREV_B, pb)]:
        gpu.upload(which, arr)
    kt = key(_abi.RESTIR_STAGE_TEMPORAL, 0, 1)
    gpu.stage_temporal(cam, f, kt)
    oa, ob, od = oracle.temporal(osc, f, kt, origin(oracle, cam), W, H, n_t, p_mat, (ca, cb), (pa, pb))
    assert_bits(gpu.download(_abi.BUF_RES_A), oa, "res_a")
    assert_bits(gpu.download(_abi.BUF_RES_B), ob, "res_b")
    assert_bits(gpu.download(_abi.BUF_RES_DBG), od, "wSum/chosen")


# spatial kernels of a stage-API pass (no sample handles: those are restir_render's, test_spatial_handles_*):
# k_spatial1_ntl (n_t staged, N = 1 biased; _t2: 32x16 tiles) in several XCD tile orders, k_spatial2_ntl, k_spatial1u,
# the general kernels
SPATIAL_VARIANTS = {"default": {},
                    "ntl": {"spatial.lean": 1, "spatial.th": 1},
                    "ntl_band": {"spatial.lean": 1, "spatial.th": 1, "spatial.xcd_rows": 0},
                    "ntl_rows2": {"spatial.lean": 1, "spatial.xcd_rows": 2},
                    "ntl_t2": {"spatial.lean": 1, "spatial.th": 2},
                    "ntl_t2_band": {"spatial.lean": 1, "spatial.th": 2, "spatial.xcd_rows": 0},
                    # 2-D XCD chunks (2 x 2 tiles; the image's 3 tile columns leave a partial chunk on the right)
                    "ntl_2d": {"spatial.lean": 1, "spatial.th": 1, "spatial.xcd_rows": 2, "spatial.xcd_cols": 2},
                    "ntl_t2_2d": {"spatial.lean": 1, "spatial.th": 2, "spatial.xcd_rows": 1, "spatial.xcd_cols": 2},
                    "general": {"spatial.lean": 0}}
SPATIAL_DEFAULTS = {"spatial.lean": 1, "spatial.xcd_rows": 255, "spatial.xcd_cols": 255, "spatial.th": 0}


# every (scene, N, combine mode) through the default knobs; the other variants differ only for N = 1 biased passes,
# so they run only there
SPATIAL_CASES = ([("default", name, N, mode) for name in ("nightclub_128pt", "cornell_parallelogram") for N in (1, 2, 3)
                  for mode in ("biased", "unbiased", "unbiased_vis")] +
                 [(lean, name, 1, "biased") for lean in SPATIAL_VARIANTS if lean != "default"
                  for name in ("nightclub_128pt", "cornell_parallelogram")] +
                 [("ntl_2d", "cornell_parallelogram", N, mode) for N in (1, 2) for mode in ("unbiased_vis", "biased")
                  if (N, mode) != (1, "biased")])


@pytest.mark.parametrize("lean,name,N,mode", SPATIAL_CASES)
def test_spatial_pass_bit_exact(gpu, oracle, name, N, mode, lean):
    for k, v in SPATIAL_VARIANTS[lean].items():
        gpu.set_tuning(k, v)
    try:
        _, osc, cam = setup(gpu, oracle, name, N)
        n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
        f = _abi.default_features(num_samples_in_reservoir=N, unbiased_combination=int(mode != "biased"),
                                  spatial_reuse_visibility_check=int(mode == "unbiased_vis"))
        a, b, _ = oracle_ris(oracle, osc, f, cam, n_t, p_mat)
        for which, arr in [(_abi.BUF_GBUF_N_T, n_t), (_abi.BUF_GBUF_P_MAT, p_mat), (_abi.BUF_RES_A, a),
                           (_abi.BUF_RES_B, b)]:
            gpu.upload(which, arr)
        for p in range(2):
            kp = key(_abi.RESTIR_STAGE_SPATIAL, p)
            gpu.stage_spatial(cam, f, kp)
            a, b, d = oracle.spatial_pass(osc, f, kp, origin(oracle, cam), W, H, n_t, p_mat, (a, b))
            assert_bits(gpu.download(_abi.BUF_RES_A), a, f"pass {p} res_a")
            assert_bits(gpu.download(_abi.BUF_RES_B), b, f"pass {p} res_b")
            assert_bits(gpu.download(_abi.BUF_RES_DBG), d, f"pass {p} wSum/chosen")
    finally:
        for k, v in SPATIAL_DEFAULTS.items():
            gpu.set_tuning(k, v)


@pytest.mark.parametrize("k,r", [(0, 10), (10, 30), (5, 1)])
def test_spatial_neighbour_ranges(gpu, oracle, k, r):
    N = 1
    _, osc, cam = setup(gpu, oracle, "nightclub_128pt", N)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    f = _abi.default_features(num_samples_in_reservoir=N, num_neighbours_to_sample=k, spatial_resample_radius=r)
    a, b, _ = oracle_ris(oracle, osc, f, cam, n_t, p_mat)
    for which, arr in [(_abi.BUF_GBUF_N_T, n_t), (_abi.BUF_GBUF_P_MAT, p_mat), (_abi.BUF_RES_A, a), (_abi.BUF_RES_B, b)]:
        gpu.upload(which, arr)
    kp = key(_abi.RESTIR_STAGE_SPATIAL, 0)
    gpu.stage_spatial(cam, f, kp)
    a2, b2, _ = oracle.spatial_pass(osc, f, kp, origin(oracle, cam), W, H, n_t, p_mat, (a, b))
    assert_bits(gpu.download(_abi.BUF_RES_A), a2, "res_a")
    assert_bits(gpu.download(_abi.BUF_RES_B), b2, "res_b")


@pytest.mark.parametrize("N", [1, 2])
@pytest.mark.parametrize("tonemap", [1, 0])
def test_final_shading(gpu, oracle, N, tonemap):
    _, osc, cam = setup(gpu, oracle, "nightclub_512", N)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    f = _abi.default_features(num_samples_in_reservoir=N, enable_tone_mapping=tonemap, gamma=2.2)
    a, b, _ = oracle_ris(oracle, osc, f, cam, n_t, p_mat)
    for which, arr in [(_abi.BUF_GBUF_N_T, n_t), (_abi.BUF_GBUF_P_MAT, p_mat), (_abi.BUF_RES_A, a), (_abi.BUF_RES_B, b)]:
        gpu.upload(which, arr)
    gpu.stage_final(cam, f)
    got = gpu.download(_abi.BUF_RGB)
    want = oracle.final(osc, f, origin(oracle, cam), W, H, n_t, p_mat, (a, b))
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-7)
    assert_bits(got, want, "rgb")


@pytest.mark.parametrize("name", ["nightclub_128pt", "cornell_1024"])
@pytest.mark.parametrize("binned", [1, 0])
@pytest.mark.parametrize("N", [1, 2])
def test_final_shading_binned_rays(gpu, oracle, name, binned, N):
    """final.sort (N = 1 and 2, the default): rays traced in target-bin order by other lanes -- the image must not
    change; final.sort 0: the unbinned kernel."""
    _, osc, cam = setup(gpu, oracle, name, N)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    f = _abi.default_features(num_samples_in_reservoir=N)
    a, b, _ = oracle_ris(oracle, osc, f, cam, n_t, p_mat)
    for which, arr in [(_abi.BUF_GBUF_N_T, n_t), (_abi.BUF_GBUF_P_MAT, p_mat), (_abi.BUF_RES_A, a), (_abi.BUF_RES_B, b)]:
        gpu.upload(which, arr)
    gpu.set_tuning("final.sort", binned)
    try:
        gpu.stage_final(cam, f)
    finally:
        gpu.set_tuning("final.sort", 1)
    want = oracle.final(osc, f, origin(oracle, cam), W, H, n_t, p_mat, (a, b))
    assert_bits(gpu.download(_abi.BUF_RGB), want, "rgb")


@pytest.mark.parametrize("name,N,compact,lds", [
    ("nightclub_128pt", 1, 1, 1), ("nightclub_128pt", 2, 1, 1), ("nightclub_128pt", 1, 1, 0), ("nightclub_128pt", 1, 0, 1),
    ("cornell_1024", 1, 1, 1), ("cornell_1024", 2, 1, 1), ("cornell_1024", 1, 1, 0), ("cornell_1024", 2, 0, 1),
    ("cornell_1024", 1, 2, 1), ("cornell_1024", 1, 2, 0), ("cornell_4096", 1, 1, 1), ("cornell_4096", 1, 2, 1),
    ("cornell_1024_shuffled", 1, 1, 1),
    ("nightclub_512", 1, 1, 1), ("nightclub_512", 2, 1, 1), ("nightclub_512", 2, 1, 0), ("nightclub_512", 2, 0, 1)])
def test_ris_compact_light_tables(gpu, oracle, name, N, compact, lds):
    """ris.compact (default 1): point-light-only scenes (C2), light grids (C4 / C5: parallelograms sharing their
    edges, one colour per light) and one-colour parallelograms (the reference's 512-light nightclub) run the _pt /
    _grid / _pg RIS kernels over the compact light tables, staged
    in LDS (ris.lds 1) or read from global memory (0); ris.compact 0: the general kernels on the same scene.  Light
    grids in regularLightGrid's order (cornell_1024 / _4096) take the _reg kernels at N = 1 (corner by arithmetic,
    colour table only; ris.compact 2 keeps the _grid table form), a shuffled grid the _grid form.  Each bit-exact vs
    the oracle, through the unfused k_ris (stage_ris) and the fused k_primary_ris of a whole frame."""
    s = get_scene(name)
    if name.startswith("cornell_"):   # the scene must qualify as a light grid, or this would test the general form
        e = np.array([[*l.p1, *l.p2] for l in s.lights], np.float32)
        c = np.array([[*l.c0, *l.c1, *l.c2, *l.c3] for l in s.lights], np.float32).reshape(-1, 4, 3)
        assert (e.view(np.uint32) == e[0].view(np.uint32)).all() and (c.view(np.uint32) == c[:, :1].view(np.uint32)).all()
    if name == "nightclub_512":   # one colour per light, edges not shared: the kLtPgram form
        e = np.array([[*l.p1, *l.p2] for l in s.lights], np.float32)
        c = np.array([[*l.c0, *l.c1, *l.c2, *l.c3] for l in s.lights], np.float32).reshape(-1, 4, 3)
        assert (c.view(np.uint32) == c[:, :1].view(np.uint32)).all() and not (e.view(np.uint32) == e[0].view(np.uint32)).all()
    _, osc, cam = setup(gpu, oracle, name, N)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    gpu.upload(_abi.BUF_GBUF_N_T, n_t)
    gpu.upload(_abi.BUF_GBUF_P_MAT, p_mat)
    f = _abi.default_features(num_samples_in_reservoir=N)
    gpu.set_tuning("ris.compact", compact)
    gpu.set_tuning("ris.lds", lds)
    try:
        gpu.stage_ris(cam, f, key(_abi.RESTIR_STAGE_RIS))
        a, b, d = oracle_ris(oracle, osc, f, cam, n_t, p_mat)
        assert_bits(gpu.download(_abi.BUF_RES_A), a, "res_a")
        assert_bits(gpu.download(_abi.BUF_RES_B), b, "res_b")
        assert_bits(gpu.download(_abi.BUF_RES_DBG), d, "wSum/chosen")
        fr = _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=1, spatial_reuse=1,
                                   temporal_reuse=0)
        gpu.set_seed(SEED, 0)
        rgb, grid = gpu.render_restir(None, cam, W, H, fr)
        want, res, _ = oracle.render_frame(osc, cam, fr, W, H, SEED, 0)
        assert_bits(rgb, want, "frame rgb")
        assert_grid(grid, res, "frame")
    finally:
        gpu.set_tuning("ris.compact", 1)
        gpu.set_tuning("ris.lds", 1)


def test_device_math_matches_oracle(gpu, oracle):
    """gl_powf / gl_expf on the GPU == the oracle's glibc restatement (== this image's libm, bit for bit:
    tests/test_oracle_pinning.py) -- the scenes' exponents over 2^20 random bit patterns each, random exponents,
    and the special cases."""
    rng = np.random.default_rng(3)
    bits = lambda n: rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    n = 1 << 20
    xs, ys = [], []
    for e in (1.0, 4.0, 10.0, 250.0, 1 / 2.2, 1 / 2.4):
        xs += [bits(n), rng.uniform(-1, 1, n // 4)]
        ys += [np.full(n, e), np.full(n // 4, e)]
    xs += [rng.uniform(0, 50, 4096), bits(n), [0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-40, -3.0, 2.0]]
    ys += [rng.uniform(-3, 3, 4096), bits(n), [2.0, 3.0, np.nan, np.inf, -1.0, 3.0, 0.0, 5.0, 0.5, -np.inf]]
    x = np.concatenate([np.asarray(a, np.float32) for a in xs])
    y = np.concatenate([np.asarray(a, np.float32) for a in ys])
    pw, ex = gpu.debug_math(x, y)
    lib = oracle.lib()
    want_pw, want_ex = np.empty_like(x), np.empty_like(x)
    lib.or_powf_n(x.ctypes.data, y.ctypes.data, want_pw.ctypes.data, x.size)
    lib.or_expf_n(x.ctypes.data, want_ex.ctypes.data, x.size)
    assert_bits(pw, want_pw, "powf")
    assert_bits(ex, want_ex, "expf")


def assert_grid(grid, res, what):
    """The device grid renderReSTIR returns (restir_frame_download) == the oracle's reservoirs: selected light
    sample (position, colour), W and M of every sub-reservoir of every pixel, bit for bit."""
    a, b = res
    pos, col, w, m = grid.download()
    N, vh, vw = w.shape
    a = a.reshape(N, vh, vw, 4)
    b = b.reshape(N, vh, vw, 4)
    assert_bits(pos, np.ascontiguousarray(a[..., :3]), f"{what} grid position")
    assert_bits(w, np.ascontiguousarray(a[..., 3]), f"{what} grid W")
    assert_bits(col, np.ascontiguousarray(b[..., :3]), f"{what} grid colour")
    assert np.array_equal(m, np.ascontiguousarray(b[..., 3]).view(np.uint32)), f"{what} grid M"


# --------------------------------------------------------------------------------------------------------
# whole frames through restir_render (renderReSTIR)
# the BASELINE.json configs at parity-test size: C1 (RIS only), C2, the 512-parallelogram nightclub, C4 (1024
# ceiling lights), C5 (4096 lights, M=64, unbiased + visibility reuse), plus the default N=2 / two passes
@pytest.mark.parametrize("name,N,passes,unbiased,M,vis", [
    ("cornell_parallelogram", 1, 0, 0, 32, 0), ("nightclub_128pt", 1, 1, 0, 32, 0), ("nightclub_512", 2, 2, 0, 32, 0),
    ("cornell_parallelogram", 1, 2, 1, 32, 0), ("cornell_1024", 1, 1, 0, 32, 0), ("cornell_4096", 1, 1, 1, 64, 1),
    ("nightclub_128pt", 1, 2, 1, 32, 1), ("cornell_parallelogram", 1, 1, 1, 32, 1)])
def test_render_frame_matches_oracle(gpu, oracle, name, N, passes, unbiased, M, vis):
    s = get_scene(name)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.camera_for(name, W, H)
    f = _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=passes, unbiased_combination=unbiased,
                              temporal_reuse=0, initial_light_samples=M, spatial_reuse=1 if passes else 0,
                              spatial_reuse_visibility_check=vis)
    gpu.set_seed(SEED, 0)
    rgb, grid = gpu.render_restir(None, cam, W, H, f)
    want, res, _ = oracle.render_frame(osc, cam, f, W, H, SEED, 0)
    np.testing.assert_allclose(rgb, want, rtol=1e-5, atol=1e-7)
    assert_bits(rgb, want, "rgb")
    assert_grid(grid, res, name)


@pytest.mark.parametrize("name,framing", [("nightclub_128pt", None), ("cornell_1024", "framed"), ("cornell_4096", "framed")])
@pytest.mark.parametrize("th", [1, 2, "lds"])
@pytest.mark.parametrize("w,h,passes,M", [(96, 64, 1, 32), (37, 23, 2, 32), (130, 70, 2, 1), (64, 1, 1, 16),
                                          (70, 150, 1, 32)])
def test_spatial_handles_frames_match_oracle(gpu, oracle, name, framing, th, w, h, passes, M):
    """The biased passes over sample handles (k_spatial1h[_tN], round 5: W and M | light index planes staged in LDS
    beside the n_t window, point lights) at every tile height, ragged sizes, 1 and 2 passes: RGB and the returned grid
    bit-exact with the oracle (render_utils.cpp:87-140, reservoir.cpp:40-66); a pass before the last writes only its
    handles.  The RGB without a returned grid (bench.py's render) too.  cornell_1024 (C4's regular light grid, camera
    into the box): the grid handles (W, M | i, a, b) of k_spatial1g_t2, whose samples are rebuilt from RIS's draws of
    the light's fractions (32 x 16 tiles only: th = 1 runs the n_t-window pass instead); cornell_4096 (4,096 lights, past
    the handle pass's 1,024-colour table): the reservoir form, as the host falls back.  At 32 x 16 the point-light handle
    pass gathers the neighbours' handles from global memory (k_spatial1hg_t2, the default since round 6); "lds": the
    round-5 form with the handle windows staged in LDS beside the n_t window (k_spatial1h_t2)."""
    s = get_scene(name)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.camera_for(name, w, h, framing)
    f = _abi.default_features(num_samples_in_reservoir=1, spatial_resampling_passes=passes, temporal_reuse=0,
                              initial_light_samples=M)
    lds = th == "lds"   # 32 x 16 with the handle windows staged in LDS (k_spatial1h_t2) instead of gathered
    gpu.set_tuning("spatial.th", 2 if lds else th)
    gpu.set_tuning("spatial.gather", 0 if lds else DEFAULT_GATHER)
    try:
        gpu.set_seed(SEED, 0)
        rgb, grid = gpu.render_restir(None, cam, w, h, f)
        gpu.set_seed(SEED, 0)
        rgb_ng, _ = gpu.render_restir(None, cam, w, h, f, want_grid=False)
    finally:
        gpu.set_tuning("spatial.th", 0)
        gpu.set_tuning("spatial.gather", DEFAULT_GATHER)
    want, res, _ = oracle.render_frame(osc, cam, f, w, h, SEED, 0)
    assert_bits(rgb, want, f"th={th} {w}x{h} passes={passes}")
    assert_grid(grid, res, f"th={th} {w}x{h} passes={passes}")
    assert_bits(rgb_ng, want, f"no grid th={th} {w}x{h} passes={passes}")


@pytest.mark.parametrize("name,framing,N,temporal", [("nightclub_128pt", None, 1, 0), ("nightclub_128pt", None, 2, 0),
                                                    ("nightclub_128pt", None, 1, 1), ("cornell_1024", "framed", 1, 0),
                                                    ("cornell_1024", None, 1, 0), ("cornell_parallelogram", None, 1, 0),
                                                    ("nightclub_512", None, 2, 0)])
@pytest.mark.parametrize("w,h,tiled", [(96, 64, 0), (37, 23, 0), (333, 190, 1), (640, 360, 0)])
def test_primary_tile_lists_match_bvh(gpu, oracle, name, framing, N, temporal, w, h, tiled):
    """primary.tl (round 6): the fused primary + RIS kernel's primary rays test the candidate triangles of their 32 x 8
    tile (tile_triangles: every triangle not wholly outside one side of the tile's ray pyramid widened by two pixels)
    instead of walking the BVH; closest_list's selection (minimal t, lowest original index) is closest()'s.  RGB and
    the returned grid bit-exact with primary.tl = 0 -- whole frames and ghost-zoned tiles, N = 1 / 2, temporal frames
    (the fused temporal kernel), point lights, light grids, parallelograms, the TOML camera (background tiles) and the
    camera into the box -- and the RGB with the oracle."""
    from romis_amd import restir
    s = get_scene(name)
    gpu.set_scene(s)
    cam = scene.camera_for(name, w, h, framing)
    f = _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=1, temporal_reuse=temporal)
    tile = restir.tile_plan(w, h, 2, 2, 2, f.spatial_resample_radius) if tiled else None
    out = {}
    try:
        for on in (0, 1):
            gpu.set_tuning("primary.tl", on)
            gpu.set_seed(SEED, 0)
            prev = None
            for fr in range(2 if temporal else 1):   # a temporal frame needs its predecessor
                rgb, grid = gpu.render_restir(prev, cam, w, h, f, tile=None if temporal else tile)
                prev = grid
            out[on] = (rgb, [np.asarray(a) for a in grid.download()])
    finally:
        gpu.set_tuning("primary.tl", 1)
    assert_bits(out[1][0], out[0][0], f"{name} {w}x{h} rgb tl on / off")
    # a tiled frame's grid is defined on the owned rect (the ghost ring holds intermediate values, include/restir_c.h)
    own = (slice(None), slice(tile.y0 - tile.gy0, tile.y0 - tile.gy0 + tile.height),
           slice(tile.x0 - tile.gx0, tile.x0 - tile.gx0 + tile.width)) if (tile is not None and not temporal) else (slice(None),)
    for a, b in zip(out[0][1], out[1][1]):
        assert np.array_equal(a[own].view(np.uint32), b[own].view(np.uint32)), f"{name} {w}x{h} grid tl on / off"
    if not temporal and w * h <= 96 * 64:
        want, _, _ = oracle.render_frame(oracle.OracleScene(s), cam, f, w, h, SEED, 0)
        if tile is not None:
            r0 = h - (tile.y0 + tile.height)
            want = np.ascontiguousarray(want[r0:r0 + tile.height, tile.x0:tile.x0 + tile.width])
        assert_bits(out[1][0], want, f"{name} {w}x{h} against the oracle")


@pytest.mark.parametrize("th", [1, 2])
@pytest.mark.parametrize("w,h,passes,M", [(96, 64, 1, 32), (37, 23, 2, 32), (130, 70, 3, 1), (64, 1, 1, 16)])
def test_spatial_n2_handles_frames_match_oracle(gpu, oracle, th, w, h, passes, M):
    """N = 2 (the reference's default, common.h:105) biased passes over 16-byte handle records (k_spatial2hg[_t2], round
    6): RIS writes (W_0, M_0 | i_0, W_1, M_1 | i_1) instead of its reservoirs, each pass gathers an accepted neighbour's
    record and rebuilds both samples from the light table; a pass before the last writes only records.  RGB and the
    returned grid bit-exact with the oracle (render_utils.cpp:87-140, reservoir.cpp:10-66), and with the handle path off
    (spatial.n2h = 0: k_spatial2_ntl over the reservoirs)."""
    name = "nightclub_128pt"
    s = get_scene(name)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.camera_for(name, w, h)
    f = _abi.default_features(num_samples_in_reservoir=2, spatial_resampling_passes=passes, temporal_reuse=0,
                              initial_light_samples=M)
    gpu.set_tuning("spatial.th", th)
    try:
        gpu.set_seed(SEED, 0)
        rgb, grid = gpu.render_restir(None, cam, w, h, f)
        gpu.set_tuning("spatial.n2h", 0)
        gpu.set_seed(SEED, 0)
        rgb_off, _ = gpu.render_restir(None, cam, w, h, f, want_grid=False)
    finally:
        gpu.set_tuning("spatial.th", 0)
        gpu.set_tuning("spatial.n2h", 1)
    want, res, _ = oracle.render_frame(osc, cam, f, w, h, SEED, 0)
    assert_bits(rgb, want, f"N=2 th={th} {w}x{h} passes={passes}")
    assert_grid(grid, res, f"N=2 th={th} {w}x{h} passes={passes}")
    assert_bits(rgb_off, want, f"N=2 reservoir form th={th} {w}x{h} passes={passes}")


@pytest.mark.parametrize("w,h,N,passes,M", [(1, 1, 1, 2, 32), (37, 23, 2, 2, 32), (33, 9, 1, 1, 1), (40, 24, 32, 1, 8),
                                          (64, 1, 3, 2, 16), (1, 50, 1, 1, 32)])
def test_odd_sizes_and_extremes_match_oracle(gpu, oracle, w, h, N, passes, M):
    """Image sizes that are not tile multiples (1x1, 1-pixel rows / columns, ragged 32x8 tiles), the largest N
    (RESTIR_MAX_N = 32), M = 1 -- two temporal frames each."""
    name = "nightclub_512"
    s = get_scene(name)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.camera_for(name, w, h)
    f = _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=passes, temporal_reuse=1,
                              initial_light_samples=M)
    gpu.set_seed(SEED, 0)
    prev_gpu, prev_or = None, None
    for frame in range(2):
        rgb, grid = gpu.render_restir(prev_gpu, cam, w, h, f)
        want, res, _ = oracle.render_frame(osc, cam, f, w, h, SEED, frame, prev=prev_or)
        assert_bits(rgb, want, f"{w}x{h} N={N} frame {frame}")
        assert_grid(grid, res, f"{w}x{h} N={N} frame {frame}")
        prev_gpu, prev_or = grid, res


@pytest.mark.parametrize("records,fuse,N,variant", [(0, 1, 1, ""), (0, 1, 1, "rescene"), (0, 1, 1, "nohandles"),
                                                    (1, 1, 1, ""), (0, 0, 1, ""), (0, 1, 2, ""), (0, 0, 2, ""),
                                                    (0, 1, 1, "moving"), (0, 1, 1, "moving_ragged"), (0, 1, 2, "moving_ragged"),
                                                    (0, 1, 1, "mbound_in"), (0, 1, 1, "mbound_out"),
                                                    (0, 1, 2, "rescene"), (0, 1, 2, "nohandles"), (0, 1, 2, "moving"),
                                                    (0, 1, 2, "mbound_in"), (0, 1, 2, "mbound_out")])
def test_temporal_sequence_matches_oracle(gpu, oracle, records, fuse, N, variant):
    """C3-style: 4 static frames, temporal reuse threading the previous frame's grid (main.cpp:165); both frame
    buffer layouts (SoA planes, per-pixel records); temporal reuse fused into the primary + RIS kernel (fuse.temporal,
    the default for point lights) and as its own pass; N = 1 and 2.  N = 1 fused: the predecessor is rebuilt from the
    frame handles its last pass wrote and the passes read sample handles; "rescene" re-uploads the scene mid-sequence
    (the handles' light table is stale: the reservoir planes are read), "nohandles" turns the handle passes off.
    "moving" / "moving_ragged" pan the camera between frames (96 x 64 and a 37 x 23 frame that is no multiple of the 32 x 8
    / 32 x 16 tiles, clampM = 1): RIS tiles whose every pixel misses now while the predecessor held real lights there, so
    the fused kernel rebuilds those predecessors from its light table (the table must be staged for such
    tiles too).  "mbound_in" / "mbound_out": 5 and 6 passes at clampM = 20, the last M bound (M + clampM M + 1)(K + 1)^P
    that fits the handles' 24 bits and the first that does not (frame handles on / reservoir planes).  N = 2 fused (round 6):
    the predecessor is rebuilt from the 16-byte frame handle records and the passes read handle records (k_spatial2hg);
    its M bound counts both predecessor sub-reservoirs, M + 2 (clampM M + 1), and crosses 24 bits at the same pass count."""
    gpu.set_tuning("layout.records", records)
    gpu.set_tuning("fuse.temporal", fuse)
    if variant == "nohandles":
        gpu.set_tuning("spatial.handles", 0)
    try:
        if variant.startswith("moving"):
            w, h = (37, 23) if variant == "moving_ragged" else (W, H)
            _temporal_sequence(gpu, oracle, N, w=w, h=h, moving=True, clamp=1)
        elif variant.startswith("mbound"):
            _temporal_sequence(gpu, oracle, N, passes=5 if variant == "mbound_in" else 6, clamp=20)
        else:
            _temporal_sequence(gpu, oracle, N, rescene=variant == "rescene")
    finally:
        gpu.set_tuning("layout.records", 0)
        gpu.set_tuning("fuse.temporal", 1)
        gpu.set_tuning("spatial.handles", 1)


# a camera panning across the nightclub (lookAt offsets per frame): 40-80 % of the pixels change from hit to miss or back
_PAN = [(0.0, 0.0), (9.0, 4.0), (3.0, -2.0), (12.0, 6.0)]


def _temporal_sequence(gpu, oracle, N=1, rescene=False, w=W, h=H, moving=False, clamp=20, passes=2):
    name = "nightclub_128pt"
    s = get_scene(name)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.camera_for(name, w, h)
    f = _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=passes, temporal_reuse=1,
                              temporal_clamp_m=clamp)
    gpu.set_seed(SEED, 0)
    prev_gpu, prev_or = None, None
    for frame in range(4):
        if rescene and frame == 2:
            gpu.set_scene(s)   # a new upload: the predecessor's frame handles name the old one (reservoir planes read)
        if moving:
            dx, dy = _PAN[frame]
            cam = scene.make_camera(30.0, 25.0, (2.57 + dx, 1.23 + dy, -1.35), (10.3, 30.0, 0.0), w, h)
        rgb, grid = gpu.render_restir(prev_gpu, cam, w, h, f)
        want, res, _ = oracle.render_frame(osc, cam, f, w, h, SEED, frame, prev=prev_or)
        assert_bits(rgb, want, f"frame {frame} rgb")
        assert_grid(grid, res, f"frame {frame}")
        prev_gpu, prev_or = grid, res


@pytest.mark.parametrize("tiles,N", [((2, 1), 1), ((2, 2), 1), ((4, 2), 1), ((2, 2), 2), ((4, 2), 2)])
def test_tiles_stitch_to_full_frame(gpu, oracle, tiles, N):
    """Screen tiles with ghost zones (the multi-GPU decomposition) reproduce the single-GPU frame bit-exactly (N = 2:
    the handle-record passes, k_spatial2hg, on the ghost-zoned views too)."""
    from romis_amd import restir
    name = "nightclub_128pt"
    s = get_scene(name)
    gpu.set_scene(s)
    cam = scene.camera_for(name, W, H)
    f = _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=2, temporal_reuse=0)
    gpu.set_seed(SEED, 0)
    full, _ = gpu.render_restir(None, cam, W, H, f, want_grid=False)
    stitched = np.zeros_like(full)
    tx, ty = tiles
    for rank in range(tx * ty):
        t = restir.tile_plan(W, H, tx, ty, rank, f.spatial_resampling_passes * f.spatial_resample_radius)
        gpu.set_seed(SEED, 0)
        rgb, _ = gpu.render_restir(None, cam, W, H, f, tile=t, want_grid=False)
        # rgb rows: row 0 = top of the tile; the full image's row 0 = top (global y = H - 1)
        r0 = H - (t.y0 + t.height)
        stitched[r0:r0 + t.height, t.x0:t.x0 + t.width] = rgb
    assert_bits(stitched, full, "stitched tiles")


# --------------------------------------------------------------------------------------------------------
# full-size (BASELINE configs) checks: size-independent properties + oracle on sampled row bands
def test_full_1080p_spatial_properties_and_sampled_parity(gpu, oracle):
    Wf, Hf, N = 1920, 1080, 1
    name = "nightclub_128pt"
    s = get_scene(name)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.camera_for(name, Wf, Hf)
    gpu.stage_configure(Wf, Hf, N)
    f = _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=1)
    gpu.stage_primary(cam)
    gpu.stage_ris(cam, f, key(_abi.RESTIR_STAGE_RIS))
    n_t = gpu.download(_abi.BUF_GBUF_N_T)
    p_mat = gpu.download(_abi.BUF_GBUF_P_MAT)
    a0 = gpu.download(_abi.BUF_RES_A)
    b0 = gpu.download(_abi.BUF_RES_B)
    kp = key(_abi.RESTIR_STAGE_SPATIAL, 0)
    gpu.stage_spatial(cam, f, kp)
    a1 = gpu.download(_abi.BUF_RES_A)
    b1 = gpu.download(_abi.BUF_RES_B)
    M0 = b0[0, :, 3].view(np.uint32).astype(np.int64)
    M1 = b1[0, :, 3].view(np.uint32).astype(np.int64)
    # properties: M only grows, by whole input Ms, bounded by (k+1) * max input M; W finite, non-negative
    assert (M1 >= M0).all() and (M1 <= (f.num_neighbours_to_sample + 1) * M0.max()).all()
    assert np.isfinite(a1[0, :, 3]).all() and (a1[0, :, 3] >= 0).all()
    # the selected light sample of every pixel is the sample of a pixel inside its (2r+1)^2 window
    pos0 = a0[0, :, :3].reshape(Hf, Wf, 3)
    pos1 = a1[0, :, :3].reshape(Hf, Wf, 3)
    rng = np.random.default_rng(0)
    r = f.spatial_resample_radius
    for _ in range(200):
        y, x = int(rng.integers(0, Hf)), int(rng.integers(0, Wf))
        win = pos0[max(0, y - r):y + r + 1, max(0, x - r):x + r + 1].reshape(-1, 3)
        assert (win == pos1[y, x]).all(axis=1).any()
    # oracle parity on sampled row bands of the full-size frame
    o = origin(oracle, cam)
    for y0 in (0, 517, Hf - 8):
        rect = oracle.Rect(0, y0, Wf, 8)
        view = oracle.Rect(0, 0, Wf, Hf)
        a2, b2, _ = oracle.spatial_pass(osc, f, kp, o, Wf, Hf, n_t, p_mat, (a0, b0), view=view, rect=rect)
        sl = slice(y0 * Wf, (y0 + 8) * Wf)
        assert_bits(a1[:, sl], a2[:, sl], f"band {y0} res_a")
        assert_bits(b1[:, sl], b2[:, sl], f"band {y0} res_b")
    # initial RIS at full size on sampled bands: the GPU's own G-buffer fed to the oracle's RIS for those rows
    import ctypes as C
    from oracle import pyoracle
    for y0 in (0, 391, 806, Hf - 4):
        rect = oracle.Rect(0, y0, Wf, 4)
        view = oracle.Rect(0, 0, Wf, Hf)
        a_or = np.zeros_like(a0)
        b_or = np.zeros_like(b0)
        pyoracle.lib().or_ris(osc.handle, C.byref(f), key(_abi.RESTIR_STAGE_RIS), pyoracle.fp(o), Wf, Hf, view, rect,
                              pyoracle.fp(n_t), pyoracle.fp(p_mat), pyoracle.fp(a_or), pyoracle.fp(b_or), None)
        sl = slice(y0 * Wf, (y0 + 4) * Wf)
        assert_bits(a0[:, sl], a_or[:, sl], f"RIS band {y0} res_a")
        assert_bits(b0[:, sl], b_or[:, sl], f"RIS band {y0} res_b")
    # G-buffer on sampled bands too
    n_t_or = np.zeros_like(n_t)
    p_mat_or = np.zeros_like(p_mat)
    cf = pyoracle.camera_frame(cam)
    for y0 in (3, 700):
        rect = oracle.Rect(0, y0, Wf, 4)
        view = oracle.Rect(0, 0, Wf, Hf)
        pyoracle.lib().or_primary(osc.handle, C.byref(cf), Wf, Hf, view, rect, pyoracle.fp(n_t_or), pyoracle.fp(p_mat_or))
        sl = slice(y0 * Wf, (y0 + 4) * Wf)
        assert_bits(n_t[sl], n_t_or[sl], f"band {y0} n_t")
        assert_bits(p_mat[sl], p_mat_or[sl], f"band {y0} p_mat")


def test_full_1080p_render_deterministic(gpu):
    name = "nightclub_128pt"
    gpu.set_scene(get_scene(name))
    cam = scene.camera_for(name, 1920, 1080)
    f = _abi.default_features(num_samples_in_reservoir=1, spatial_resampling_passes=1, temporal_reuse=0)
    gpu.set_seed(SEED, 0)
    a, _ = gpu.render_restir(None, cam, 1920, 1080, f, want_grid=False)
    gpu.set_seed(SEED, 0)
    b, _ = gpu.render_restir(None, cam, 1920, 1080, f, want_grid=False)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.isfinite(a).all() and (a >= 0).all() and a.mean() > 0.01


def test_measured_read_bandwidth_is_plausible(gpu):
    gbs = gpu.measure_read_bandwidth(1 << 30, 3)
    assert 1000.0 < gbs < 9000.0, gbs     # MI355X HBM3E: 8 TB/s spec


def test_errors_are_reported(gpu):
    from romis_amd._abi import RestirError
    cam = scene.nightclub_camera(W, H)
    with pytest.raises(RestirError, match="UNSUPPORTED"):   # R-MIS / R-OMIS render whole images only
        tile = _abi.Tile(W, H, 0, 0, W // 2, H, 0, 0, W // 2 + 10, H)
        gpu.render_restir(None, cam, W, H, _abi.default_features(ray_trace_mode=_abi.MODE_ROMIS), tile=tile)
    with pytest.raises(RestirError, match="INVALID"):
        gpu.render_restir(None, cam, W, H, _abi.default_features(ray_trace_mode=7))
    with pytest.raises(RestirError, match="INVALID"):
        gpu.render_restir(None, cam, W, H, _abi.default_features(num_samples_in_reservoir=0))


def test_render_invalidates_stage_state(gpu, oracle):
    """A frame render re-sizes the context's shared view state: the stage API reports RESTIR_ERR_STATE until
    restir_stage_configure runs again, instead of copying with the frame's sizes (advisor finding)."""
    from romis_amd._abi import RestirError
    name = "nightclub_128pt"
    _, osc, cam = setup(gpu, oracle, name, 1)
    gpu.stage_configure(W, H, 1)
    big = scene.camera_for(name, 2 * W, 2 * H)
    gpu.render_restir(None, big, 2 * W, 2 * H, _abi.default_features(num_samples_in_reservoir=1, temporal_reuse=0))
    with pytest.raises(RestirError, match="STATE"):
        gpu.download(_abi.BUF_RES_A)


def test_temporal_frames_recycle_records(gpu, oracle):
    """Released temporal frames hand their records back to the context (stream-ordered): a long sequence whose
    predecessors are dropped as it goes stays bit-exact, and a predecessor read by a second context (its own
    stream) is waited for, not raced."""
    from romis_amd import restir
    name = "nightclub_128pt"
    s = get_scene(name)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.camera_for(name, W, H)
    f = _abi.default_features(num_samples_in_reservoir=1, spatial_resampling_passes=1, temporal_reuse=1)
    gpu.set_seed(SEED, 0)
    other = restir.Renderer(0)
    try:
        other.set_scene(s)
        prev_gpu, prev_or = None, None
        for frame in range(6):
            rgb, grid = gpu.render_restir(prev_gpu, cam, W, H, f, want_rgb=frame % 2 == 1)
            _, res, _ = oracle.render_frame(osc, cam, f, W, H, SEED, frame, prev=prev_or)
            if frame % 2 == 1:
                assert_grid(grid, res, f"frame {frame}")
            # the second context renders its frame `frame + 1` from this grid before the first context's
            # stream has necessarily finished writing it
            other.set_seed(SEED, frame + 1)
            rgb2, grid2 = other.render_restir(grid, cam, W, H, f)
            want2, res2, _ = oracle.render_frame(osc, cam, f, W, H, SEED, frame + 1, prev=res)
            assert_bits(rgb2, want2, f"second context frame {frame + 1}")
            del grid2
            prev_gpu, prev_or = grid, res   # the previous predecessor is released here
    finally:
        other.close()



# --------------------------------------------------------------------------------------------------------
# textures: diffuseAlbedo = acquireTexel(kdTexture, texCoord) on CubeTextured (scene.cpp:91-95)
TEX = "CubeTextured"


def test_textured_gbuffer_bit_exact(gpu, oracle):
    """genPrimaryRayHits on a textured scene also interpolates the hit's texCoord (embree_interface.cpp:80-81)."""
    _, osc, cam = setup(gpu, oracle, TEX, 1)
    gpu.stage_primary(cam)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    assert_bits(gpu.download(_abi.BUF_GBUF_N_T), n_t, "n_t")
    assert_bits(gpu.download(_abi.BUF_GBUF_P_MAT), p_mat, "p_mat")
    assert_bits(gpu.download(_abi.BUF_GBUF_UV), osc.uv, "texCoord")
    hit = n_t[:, 3] < 1e30
    assert hit.mean() > 0.05 and len(np.unique(osc.uv[hit], axis=0)) > 100


@pytest.mark.parametrize("texture", [1, 0])
@pytest.mark.parametrize("N", [1, 2])
def test_textured_stages_bit_exact(gpu, oracle, texture, N):
    """RIS, a spatial pass and final shading on CubeTextured with texture mapping on (texel albedo) and off
    (kd), each stage on the oracle's inputs."""
    _, osc, cam = setup(gpu, oracle, TEX, N)
    n_t, p_mat = oracle.gbuffer(osc, cam, W, H)
    for which, arr in [(_abi.BUF_GBUF_N_T, n_t), (_abi.BUF_GBUF_P_MAT, p_mat), (_abi.BUF_GBUF_UV, osc.uv)]:
        gpu.upload(which, arr)
    f = _abi.default_features(num_samples_in_reservoir=N, enable_texture_mapping=texture)
    gpu.stage_ris(cam, f, key(_abi.RESTIR_STAGE_RIS))
    a, b, d = oracle_ris(oracle, osc, f, cam, n_t, p_mat)
    assert_bits(gpu.download(_abi.BUF_RES_A), a, "ris res_a")
    assert_bits(gpu.download(_abi.BUF_RES_B), b, "ris res_b")
    assert_bits(gpu.download(_abi.BUF_RES_DBG), d, "ris wSum/chosen")
    kp = key(_abi.RESTIR_STAGE_SPATIAL, 0)
    gpu.stage_spatial(cam, f, kp)
    a, b, d = oracle.spatial_pass(osc, f, kp, origin(oracle, cam), W, H, n_t, p_mat, (a, b))
    assert_bits(gpu.download(_abi.BUF_RES_A), a, "spatial res_a")
    assert_bits(gpu.download(_abi.BUF_RES_B), b, "spatial res_b")
    gpu.stage_final(cam, f)
    want = oracle.final(osc, f, origin(oracle, cam), W, H, n_t, p_mat, (a, b))
    assert_bits(gpu.download(_abi.BUF_RGB), want, "rgb")


@pytest.mark.parametrize("texture", [1, 0])
def test_textured_frames_match_oracle(gpu, oracle, texture):
    """Whole CubeTextured frames (2 temporal frames, 2 spatial passes): images and returned grids bit-exact; the
    texture visibly changes the image."""
    s = get_scene(TEX)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.camera_for(TEX, W, H)
    f = _abi.default_features(num_samples_in_reservoir=1, spatial_resampling_passes=2, temporal_reuse=1,
                              enable_texture_mapping=texture)
    gpu.set_seed(SEED, 0)
    prev_gpu, prev_or = None, None
    first = None
    for frame in range(2):
        rgb, grid = gpu.render_restir(prev_gpu, cam, W, H, f)
        want, res, _ = oracle.render_frame(osc, cam, f, W, H, SEED, frame, prev=prev_or)
        assert_bits(rgb, want, f"frame {frame} rgb")
        assert_grid(grid, res, f"frame {frame}")
        prev_gpu, prev_or = grid, res
        first = want if first is None else first
    f0 = _abi.default_features(num_samples_in_reservoir=1, spatial_resampling_passes=2, temporal_reuse=1,
                               enable_texture_mapping=1 - texture)
    other, _, _ = oracle.render_frame(osc, cam, f0, W, H, SEED, 0, prev=None)
    assert not np.array_equal(other, first)


def geometry_bands(oracle, osc, cam, Wf, Hf, rows, n, min_hits=0.2):
    """n row bands of `rows` rows spread over the rows whose oracle primary rays hit the scene: every band's pixels
    are >= min_hits geometry (the oracle G-buffer of 64 candidate bands, not the GPU's)."""
    cands = []
    for y0 in np.linspace(0, Hf - rows, 64).astype(int):
        _, p_mat = oracle.gbuffer(osc, cam, Wf, Hf, oracle.Rect(0, int(y0), Wf, rows))
        if (p_mat[:, 3].view(np.uint32) != osc.miss_material).mean() >= min_hits:
            cands.append(int(y0))
    assert len(cands) >= n, f"only {len(cands)} bands hold >= {min_hits:.0%} geometry"
    return [cands[i] for i in np.linspace(0, len(cands) - 1, n).astype(int)]


# C4 (4K, 1024 parallelogram lights, k = 5 x1 biased) and C5 (8K, 4096 lights, M = 64, unbiased + spatial
# visibility reuse) at their full sizes, with the TOML camera (c4, c5: 13 % geometry) and looking into the box (c4f,
# c5f: 99.9 %): the GPU frame's RGB and returned grid (position, W, colour, M) on four row bands that each hold
# >= 20 % geometry by the oracle's G-buffer, against the oracle rendering those rows (with the ghost rows its spatial
# pass reads), bit for bit.
@pytest.mark.parametrize("cfg", ["c4", "c5", "c4f", "c5f"])
def test_full_size_frames_c4_c5_band_parity(gpu, oracle, cfg):
    name, Wf, Hf, M, unb = {"c4": ("cornell_1024", 3840, 2160, 32, 0), "c5": ("cornell_4096", 7680, 4320, 64, 1)}[cfg[:2]]
    s = get_scene(name)
    gpu.set_scene(s)
    gpu.set_seed(SEED, 0)
    cam = scene.camera_for(name, Wf, Hf, "framed" if cfg.endswith("f") else None)
    f = _abi.default_features(initial_light_samples=M, num_samples_in_reservoir=1, spatial_resampling_passes=1,
                              temporal_reuse=0, unbiased_combination=unb, spatial_reuse_visibility_check=unb)
    rgb, grid = gpu.render_restir(None, cam, Wf, Hf, f)
    assert rgb.shape == (Hf, Wf, 3) and np.isfinite(rgb).all()
    pos, col, w, m = grid.download()
    del grid
    osc = oracle.OracleScene(s)
    g = f.spatial_resample_radius
    rows = 4
    for y0 in geometry_bands(oracle, osc, cam, Wf, Hf, rows, 4):
        vy0 = max(0, y0 - g)
        view = oracle.Rect(0, vy0, Wf, min(Hf, y0 + rows + g) - vy0)
        rect = oracle.Rect(0, y0, Wf, rows)
        want, res, _ = oracle.render_frame(osc, cam, f, Wf, Hf, SEED, 0, view=view, rect=rect, threads=16)
        r0 = Hf - (y0 + rows)          # RGB row 0 = top of the image
        assert_bits(rgb[r0:r0 + rows], want, f"{cfg} rows {y0}..{y0 + rows - 1}")
        a, b = res
        sl = slice((y0 - vy0) * Wf, (y0 - vy0 + rows) * Wf)
        a = a[:, sl].reshape(1, rows, Wf, 4)
        b = b[:, sl].reshape(1, rows, Wf, 4)
        gs = slice(y0, y0 + rows)
        assert_bits(pos[:, gs], np.ascontiguousarray(a[..., :3]), f"{cfg} grid position rows {y0}..")
        assert_bits(w[:, gs], np.ascontiguousarray(a[..., 3]), f"{cfg} grid W rows {y0}..")
        assert_bits(col[:, gs], np.ascontiguousarray(b[..., :3]), f"{cfg} grid colour rows {y0}..")
        assert np.array_equal(m[:, gs], np.ascontiguousarray(b[..., 3]).view(np.uint32)), f"{cfg} grid M rows {y0}.."


def test_full_size_c2_frame_band_parity(gpu, oracle):
    """C2, the headline (BASELINE configs[1]), at its full size through the bench's own path: restir_render with the
    fused primary + RIS kernel writing the pdf cache, k_spatial1_ntl reading it (no temporal pass between), final
    shading.  The frame's RGB (want_grid=False, as bench.py renders it) and, from a second render of the same
    frame, its returned grid, on sampled row bands against the oracle rendering those rows with the ghost rows its
    spatial pass reads, bit for bit."""
    name, Wf, Hf = "nightclub_128pt", 1920, 1080
    s = get_scene(name)
    gpu.set_scene(s)
    cam = scene.camera_for(name, Wf, Hf)
    f = _abi.default_features(initial_light_samples=32, num_samples_in_reservoir=1, num_neighbours_to_sample=5,
                              spatial_resample_radius=10, spatial_resampling_passes=1, temporal_reuse=0)
    gpu.set_seed(SEED, 0)
    rgb, _ = gpu.render_restir(None, cam, Wf, Hf, f, want_grid=False)
    gpu.set_seed(SEED, 0)
    rgb2, grid = gpu.render_restir(None, cam, Wf, Hf, f)
    assert_bits(rgb2, rgb, "C2 rgb with and without the returned grid")
    pos, col, w, m = grid.download()
    osc = oracle.OracleScene(s)
    g = f.spatial_resample_radius
    rows = 6
    for y0 in (0, 97, 355, Hf // 2 - 3, 811, Hf - rows):
        vy0 = max(0, y0 - g)
        view = oracle.Rect(0, vy0, Wf, min(Hf, y0 + rows + g) - vy0)
        rect = oracle.Rect(0, y0, Wf, rows)
        want, res, _ = oracle.render_frame(osc, cam, f, Wf, Hf, SEED, 0, view=view, rect=rect, threads=16)
        r0 = Hf - (y0 + rows)          # RGB row 0 = top of the image
        assert_bits(rgb[r0:r0 + rows], want, f"C2 rgb rows {y0}..{y0 + rows - 1}")
        a, b = res
        sl = slice((y0 - vy0) * Wf, (y0 - vy0 + rows) * Wf)
        a = a[:, sl].reshape(1, rows, Wf, 4)
        b = b[:, sl].reshape(1, rows, Wf, 4)
        gs = slice(y0, y0 + rows)
        assert_bits(pos[:, gs], np.ascontiguousarray(a[..., :3]), f"C2 grid position rows {y0}..")
        assert_bits(w[:, gs], np.ascontiguousarray(a[..., 3]), f"C2 grid W rows {y0}..")
        assert_bits(col[:, gs], np.ascontiguousarray(b[..., :3]), f"C2 grid colour rows {y0}..")
        assert np.array_equal(m[:, gs], np.ascontiguousarray(b[..., 3]).view(np.uint32)), f"C2 grid M rows {y0}.."
    assert rgb.mean() > 0.01


def test_full_size_c1_frame_matches_oracle(gpu, oracle):
    """C1 (BASELINE configs[0]) at its full size: CornellBox-Mirror 512x512, 1 parallelogram light, M = 32, RIS
    only -- the whole frame's RGB and returned grid against the oracle, bit for bit."""
    name, Wf, Hf = "cornell_parallelogram", 512, 512
    s = get_scene(name)
    gpu.set_scene(s)
    cam = scene.camera_for(name, Wf, Hf)
    f = _abi.default_features(initial_light_samples=32, num_samples_in_reservoir=1, spatial_resampling_passes=0,
                              spatial_reuse=0, temporal_reuse=0)
    gpu.set_seed(SEED, 0)
    rgb, grid = gpu.render_restir(None, cam, Wf, Hf, f)
    want, res, _ = oracle.render_frame(oracle.OracleScene(s), cam, f, Wf, Hf, SEED, 0, threads=16)
    assert_bits(rgb, want, "C1 rgb")
    assert_grid(grid, res, "C1")
    assert rgb.mean() > 0.01


@pytest.mark.parametrize("N", [1, 2])
def test_full_size_c3_sequence_band_parity(gpu, oracle, N):
    """C3 at its full size: 1080p nightclub, 128 point lights, M = 32, two spatial passes, temporal reuse over 4
    frames threaded through the frame pool (each predecessor released as the sequence goes, and an unrelated frame
    rendered between frames 1 and 2 so recycled records are reused).  Checked on sampled row bands: frame f's rows
    depend on frame f - 1's grid within passes * r = 20 rows (temporal reuse is same-pixel, render_utils.cpp:155;
    spatial reuse reads +-r per pass, :91), so the oracle renders frame 0 on the band grown by 4 * 20 = 80 rows,
    frame 1 on the band grown by 60, ... each frame's view being the previous frame's owned rows.  Every frame's
    RGB and the last frame's grid are compared on the band, bit for bit.  N = 2 is the reference's default
    (common.h:105): k_temporal_n2, k_spatial2_ntl and k_final_n2_sorted at full size."""
    name, Wf, Hf, P, R, frames = "nightclub_128pt", 1920, 1080, 2, 10, 4
    s = get_scene(name)
    gpu.set_scene(s)
    osc = oracle.OracleScene(s)
    cam = scene.camera_for(name, Wf, Hf)
    f = _abi.default_features(initial_light_samples=32, num_samples_in_reservoir=N, spatial_resampling_passes=P,
                              spatial_resample_radius=R, temporal_reuse=1)
    gpu.set_seed(SEED, 0)
    rgbs, grid = [], None
    for fr in range(frames):
        rgb, nxt = gpu.render_restir(grid, cam, Wf, Hf, f)
        grid = nxt                      # the predecessor is released here (records back to the pool)
        rgbs.append(rgb)
        if fr == 1:                     # an unrelated frame takes recycled records, then hands them back
            other, _ = gpu.render_restir(None, scene.camera_for("cornell_1024", Wf, Hf), Wf, Hf, f)
            del other
            gpu.set_seed(SEED, fr + 1)
    pos, col, w, m = grid.download()
    rows, grow = 6, P * R
    for y0 in (0, 531, Hf - rows):
        prev = None
        for fr in range(frames):
            g_rect = (frames - 1 - fr) * grow          # owned rows of frame fr: the band grown by this
            ry0, ry1 = max(0, y0 - g_rect), min(Hf, y0 + rows + g_rect)
            vy0, vy1 = max(0, ry0 - grow), min(Hf, ry1 + grow)
            view, rect = oracle.Rect(0, vy0, Wf, vy1 - vy0), oracle.Rect(0, ry0, Wf, ry1 - ry0)
            want, res, _ = oracle.render_frame(osc, cam, f, Wf, Hf, SEED, fr, prev=prev, view=view, rect=rect,
                                               threads=16)
            top = Hf - ry1                             # RGB row 0 = top of the image
            assert_bits(rgbs[fr][top:top + (ry1 - ry0)], want, f"C3 frame {fr} rows {ry0}..{ry1 - 1}")
            # the next frame's view is this frame's owned rows: its predecessor grid is those rows of `res`
            a, b = res
            sl = slice((ry0 - vy0) * Wf, (ry1 - vy0) * Wf)
            prev = (np.ascontiguousarray(a[:, sl]), np.ascontiguousarray(b[:, sl]))
        a, b = prev                                    # frame 3's grid on its owned band (= the checked rows)
        a = a.reshape(N, -1, Wf, 4)
        b = b.reshape(N, -1, Wf, 4)
        gs = slice(y0, y0 + rows)
        assert_bits(pos[:, gs], np.ascontiguousarray(a[..., :3]), f"C3 grid position rows {y0}..")
        assert_bits(w[:, gs], np.ascontiguousarray(a[..., 3]), f"C3 grid W rows {y0}..")
        assert_bits(col[:, gs], np.ascontiguousarray(b[..., :3]), f"C3 grid colour rows {y0}..")
        assert np.array_equal(m[:, gs], np.ascontiguousarray(b[..., 3]).view(np.uint32)), f"C3 grid M rows {y0}.."


@pytest.mark.parametrize("name,passes,unbiased,vis,tiled,tune", [
    ("cornell_1024", 1, 0, 0, 0, {}), ("cornell_1024", 2, 0, 0, 0, {}), ("cornell_4096", 1, 1, 1, 0, {}),
    ("cornell_4096", 2, 1, 1, 0, {}), ("cornell_4096", 1, 1, 0, 0, {}), ("nightclub_128pt", 1, 0, 0, 0, {}),
    ("cornell_1024", 2, 0, 0, 1, {}), ("cornell_4096", 2, 1, 1, 1, {}),
    # sample-handle passes (point lights / the light grid) on a ghost-zoned tile: the returned ring keeps RIS's reservoirs
    ("nightclub_128pt", 2, 0, 0, 1, {}), ("cornell_1024", 3, 0, 0, 1, {}),
    # biased passes with the G-buffer stores skipped too (miss.gbuf = 1; the default does so only from 2048 px wide):
    # the window fix-up, on 32 x 8 and on 32 x 16 tiles
    ("cornell_1024", 1, 0, 0, 0, {"miss.gbuf": 1}), ("cornell_1024", 2, 0, 0, 0, {"miss.gbuf": 1}),
    ("cornell_1024", 1, 0, 0, 0, {"miss.gbuf": 1, "spatial.th": 2}), ("nightclub_128pt", 1, 0, 0, 0, {"miss.gbuf": 1}),
    # N = 2 (the reference default): k_spatial2_ntl and k_final_n2_sorted read the flags too
    ("cornell_1024", 1, 0, 0, 0, {"N": 2}), ("cornell_1024", 2, 0, 0, 0, {"N": 2}), ("nightclub_128pt", 1, 0, 0, 0, {"N": 2}),
    ("cornell_1024", 2, 0, 0, 1, {"N": 2}), ("cornell_4096", 1, 1, 1, 0, {"N": 2}),
    # final shading's shadow rays over the 16-byte quantized nodes at N = 1 (final.qbvh = 1; the default takes them at
    # N = 2 only) and over the 32-byte float nodes at N = 2 (final.qbvh = 0)
    ("cornell_1024", 1, 0, 0, 0, {"final.qbvh": 1}), ("nightclub_128pt", 1, 0, 0, 0, {"final.qbvh": 1}),
    ("nightclub_128pt", 1, 0, 0, 0, {"N": 2, "final.qbvh": 0})])
def test_miss_tiles_match_full_reads(gpu, oracle, name, passes, unbiased, vis, tiled, tune):
    """MissTiles (miss.tiles = 1, the default): RIS flags the 32 x 8 tiles whose pixels all missed the scene, and the
    spatial passes and final shading write those tiles' known results without reading them.  Frames at 640 x 360
    (the Cornell box fills the middle: most tiles, and most unbiased neighbourhoods, are background), whole and as a
    ghost-zoned screen tile (2 x 2 plan, rank 3: the RIS, spatial and final regions start at different offsets), must
    equal the frames rendered with the flags off bit for bit -- RGB and the returned grid -- and the oracle's frame (RGB;
    a tile against the oracle's whole frame cropped to its owned rect)."""
    from romis_amd import restir
    tune = dict(tune)
    N = tune.pop("N", 1)
    w, h = 640, 360
    s = get_scene(name)
    gpu.set_scene(s)
    cam = scene.camera_for(name, w, h)
    f = _abi.default_features(num_samples_in_reservoir=N, spatial_resampling_passes=passes, unbiased_combination=unbiased,
                              temporal_reuse=0, spatial_reuse_visibility_check=vis)
    tile = restir.tile_plan(w, h, 2, 2, 3, passes * f.spatial_resample_radius) if tiled else None

    def run(on):
        gpu.set_tuning("miss.tiles", on)
        gpu.set_seed(SEED, 0)
        rgb, grid = gpu.render_restir(None, cam, w, h, f, tile=tile)
        return rgb, grid.download()

    try:
        for k, v in tune.items():
            gpu.set_tuning(k, v)
        off_rgb, off_grid = run(0)
        on_rgb, on_grid = run(1)
    finally:
        gpu.set_tuning("miss.tiles", 1)
        gpu.set_tuning("miss.gbuf", 2)
        gpu.set_tuning("spatial.th", 0)
        gpu.set_tuning("final.qbvh", 2)
    want, _, _ = oracle.render_frame(oracle.OracleScene(s), cam, f, w, h, SEED, 0, threads=16)
    if tile is not None:   # the tile's rows (row 0 = its top) against the oracle's whole frame (row 0 = global y = h - 1)
        r0 = h - (tile.y0 + tile.height)
        want = np.ascontiguousarray(want[r0:r0 + tile.height, tile.x0:tile.x0 + tile.width])
    assert_bits(on_rgb, want, f"{name} rgb against the oracle")
    assert_bits(on_rgb, off_rgb, f"{name} rgb")
    # a tiled frame's grid is defined on the owned rect (the ghost ring holds intermediate values, include/restir_c.h)
    own = (slice(None), slice(tile.y0 - tile.gy0, tile.y0 - tile.gy0 + tile.height),
           slice(tile.x0 - tile.gx0, tile.x0 - tile.gx0 + tile.width)) if tile is not None else (slice(None),)
    for a, b in zip(off_grid, on_grid):
        assert np.array_equal(np.asarray(a)[own].view(np.uint32), np.asarray(b)[own].view(np.uint32)), f"{name} grid"
