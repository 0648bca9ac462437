"""Frame output against the reference's own code (tests/golden/screen_fixtures.json, written by
oracle/_ref/screen_ref from the reference's glm / stb / cereal / struct Features -- make_screen_fixtures.py):
  - restir_encode_bmp / restir_write_bmp = Screen::writeBitmapToFile (screen.cpp:45-56): clamp, x255, truncate,
    stbi_write_bmp with 4 components -- byte for byte;
  - restir_features_json = the configuration record of renderRayTraced (render.cpp:281-287) -- byte for byte.
Host-only entry points of libromis_amd: no GPU needed."""
import base64
import ctypes as C
import json
import os
import struct

import numpy as np
import pytest

from romis_amd import _abi

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def fx():
    with open(os.path.join(HERE, "golden", "screen_fixtures.json")) as fh:
        return json.load(fh)


def encode_bmp(lib, img):
    H, W, _ = img.shape
    img = np.ascontiguousarray(img, np.float32)
    n = C.c_size_t()
    _abi.check(lib, lib.restir_encode_bmp(img.ctypes.data, W, H, None, 0, C.byref(n)), "size")
    out = (C.c_uint8 * n.value)()
    _abi.check(lib, lib.restir_encode_bmp(img.ctypes.data, W, H, out, n.value, C.byref(n)), "encode")
    return bytes(out)


def test_bmp_matches_reference_stb(abi_lib, fx):
    for case in fx["bmp"]:
        img = np.frombuffer(base64.b64decode(case["rgb_bits"]), np.float32).reshape(case["height"], case["width"], 3)
        got = encode_bmp(abi_lib, img)
        want = base64.b64decode(case["bmp"])
        assert got == want, f"{case['name']}: BMP bytes differ"


def test_write_bmp_file(abi_lib, fx, tmp_path):
    case = fx["bmp"][-1]
    img = np.frombuffer(base64.b64decode(case["rgb_bits"]), np.float32).reshape(case["height"], case["width"], 3)
    path = str(tmp_path / "frame.bmp")
    _abi.check(abi_lib, abi_lib.restir_write_bmp(path.encode(), np.ascontiguousarray(img).ctypes.data,
                                                 case["width"], case["height"]), "write")
    with open(path, "rb") as fh:
        assert fh.read() == base64.b64decode(case["bmp"])


def test_rgba8_conversion_edges(abi_lib):
    # glm::clamp then truncation: -0.1 -> 0, 1.7 -> 255, k/255 -> k (exactly representable products only)
    rgb = np.float32([[-0.1, 1.7, 0.5], [1.0, 0.0, 254.5 / 255.0]])
    out = (C.c_uint8 * 8)()
    _abi.check(abi_lib, abi_lib.restir_rgb_to_rgba8(rgb.ctypes.data, 2, out), "rgba8")
    assert list(out) == [0, 255, 127, 255, 255, 0, 254, 255]


FEATURE_FIELDS = {   # Features (common.h) name -> (restir_features field, or "x." + restir_features_record_extra field)
    "enableShading": "enable_shading", "enableRecursive": "x.enable_recursive",
    "enableHardShadow": "x.enable_hard_shadow", "enableSoftShadow": "x.enable_soft_shadow",
    "enableNormalInterp": "x.enable_normal_interp", "enableTextureMapping": "enable_texture_mapping",
    "enableAccelStructure": "x.enable_accel_structure", "maxReflectionRecursion": "x.max_reflection_recursion",
    "rayTraceMode": "ray_trace_mode", "initialSamplesVisibilityCheck": "initial_samples_visibility_check",
    "numSamplesInReservoir": "num_samples_in_reservoir", "initialLightSamples": "initial_light_samples",
    "numNeighboursToSample": "num_neighbours_to_sample", "spatialResampleRadius": "spatial_resample_radius",
    "maxIterationsMIS": "max_iterations_mis", "neighbourSelectionStrategy": "neighbour_selection_strategy",
    "misWeightRMIS": "mis_weight_rmis", "useProgressiveROMIS": "use_progressive_romis",
    "progressiveUpdateMod": "progressive_update_mod", "saveAlphasVisualisation": "save_alphas_visualisation",
    "unbiasedCombination": "unbiased_combination", "spatialReuse": "spatial_reuse",
    "spatialReuseVisibilityCheck": "spatial_reuse_visibility_check", "temporalReuse": "temporal_reuse",
    "spatialResamplingPasses": "spatial_resampling_passes", "temporalClampM": "temporal_clamp_m",
    "enableToneMapping": "enable_tone_mapping", "gamma": "gamma", "exposure": "exposure"}


def features_json(lib, s):
    f = _abi.Features()
    lib.restir_features_default(C.byref(f))
    f.ray_trace_mode = 2   # struct Features' own default (ROMIS, common.h:104); restir_features_default sets ReSTIR
    x = _abi.FeaturesRecordExtra(0, 1, 1, 1, 1, (C.c_uint8 * 3)(), 5)
    for k, v in s.items():
        field = FEATURE_FIELDS[k]
        if k in ("gamma", "exposure"):
            v = struct.unpack("<f", struct.pack("<I", v))[0]
        if field.startswith("x."):
            setattr(x, field[2:], v)
        else:
            setattr(f, field, v)
    n = C.c_size_t()
    _abi.check(lib, lib.restir_features_json(C.byref(f), C.byref(x), None, 0, C.byref(n)), "size")
    buf = C.create_string_buffer(n.value + 1)
    _abi.check(lib, lib.restir_features_json(C.byref(f), C.byref(x), buf, n.value + 1, C.byref(n)), "json")
    return buf.value.decode()


def test_features_json_matches_reference_cereal(abi_lib, fx):
    for case in fx["json"]:
        assert features_json(abi_lib, case["set"]) == case["json"], case["set"]


def test_features_json_defaults_and_errors(abi_lib):
    f = _abi.Features()
    abi_lib.restir_features_default(C.byref(f))
    n = C.c_size_t()
    assert abi_lib.restir_features_json(C.byref(f), None, None, 0, C.byref(n)) == 0
    buf = C.create_string_buffer(n.value + 1)
    assert abi_lib.restir_features_json(C.byref(f), None, buf, n.value + 1, C.byref(n)) == 0
    rec = json.loads(buf.value.decode())
    assert rec["enableHardShadow"] is True and rec["maxReflectionRecursion"] == 5 and rec["rayTraceMode"] == 0
    assert abi_lib.restir_features_json(C.byref(f), None, buf, 3, C.byref(n)) == 1
    f.gamma = float("nan")
    assert abi_lib.restir_features_json(C.byref(f), None, None, 0, C.byref(n)) == 1


@pytest.mark.gpu
def test_gpu_frame_bitmap_matches_oracle_bitmap(abi_lib, oracle):
    """A rendered frame's 8-bit bitmap (f2): the GPU frame through restir_encode_bmp equals the oracle frame's
    bitmap byte for byte (tone mapping on, and off so that the clamp matters)."""
    from romis_amd import restir, scene
    name, W, H = "nightclub_128pt", 96, 64
    osc = oracle.OracleScene(scene.bench_scene(name))
    cam = scene.camera_for(name, W, H)
    r = restir.Renderer(0)
    try:
        r.set_scene(scene.bench_scene(name))
        r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
        for tone in (1, 0):
            r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)   # both renders are frame 0 (the oracle's keys)
            f = _abi.default_features(num_samples_in_reservoir=1, enable_tone_mapping=tone, temporal_reuse=0)
            got, _ = r.render_restir(None, cam, W, H, f, want_grid=False)
            want, _, _ = oracle.render_frame(osc, cam, f, W, H, threads=4)
            assert encode_bmp(abi_lib, got) == encode_bmp(abi_lib, want), f"tone mapping {tone}"
            if not tone:
                assert (want > 1.0).any()   # the clamp is exercised
    finally:
        r.close()
