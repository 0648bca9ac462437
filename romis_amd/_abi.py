"""ctypes mirror of include/restir_c.h (the C ABI of libromis_amd.so).

The library is built in-tree (romis_amd/_build/libromis_amd.so, see romis_amd/build.py).  Loading fails loudly
when it is missing: there is no CPU fallback for the product path.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libromis_amd.so")

RESTIR_STAGE_RIS = 1
RESTIR_STAGE_TEMPORAL = 2
RESTIR_STAGE_SPATIAL = 3
RESTIR_STAGE_NEIGHBOURS = 4
RESTIR_DEFAULT_SEED = 0x5EED0001
RESTIR_MAX_N = 32
RESTIR_ROMIS_MAX_TECHNIQUES = 8
RESTIR_RCCL_ID_BYTES = 128
RESTIR_ABI_VERSION = 5
RESTIR_HALO_OP_SEND, RESTIR_HALO_OP_RECV = 0, 1
# restir_halo_event.what (include/restir_c.h)
(RESTIR_HALO_EV_PACK, RESTIR_HALO_EV_RECORD, RESTIR_HALO_EV_WAIT, RESTIR_HALO_EV_GROUP_START, RESTIR_HALO_EV_SEND,
 RESTIR_HALO_EV_RECV, RESTIR_HALO_EV_GROUP_END, RESTIR_HALO_EV_INTERIOR, RESTIR_HALO_EV_UNPACK,
 RESTIR_HALO_EV_BORDER) = range(10)

LIGHT_POINT, LIGHT_SEGMENT, LIGHT_PARALLELOGRAM = 0, 1, 2
MODE_RESTIR, MODE_RMIS, MODE_ROMIS = 0, 1, 2
MIS_EQUAL, MIS_BALANCE = 0, 1
NEIGHBOURS_RANDOM, NEIGHBOURS_SIMILAR, NEIGHBOURS_DISSIMILAR, NEIGHBOURS_EQUAL_SIMILAR_DISSIMILAR = 0, 1, 2, 3

BUF_GBUF_N_T, BUF_GBUF_P_MAT, BUF_RES_A, BUF_RES_B, BUF_RES_DBG = 0, 1, 2, 3, 4
BUF_PREV_A, BUF_PREV_B, BUF_PREV_DBG, BUF_RGB = 5, 6, 7, 8
BUF_MIS_NBR, BUF_MIS_ACC = 9, 10
BUF_GBUF_UV = 11

K_PRIMARY, K_RIS, K_TEMPORAL, K_SPATIAL, K_FINAL, K_PRIMARY_RIS, K_MIS, K_COUNT = 0, 1, 2, 3, 4, 5, 6, 7
KERNEL_NAMES = ["primary", "ris", "temporal", "spatial", "final", "primary_ris", "mis"]

STATUS_NAMES = {0: "OK", 1: "INVALID", 2: "HIP", 3: "NO_DEVICE", 4: "STATE", 5: "UNSUPPORTED", 6: "COMM"}

F3 = C.c_float * 3


class Light(C.Structure):
    _fields_ = [("type", C.c_uint32), ("p0", F3), ("p1", F3), ("p2", F3),
                ("c0", F3), ("c1", F3), ("c2", F3), ("c3", F3)]


class Material(C.Structure):
    _fields_ = [("kd", F3), ("ks", F3), ("shininess", C.c_float), ("transparency", C.c_float),
                ("kd_texture", C.c_uint32)]


class Mesh(C.Structure):
    _fields_ = [("positions", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
                ("num_vertices", C.c_uint32), ("triangles", C.POINTER(C.c_uint32)),
                ("num_triangles", C.c_uint32), ("material", Material), ("texcoords", C.POINTER(C.c_float))]


class Texture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("rgb", C.POINTER(C.c_float))]


class Camera(C.Structure):
    _fields_ = [("fovy", C.c_float), ("aspect", C.c_float), ("look_at", F3), ("distance", C.c_float),
                ("rotation", F3)]


class CameraFrame(C.Structure):
    _fields_ = [("origin", F3), ("quat", C.c_float * 4), ("half_w", C.c_float), ("half_h", C.c_float)]


class Features(C.Structure):
    _fields_ = [("ray_trace_mode", C.c_uint32), ("initial_light_samples", C.c_uint32),
                ("num_samples_in_reservoir", C.c_uint32), ("num_neighbours_to_sample", C.c_uint32),
                ("spatial_resample_radius", C.c_uint32), ("spatial_resampling_passes", C.c_uint32),
                ("temporal_clamp_m", C.c_uint32),
                ("initial_samples_visibility_check", C.c_uint8), ("unbiased_combination", C.c_uint8),
                ("spatial_reuse", C.c_uint8), ("spatial_reuse_visibility_check", C.c_uint8),
                ("temporal_reuse", C.c_uint8), ("enable_shading", C.c_uint8),
                ("enable_texture_mapping", C.c_uint8), ("enable_tone_mapping", C.c_uint8),
                ("gamma", C.c_float), ("exposure", C.c_float),
                ("neighbour_same_geometry", C.c_uint8), ("use_progressive_romis", C.c_uint8),
                ("save_alphas_visualisation", C.c_uint8), ("reserved0", C.c_uint8),
                ("neighbour_max_depth_difference_fraction", C.c_float),
                ("neighbour_max_normal_angle_difference_radians", C.c_float),
                ("max_iterations_mis", C.c_uint32), ("neighbour_selection_strategy", C.c_uint32),
                ("mis_weight_rmis", C.c_uint32), ("progressive_update_mod", C.c_uint32)]


class FeaturesRecordExtra(C.Structure):
    """restir_features_record_extra: the Features fields only the configuration record carries."""
    _fields_ = [("enable_recursive", C.c_uint8), ("enable_hard_shadow", C.c_uint8), ("enable_soft_shadow", C.c_uint8),
                ("enable_normal_interp", C.c_uint8), ("enable_accel_structure", C.c_uint8),
                ("reserved", C.c_uint8 * 3), ("max_reflection_recursion", C.c_uint32)]


class HaloSegment(C.Structure):
    _fields_ = [("rank", C.c_uint32), ("x0", C.c_uint32), ("y0", C.c_uint32), ("width", C.c_uint32),
                ("height", C.c_uint32), ("offset", C.c_uint64), ("bytes", C.c_uint64)]


class HaloOp(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("peer", C.c_uint32), ("offset", C.c_uint64), ("bytes", C.c_uint64),
                ("x0", C.c_uint32), ("y0", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32)]


class HaloEvent(C.Structure):
    _fields_ = [("what", C.c_uint32), ("stream", C.c_uint32), ("peer", C.c_uint32), ("pass_", C.c_uint32),
                ("offset", C.c_uint64), ("bytes", C.c_uint64)]


class Tile(C.Structure):
    _fields_ = [("global_width", C.c_uint32), ("global_height", C.c_uint32),
                ("x0", C.c_uint32), ("y0", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32),
                ("gx0", C.c_uint32), ("gy0", C.c_uint32), ("gwidth", C.c_uint32), ("gheight", C.c_uint32)]


RESTIR_MAX_TILES_X = 16
RESTIR_MAX_TILES_Y = 16


class TileLayout(C.Structure):
    """restir_tile_layout: column cuts x_cuts[0..tiles_x], per-column row cuts y_cuts[c][0..tiles_y]."""
    _fields_ = [("global_width", C.c_uint32), ("global_height", C.c_uint32), ("tiles_x", C.c_uint32),
                ("tiles_y", C.c_uint32), ("x_cuts", C.c_uint32 * (RESTIR_MAX_TILES_X + 1)),
                ("y_cuts", (C.c_uint32 * (RESTIR_MAX_TILES_Y + 1)) * RESTIR_MAX_TILES_X)]

    def cuts(self) -> dict:
        """JSON form: {"x": [...], "y": [[...] per column]}."""
        tx, ty = self.tiles_x, self.tiles_y
        return {"x": list(self.x_cuts[:tx + 1]), "y": [list(self.y_cuts[c][:ty + 1]) for c in range(tx)]}

    @classmethod
    def from_cuts(cls, width: int, height: int, cuts: dict) -> "TileLayout":
        L = cls()
        L.global_width, L.global_height = width, height
        L.tiles_x, L.tiles_y = len(cuts["x"]) - 1, len(cuts["y"][0]) - 1
        for i, v in enumerate(cuts["x"]):
            L.x_cuts[i] = v
        for c, col in enumerate(cuts["y"]):
            for i, v in enumerate(col):
                L.y_cuts[c][i] = v
        return L


assert C.sizeof(HaloOp) == 40 and C.sizeof(HaloEvent) == 32
assert C.sizeof(TileLayout) == 4 * (4 + 17 + 16 * 17)
assert C.sizeof(Light) == 88
assert C.sizeof(Material) == 36
assert C.sizeof(Mesh) == 80 and C.sizeof(Texture) == 16
assert C.sizeof(Features) == 72


def default_features(**overrides) -> Features:
    """struct Features defaults (src/utils/common.h:89-136) with rayTraceMode = ReSTIR."""
    f = Features(ray_trace_mode=MODE_RESTIR, initial_light_samples=32, num_samples_in_reservoir=2,
                 num_neighbours_to_sample=5, spatial_resample_radius=10, spatial_resampling_passes=2,
                 temporal_clamp_m=20, initial_samples_visibility_check=0, unbiased_combination=0,
                 spatial_reuse=1, spatial_reuse_visibility_check=0, temporal_reuse=1, enable_shading=1,
                 enable_texture_mapping=1, enable_tone_mapping=1, gamma=1.0, exposure=1.5,
                 neighbour_same_geometry=1, use_progressive_romis=0, save_alphas_visualisation=1,
                 neighbour_max_depth_difference_fraction=0.10, neighbour_max_normal_angle_difference_radians=0.436332,
                 max_iterations_mis=5, neighbour_selection_strategy=NEIGHBOURS_SIMILAR, mis_weight_rmis=MIS_EQUAL,
                 progressive_update_mod=1)
    for k, v in overrides.items():
        if not hasattr(f, k):
            raise AttributeError(f"Features has no field {k!r}")
        setattr(f, k, v)
    return f


# Exported symbols of include/restir_c.h with their ctypes signatures.
_P = C.c_void_p
SIGNATURES = {
    "restir_features_default": (None, [C.POINTER(Features)]),
    "restir_rng_key": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "restir_rng_draw": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32]),
    "restir_camera_derive": (None, [C.POINTER(Camera), C.POINTER(CameraFrame)]),
    "restir_tile_plan": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.POINTER(Tile)]),
    "restir_last_error": (C.c_char_p, []),
    "restir_abi_version": (C.c_int, []),
    "restir_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "restir_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "restir_destroy": (None, [_P]),
    "restir_set_seed": (C.c_int, [_P, C.c_uint32, C.c_uint32]),
    "restir_set_renders_dir": (C.c_int, [_P, C.c_char_p]),
    "restir_set_scene": (C.c_int, [_P, C.POINTER(Mesh), C.c_uint32, C.POINTER(Light), C.c_uint32]),
    "restir_set_scene_textured": (C.c_int, [_P, C.POINTER(Mesh), C.c_uint32, C.POINTER(Light), C.c_uint32,
                                            C.POINTER(Texture), C.c_uint32]),
    "restir_render": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Features), C.c_uint32, C.c_uint32,
                                C.POINTER(Tile), _P, C.POINTER(_P), C.POINTER(C.c_float)]),
    "restir_frame_retain": (C.c_int, [_P]),
    "restir_frame_release": (None, [_P]),
    "restir_frame_info": (C.c_int, [_P] + [C.POINTER(C.c_uint32)] * 7),
    "restir_frame_download": (C.c_int, [_P, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                        C.POINTER(C.c_uint32)]),
    "restir_synchronize": (C.c_int, [_P]),
    "restir_download_rgb": (C.c_int, [_P, C.POINTER(C.c_float), C.c_size_t]),
    "restir_stage_configure": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32]),
    "restir_stage_upload": (C.c_int, [_P, C.c_int, _P, C.c_size_t]),
    "restir_stage_download": (C.c_int, [_P, C.c_int, _P, C.c_size_t]),
    "restir_stage_primary": (C.c_int, [_P, C.POINTER(Camera)]),
    "restir_stage_ris": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Features), C.c_uint32, C.c_int]),
    "restir_stage_temporal": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Features), C.c_uint32, C.c_int]),
    "restir_stage_spatial": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Features), C.c_uint32, C.c_int]),
    "restir_stage_final": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Features)]),
    "restir_debug_math": (C.c_int, [_P, C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                    C.POINTER(C.c_float), C.c_size_t]),
    "restir_stage_neighbours": (C.c_int, [_P, C.POINTER(Features), C.c_uint32, C.c_uint32]),
    "restir_stage_mis_accumulate": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Features), C.c_uint32]),
    "restir_stage_mis_finish": (C.c_int, [_P, C.POINTER(Features)]),
    "restir_stage_mis_capacity": (C.c_int, [_P, C.POINTER(Features), C.POINTER(C.c_uint32)]),
    "restir_debug_cod_solve": (C.c_int, [_P, C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                         C.POINTER(C.c_float), C.c_size_t]),
    "restir_halo_plan": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                   C.c_uint32, C.POINTER(HaloSegment), C.POINTER(HaloSegment),
                                   C.POINTER(C.c_uint32)]),
    "restir_halo_begin": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Features), C.c_uint32, C.c_uint32, C.c_uint32,
                                    C.c_uint32, C.c_uint32, _P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "restir_halo_pack": (C.c_int, [_P, _P, C.c_uint64, C.c_int]),
    "restir_halo_unpack": (C.c_int, [_P, _P, C.c_uint64, C.c_int]),
    "restir_halo_spatial": (C.c_int, [_P]),
    "restir_halo_spatial_interior": (C.c_int, [_P]),
    "restir_halo_spatial_border": (C.c_int, [_P]),
    "restir_rccl_unique_id": (C.c_int, [_P, C.c_size_t]),
    "restir_halo_attach_rccl": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32]),
    "restir_halo_attach_comm": (C.c_int, [_P, _P]),
    "restir_halo_pass": (C.c_int, [_P]),
    "restir_halo_ops": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                  C.POINTER(HaloOp), C.POINTER(C.c_uint32)]),
    "restir_halo_record": (C.c_int, [_P, C.c_int]),
    "restir_halo_log": (C.c_int, [_P, C.POINTER(HaloEvent), C.POINTER(C.c_uint32)]),
    "restir_rgb_to_rgba8": (C.c_int, [_P, C.c_size_t, _P]),
    "restir_encode_bmp": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "restir_write_bmp": (C.c_int, [C.c_char_p, _P, C.c_uint32, C.c_uint32]),
    "restir_features_json": (C.c_int, [C.POINTER(Features), C.POINTER(FeaturesRecordExtra), C.c_char_p, C.c_size_t,
                                       C.POINTER(C.c_size_t)]),
    "restir_halo_end": (C.c_int, [_P, C.POINTER(_P), C.POINTER(C.c_float)]),
    "restir_measure_read_bandwidth": (C.c_int, [_P, C.c_uint64, C.c_uint32, C.POINTER(C.c_double)]),
    "restir_layout_even": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(TileLayout)]),
    "restir_layout_balanced": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_float), C.c_uint32,
                                         C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(TileLayout),
                                         C.POINTER(C.c_double)]),
    "restir_layout_shares": (C.c_int, [C.POINTER(TileLayout), C.POINTER(C.c_float), C.c_uint32, C.c_uint32,
                                       C.POINTER(C.c_double)]),
    "restir_layout_tile": (C.c_int, [C.POINTER(TileLayout), C.c_uint32, C.c_uint32, C.POINTER(Tile)]),
    "restir_layout_halo_plan": (C.c_int, [C.POINTER(TileLayout), C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.POINTER(HaloSegment), C.POINTER(HaloSegment), C.POINTER(C.c_uint32)]),
    "restir_layout_halo_ops": (C.c_int, [C.POINTER(TileLayout), C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(HaloOp),
                                         C.POINTER(C.c_uint32)]),
    "restir_halo_begin_layout": (C.c_int, [_P, C.POINTER(Camera), C.POINTER(Features), C.POINTER(TileLayout), C.c_uint32,
                                           _P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "restir_background_pixels": (C.c_int, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "restir_enable_timing": (C.c_int, [_P, C.c_int]),
    "restir_set_tuning": (C.c_int, [_P, C.c_char_p, C.c_int]),
    "restir_timings": (C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "restir_reset_timings": (C.c_int, [_P]),
}


class RestirError(RuntimeError):
    """Mirrors the reference's std::runtime_error convention (render.cpp:99,278)."""


_lib = None


def load_library(path: str | None = None) -> C.CDLL:
    """Load libromis_amd.so and bind every symbol of include/restir_c.h.  Raises if it is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("ROMIS_AMD_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise RestirError(f"libromis_amd.so not found at {p}: build it with `python -m romis_amd.build` "
                          "(there is no CPU fallback for the HIP path)")
    lib = C.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(lib: C.CDLL, status: int, what: str = "") -> None:
    if status != 0:
        msg = lib.restir_last_error()
        raise RestirError(f"{what}: {STATUS_NAMES.get(status, status)}: {msg.decode() if msg else ''}")
