"""TEST INFRASTRUCTURE ONLY -- ctypes binding of oracle/_build/liboracle.so (the C restatement of the
reference ReSTIR path, oracle/restir_oracle.c).  Imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; never by the product package romis_amd.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from romis_amd import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")

FP = C.POINTER(C.c_float)
UP = C.POINTER(C.c_uint32)


class Rect(C.Structure):
    _fields_ = [("x0", C.c_uint32), ("y0", C.c_uint32), ("w", C.c_uint32), ("h", C.c_uint32)]


_lib = None


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE, "oracle"])


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        l = C.CDLL(LIB)
        P = C.c_void_p
        u32 = C.c_uint32
        sig = {
            "or_scene_create": (P, [C.POINTER(_abi.Mesh), u32, C.POINTER(_abi.Light), u32]),
            "or_scene_destroy": (None, [P]),
            "or_scene_create_textured": (P, [C.POINTER(_abi.Mesh), u32, C.POINTER(_abi.Light), u32,
                                             C.POINTER(_abi.Texture), u32]),
            "or_scene_bind_uv": (None, [P, FP]),
            "or_acquire_texel": (None, [P, u32, FP, FP]),
            "or_primary_uv": (None, [P, C.POINTER(_abi.CameraFrame), u32, u32, Rect, Rect, FP, FP, FP]),
            "or_scene_num_triangles": (u32, [P]),
            "or_scene_miss_material": (u32, [P]),
            "or_rng_key": (u32, [u32, u32, u32, u32]),
            "or_set_rng_mode": (None, [C.c_int]),
            "or_rng_draw": (u32, [u32, u32, u32]),
            "or_glm_probe": (None, [FP, FP, C.c_float, FP, FP]),
            "or_tonemap": (None, [FP, C.c_float, C.c_float, FP]),
            "or_powf": (C.c_float, [C.c_float, C.c_float]),
            "or_expf": (C.c_float, [C.c_float]),
            "or_powf_n": (None, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
            "or_expf_n": (None, [C.c_void_p, C.c_void_p, C.c_size_t]),
            "or_camera_derive": (None, [C.POINTER(_abi.Camera), C.POINTER(_abi.CameraFrame)]),
            "or_target_pdf": (C.c_float, [P, C.POINTER(_abi.Features), FP, FP, FP, FP, FP]),
            "or_primary": (None, [P, C.POINTER(_abi.CameraFrame), u32, u32, Rect, Rect, FP, FP]),
            "or_ris": (None, [P, C.POINTER(_abi.Features), u32, FP, u32, u32, Rect, Rect, FP, FP, FP, FP, FP]),
            "or_temporal": (None, [P, C.POINTER(_abi.Features), u32, FP, u32, u32, Rect, Rect, FP, FP, FP, FP,
                                   FP, FP, FP, FP, FP]),
            "or_spatial_pass": (C.c_int, [P, C.POINTER(_abi.Features), u32, FP, u32, u32, Rect, Rect, FP, FP,
                                          FP, FP, FP, FP, FP]),
            "or_final": (None, [P, C.POINTER(_abi.Features), FP, u32, u32, Rect, Rect, FP, FP, FP, FP, FP]),
            "or_render_frame": (C.c_int, [P, C.POINTER(_abi.Camera), C.POINTER(_abi.Features), u32, u32, u32,
                                          u32, Rect, Rect, FP, FP, FP, FP, FP, FP, FP, C.c_int]),
            "or_mis_capacity": (u32, [C.POINTER(_abi.Features), u32, u32]),
            "or_mis_acc_rows": (u32, [C.POINTER(_abi.Features)]),
            "or_neighbours": (None, [P, C.POINTER(_abi.Features), u32, u32, u32, u32, FP, FP, u32, UP]),
            "or_rmis_accumulate": (None, [P, C.POINTER(_abi.Features), FP, u32, u32, FP, FP, UP, FP, FP, FP]),
            "or_romis_accumulate": (None, [P, C.POINTER(_abi.Features), FP, u32, u32, FP, FP, UP, FP, FP, FP, u32,
                                           FP]),
            "or_mis_finish": (None, [C.POINTER(_abi.Features), u32, u32, FP, FP]),
            "or_cod_solve": (None, [u32, FP, FP, FP]),
            "or_render_mis": (C.c_int, [P, C.POINTER(_abi.Camera), C.POINTER(_abi.Features), u32, u32, u32, u32, FP,
                                        C.c_int]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def set_rng_mode(reference: bool) -> None:
    """CPU-baseline timing mode: the reference's own generators (oracle/ref_rng.cpp) instead of the keyed draws.
    Results are then not reproducible; bench.py only times it."""
    lib().or_set_rng_mode(1 if reference else 0)


def fp(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(FP)


class OracleScene:
    def __init__(self, scene):
        meshes, nm, lights, nl, keep = scene.to_abi()
        texs, ntex, tkeep = scene.textures_abi()
        self._keep = (meshes, lights, keep, texs, tkeep)
        self.handle = lib().or_scene_create_textured(meshes, nm, lights, nl, texs, ntex)
        self.num_lights = nl
        self.num_textures = ntex
        self.miss_material = lib().or_scene_miss_material(self.handle)
        self.uv = None   # the bound G-buffer texCoord plane (textured scenes; set by gbuffer / bind_uv)

    def bind_uv(self, uv: np.ndarray | None) -> None:
        """The texCoord plane ([pixels][2], like n_t / p_mat) the following stage calls read."""
        self.uv = None if uv is None else np.ascontiguousarray(uv, np.float32)
        lib().or_scene_bind_uv(self.handle, fp(self.uv))

    def __del__(self):
        if getattr(self, "handle", None):
            lib().or_scene_destroy(self.handle)
            self.handle = None


def camera_frame(cam: _abi.Camera) -> _abi.CameraFrame:
    cf = _abi.CameraFrame()
    lib().or_camera_derive(C.byref(cam), C.byref(cf))
    return cf


def full_rect(W, H) -> Rect:
    return Rect(0, 0, W, H)


def gbuffer(osc: OracleScene, cam: _abi.Camera, W: int, H: int, view: Rect | None = None):
    """(n_t, p_mat) of genPrimaryRayHits; for textured scenes the texCoord plane is bound to `osc` (osc.uv) for
    the stage calls that follow."""
    view = view or full_rect(W, H)
    n = view.w * view.h
    n_t = np.zeros((n, 4), np.float32)
    p_mat = np.zeros((n, 4), np.float32)
    uv = np.zeros((n, 2), np.float32) if osc.num_textures else None
    lib().or_primary_uv(osc.handle, C.byref(camera_frame(cam)), W, H, view, view, fp(n_t), fp(p_mat), fp(uv))
    if osc.num_textures:
        osc.bind_uv(uv)
    return n_t, p_mat


def acquire_texel(osc: OracleScene, texture: int, tc) -> np.ndarray:
    out = np.zeros(3, np.float32)
    t = np.ascontiguousarray(tc, np.float32)
    lib().or_acquire_texel(osc.handle, texture, fp(t), fp(out))
    return out


def empty_reservoirs(N: int, npx: int):
    return (np.zeros((N, npx, 4), np.float32), np.zeros((N, npx, 4), np.float32), np.zeros((N, npx, 2), np.float32))


def ris(osc, f, key, origin, W, H, n_t, p_mat, view=None):
    view = view or full_rect(W, H)
    a, b, d = empty_reservoirs(f.num_samples_in_reservoir, view.w * view.h)
    o = np.asarray(origin, np.float32)
    lib().or_ris(osc.handle, C.byref(f), key, fp(o), W, H, view, view, fp(n_t), fp(p_mat), fp(a), fp(b), fp(d))
    return a, b, d


def temporal(osc, f, key, origin, W, H, n_t, p_mat, cur, prev, view=None):
    view = view or full_rect(W, H)
    a, b, d = empty_reservoirs(f.num_samples_in_reservoir, view.w * view.h)
    o = np.asarray(origin, np.float32)
    lib().or_temporal(osc.handle, C.byref(f), key, fp(o), W, H, view, view, fp(n_t), fp(p_mat),
                      fp(cur[0]), fp(cur[1]), fp(prev[0]), fp(prev[1]), fp(a), fp(b), fp(d))
    return a, b, d


def spatial_pass(osc, f, key, origin, W, H, n_t, p_mat, res_in, view=None, rect=None):
    view = view or full_rect(W, H)
    rect = rect or view
    a, b, d = (x.copy() for x in empty_reservoirs(f.num_samples_in_reservoir, view.w * view.h))
    o = np.asarray(origin, np.float32)
    rc = lib().or_spatial_pass(osc.handle, C.byref(f), key, fp(o), W, H, view, rect, fp(n_t), fp(p_mat),
                               fp(res_in[0]), fp(res_in[1]), fp(a), fp(b), fp(d))
    if rc != 0:
        raise RuntimeError("oracle spatial pass: neighbour outside the view")
    return a, b, d


def final(osc, f, origin, W, H, n_t, p_mat, res, view=None, rect=None):
    view = view or full_rect(W, H)
    rect = rect or view
    rgb = np.zeros((rect.h, rect.w, 3), np.float32)
    o = np.asarray(origin, np.float32)
    lib().or_final(osc.handle, C.byref(f), fp(o), W, H, view, rect, fp(n_t), fp(p_mat), fp(res[0]),
                   fp(res[1]), fp(rgb))
    return rgb


def render_frame(osc, cam, f, W, H, seed=_abi.RESTIR_DEFAULT_SEED, frame=0, prev=None, view=None, rect=None,
                 threads=0):
    """renderReSTIR over `view`, owned pixels `rect`.  Returns (rgb, (res_a, res_b), (n_t, p_mat))."""
    view = view or full_rect(W, H)
    rect = rect or view
    N = f.num_samples_in_reservoir
    npx = view.w * view.h
    n_t = np.zeros((npx, 4), np.float32)
    p_mat = np.zeros((npx, 4), np.float32)
    a = np.zeros((N, npx, 4), np.float32)
    b = np.zeros((N, npx, 4), np.float32)
    rgb = np.zeros((rect.h, rect.w, 3), np.float32)
    pa = fp(prev[0]) if prev is not None else None
    pb = fp(prev[1]) if prev is not None else None
    rc = lib().or_render_frame(osc.handle, C.byref(cam), C.byref(f), seed, frame, W, H, view, rect, pa, pb,
                               fp(n_t), fp(p_mat), fp(a), fp(b), fp(rgb), threads)
    if rc != 0:
        raise RuntimeError(f"oracle render_frame failed ({rc})")
    return rgb, (a, b), (n_t, p_mat)


# ---- R-MIS / R-OMIS (render.cpp:64-265) -------------------------------------------------------------------
def up(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.uint32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(UP)


def mis_capacity(f, W, H) -> int:
    return int(lib().or_mis_capacity(C.byref(f), W, H))


def mis_acc_rows(f) -> int:
    return int(lib().or_mis_acc_rows(C.byref(f)))


def neighbours(osc, f, key_sim, key_dis, W, H, n_t, p_mat):
    cap = mis_capacity(f, W, H)
    nbr = np.zeros(((1 + cap), W * H), np.uint32)
    lib().or_neighbours(osc.handle, C.byref(f), key_sim, key_dis, W, H, fp(n_t), fp(p_mat), cap, up(nbr))
    return nbr


def rmis_accumulate(osc, f, origin, W, H, n_t, p_mat, nbr, res_a, res_b, acc):
    o = np.asarray(origin, np.float32)
    lib().or_rmis_accumulate(osc.handle, C.byref(f), fp(o), W, H, fp(n_t), fp(p_mat), up(nbr), fp(res_a), fp(res_b),
                             fp(acc))


def romis_accumulate(osc, f, origin, W, H, n_t, p_mat, nbr, res_a, res_b, res_dbg, iteration, acc):
    o = np.asarray(origin, np.float32)
    lib().or_romis_accumulate(osc.handle, C.byref(f), fp(o), W, H, fp(n_t), fp(p_mat), up(nbr), fp(res_a),
                              fp(res_b), fp(res_dbg), iteration, fp(acc))


def mis_finish(f, W, H, acc):
    rgb = np.zeros((H, W, 3), np.float32)
    lib().or_mis_finish(C.byref(f), W, H, fp(acc), fp(rgb))
    return rgb


def cod_solve(A: np.ndarray, b: np.ndarray) -> np.ndarray:
    """A: [n, n] (row-major numpy; passed column-major), b: [n] -> x"""
    n = A.shape[0]
    Ac = np.ascontiguousarray(A.T, np.float32)
    bc = np.ascontiguousarray(b, np.float32)
    x = np.zeros(n, np.float32)
    lib().or_cod_solve(n, fp(Ac), fp(bc), fp(x))
    return x


def render_mis(osc, cam, f, W, H, seed=_abi.RESTIR_DEFAULT_SEED, frame=0, threads=0):
    rgb = np.zeros((H, W, 3), np.float32)
    rc = lib().or_render_mis(osc.handle, C.byref(cam), C.byref(f), seed, frame, W, H, fp(rgb), threads)
    if rc != 0:
        raise RuntimeError(f"oracle render_mis failed ({rc})")
    return rgb
