"""Python host binding of the C ABI (include/restir_c.h) -- mirrors the reference's render surface.

    renderer = Renderer(device=0)
    renderer.set_scene(scene)                                  # EmbreeInterface(scene) (embree_interface.cpp:14-51)
    rgb, grid = renderer.render_restir(prev_grid, camera, W, H, features)   # renderReSTIR (render.cpp:28-62)

Errors raise RestirError (the reference throws std::runtime_error, render.cpp:99/278).  Everything runs in
libromis_amd.so on the GPU; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi
from ._abi import RestirError, check  # noqa: F401


class ReservoirGrid:
    """Device-resident ReservoirGrid (reservoir.h:75) -- a reference-counted restir_frame handle."""

    def __init__(self, lib, handle):
        self._lib = lib
        self.handle = handle

    def __del__(self):
        if getattr(self, "handle", None):
            self._lib.restir_frame_release(self.handle)
            self.handle = None

    def info(self) -> dict:
        """(W, H) of the image and the (vx0, vy0, vw, vh) view the grid covers, N sub-reservoirs per pixel."""
        v = [C.c_uint32() for _ in range(7)]
        check(self._lib, self._lib.restir_frame_info(self.handle, *[C.byref(x) for x in v]), "restir_frame_info")
        return dict(zip(("W", "H", "vx0", "vy0", "vw", "vh", "N"), (x.value for x in v)))

    def download(self):
        """The grid's (pos [N][vh][vw][3], color [N][vh][vw][3], W [N][vh][vw], M [N][vh][vw] uint32), rows y = 0
        bottom -- the per-pixel Reservoir state renderReSTIR returns (render.cpp:61)."""
        i = self.info()
        n = i["N"] * i["vh"] * i["vw"]
        pos, col = np.zeros((n, 3), np.float32), np.zeros((n, 3), np.float32)
        w, m = np.zeros(n, np.float32), np.zeros(n, np.uint32)
        FP, UP = C.POINTER(C.c_float), C.POINTER(C.c_uint32)
        check(self._lib, self._lib.restir_frame_download(self.handle, pos.ctypes.data_as(FP), col.ctypes.data_as(FP),
                                                         w.ctypes.data_as(FP), m.ctypes.data_as(UP)),
              "restir_frame_download")
        shp = (i["N"], i["vh"], i["vw"])
        return pos.reshape(shp + (3,)), col.reshape(shp + (3,)), w.reshape(shp), m.reshape(shp)


class Renderer:
    def __init__(self, device: int = 0):
        self.lib = _abi.load_library()
        h = C.c_void_p()
        check(self.lib, self.lib.restir_create(device, C.byref(h)), "restir_create")
        self.ctx = h
        self._scene_keep = None
        self.stage_shape = None

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.restir_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        self.close()

    # ---- scene / seed -------------------------------------------------------------------------------
    def set_scene(self, scene) -> None:
        """EmbreeInterface(scene): meshes, lights and the Images of textured materials (restir_set_scene_textured)."""
        meshes, nm, lights, nl, keep = scene.to_abi()
        texs, ntex, tkeep = scene.textures_abi()
        check(self.lib, self.lib.restir_set_scene_textured(self.ctx, meshes, nm, lights, nl, texs, ntex),
              "restir_set_scene_textured")
        self._scene_keep = (meshes, lights, keep, texs, tkeep)

    def set_seed(self, seed: int = _abi.RESTIR_DEFAULT_SEED, frame: int = 0) -> None:
        check(self.lib, self.lib.restir_set_seed(self.ctx, seed, frame), "restir_set_seed")

    def set_renders_dir(self, path) -> None:
        """The reference's RENDERS_DIR for file side outputs (None = none): R-OMIS renders with
        save_alphas_visualisation write visualiseAlphas' bitmaps there after every iteration."""
        d = None if path is None else os.fsencode(path)
        check(self.lib, self.lib.restir_set_renders_dir(self.ctx, d), "restir_set_renders_dir")

    # ---- frame ----------------------------------------------------------------------------------------
    def render_restir(self, prev: ReservoirGrid | None, camera, width: int, height: int, features,
                      tile=None, want_rgb: bool = True, want_grid: bool = True):
        """renderReSTIR: returns (rgb [h][w][3] row 0 = top, or None; ReservoirGrid or None)."""
        out = C.c_void_p()
        rgb = None
        rgb_ptr = None
        if want_rgb:
            h_ = tile.height if tile is not None else height
            w_ = tile.width if tile is not None else width
            rgb = np.zeros((h_, w_, 3), np.float32)
            rgb_ptr = rgb.ctypes.data_as(C.POINTER(C.c_float))
        st = self.lib.restir_render(self.ctx, C.byref(camera), C.byref(features), width, height,
                                    C.byref(tile) if tile is not None else None,
                                    prev.handle if prev is not None else None,
                                    C.byref(out) if want_grid else None, rgb_ptr)
        check(self.lib, st, "restir_render")
        grid = ReservoirGrid(self.lib, out) if want_grid and out.value else None
        return rgb, grid

    def synchronize(self) -> None:
        check(self.lib, self.lib.restir_synchronize(self.ctx), "restir_synchronize")

    def download_rgb(self, width: int, height: int) -> np.ndarray:
        rgb = np.zeros((height, width, 3), np.float32)
        check(self.lib, self.lib.restir_download_rgb(self.ctx, rgb.ctypes.data_as(C.POINTER(C.c_float)), rgb.size),
              "restir_download_rgb")
        return rgb

    # ---- halo-mode frames (include/restir_c.h "halo-mode frames") -------------------------------------
    def halo_begin(self, prev, camera, width, height, features, tiles, rank, layout=None):
        """Primary rays on the tile + ring, RIS / temporal on the owned tile.  Returns (send_bytes, recv_bytes).
        layout: an uneven restir_tile_layout (layout_balanced) instead of the even tiles split."""
        sb, rb_ = C.c_uint64(), C.c_uint64()
        ph = prev.handle if prev is not None else None
        if layout is not None:
            check(self.lib, self.lib.restir_halo_begin_layout(self.ctx, C.byref(camera), C.byref(features), C.byref(layout),
                                                              rank, ph, C.byref(sb), C.byref(rb_)), "restir_halo_begin_layout")
        else:
            check(self.lib, self.lib.restir_halo_begin(self.ctx, C.byref(camera), C.byref(features), width, height,
                                                       tiles[0], tiles[1], rank, ph, C.byref(sb), C.byref(rb_)),
                  "restir_halo_begin")
        return sb.value, rb_.value

    def halo_pack(self, buf_ptr: int, nbytes: int, host: bool) -> None:
        check(self.lib, self.lib.restir_halo_pack(self.ctx, buf_ptr, nbytes, int(host)), "restir_halo_pack")

    def halo_unpack(self, buf_ptr: int, nbytes: int, host: bool) -> None:
        check(self.lib, self.lib.restir_halo_unpack(self.ctx, buf_ptr, nbytes, int(host)), "restir_halo_unpack")

    def halo_spatial(self) -> None:
        check(self.lib, self.lib.restir_halo_spatial(self.ctx), "restir_halo_spatial")

    def halo_spatial_interior(self) -> None:
        """The current pass's interior (reads no exchanged reservoir): issue it before waiting on the exchange."""
        check(self.lib, self.lib.restir_halo_spatial_interior(self.ctx), "restir_halo_spatial_interior")

    def halo_spatial_border(self) -> None:
        """The current pass's border strips (after the unpack); completes the pass."""
        check(self.lib, self.lib.restir_halo_spatial_border(self.ctx), "restir_halo_spatial_border")

    def halo_attach_rccl(self, unique_id: bytes, nranks: int, rank: int) -> None:
        """Native RCCL halo transport: ncclCommInitRank on this context's device (restir_halo_attach_rccl)."""
        buf = C.create_string_buffer(bytes(unique_id), _abi.RESTIR_RCCL_ID_BYTES)
        check(self.lib, self.lib.restir_halo_attach_rccl(self.ctx, C.cast(buf, C.c_void_p), nranks, rank),
              "restir_halo_attach_rccl")

    def halo_pass(self) -> None:
        """One spatial pass with the exchange over the attached communicator, overlapped with the interior."""
        check(self.lib, self.lib.restir_halo_pass(self.ctx), "restir_halo_pass")

    def halo_record(self, on: bool = True) -> None:
        """restir_halo_record: halo_pass logs the steps it issues instead of calling RCCL (no communicator needed)."""
        check(self.lib, self.lib.restir_halo_record(self.ctx, 1 if on else 0), "restir_halo_record")

    def halo_log(self) -> list:
        """restir_halo_log: the record-only passes' steps in issue order (then cleared), as HaloEvent structs."""
        n = C.c_uint32(0)
        rc = self.lib.restir_halo_log(self.ctx, None, C.byref(n))
        if rc != 0 and n.value == 0:
            check(self.lib, rc, "restir_halo_log")
        buf = (_abi.HaloEvent * max(1, n.value))()
        n2 = C.c_uint32(n.value)
        check(self.lib, self.lib.restir_halo_log(self.ctx, buf, C.byref(n2)), "restir_halo_log")
        return list(buf[:n2.value])

    def halo_end(self, tile, want_rgb: bool = True, want_grid: bool = True):
        out = C.c_void_p()
        rgb = np.zeros((tile.height, tile.width, 3), np.float32) if want_rgb else None
        check(self.lib, self.lib.restir_halo_end(self.ctx, C.byref(out) if want_grid else None,
                                                 rgb.ctypes.data_as(C.POINTER(C.c_float)) if want_rgb else None),
              "restir_halo_end")
        return rgb, (ReservoirGrid(self.lib, out) if want_grid and out.value else None)

    def measure_read_bandwidth(self, nbytes: int = 4 << 30, iters: int = 10) -> float:
        """GB/s of a streaming-read kernel over `nbytes` of HBM (restir_measure_read_bandwidth)."""
        out = C.c_double()
        check(self.lib, self.lib.restir_measure_read_bandwidth(self.ctx, int(nbytes), int(iters), C.byref(out)),
              "restir_measure_read_bandwidth")
        return out.value

    def background_pixels(self) -> tuple[int, int]:
        """(background, computed) pixels of the last render_restir frame (restir_background_pixels): the pixels of its
        RIS tiles flagged all-miss, which the spatial passes and final shading write without reading."""
        bg, px = C.c_uint64(), C.c_uint64()
        check(self.lib, self.lib.restir_background_pixels(self.ctx, C.byref(bg), C.byref(px)), "restir_background_pixels")
        return int(bg.value), int(px.value)

    # ---- timing ---------------------------------------------------------------------------------------
    def enable_timing(self, on: bool = True) -> None:
        check(self.lib, self.lib.restir_enable_timing(self.ctx, 1 if on else 0), "restir_enable_timing")

    def timings(self):
        ms = (C.c_double * _abi.K_COUNT)()
        n = (C.c_uint64 * _abi.K_COUNT)()
        check(self.lib, self.lib.restir_timings(self.ctx, ms, n), "restir_timings")
        return {name: (ms[i], n[i]) for i, name in enumerate(_abi.KERNEL_NAMES)}

    def set_tuning(self, key: str, value: int) -> None:
        check(self.lib, self.lib.restir_set_tuning(self.ctx, key.encode(), int(value)), "restir_set_tuning")

    def reset_timings(self) -> None:
        check(self.lib, self.lib.restir_reset_timings(self.ctx), "restir_reset_timings")

    # ---- stage API (parity tests) ---------------------------------------------------------------------
    def stage_configure(self, width: int, height: int, n: int) -> None:
        check(self.lib, self.lib.restir_stage_configure(self.ctx, width, height, n), "restir_stage_configure")
        self.stage_shape = (width, height, n)

    def _shape(self, which):
        w, h, n = self.stage_shape
        npx = w * h
        return {
            _abi.BUF_GBUF_N_T: (npx, 4), _abi.BUF_GBUF_P_MAT: (npx, 4),
            _abi.BUF_RES_A: (n, npx, 4), _abi.BUF_RES_B: (n, npx, 4), _abi.BUF_RES_DBG: (n, npx, 2),
            _abi.BUF_PREV_A: (n, npx, 4), _abi.BUF_PREV_B: (n, npx, 4), _abi.BUF_PREV_DBG: (n, npx, 2),
            _abi.BUF_RGB: (h, w, 3), _abi.BUF_GBUF_UV: (npx, 2),
        }[which]

    def upload(self, which: int, arr: np.ndarray) -> None:
        a = np.ascontiguousarray(arr, dtype=np.float32).reshape(self._shape(which))
        check(self.lib, self.lib.restir_stage_upload(self.ctx, which, a.ctypes.data, a.nbytes), "restir_stage_upload")

    def download(self, which: int) -> np.ndarray:
        a = np.zeros(self._shape(which), np.float32)
        check(self.lib, self.lib.restir_stage_download(self.ctx, which, a.ctypes.data, a.nbytes),
              "restir_stage_download")
        return a

    def stage_primary(self, camera) -> None:
        check(self.lib, self.lib.restir_stage_primary(self.ctx, C.byref(camera)), "restir_stage_primary")

    def stage_ris(self, camera, features, key: int, debug: bool = True) -> None:
        check(self.lib, self.lib.restir_stage_ris(self.ctx, C.byref(camera), C.byref(features), key, int(debug)),
              "restir_stage_ris")

    def stage_temporal(self, camera, features, key: int, debug: bool = True) -> None:
        check(self.lib, self.lib.restir_stage_temporal(self.ctx, C.byref(camera), C.byref(features), key,
                                                       int(debug)), "restir_stage_temporal")

    def stage_spatial(self, camera, features, key: int, debug: bool = True) -> None:
        check(self.lib, self.lib.restir_stage_spatial(self.ctx, C.byref(camera), C.byref(features), key,
                                                      int(debug)), "restir_stage_spatial")

    def stage_final(self, camera, features) -> None:
        check(self.lib, self.lib.restir_stage_final(self.ctx, C.byref(camera), C.byref(features)),
              "restir_stage_final")

    # ---- R-MIS / R-OMIS (render.cpp:64-265) ------------------------------------------------------------
    def render_mis(self, camera, width: int, height: int, features) -> np.ndarray:
        """renderRMIS / renderROMIS by features.ray_trace_mode: the screen image (row 0 = top).  No grid is
        returned, as renderRayTraced returns std::nullopt for these modes (render.cpp:274-279)."""
        rgb, _ = self.render_restir(None, camera, width, height, features, want_grid=False)
        return rgb

    def mis_capacity(self, features) -> int:
        cap = C.c_uint32()
        check(self.lib, self.lib.restir_stage_mis_capacity(self.ctx, C.byref(features), C.byref(cap)),
              "restir_stage_mis_capacity")
        return cap.value

    def stage_neighbours(self, features, key_similar: int, key_dissimilar: int) -> None:
        check(self.lib, self.lib.restir_stage_neighbours(self.ctx, C.byref(features), key_similar, key_dissimilar),
              "restir_stage_neighbours")

    def stage_mis_accumulate(self, camera, features, iteration: int) -> None:
        check(self.lib, self.lib.restir_stage_mis_accumulate(self.ctx, C.byref(camera), C.byref(features), iteration),
              "restir_stage_mis_accumulate")

    def stage_mis_finish(self, features) -> None:
        check(self.lib, self.lib.restir_stage_mis_finish(self.ctx, C.byref(features)), "restir_stage_mis_finish")

    def mis_buffers(self, features, nbr: np.ndarray | None = None, acc: np.ndarray | None = None):
        """Upload (when given) and download the MIS_NBR (uint32 [1 + cap][pixels]) and MIS_ACC (float
        [rows][pixels]) stage buffers."""
        w, h, _ = self.stage_shape
        cap = self.mis_capacity(features)
        T = features.num_neighbours_to_sample + 1
        rows = T * T + 6 * T + 3 if features.ray_trace_mode == _abi.MODE_ROMIS else 3
        for which, arr, dt, shape in [(_abi.BUF_MIS_NBR, nbr, np.uint32, (1 + cap, w * h)),
                                      (_abi.BUF_MIS_ACC, acc, np.float32, (rows, w * h))]:
            if arr is not None:
                a = np.ascontiguousarray(arr, dtype=dt).reshape(shape)
                check(self.lib, self.lib.restir_stage_upload(self.ctx, which, a.ctypes.data, a.nbytes),
                      "restir_stage_upload")
        out = []
        for which, dt, shape in [(_abi.BUF_MIS_NBR, np.uint32, (1 + cap, w * h)),
                                 (_abi.BUF_MIS_ACC, np.float32, (rows, w * h))]:
            a = np.zeros(shape, dt)
            check(self.lib, self.lib.restir_stage_download(self.ctx, which, a.ctypes.data, a.nbytes),
                  "restir_stage_download")
            out.append(a)
        return tuple(out)

    def debug_cod_solve(self, A: np.ndarray, b: np.ndarray) -> np.ndarray:
        """Batched least squares (A [count][n][n] row-major numpy, b [count][n]) with the device routine of the
        R-OMIS finish (Eigen CompleteOrthogonalDecomposition::solve, render_utils.h:52)."""
        A = np.asarray(A, np.float32)
        count, n, _ = A.shape
        Ac = np.ascontiguousarray(np.transpose(A, (0, 2, 1)), np.float32)   # column-major per system
        bc = np.ascontiguousarray(b, np.float32).reshape(count, n)
        x = np.zeros((count, n), np.float32)
        FP = C.POINTER(C.c_float)
        check(self.lib, self.lib.restir_debug_cod_solve(self.ctx, n, Ac.ctypes.data_as(FP), bc.ctypes.data_as(FP),
                                                        x.ctypes.data_as(FP), count), "restir_debug_cod_solve")
        return x

    def debug_math(self, x: np.ndarray, y: np.ndarray):
        x = np.ascontiguousarray(x, np.float32)
        y = np.ascontiguousarray(y, np.float32)
        pw = np.zeros_like(x)
        ex = np.zeros_like(x)
        FP = C.POINTER(C.c_float)
        check(self.lib, self.lib.restir_debug_math(self.ctx, x.ctypes.data_as(FP), y.ctypes.data_as(FP),
                                                   pw.ctypes.data_as(FP), ex.ctypes.data_as(FP), x.size),
              "restir_debug_math")
        return pw, ex


def rng_key(seed: int, frame: int, stage: int, pass_: int = 0) -> int:
    return _abi.load_library().restir_rng_key(seed, frame, stage, pass_)


def rccl_unique_id() -> bytes:
    """restir_rccl_unique_id: the RESTIR_RCCL_ID_BYTES bytes one rank hands to all (ncclGetUniqueId)."""
    lib = _abi.load_library()
    buf = C.create_string_buffer(_abi.RESTIR_RCCL_ID_BYTES)
    check(lib, lib.restir_rccl_unique_id(C.cast(buf, C.c_void_p), _abi.RESTIR_RCCL_ID_BYTES), "restir_rccl_unique_id")
    return buf.raw


def halo_plan(width: int, height: int, tiles_x: int, tiles_y: int, rank: int, radius: int, N: int, layout=None):
    """restir_halo_plan: ([send segments], [recv segments]) for `rank`, one pair per adjacent rank (layout: an
    uneven restir_tile_layout instead of the even tiles_x x tiles_y split)."""
    lib = _abi.load_library()
    send = (_abi.HaloSegment * 8)()
    recv = (_abi.HaloSegment * 8)()
    n = C.c_uint32(8)
    if layout is not None:
        check(lib, lib.restir_layout_halo_plan(C.byref(layout), rank, radius, N, send, recv, C.byref(n)),
              "restir_layout_halo_plan")
    else:
        check(lib, lib.restir_halo_plan(width, height, tiles_x, tiles_y, rank, radius, N, send, recv, C.byref(n)),
              "restir_halo_plan")
    return list(send[:n.value]), list(recv[:n.value])


def halo_ops(width: int, height: int, tiles_x: int, tiles_y: int, rank: int, radius: int, N: int, layout=None) -> list:
    """restir_halo_ops: the sends / receives restir_halo_pass posts per spatial pass, in posting order."""
    lib = _abi.load_library()
    ops = (_abi.HaloOp * 16)()
    n = C.c_uint32(16)
    if layout is not None:
        check(lib, lib.restir_layout_halo_ops(C.byref(layout), rank, radius, N, ops, C.byref(n)), "restir_layout_halo_ops")
    else:
        check(lib, lib.restir_halo_ops(width, height, tiles_x, tiles_y, rank, radius, N, ops, C.byref(n)),
              "restir_halo_ops")
    return list(ops[:n.value])


def tile_plan(width: int, height: int, tiles_x: int, tiles_y: int, rank: int, ghost: int, layout=None) -> _abi.Tile:
    lib = _abi.load_library()
    t = _abi.Tile()
    if layout is not None:
        check(lib, lib.restir_layout_tile(C.byref(layout), rank, ghost, C.byref(t)), "restir_layout_tile")
    else:
        check(lib, lib.restir_tile_plan(width, height, tiles_x, tiles_y, rank, ghost, C.byref(t)), "restir_tile_plan")
    return t


def layout_even(width: int, height: int, tiles_x: int, tiles_y: int) -> _abi.TileLayout:
    """restir_layout_even: restir_tile_plan's even split as a layout."""
    lib = _abi.load_library()
    L = _abi.TileLayout()
    check(lib, lib.restir_layout_even(width, height, tiles_x, tiles_y, C.byref(L)), "restir_layout_even")
    return L


def _cost_arg(cost):
    c = np.ascontiguousarray(cost, dtype=np.float32)
    if c.ndim != 2:
        raise ValueError("cost grid must be 2-D [rows (row 0 = bottom)][columns]")
    return c, c.ctypes.data_as(C.POINTER(C.c_float))


def layout_balanced(width: int, height: int, tiles_x: int, tiles_y: int, cost, align=(32, 8)):
    """restir_layout_balanced: (layout, implied efficiency) balancing the cost grid [rows][cols] (row 0 = bottom)."""
    lib = _abi.load_library()
    c, ptr = _cost_arg(cost)
    L = _abi.TileLayout()
    eff = C.c_double()
    check(lib, lib.restir_layout_balanced(width, height, tiles_x, tiles_y, ptr, c.shape[1], c.shape[0], align[0], align[1],
                                          C.byref(L), C.byref(eff)), "restir_layout_balanced")
    return L, eff.value


def layout_shares(layout, cost) -> np.ndarray:
    """restir_layout_shares: each rank's share of the cost grid under `layout` (sums to 1)."""
    lib = _abi.load_library()
    c, ptr = _cost_arg(cost)
    out = np.zeros(layout.tiles_x * layout.tiles_y, np.float64)
    check(lib, lib.restir_layout_shares(C.byref(layout), ptr, c.shape[1], c.shape[0],
                                        out.ctypes.data_as(C.POINTER(C.c_double))), "restir_layout_shares")
    return out


def tile_grid(n: int) -> tuple:
    """Screen tiling for n ranks: 1x1, 2x1, 2x2, 4x2 (tiles_x, tiles_y)."""
    return {1: (1, 1), 2: (2, 1), 4: (2, 2), 8: (4, 2)}.get(n) or (n, 1)
