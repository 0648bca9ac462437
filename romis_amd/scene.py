"""Host-side scene model: the reference's Scene (src/scene/scene.h:28-33) as numpy arrays.

Prebuilt scenes are the reference's own loadScenePrebuilt() results (scene.cpp:68-132), dumped by the
reference's loader itself (tests/golden/make_ref_fixtures.py) into romis_amd/scenes/prebuilt_scenes.json.
The synthetic many-light configurations of BASELINE.json are built here from
regularLightGrid (scene.cpp:5-28), restated in float32 and pinned by tests/test_oracle_pinning.py.
"""
from __future__ import annotations

import ctypes as C
import json
import os
from dataclasses import dataclass, field

import numpy as np

from . import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
PREBUILT_JSON = os.path.join(HERE, "scenes", "prebuilt_scenes.json")
f32 = np.float32


@dataclass
class MeshData:
    positions: np.ndarray        # [V, 3] float32
    normals: np.ndarray          # [V, 3] float32
    triangles: np.ndarray        # [T, 3] uint32
    kd: np.ndarray               # [3] float32
    ks: np.ndarray               # [3] float32
    shininess: np.float32
    transparency: np.float32
    name: str = ""
    texcoords: np.ndarray | None = None   # [V, 2] float32 Vertex::texCoord (None: loadMesh's (0, 0))
    texture: object = None                # Texture (Material::kdTexture) or None


@dataclass
class Texture:
    """Image (framework/include/framework/image.h): rgb [height][width][3] float32, row 0 = the file's first row."""
    rgb: np.ndarray


@dataclass
class Scene:
    meshes: list = field(default_factory=list)
    lights: list = field(default_factory=list)   # list of _abi.Light
    name: str = ""

    @property
    def num_triangles(self) -> int:
        return int(sum(len(m.triangles) for m in self.meshes))

    def textures(self) -> list:
        """The distinct Images the meshes' materials point at (restir_material.kd_texture = 1 + index)."""
        out = []
        for m in self.meshes:
            if m.texture is not None and not any(t is m.texture for t in out):
                out.append(m.texture)
        return out

    def to_abi(self):
        """(Mesh array, Light array, keepalive) for restir_set_scene / or_scene_create."""
        keep = []
        texs = self.textures()
        meshes = (_abi.Mesh * max(1, len(self.meshes)))()
        for i, m in enumerate(self.meshes):
            pos = np.ascontiguousarray(m.positions, dtype=f32)
            nrm = np.ascontiguousarray(m.normals, dtype=f32)
            tri = np.ascontiguousarray(m.triangles, dtype=np.uint32)
            keep += [pos, nrm, tri]
            meshes[i].positions = pos.ctypes.data_as(C.POINTER(C.c_float))
            meshes[i].normals = nrm.ctypes.data_as(C.POINTER(C.c_float))
            meshes[i].num_vertices = len(pos)
            meshes[i].triangles = tri.ctypes.data_as(C.POINTER(C.c_uint32))
            meshes[i].num_triangles = len(tri)
            meshes[i].material.kd[:] = [float(x) for x in m.kd]
            meshes[i].material.ks[:] = [float(x) for x in m.ks]
            meshes[i].material.shininess = float(m.shininess)
            meshes[i].material.transparency = float(m.transparency)
            meshes[i].material.kd_texture = 0 if m.texture is None else 1 + next(
                k for k, t in enumerate(texs) if t is m.texture)
            if m.texcoords is not None:
                tc = np.ascontiguousarray(m.texcoords, dtype=f32)
                keep.append(tc)
                meshes[i].texcoords = tc.ctypes.data_as(C.POINTER(C.c_float))
        lights = (_abi.Light * max(1, len(self.lights)))()
        for i, l in enumerate(self.lights):
            lights[i] = l
        return meshes, len(self.meshes), lights, len(self.lights), keep

    def textures_abi(self):
        """(Texture array, count, keepalive) for restir_set_scene_textured / or_scene_create_textured."""
        texs = self.textures()
        arr = (_abi.Texture * max(1, len(texs)))()
        keep = []
        for i, t in enumerate(texs):
            rgb = np.ascontiguousarray(t.rgb, dtype=f32)
            keep.append(rgb)
            arr[i].width, arr[i].height = rgb.shape[1], rgb.shape[0]
            arr[i].rgb = rgb.ctypes.data_as(C.POINTER(C.c_float))
        return arr, len(texs), keep


def _bits(a) -> np.ndarray:
    return np.asarray(a, dtype=np.uint32).view(np.float32)


_prebuilt_cache: dict = {}


def _prebuilt_json() -> dict:
    if "d" not in _prebuilt_cache:
        with open(PREBUILT_JSON) as fh:
            _prebuilt_cache["d"] = json.load(fh)["scenes"]
    return _prebuilt_cache["d"]


def light_from_record(rec: dict) -> _abi.Light:
    v = [_bits(x) for x in rec["v"]]
    l = _abi.Light(type=rec["type"])
    if rec["type"] == _abi.LIGHT_POINT:
        l.p0[:], l.c0[:] = v[0].tolist(), v[1].tolist()
    elif rec["type"] == _abi.LIGHT_SEGMENT:
        l.p0[:], l.p1[:], l.c0[:], l.c1[:] = (x.tolist() for x in v)
    else:
        l.p0[:], l.p1[:], l.p2[:], l.c0[:], l.c1[:], l.c2[:], l.c3[:] = (x.tolist() for x in v)
    return l


def prebuilt_names() -> list:
    return list(_prebuilt_json().keys())


def load_prebuilt(name: str) -> Scene:
    """loadScenePrebuilt(SceneType, DATA_DIR) (scene.cpp:68-132), as the reference's own loader produced it."""
    d = _prebuilt_json()[name]
    meshes = []
    for i, m in enumerate(d["meshes"]):
        pos = _bits([v[0] for v in m["vertices"]]).reshape(-1, 3)
        nrm = _bits([v[1] for v in m["vertices"]]).reshape(-1, 3)
        tri = np.asarray(m["triangles"], dtype=np.uint32).reshape(-1, 3)
        tc = _bits([v[2] for v in m["vertices"]]).reshape(-1, 2)
        tex = None
        if "texture" in m:   # Image: stb RGB bytes / 255.0f (image.cpp:22-31), bytes from the reference's load
            t = m["texture"]
            b = np.frombuffer(bytes.fromhex(t["rgb_u8"]), dtype=np.uint8).astype(f32)
            tex = Texture((b / f32(255.0)).astype(f32).reshape(t["height"], t["width"], 3))
        meshes.append(MeshData(pos, nrm, tri, _bits(m["kd"]), _bits(m["ks"]), _bits([m["shininess"]])[0],
                               _bits([m["transparency"]])[0], name=f"{name}:{i}",
                               texcoords=tc if np.any(tc) or tex is not None else None, texture=tex))
    lights = [light_from_record(r) for r in d["lights"]]
    return Scene(meshes, lights, name)


def regular_light_grid(start, counts, edge01, edge02, color, empty_space=0.1):
    """regularLightGrid (scene.cpp:5-28) in float32, same operation order.  Returns parallelogram lights."""
    start, e01, e02, color = (np.asarray(x, dtype=f32) for x in (start, edge01, edge02, color))
    empty_space = f32(empty_space)
    cx, cy = f32(counts[0]), f32(counts[1])
    space01 = e01 / cx
    space02 = e02 / cy
    light01 = (e01 * (f32(1.0) - empty_space)) / cx
    light02 = (e02 * (f32(1.0) - empty_space)) / cy
    out = []
    for xl in range(int(counts[0])):
        for yl in range(int(counts[1])):
            origin = (start + space01 * f32(xl)) + space02 * f32(yl)
            l = _abi.Light(type=_abi.LIGHT_PARALLELOGRAM)
            l.p0[:] = origin.tolist()
            l.p1[:] = light01.tolist()
            l.p2[:] = light02.tolist()
            for c in ("c0", "c1", "c2", "c3"):
                getattr(l, c)[:] = color.tolist()
            out.append(l)
    return out


def nightclub_wall_grids(counts=(16, 16)):
    """The two lit walls of constructNightClubLights (scene.cpp:30-66): right (0.65) and back (0.4)."""
    free = 0.30
    right = regular_light_grid((-8.7, 6.4, -9.1), counts, (0.0, 0.0, 17.0), (0.0, -6.0, 0.0), (0.65,) * 3, free)
    back = regular_light_grid((9.2, 6.4, 8.6), counts, (-17.0, 0.0, 0.0), (0.0, -6.0, 0.0), (0.4,) * 3, free)
    return right + back


def parallelogram_centre_points(lights):
    """Point lights at the centres v0 + 0.5 e01 + 0.5 e02 of parallelogram lights."""
    out = []
    h = f32(0.5)
    for l in lights:
        v0, e1, e2 = (np.asarray(list(getattr(l, k)), dtype=f32) for k in ("p0", "p1", "p2"))
        c = (v0 + e1 * h) + e2 * h
        p = _abi.Light(type=_abi.LIGHT_POINT)
        p.p0[:] = c.tolist()
        p.c0[:] = list(l.c0)
        out.append(p)
    return out


def _keyed_colour(i: int, seed: int = 0x5EED0001) -> list:
    """Deterministic per-light colour ~ U[0.2, 1]^3 from the keyed RNG (murmur3 fmix32)."""
    def mix32(h):
        h &= 0xFFFFFFFF
        h ^= h >> 16; h = (h * 0x85EBCA6B) & 0xFFFFFFFF
        h ^= h >> 13; h = (h * 0xC2B2AE35) & 0xFFFFFFFF
        h ^= h >> 16
        return h
    out = []
    for c in range(3):
        u = f32(mix32(seed ^ mix32(i * 3 + c + 1)) >> 8) * f32(1.0 / 16777216.0)
        out.append(float(f32(0.2) + f32(0.8) * u))
    return out


def cornell_ceiling_grid(n: int) -> Scene:
    """C4/C5: normalised Cornell box + n x n parallelogram lights under the ceiling covering
    90% of the ceiling AABB, free space 0.3, y = ceiling - 0.01, per-light colours ~ U[0.2, 1]^3."""
    s = load_prebuilt("CornellBoxParallelogramLight")
    # the ceiling is the sub-mesh whose lowest vertex is highest
    ceiling = max(s.meshes, key=lambda m: float(np.min(m.positions[:, 1])))
    lo, hi = ceiling.positions.min(axis=0), ceiling.positions.max(axis=0)
    ext = (hi - lo).astype(f32)
    start = (lo + ext * f32(0.05)).astype(f32)
    start[1] = f32(lo[1] - f32(0.01))
    e01 = np.array([ext[0] * f32(0.9), 0, 0], dtype=f32)
    e02 = np.array([0, 0, ext[2] * f32(0.9)], dtype=f32)
    lights = regular_light_grid(start, (n, n), e01, e02, (1.0, 1.0, 1.0), 0.3)
    for i, l in enumerate(lights):
        col = _keyed_colour(i)
        for c in ("c0", "c1", "c2", "c3"):
            getattr(l, c)[:] = col
    return Scene(s.meshes, lights, f"cornell_{n}x{n}")


def bench_scene(name: str) -> Scene:
    """Named workloads of BASELINE.json / SURVEY.md §8d."""
    if name == "cornell_parallelogram":          # C1
        return load_prebuilt("CornellBoxParallelogramLight")
    if name == "nightclub_128pt":                # C2 / C3
        s = load_prebuilt("CornellNightClub")
        return Scene(s.meshes, parallelogram_centre_points(nightclub_wall_grids((8, 8))), name)
    if name == "nightclub_512":                  # shipped 512-parallelogram set
        return load_prebuilt("CornellNightClub")
    if name == "cornell_1024":                   # C4
        return cornell_ceiling_grid(32)
    if name == "cornell_4096":                   # C5
        return cornell_ceiling_grid(64)
    return load_prebuilt(name)


def nightclub_camera(width: int, height: int) -> _abi.Camera:
    """CameraConfig defaults (src/utils/config.h:21-26) through Trackball(radians(fov)) + setCamera."""
    return make_camera(30.0, 25.0, (2.57, 1.23, -1.35), (10.3, 30.0, 0.0), width, height)


def cornell_camera(width: int, height: int) -> _abi.Camera:
    """TOML camera defaults (config.cpp:249-252): fov 50, distance 3, lookAt 0, rotation (20, 20, 0)."""
    return make_camera(50.0, 3.0, (0.0, 0.0, 0.0), (20.0, 20.0, 0.0), width, height)


# The framed Cornell camera of bench.py's c4f / c5f: the TOML camera sees the box in the middle of a
# 16:9 frame -- 13 % of C4's pixels hit geometry -- so its 4K / 8K spatial passes mostly write background tiles.  This
# one looks into the box from 1.5 units with a 30 degree field of view, rotation (20, 10, 0): 99.9 % of the pixels
# hit geometry (7 materials; oracle primary rays at 384 x 216), 91 % are lit.  Not a reference camera: the same
# Trackball parameters the reference's UI sets (trackball.cpp:20-29), chosen so the pass reads HBM, not background.
CORNELL_FRAMED = dict(fov_deg=30.0, dist=1.5, look_at=(0.0, 0.0, 0.0), rot_deg=(20.0, 10.0, 0.0))


def cornell_framed_camera(width: int, height: int) -> _abi.Camera:
    c = CORNELL_FRAMED
    return make_camera(c["fov_deg"], c["dist"], c["look_at"], c["rot_deg"], width, height)


def make_camera(fov_deg, dist, look_at, rot_deg, width, height) -> _abi.Camera:
    rad = f32(0.01745329251994329576923690768489)   # glm::radians
    cam = _abi.Camera()
    cam.fovy = float(f32(fov_deg) * rad)
    cam.aspect = float(f32(width) / f32(height)) if width and height else 1.0
    cam.look_at[:] = [float(f32(x)) for x in look_at]
    cam.distance = float(f32(dist))
    cam.rotation[:] = [float(f32(x) * rad) for x in rot_deg]
    return cam


def camera_for(scene_name: str, width: int, height: int, framing: str | None = None) -> _abi.Camera:
    """The workload's camera: the scene's default, or framing "framed" (the Cornell scenes: CORNELL_FRAMED)."""
    if framing == "framed":
        if scene_name.startswith("nightclub") or scene_name == "CornellNightClub":
            raise ValueError("framing 'framed' is defined for the Cornell scenes")
        return cornell_framed_camera(width, height)
    if scene_name.startswith("nightclub") or scene_name == "CornellNightClub":
        return nightclub_camera(width, height)
    return cornell_camera(width, height)
