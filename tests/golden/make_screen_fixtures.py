#!/usr/bin/env python3
"""Generate tests/golden/screen_fixtures.json: frame output written by the REFERENCE's own code paths
(oracle/_ref/screen_ref, built by `make -C oracle ref` from /root/reference):
  - bmp:  float RGB images (row 0 = top) -> Screen::writeBitmapToFile's 8-bit conversion (screen.cpp:47-51) on the
          reference's glm -> its vendored stb_image_write BMP (screen.cpp:55).  Values cover [-0.5, 1.5], the
          k / 255 boundaries and their float neighbours, exact 0 / 1, and a tone-mapped frame of the oracle.
  - json: struct Features with fields set -> the reference's vendored cereal JSONOutputArchive (render.cpp:284-286).
Run in the build container only (the GPU box has no /root/reference):  python tests/golden/make_screen_fixtures.py
"""
import base64
import json
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
TOOL = os.path.join(ROOT, "oracle", "_ref", "screen_ref")
OUT = os.path.join(ROOT, "tests", "golden", "screen_fixtures.json")


def images():
    rng = np.random.default_rng(20261016)
    out = []
    out.append(("random", rng.uniform(-0.5, 1.5, (7, 13, 3)).astype(np.float32)))
    k = np.arange(256, dtype=np.float32) / np.float32(255.0)
    edges = np.concatenate([k, np.nextafter(k, np.float32(-1)), np.nextafter(k, np.float32(2)),
                            np.float32([0.0, -0.0, 1.0, 2.0, -1.0, 1e-30, 0.99999994])]).astype(np.float32)
    pad = (-edges.size) % 48
    edges = np.concatenate([edges, np.zeros(pad, np.float32)]).reshape(-1, 16, 3)
    out.append(("boundaries", edges))
    out.append(("one_pixel", np.float32([[[0.25, 0.5, 0.75]]])))
    from oracle import pyoracle
    from romis_amd import _abi, scene
    name, W, H = "nightclub_128pt", 24, 16
    osc = pyoracle.OracleScene(scene.bench_scene(name))
    f = _abi.default_features(initial_light_samples=8, num_samples_in_reservoir=1)
    rgb, _, _ = pyoracle.render_frame(osc, scene.camera_for(name, W, H), f, W, H, threads=1)
    out.append(("oracle_frame", rgb.astype(np.float32)))
    return out


def bits(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def feature_sets():
    rng = np.random.default_rng(7)
    sets = [{}, {"gamma": bits(2.2), "exposure": bits(0.1)}, {"rayTraceMode": 2, "numSamplesInReservoir": 7,
            "enableShading": 0, "temporalReuse": 0, "maxIterationsMIS": 12, "neighbourSelectionStrategy": 3,
            "misWeightRMIS": 1, "useProgressiveROMIS": 1, "enableRecursive": 1, "maxReflectionRecursion": 9,
            "gamma": bits(1e-7), "exposure": bits(3e25)},
            {"gamma": bits(123456.789), "exposure": bits(-0.0)}, {"gamma": bits(1e21), "exposure": bits(1e-6)},
            {"gamma": bits(0.5), "exposure": bits(100.0)}]
    for _ in range(200):
        g = float(np.float32(rng.uniform(0.0, 4.0)))
        e = float(np.float32(10.0 ** rng.uniform(-9, 25)))
        sets.append({"gamma": bits(g), "exposure": bits(e), "initialLightSamples": int(rng.integers(1, 1 << 20)),
                     "spatialReuse": int(rng.integers(0, 2))})
    return sets


def main():
    if not os.path.exists(TOOL):
        sys.exit(f"{TOOL} missing: run `make -C oracle ref` first")
    fx = {"generator": "tests/golden/make_screen_fixtures.py (oracle/_ref/screen_ref: the reference's glm + stb + "
                       "cereal + struct Features)", "bmp": [], "json": []}
    for name, img in images():
        H, W, _ = img.shape
        r = subprocess.run([TOOL, "bmp", str(W), str(H)], input=img.tobytes(), capture_output=True, check=True)
        fx["bmp"].append({"name": name, "width": W, "height": H,
                          "rgb_bits": base64.b64encode(img.tobytes()).decode(),
                          "bmp": base64.b64encode(r.stdout).decode()})
    for s in feature_sets():
        args = [f"{k}={v}" for k, v in s.items()]
        r = subprocess.run([TOOL, "json"] + args, capture_output=True, check=True, text=True)
        fx["json"].append({"set": s, "json": r.stdout})
    with open(OUT, "w") as fh:
        json.dump(fx, fh, indent=0)
    print(OUT, len(fx["bmp"]), "images", len(fx["json"]), "feature sets")


if __name__ == "__main__":
    main()
