#!/usr/bin/env python3
"""Geometry share per rank of the strong-scaling configs' screen-tile plans (VERDICT r4 missing #3): the oracle's
primary rays over the config's image at a quarter of its resolution (same camera and aspect), the fraction of each
tile_plan tile's pixels that hit the scene, and the parallel efficiency that implies if a rank's time follows its
geometry pixels (mean share / max share; background tiles cost almost nothing with MissTiles).

    python scripts/balance.py > profiles/r5/balance.json
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import pyoracle  # noqa: E402
from romis_amd import restir, scene  # noqa: E402

import bench  # noqa: E402


def main():
    out = {"method": "oracle primary rays at 1/4 resolution; share = geometry pixels / tile pixels; efficiency = "
                     "mean over ranks of geometry pixels / max over ranks (time proportional to geometry pixels)"}
    for name in ("c4", "c5", "c4f", "c5f"):
        cf = bench.CONFIGS[name]
        W, H = cf["image"]
        w, h = W // 4, H // 4
        osc = pyoracle.OracleScene(scene.bench_scene(cf["scene"]))
        cam = scene.camera_for(cf["scene"], w, h, cf.get("camera"))
        _, p_mat = pyoracle.gbuffer(osc, cam, w, h)
        hit = (p_mat[:, 3].view(np.uint32) != osc.miss_material).reshape(h, w)   # row 0 = bottom
        rec = {"image": [W, H], "sampled": [w, h], "geometry": round(float(hit.mean()), 4), "plans": {}}
        for world in (2, 4, 8):
            tx, ty = restir.tile_grid(world)
            shares, pix = [], []
            for rank in range(world):
                t = restir.tile_plan(w, h, tx, ty, rank, 0)
                blk = hit[t.y0:t.y0 + t.height, t.x0:t.x0 + t.width]
                shares.append(round(float(blk.mean()), 4))
                pix.append(int(blk.sum()))
            eff = float(np.mean(pix) / max(1, max(pix)))
            rec["plans"][f"{tx}x{ty}"] = {"share_per_rank": shares, "geometry_px_per_rank": pix,
                                          "implied_efficiency": round(eff, 3)}
        out[name] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
