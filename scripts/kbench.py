#!/usr/bin/env python3
"""Interleaved in-process A/B of launch-shape knobs (restir_set_tuning) on the headline 1080p frame.

    python scripts/kbench.py [--rounds 5] [--frames 10]

Every variant renders the same frames; per-kernel times come from HIP events on the context's stream.
Prints one JSON object: {variant: {kernel: median us per launch}}.  Knobs never change results (the GPU
parity suite checks that under the defaults; this script also checks the RGB of every variant is identical).
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from romis_amd import _abi, restir, scene  # noqa: E402

DEFAULTS = {"primary.lds": 1, "ris.lds": 1, "ris.compact": 1, "ris.late": 1, "miss.tiles": 1, "miss.gbuf": 2,
            "spatial.xcd_rows": 255, "spatial.xcd_cols": 255, "spatial.lean": 1, "spatial.th": 0, "spatial.handles": 1, "spatial.gather": 1, "spatial.n2h": 1,
            "fuse.primary_ris": 1, "fuse.temporal": 1, "bvh.max_leaf": 2, "final.lds": 1, "final.sort": 1, "final.qbvh": 2, "primary.tl": 1, "final.miss": 1, "layout.records": 0}

VARIANTS = {
    "default": {},
    "handles_off": {"spatial.handles": 0},
    "handles_t1": {"spatial.th": 1},
    "handles_lds": {"spatial.gather": 0},
    "tl_off": {"primary.tl": 0},
    "ntl_t2": {"spatial.handles": 0, "spatial.th": 2},
    "feat_no_tonemap": {"@enable_tone_mapping": 0},
    "primary_2d_global": {"primary.lds": 0},
    "ris_nolds": {"ris.lds": 0},
    "spatial_band": {"spatial.xcd_rows": 0},

    "spatial_rows1": {"spatial.xcd_rows": 1},
    "spatial_rows2": {"spatial.xcd_rows": 2},
    "spatial_rows8": {"spatial.xcd_rows": 8},
    "spatial_rows4": {"spatial.xcd_rows": 4},
    "spatial_rows3": {"spatial.xcd_rows": 3},
    "spatial_rows5": {"spatial.xcd_rows": 5},
    "spatial_rows6": {"spatial.xcd_rows": 6},
    "spatial_general": {"spatial.lean": 0},
    "unfused": {"fuse.primary_ris": 0},
    "final_unsorted": {"final.sort": 0},
    "layout_records": {"layout.records": 1},
    "bvh_leaf1": {"bvh.max_leaf": 1},
    "bvh_leaf3": {"bvh.max_leaf": 3},
    "bvh_leaf4": {"bvh.max_leaf": 4},
    "bvh_leaf1_sort": {"bvh.max_leaf": 1, "final.sort": 1},
    "bvh_leaf8": {"bvh.max_leaf": 8},
    "final_2d_global": {"final.lds": 0},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--scene", default="nightclub_128pt")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--only", nargs="*", help="run only these variants")
    args = ap.parse_args()
    variants = {k: v for k, v in VARIANTS.items() if not args.only or k in args.only}
    W, H = args.width, args.height
    r = restir.Renderer(0)
    sc = scene.bench_scene(args.scene)
    r.set_scene(sc)
    prev_leaf = 2
    cam = scene.camera_for(args.scene, W, H)
    f = _abi.default_features(num_samples_in_reservoir=1, spatial_resampling_passes=1, temporal_reuse=0)
    ref_rgb = None
    samples = {v: {k: [] for k in _abi.KERNEL_NAMES} for v in variants}
    for rnd in range(args.rounds):
        for name, knobs in variants.items():
            fv = _abi.default_features(num_samples_in_reservoir=1, spatial_resampling_passes=1, temporal_reuse=0)
            for k, v in {**DEFAULTS, **knobs}.items():
                if k.startswith("@"):          # a Features override (changes results: not image-checked)
                    setattr(fv, k[1:], v)
                else:
                    r.set_tuning(k, v)
            if "bvh.max_leaf" in knobs or prev_leaf != knobs.get("bvh.max_leaf", 2):
                r.set_scene(sc)            # the BVH is built at set_scene
                prev_leaf = knobs.get("bvh.max_leaf", 2)
            r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
            rgb, _ = r.render_restir(None, cam, W, H, fv, want_grid=False)   # warm + result check
            if ref_rgb is None:
                ref_rgb = rgb
            elif not any(k.startswith("@") for k in knobs) and not np.array_equal(rgb.view(np.uint32),
                                                                                ref_rgb.view(np.uint32)):
                raise SystemExit(f"variant {name} changed the image")
            r.reset_timings()
            r.enable_timing(True)
            for _ in range(args.frames):
                r.render_restir(None, cam, W, H, fv, want_rgb=False, want_grid=False)
            r.synchronize()
            r.enable_timing(False)
            for k, (ms, n) in r.timings().items():
                if n:
                    samples[name][k].append(ms / n * 1e3)
    out = {name: {k: round(statistics.median(v), 2) for k, v in ks.items() if v} for name, ks in samples.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
