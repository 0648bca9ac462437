#!/usr/bin/env python3
"""Interleaved in-process A/B of restir_set_tuning knobs on a BASELINE.json config's frame (bench.py CONFIGS):
per-kernel median microseconds per launch over rounds; every variant's RGB must equal the first's.

    python scripts/cfg_kbench.py --config c5 --variants default:spatial.lean=1 general:spatial.lean=0
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import bench  # noqa: E402
from romis_amd import _abi, restir, scene  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "scripts"))
from kbench import DEFAULTS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2", choices=list(bench.CONFIGS))
    ap.add_argument("--N", type=int, default=1)
    ap.add_argument("--scene", default=None, help="another bench scene under the config's settings")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--variants", nargs="+", default=["default:"])
    args = ap.parse_args()
    cf = dict(bench.CONFIGS[args.config])
    if args.scene:
        cf["scene"] = args.scene
    W, H = cf.get("image") or cf["tile"]
    passes = cf["passes"]
    f = _abi.default_features(initial_light_samples=cf["M"], num_samples_in_reservoir=args.N, spatial_resampling_passes=passes,
                              spatial_reuse=1 if passes else 0, temporal_reuse=cf["temporal"],
                              unbiased_combination=cf["unbiased"], spatial_reuse_visibility_check=cf["vis"])
    variants = {}
    for v in args.variants:
        name, _, knobs = v.partition(":")
        variants[name] = dict((k, int(x)) for k, x in (kv.split("=") for kv in knobs.split(",") if kv))
    keys = sorted({k for kn in variants.values() for k in kn})
    missing = [k for k in keys if k not in DEFAULTS]
    if missing:   # every knob a variant sets needs its library default (scripts/kbench.py DEFAULTS) for the others
        raise SystemExit(f"cfg_kbench: no default for {missing} in scripts/kbench.py DEFAULTS")
    r = restir.Renderer(0)
    r.set_scene(scene.bench_scene(cf["scene"]))
    cam = scene.camera_for(cf["scene"], W, H, cf.get("camera"))
    ref = None
    samples = {v: {} for v in variants}
    for _ in range(args.rounds):
        for name, knobs in variants.items():
            for k in keys:   # every knob any variant sets: this variant's value or the default
                r.set_tuning(k, knobs.get(k, DEFAULTS[k]))
            if any(k.startswith("bvh.") for k in keys):   # BVH knobs apply at the next set_scene
                r.set_scene(scene.bench_scene(cf["scene"]))
            r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
            # temporal configs (c3): the second frame reuses the first's grid, so its image checks the temporal path
            rgb, g = r.render_restir(None, cam, W, H, f, want_grid=bool(cf["temporal"]))
            if cf["temporal"]:
                rgb, g = r.render_restir(g, cam, W, H, f, want_grid=True)
            if ref is None:
                ref = rgb
            elif not np.array_equal(rgb.view(np.uint32), ref.view(np.uint32)):
                raise SystemExit(f"variant {name} changed the image")
            r.reset_timings()
            r.enable_timing(True)
            for _ in range(args.frames):   # temporal configs thread the previous frame's grid (main.cpp:165)
                if cf["temporal"]:
                    _, g = r.render_restir(g, cam, W, H, f, want_rgb=False, want_grid=True)
                else:
                    r.render_restir(None, cam, W, H, f, want_rgb=False, want_grid=False)
            r.synchronize()
            g = None
            r.enable_timing(False)
            for k, (ms, n) in r.timings().items():
                if n:
                    samples[name].setdefault(k, []).append(ms / n * 1e3)
    out = {name: {k: round(statistics.median(v), 2) for k, v in ks.items()} for name, ks in samples.items()}
    print(json.dumps({"config": args.config, "scene": cf["scene"], "N": args.N, "us_per_launch": out}))
    r.close()


if __name__ == "__main__":
    main()
