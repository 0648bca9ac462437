#!/usr/bin/env python3
"""Frame time of the C2 workload with no kernel timing, with the spatial kernel's launch events (bench.py's timed
region), and with every kernel timed; plus the per-kernel sum, so the inter-kernel overhead per frame shows."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from romis_amd import _abi, restir, scene  # noqa: E402

cf = bench.CONFIGS["c2"]
W, H = cf["tile"]
f = _abi.default_features(initial_light_samples=cf["M"], num_samples_in_reservoir=1, spatial_resampling_passes=1,
                          spatial_reuse=1, temporal_reuse=0)
r = restir.Renderer(0)
r.set_scene(scene.bench_scene(cf["scene"]))
cam = scene.camera_for(cf["scene"], W, H)
out = {}
for mode in ("none", "spatial", "all", "none", "spatial", "all"):
    for _ in range(5):
        r.render_restir(None, cam, W, H, f, want_rgb=False, want_grid=False)
    r.synchronize()
    r.reset_timings()
    if mode != "none":
        r.set_tuning("timing.mask", -1 if mode == "all" else 1 << _abi.K_SPATIAL)
    r.enable_timing(mode != "none")
    t0 = time.perf_counter()
    for _ in range(100):
        r.render_restir(None, cam, W, H, f, want_rgb=False, want_grid=False)
    r.synchronize()
    t1 = time.perf_counter()
    r.enable_timing(False)
    kt = r.timings()
    r.set_tuning("timing.mask", -1)
    ms = (t1 - t0) / 100 * 1e3
    rec = {"ms_per_frame": round(ms, 4)}
    if mode == "all":
        tot = sum(ms_k * 1e3 for ms_k, n in kt.values() if n) / 100
        rec["kernel_sum_us"] = round(tot, 1)
        rec["overhead_us"] = round(ms * 1e3 - tot, 1)
    out.setdefault(mode, []).append(rec)
print(json.dumps(out))
