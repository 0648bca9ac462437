#!/usr/bin/env python3
"""C5's spatial pass with and without its visibility reuse (spatial_reuse_visibility_check): how much of the
unbiased pass's time the (k + 1) shadow rays per pixel take.  Per-kernel HIP-event times, median of rounds."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from romis_amd import _abi, restir, scene  # noqa: E402

cf = bench.CONFIGS["c5"]
W, H = cf.get("image") or cf["tile"]
r = restir.Renderer(0)
r.set_scene(scene.bench_scene(cf["scene"]))
cam = scene.camera_for(cf["scene"], W, H)
out = {}
for vis in (1, 0, 1, 0):
    f = _abi.default_features(initial_light_samples=cf["M"], num_samples_in_reservoir=1, spatial_resampling_passes=1,
                              spatial_reuse=1, temporal_reuse=0, unbiased_combination=1,
                              spatial_reuse_visibility_check=vis)
    r.render_restir(None, cam, W, H, f, want_rgb=False, want_grid=False)
    r.synchronize()
    r.reset_timings()
    r.enable_timing(True)
    for _ in range(3):
        r.render_restir(None, cam, W, H, f, want_rgb=False, want_grid=False)
    r.synchronize()
    r.enable_timing(False)
    kt = r.timings()
    out.setdefault(f"vis{vis}", []).append({k: round(ms * 1e3 / n, 1) for k, (ms, n) in kt.items() if n})
print(json.dumps(out))
