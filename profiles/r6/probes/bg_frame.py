#!/usr/bin/env python3
"""Round 6 probe: the cost of background tiles -- C4's frame (cornell_1024, 3840 x 2160, M = 32, one biased pass) with
the TOML camera (13 % geometry), the framed camera (99.9 %) and a camera looking at empty space (0 %), per-kernel
median microseconds over rounds (HIP events on every launch)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime with the library)
from romis_amd import _abi, restir, scene  # noqa: E402

W, H = 3840, 2160
r = restir.Renderer(0)
r.set_scene(scene.bench_scene("cornell_1024"))
f = _abi.default_features(initial_light_samples=32, num_samples_in_reservoir=1, spatial_resampling_passes=1,
                          temporal_reuse=0)
cams = {"toml": scene.camera_for("cornell_1024", W, H), "framed": scene.camera_for("cornell_1024", W, H, "framed"),
        "empty": scene.make_camera(50.0, 3.0, (0.0, 50.0, 0.0), (0.0, 0.0, 0.0), W, H)}
out = {k: {} for k in cams}
for rnd in range(5):
    for name, cam in cams.items():
        r.render_restir(None, cam, W, H, f, want_rgb=False, want_grid=False)
        r.reset_timings()
        r.set_tuning("timing.mask", -1)
        r.enable_timing(True)
        for _ in range(5):
            r.render_restir(None, cam, W, H, f, want_rgb=False, want_grid=False)
        r.synchronize()
        r.enable_timing(False)
        for k, (ms, n) in r.timings().items():
            if n:
                out[name].setdefault(k, []).append(ms / n * 1e3)
print(json.dumps({name: {k: round(statistics.median(v), 2) for k, v in d.items()} for name, d in out.items()}))
r.close()
