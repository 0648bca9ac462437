"""Probe: C2 frames alternated over n contexts on one GPU (frames in flight), throughput only."""
import sys, time, json
sys.path.insert(0, '.')
import torch
from romis_amd import _abi, restir, scene
sc = scene.bench_scene("nightclub_128pt")
cam = scene.camera_for("nightclub_128pt", 1920, 1080)
f = _abi.default_features(initial_light_samples=32, num_samples_in_reservoir=1, num_neighbours_to_sample=5,
                          spatial_resample_radius=10, spatial_resampling_passes=1, spatial_reuse=1, temporal_reuse=0)
out = {}
for n in (1, 2, 3):
    rs = []
    for i in range(n):
        r = restir.Renderer(0); r.set_scene(sc); r.set_seed(_abi.RESTIR_DEFAULT_SEED, i); rs.append(r)
    for k in range(6):
        rs[k % n].render_restir(None, cam, 1920, 1080, f, want_rgb=False, want_grid=False)
    for r in rs: r.synchronize()
    best = 1e9
    for rep in range(3):
        t0 = time.perf_counter()
        K = 60
        for k in range(K):
            rs[k % n].render_restir(None, cam, 1920, 1080, f, want_rgb=False, want_grid=False)
        for r in rs: r.synchronize()
        best = min(best, (time.perf_counter() - t0) / K * 1e3)
    out[n] = round(best, 4)
    for r in rs: r.close()
print(json.dumps(out))
