#!/usr/bin/env python3
"""Time R-MIS / R-OMIS renders (renderRMIS / renderROMIS, render.cpp:64-265) on the GPU against the oracle's CPU
restatement (OpenMP) on the same host.  One JSON object per line; not the headline bench (bench.py).

    python scripts/mis_bench.py [--width 1920 --height 1080] [--cpu-width 320 --cpu-height 180] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from romis_amd import _abi, restir, scene  # noqa: E402

CASES = {
    "rmis_equal": dict(ray_trace_mode=_abi.MODE_RMIS),
    "rmis_balance": dict(ray_trace_mode=_abi.MODE_RMIS, mis_weight_rmis=_abi.MIS_BALANCE),
    "romis_direct": dict(ray_trace_mode=_abi.MODE_ROMIS),
    "romis_progressive_n6": dict(ray_trace_mode=_abi.MODE_ROMIS, use_progressive_romis=1, num_samples_in_reservoir=6),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="nightclub_128pt")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--cpu-width", type=int, default=320)
    ap.add_argument("--cpu-height", type=int, default=180)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    sc = scene.bench_scene(args.scene)
    r = restir.Renderer(0)
    r.set_scene(sc)
    osc = None
    for name, kw in CASES.items():
        f = _abi.default_features(**kw)   # reference defaults: N = 2 (unless set), k = 5, r = 10, 5 iterations
        cam = scene.camera_for(args.scene, args.width, args.height)
        r.render_mis(cam, args.width, args.height, f)   # warm-up (allocation, code load)
        r.synchronize()
        t = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            r.render_mis(cam, args.width, args.height, f)
            t.append(time.perf_counter() - t0)
        gpu_s = min(t)
        rec = {"case": name, "scene": args.scene, "image": [args.width, args.height], "N": f.num_samples_in_reservoir,
               "k": f.num_neighbours_to_sample, "iterations": f.max_iterations_mis, "gpu_ms": round(gpu_s * 1e3, 3),
               "gpu_mpx_per_s": round(args.width * args.height / gpu_s / 1e6, 2)}
        if not args.no_cpu:
            from oracle import pyoracle
            osc = osc or pyoracle.OracleScene(sc)
            cw, ch = args.cpu_width, args.cpu_height
            ccam = scene.camera_for(args.scene, cw, ch)
            threads = min(16, os.cpu_count() or 1)
            t0 = time.perf_counter()
            pyoracle.render_mis(osc, ccam, f, cw, ch, threads=threads)
            cpu_s = time.perf_counter() - t0
            rec.update({"cpu_sample": [cw, ch], "cpu_threads": threads, "cpu_s": round(cpu_s, 3),
                        "cpu_mpx_per_s": round(cw * ch / cpu_s / 1e6, 4),
                        "gpu_over_cpu": round((args.width * args.height / gpu_s) / (cw * ch / cpu_s), 1)})
        print(json.dumps(rec), flush=True)
    r.close()


if __name__ == "__main__":
    main()
