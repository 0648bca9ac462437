#!/usr/bin/env python3
"""Per-rank frame times of the strong-scaling configs' 8-GPU tile layouts, measured on ONE MI355X.

For each config (c4, c5 with the TOML camera; c4f as the evenly filled control) and each 4 x 2 layout -- the even split
(restir_layout_even) and the cost-balanced one bench.py uses at N = 8 (distributed.balanced_layout: the cost grid from the
library's primary-ray kernel, restir_layout_balanced) -- every rank's halo-mode frame (restir_halo_begin_layout ..
restir_halo_end, the passes through restir_halo_pass in record-only mode: the same kernels, the receive buffers zeroed, no
transfer) is rendered and timed alone on the GPU.  implied_efficiency = mean / max of the per-rank times: the strong-
scaling efficiency the layout allows before the halo transfers (which the interior launch overlaps).  A least-squares fit
t = a * geometry_px + b * background_px + c over all ranks gives the background weight b / a the balancer uses.

    python scripts/balance_measure.py [--frames 5] > profiles/r6/balance.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--configs", default="c4,c5,c4f")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime with the library, as bench.py)
    import bench
    from romis_amd import _abi, distributed, restir, scene

    r = restir.Renderer(0)
    out = {"method": __doc__.strip().splitlines()[2:10], "frames": args.frames, "configs": {}}
    fits = []
    for name in args.configs.split(","):
        cf = bench.CONFIGS[name]
        W, H = cf["image"]
        sc = scene.bench_scene(cf["scene"])
        r.set_scene(sc)
        cam_fn = lambda w, h: scene.camera_for(cf["scene"], w, h, cf.get("camera"))  # noqa: E731
        cam = cam_fn(W, H)
        f = _abi.default_features(initial_light_samples=cf["M"], num_samples_in_reservoir=1, num_neighbours_to_sample=5,
                                  spatial_resample_radius=10, spatial_resampling_passes=cf["passes"], spatial_reuse=1,
                                  temporal_reuse=0, unbiased_combination=cf["unbiased"],
                                  spatial_reuse_visibility_check=cf["vis"])
        # the whole frame on one GPU (restir_render, background-tile flags on): the strong-scaling reference time
        r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
        for _ in range(2):
            r.render_restir(None, cam, W, H, f, want_rgb=False, want_grid=False)
        r.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.frames):
            r.render_restir(None, cam, W, H, f, want_rgb=False, want_grid=False)
        r.synchronize()
        t_one = (time.perf_counter() - t0) / args.frames
        cost = distributed.geometry_cost(r, cam_fn, W, H, background=1.0)   # 1 everywhere: hit mask below
        gw, gh = cost.shape[1], cost.shape[0]
        cost_hit = distributed.geometry_cost(r, cam_fn, W, H, background=0.0)
        gcost = distributed.geometry_cost(r, cam_fn, W, H)
        balanced, model_eff = restir.layout_balanced(W, H, 4, 2, gcost, distributed.LAYOUT_ALIGN)

        def ghost_times_of(L):   # every rank's ghost-zone tile frame, one after another (bench.py's time_tile)
            out_t = []
            for q in range(8):
                gt = restir.tile_plan(W, H, 4, 2, q, cf["passes"] * 10, layout=L)
                r.render_restir(None, cam, W, H, f, tile=gt, want_rgb=False, want_grid=False)
                r.synchronize()
                t0 = time.perf_counter()
                for _ in range(3):
                    r.render_restir(None, cam, W, H, f, tile=gt, want_rgb=False, want_grid=False)
                r.synchronize()
                out_t.append((time.perf_counter() - t0) / 3)
            return out_t

        # distributed.balanced_layout's measured refinement, its ranks emulated one after another on this GPU
        refined, cost_r, rounds = balanced, gcost, []
        for _ in range(3):
            tt = ghost_times_of(refined)
            rounds.append({"cuts": refined.cuts(), "rank_ms": [round(v * 1e3, 4) for v in tt],
                           "measured_efficiency": round(float(np.mean(tt) / max(tt)), 4)})
            cost_r = distributed.refine_cost(cost_r, refined, tt)
            refined, _ = restir.layout_balanced(W, H, 4, 2, cost_r, distributed.LAYOUT_ALIGN)
        rec = {"image": [W, H], "whole_frame_ms_1gpu": round(t_one * 1e3, 4), "geometry": round(float(cost_hit.mean()), 4),
               "refinement_rounds": rounds, "layouts": {}}
        for kind, L in (("even", restir.layout_even(W, H, 4, 2)), ("balanced", balanced), ("refined", refined)):
            geo_share = restir.layout_shares(L, cost_hit)
            px_share = restir.layout_shares(L, cost)
            times, kern, ghost_times = [], [], []
            r.halo_record(True)
            for rank in range(8):
                tile = restir.tile_plan(W, H, 4, 2, rank, 0, layout=L)

                def frame():
                    r.halo_begin(None, cam, W, H, f, (4, 2), rank, layout=L)
                    for _ in range(cf["passes"]):
                        r.halo_pass()
                    r.halo_end(tile, False, False)

                r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
                for _ in range(2):
                    frame()
                r.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.frames):
                    frame()
                r.synchronize()
                times.append((time.perf_counter() - t0) / args.frames)
                r.halo_log()   # drop the record-only log
                # the same rank's kernels one by one (HIP events on every launch), and its tile as a ghost-zone frame
                # (restir_render over the tile + passes * r: no exchange, the ring recomputed)
                r.reset_timings()
                r.set_tuning("timing.mask", -1)
                r.set_tuning("timing.every", 1)
                r.enable_timing(True)
                for _ in range(args.frames):
                    frame()
                r.synchronize()
                r.enable_timing(False)
                kern.append({k: round(v[0] / args.frames, 4) for k, v in r.timings().items() if v[1]})
                r.halo_log()
                gt = restir.tile_plan(W, H, 4, 2, rank, cf["passes"] * 10, layout=L)
                for _ in range(2):
                    r.render_restir(None, cam, W, H, f, tile=gt, want_rgb=False, want_grid=False)
                r.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.frames):
                    r.render_restir(None, cam, W, H, f, tile=gt, want_rgb=False, want_grid=False)
                r.synchronize()
                ghost_times.append((time.perf_counter() - t0) / args.frames)
                geo_px = geo_share[rank] * cost_hit.sum() * (W * H) / (gw * gh)
                all_px = tile.width * tile.height
                fits.append((geo_px, all_px - geo_px, times[-1]))
            r.halo_record(False)
            t = np.array(times)
            tg = np.array(ghost_times)
            rec["layouts"][kind] = {
                "cuts": L.cuts(), "rank_ms": [round(v * 1e3, 4) for v in t],
                "geometry_share_per_rank": [round(float(v), 4) for v in geo_share],
                "pixel_share_per_rank": [round(float(v), 4) for v in px_share],
                "implied_efficiency": round(float(t.mean() / t.max()), 4),
                "speedup_vs_1gpu_whole_frame": round(float(t_one / t.max()), 3),
                "strong_scaling_efficiency_vs_1gpu": round(float(t_one / t.max() / 8), 4),
                "kernel_ms_per_rank": kern,
                "ghost_rank_ms": [round(v * 1e3, 4) for v in tg],
                "ghost_implied_efficiency": round(float(tg.mean() / tg.max()), 4),
                "ghost_strong_scaling_efficiency_vs_1gpu": round(float(t_one / tg.max() / 8), 4)}
            if kind == "balanced":
                rec["layouts"][kind]["model_efficiency"] = round(model_eff, 4)
        out["configs"][name] = rec
        print(json.dumps({name: {k: v["implied_efficiency"] for k, v in rec["layouts"].items()}}), file=sys.stderr,
              flush=True)
    fits = fits or [(1.0, 0.0, 1.0)]
    A = np.array([[g, b, 1.0] for g, b, _ in fits])
    y = np.array([t for _, _, t in fits])
    coef, *_ = np.linalg.lstsq(A, y, rcond=None)
    out["fit"] = {"ms_per_mpx_geometry": round(coef[0] * 1e9, 4), "ms_per_mpx_background": round(coef[1] * 1e9, 4),
                  "ms_fixed": round(coef[2] * 1e3, 4), "background_weight": round(float(coef[1] / coef[0]), 4),
                  "used_by_balancer": distributed.BACKGROUND_WEIGHT}
    r.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
