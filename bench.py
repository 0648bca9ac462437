#!/usr/bin/env python3
"""Headline benchmark: Mpixel-reservoirs/s of the ReSTIR frame (BASELINE.json metric) on 1..8 MI355X.

One step = one renderReSTIR frame (render.cpp:28-62) of configs[1] of BASELINE.json: cornell-nightclub
geometry, 128 point lights, 1920x1080 per GPU, M = 32 initial candidates, N = 1 reservoir, spatial reuse
k = 5, r = 10, one pass (biased), no temporal reuse, shading + tone mapping on -- primary rays, initial RIS,
spatial pass and final shading (shadow rays) all run on the GPU inside the timed region; inputs (scene, BVH)
are resident in HBM before it starts and no host transfer happens inside it.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): weak scaling over screen
tiles -- each rank owns a 1920x1080 tile of a (tx*1920) x (ty*1080) image (2x1, 2x2, 4x2) and computes its
tile plus a ghost zone of passes*r pixels, so no data-path collective is needed (DESIGN.md "Multi-GPU");
the barrier / max-over-ranks timing uses torch.distributed (RCCL).

Other BASELINE.json configs (--config c1|c3|c4|c5; c2 is the default): c1 CornellBox 512x512 RIS only, c3 two
spatial passes + temporal reuse threading each frame's grid into the next (1 GPU), c4 4K / 1024 lights and
c5 8K / 4096 lights / M=64 / unbiased + visibility reuse (strong scaling: the image is fixed and split).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md "Chip-level parameters")
FP32_VECTOR_PEAK_TFS = 157.3   # MI355X FP32 vector peak (MI355X_MICROARCH.md "Matrix cores", F32 row)
RIS_FLOP_PER_CANDIDATE = 160
TILE_W, TILE_H = 1920, 1080


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)   # ~0.1 s timed at C2: past the first frames after the idle sync (slower clocks; 50 steps read 2 % low, profiles/r3/r3q)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "c4f", "c5f"],
                    help="BASELINE.json config (c2 = configs[1], the headline)")
    ap.add_argument("--scene", default=None, help="override the config's scene")
    ap.add_argument("--mode", default="auto", choices=["auto", "ghost", "halo"],
                    help="multi-GPU tiles: recompute a ghost zone (no communication) or exchange reservoir halos "
                         "over RCCL before each spatial pass; auto = halo when temporal reuse is on")
    ap.add_argument("--M", type=int, default=None, help="override the config's M")
    ap.add_argument("--N", type=int, default=1)
    ap.add_argument("--k", type=int, default=5)
    ap.add_argument("--r", type=int, default=10)
    ap.add_argument("--passes", type=int, default=None, help="override the config's spatial passes")
    ap.add_argument("--tile-width", type=int, default=None)
    ap.add_argument("--tile-height", type=int, default=None)
    ap.add_argument("--cpu-baseline", dest="cpu_baseline", action="store_true", default=True)
    ap.add_argument("--no-cpu-baseline", dest="cpu_baseline", action="store_false")
    ap.add_argument("--no-cpu-stages", dest="cpu_stages", action="store_false", default=True,
                    help="skip cpu_baseline.stages (per-stage oracle rates for C1 and C2)")
    ap.add_argument("--time-kernels", default="spatial", choices=["all", "spatial"],
                    help="kernels bracketed by HIP events in the timed region")
    ap.add_argument("--cpu-rows", type=int, default=None, help="rows of the workload the CPU baseline renders "
                    "(default: ~1 Mpx worth)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group of the multi-rank bench (nccl = RCCL, the real run; gloo = a rehearsal with "
                         "several ranks sharing one GPU)")
    ap.add_argument("--halo-check", default="auto", choices=["auto", "on", "off"],
                    help="N > 1: before timing, render one frame of this rank's tile through the RCCL reservoir halo "
                         "(HaloFrames) and through the ghost zone, require them bit-identical (exit 3 otherwise) and "
                         "time the halo-mode frame and its exchange (auto = on when the frame has spatial passes)")
    ap.add_argument("--halo-transport", default="auto", choices=["auto", "native", "torch"],
                    help="halo transport: the library's own RCCL communicator (native), torch.distributed p2p (torch); "
                         "auto = native under nccl, torch under gloo")
    ap.add_argument("--layout", default="auto", choices=["auto", "even", "balanced"],
                    help="N > 1 tile layout: even cuts, or cost-balanced cuts from a low-resolution primary pass "
                         "(restir_layout_balanced, broadcast from rank 0); auto = balanced for the strong-scaling "
                         "configs (c4 / c5: one image split over the ranks), even for weak-scaling c2 / c3")
    ap.add_argument("--layout-rounds", type=int, default=3,
                    help="balanced layout: rounds of refinement from the ranks' measured tile frame times")
    ap.add_argument("--prewarm-gemm-ms", type=float, default=500.0,
                    help="GPU clock pre-warm before the warm-up frames (not frames, not timed): fp32 GEMMs through torch "
                         "for this long.  An idle box's first ~40 frames run up to 10 %% slower (profiles/r4/gap); 500 ms "
                         "of compute-bound work takes the driver's 20-frame C2 run 0.467 -> 0.451 ms (profiles/r4/r4c); "
                         "streaming reads (restir_measure_read_bandwidth) do not raise the clocks")
    ap.add_argument("--timing-every", type=int, default=4,
                    help="HIP events on every n-th spatial launch of the timed region (the event-carrying dispatch "
                         "costs ~9 us of stream gaps, profiles/r4/gap); the roofline's average launch time is over "
                         "those launches")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="restir_set_tuning knobs for A/B runs (launch shapes and timing only; results are identical)")
    ap.add_argument("--traffic-csv", default=None,
                    help="rocprofv3 --pmc CSV (FETCH_SIZE / WRITE_SIZE) of this command for roofline.traffic")
    return ap.parse_args()


def dist_setup(n_gpus, backend="nccl"):
    """(rank, world, device, torch).  torch is imported before libromis_amd so both share one HIP runtime.
    backend "gloo" (a rehearsal of the multi-rank path on a box with fewer GPUs than ranks): the ranks share the
    visible GPUs round-robin and the barrier / max-over-ranks run on the CPU."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            local = local % max(1, torch.cuda.device_count())
            dist.init_process_group("gloo")
    if world != n_gpus and rank == 0:
        print(f"warning: --gpus {n_gpus} but WORLD_SIZE {world}", file=sys.stderr)
    return rank, world, local, torch


def barrier_sync(torch, world, renderer):
    renderer.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
        torch.cuda.synchronize()


def max_over_ranks(torch, world, value, local):
    if world == 1:
        return value
    on_gpu = torch.distributed.get_backend() == "nccl"
    t = torch.tensor([value], dtype=torch.float64, device=torch.device("cuda", local) if on_gpu else "cpu")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def gemm_prewarm(torch, local, ms):
    """fp32 4096^3 GEMMs on this rank's GPU for `ms` milliseconds (not a frame, not timed): compute-bound work that
    brings an idle box's shader clocks up before the warm-up frames."""
    dev = torch.device("cuda", local)
    a = torch.randn(4096, 4096, device=dev)
    b = torch.randn(4096, 4096, device=dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(4):
            a = torch.mm(a, b) * (1.0 / 64.0)   # 1/sqrt(4096): the entries keep their magnitude (no decay to zeros)
        torch.cuda.synchronize(dev)
    del a, b


def camera_record(framing):
    """The JSON record of a config's camera framing (config.camera; JSON types, so records compare after a round trip)."""
    from romis_amd import scene
    assert framing == "framed", framing
    return json.loads(json.dumps(dict(scene.CORNELL_FRAMED, kind="framed (scene.CORNELL_FRAMED)")))


def committed_traffic(cfg):
    """The spatial kernel's HBM bytes per launch from profiles/traffic.json (written by
    scripts/collect_profiles.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench), used
    only when it was measured on these exact kernel sources (build.source_hash) and this workload."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "traffic.json")
    try:
        from romis_amd import build
        with open(path) as fh:
            rec = json.load(fh)
        keys = ("scene", "tile", "M", "N", "k", "r", "passes", "camera")
        here = build.source_hash()
        # the top-level record (scripts/collect_profiles.py: the headline's --pmc passes), then the per-config
        # entries of the attribution study (scripts/traffic_json.py), each only at these exact kernel sources;
        # the default XCD tile order is "chunks"
        groups = []
        if rec.get("source_hash") == here:
            groups.append((rec.get("entries") or [rec], rec.get("profile")))
        att = rec.get("attribution") or {}
        if att.get("source_hash") == here:
            groups.append((att.get("entries") or [], att.get("profile")))
        for entries, profile in groups:
            for e in entries:
                rc = e.get("config") or {}
                if e.get("variant", e.get("xcd_order", "chunks")) == "chunks" and all(rc.get(k) == cfg.get(k) for k in keys):
                    return e["traffic_bytes_per_launch"], profile
    except (OSError, ValueError, KeyError):
        pass
    return None, None


def committed_valu(cfg_name, n_sub, kernel):
    """VALU wave-instructions per candidate of the RIS kernel from profiles/valu.json (scripts/valu_json.py: an SQ
    counter pass over this bench), only when it was measured on these exact sources and this config."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "valu.json")
    try:
        from romis_amd import build
        with open(path) as fh:
            rec = json.load(fh)
        if rec.get("source_hash") != build.source_hash() or rec.get("config") != cfg_name or rec.get("N") != n_sub:
            return None
        for k, e in rec.get("kernels", {}).items():
            if k.startswith(kernel) and "valu_instr_per_candidate" in e:
                return {"valu_instr_per_candidate": e["valu_instr_per_candidate"], "sq_insts_valu_per_launch": e["sq_insts_valu"],
                        "kernel_variant": k, "source": rec.get("profile")}
    except (OSError, ValueError, KeyError):
        pass
    return None


def pmc_traffic(path, kernel_prefix="k_spatial"):
    """Per-launch HBM bytes of the spatial kernel from a rocprofv3 --pmc CSV (counter_collection.csv).
    FETCH_SIZE / WRITE_SIZE are KB; FETCH_SIZE is doubled for wide coalesced streams on gfx950
    (MI355X_MICROARCH.md "HBM")."""
    import csv
    fetch, write = {}, {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if not row.get("Kernel_Name", "").startswith(kernel_prefix):
                continue
            d = row.get("Dispatch_Id")
            name, val = row.get("Counter_Name"), float(row.get("Counter_Value", 0))
            if name == "FETCH_SIZE":
                fetch[d] = val
            elif name == "WRITE_SIZE":
                write[d] = val
    if not fetch and not write:
        return None
    f = sum(fetch.values()) / max(1, len(fetch)) * 1024.0 * 2.0
    w = sum(write.values()) / max(1, len(write)) * 1024.0
    return f + w


def cpu_baseline(sc, cam_fn, features, rows, W, H):
    """The oracle (C restatement, OpenMP over rows) on a band of `rows` rows of the same workload."""
    from oracle import pyoracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    osc = pyoracle.OracleScene(sc)
    cam = cam_fn(W, H)
    g = features.spatial_resampling_passes * features.spatial_resample_radius
    y0 = (H - rows) // 2

    def band(n):   # owned rows [y0, y0+n) plus the ghost rows the spatial passes read
        return pyoracle.Rect(0, y0 - g, W, n + 2 * g), pyoracle.Rect(0, y0, W, n)

    def timed(reference_rng, n):
        pyoracle.set_rng_mode(reference_rng)
        try:
            v, rc = band(2)
            pyoracle.render_frame(osc, cam, features, W, H, view=v, rect=rc, threads=threads)   # warm
            v, rc = band(n)
            t0 = time.perf_counter()
            pyoracle.render_frame(osc, cam, features, W, H, view=v, rect=rc, threads=threads)
            return time.perf_counter() - t0
        finally:
            pyoracle.set_rng_mode(False)

    px = W * rows * features.num_samples_in_reservoir
    dt = timed(False, rows)
    # the reference's generators serialise on glibc's rand() lock (~100x slower on 16 threads): an eighth of the
    # rows keeps the leg near 5 s
    rows_ref = max(32, rows // 8)
    dt_ref = timed(True, rows_ref)
    px_ref = W * rows_ref * features.num_samples_in_reservoir
    return {"value": round(px / dt / 1e6, 6), "unit": "Mpixel-reservoirs/s", "cores": threads, "kind": "port",
            "sample": f"oracle/restir_oracle.c frame (primary+RIS+spatial+final) owning rows {y0}..{y0 + rows - 1} "
                      f"of the {W}x{H} workload ({W * rows} px counted, +{2 * g} ghost rows computed, {dt:.2f} s, "
                      f"OpenMP {threads} threads, keyed counter RNG)",
            # the same frame with the reference's own generators (per-pixel std::random_device + std::mt19937,
            # process-wide rand(); light.cpp:49-51, reservoir.cpp:24, render_utils.cpp:89-91) -- how the
            # reference itself runs; not reproducible, so timed only
            "reference_rng": {"value": round(px_ref / dt_ref / 1e6, 6), "unit": "Mpixel-reservoirs/s", "cores": threads,
                              "seconds": round(dt_ref, 3), "rows": rows_ref, "ghost_rows_computed": 2 * g,
                              "rng": "per-pixel std::random_device + std::mt19937, global rand() (oracle/ref_rng.cpp)"}}


def cpu_stage_baseline(sc, cam, features, W, H, rows, reference_rng):
    """Per-stage rates of the oracle (OpenMP over rows, the thread count cpu_baseline set) on a band of `rows` owned
    rows of a W x H frame: primary rays and RIS / temporal over the band's view (owned rows + the passes * r ghost
    rows the spatial passes read), the spatial passes and final shading over the owned rows.  Mpixel-reservoirs/s
    per stage (pixels the stage computes x N / seconds) -- BASELINE.md's per-stage CPU baseline (render_utils.cpp:
    36-52, 87-140, 142-177; render.cpp:45-57)."""
    from oracle import pyoracle
    from romis_amd import _abi
    f = features
    N = f.num_samples_in_reservoir
    passes = f.spatial_resampling_passes if f.spatial_reuse else 0
    g = passes * f.spatial_resample_radius
    y0 = (H - rows) // 2
    vy0, vy1 = max(0, y0 - g), min(H, y0 + rows + g)
    view, rect = pyoracle.Rect(0, vy0, W, vy1 - vy0), pyoracle.Rect(0, y0, W, rows)
    osc = pyoracle.OracleScene(sc)
    cf = pyoracle.camera_frame(cam)
    o = np.array(list(cf.origin), np.float32)
    lib = pyoracle.lib()
    nv = view.w * view.h
    n_t, p_mat = np.zeros((nv, 4), np.float32), np.zeros((nv, 4), np.float32)
    out = {}

    def rate(name, px, fn):
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        out[name] = {"value": round(px * N / dt / 1e6, 6), "pixels": int(px), "seconds": round(dt, 4)}

    pyoracle.set_rng_mode(reference_rng)
    try:
        rate("primary", nv, lambda: lib.or_primary(osc.handle, C.byref(cf), W, H, view, view, pyoracle.fp(n_t),
                                                   pyoracle.fp(p_mat)))
        res = {}

        def ris(tag, key):
            a, b, _ = pyoracle.empty_reservoirs(N, nv)
            lib.or_ris(osc.handle, C.byref(f), key, pyoracle.fp(o), W, H, view, view, pyoracle.fp(n_t),
                       pyoracle.fp(p_mat), pyoracle.fp(a), pyoracle.fp(b), None)
            res[tag] = (a, b)
        seed = _abi.RESTIR_DEFAULT_SEED
        rate("ris", nv, lambda: ris("cur", restir_key(seed, 1, _abi.RESTIR_STAGE_RIS, 0)))
        ris("prev", restir_key(seed, 0, _abi.RESTIR_STAGE_RIS, 0))   # a predecessor grid for the temporal stage

        def temporal():
            a, b, _ = pyoracle.empty_reservoirs(N, nv)
            lib.or_temporal(osc.handle, C.byref(f), restir_key(seed, 1, _abi.RESTIR_STAGE_TEMPORAL, 0), pyoracle.fp(o), W,
                            H, view, view, pyoracle.fp(n_t), pyoracle.fp(p_mat), pyoracle.fp(res["cur"][0]),
                            pyoracle.fp(res["cur"][1]), pyoracle.fp(res["prev"][0]), pyoracle.fp(res["prev"][1]),
                            pyoracle.fp(a), pyoracle.fp(b), None)
        rate("temporal", nv, temporal)
        cur = res["cur"]
        if passes:
            px = 0
            t0 = time.perf_counter()
            for p in range(passes):
                gp = (passes - 1 - p) * f.spatial_resample_radius
                ry0, ry1 = max(0, y0 - gp), min(H, y0 + rows + gp)
                pr = pyoracle.Rect(0, ry0, W, ry1 - ry0)
                a, b, _ = pyoracle.empty_reservoirs(N, nv)
                a[:], b[:] = cur[0], cur[1]
                lib.or_spatial_pass(osc.handle, C.byref(f), restir_key(seed, 1, _abi.RESTIR_STAGE_SPATIAL, p),
                                    pyoracle.fp(o), W, H, view, pr, pyoracle.fp(n_t), pyoracle.fp(p_mat),
                                    pyoracle.fp(cur[0]), pyoracle.fp(cur[1]), pyoracle.fp(a), pyoracle.fp(b), None)
                cur = (a, b)
                px += pr.w * pr.h
            dt = time.perf_counter() - t0
            out["spatial"] = {"value": round(px * N / dt / 1e6, 6), "pixels": int(px), "seconds": round(dt, 4),
                              "passes": passes}
        rgb = np.zeros((rows, W, 3), np.float32)
        rate("final", rect.w * rect.h, lambda: lib.or_final(osc.handle, C.byref(f), pyoracle.fp(o), W, H, view, rect,
                                                            pyoracle.fp(n_t), pyoracle.fp(p_mat), pyoracle.fp(cur[0]),
                                                            pyoracle.fp(cur[1]), pyoracle.fp(rgb)))
    finally:
        pyoracle.set_rng_mode(False)
    out["rows"] = {"owned": rows, "view": view.h, "of": [W, H]}
    return out


def restir_key(seed, frame, stage, pass_):
    from romis_amd import restir
    return restir.rng_key(seed, frame, stage, pass_)


def cpu_stages(cf_name, sc_fn, cam_fn, features_fn, threads):
    """cpu_baseline.stages: per-stage oracle rates for C1 and C2 (BASELINE.md's per-stage CPU baseline), keyed RNG
    and the reference's own generators, on bounded bands (the reference generators serialise on rand()'s lock)."""
    out = {"cores": threads, "unit": "Mpixel-reservoirs/s"}
    for name in ("c1", "c2"):
        cf = CONFIGS[name]
        W, H = cf.get("image") or cf["tile"]
        sc = sc_fn(cf["scene"])
        cam = cam_fn(cf["scene"], W, H)
        f = features_fn(cf)
        rows_keyed = min(H, max(8, 1036800 // W))
        out[name] = {"keyed": cpu_stage_baseline(sc, cam, f, W, H, rows_keyed, False),
                     "reference_rng": cpu_stage_baseline(sc, cam, f, W, H, max(16, rows_keyed // 16), True)}
    return out


# BASELINE.json configs.  "weak": each rank owns a tile x tile_h tile of a (tx*tile) x (ty*tile_h) image;
# "strong": the image is fixed and split over the ranks.  c2 (configs[1]) is the headline and the default.
CONFIGS = {
    "c1": dict(scene="cornell_parallelogram", image=(512, 512), M=32, passes=0, temporal=0, unbiased=0, vis=0,
               workload="C1: CornellBox-Mirror 512x512, 1 parallelogram light, M=32, RIS only (no spatial/temporal)"),
    "c2": dict(scene="nightclub_128pt", tile=(TILE_W, TILE_H), M=32, passes=1, temporal=0, unbiased=0, vis=0,
               workload="C2: cornell-nightclub 1080p per GPU, 128 point lights, M=32, N=1, spatial k=5 r=10 x1 "
                        "biased, no temporal, frame = primary+RIS+spatial+final"),
    "c3": dict(scene="nightclub_128pt", tile=(TILE_W, TILE_H), M=32, passes=2, temporal=1, unbiased=0, vis=0,
               workload="C3: cornell-nightclub 1080p, 128 point lights, M=32, spatial k=5 x2 + temporal reuse, "
                        "every frame reuses the previous one (static camera)"),
    "c4": dict(scene="cornell_1024", image=(3840, 2160), M=32, passes=1, temporal=0, unbiased=0, vis=0, geometry=0.132,
               workload="C4: 4K Cornell box, 32x32 = 1024 ceiling parallelogram lights, M=32, k=5 x1 biased"),
    "c5": dict(scene="cornell_4096", image=(7680, 4320), M=64, passes=1, temporal=0, unbiased=1, vis=1, geometry=0.132,
               workload="C5: 8K Cornell box, 64x64 = 4096 ceiling parallelogram lights, M=64, k=5 x1 unbiased "
                        "+ spatial visibility reuse"),
    # C4 / C5 with the camera looking into the box (scene.CORNELL_FRAMED): the TOML camera's frame is 87 % background,
    # whose tiles the passes write without reading (MissTiles), so c4 / c5 do not measure the 4K / 8K pass on geometry
    # -- these do (99.9 % of the pixels hit the box).  Same scenes, lights, M, k, passes and combine.
    "c4f": dict(scene="cornell_1024", image=(3840, 2160), M=32, passes=1, temporal=0, unbiased=0, vis=0, camera="framed",
                workload="C4 framed: 4K Cornell box, 32x32 = 1024 ceiling parallelogram lights, M=32, k=5 x1 biased, "
                         "camera looking into the box (99.9 % geometry)"),
    "c5f": dict(scene="cornell_4096", image=(7680, 4320), M=64, passes=1, temporal=0, unbiased=1, vis=1, camera="framed",
                workload="C5 framed: 8K Cornell box, 64x64 = 4096 ceiling parallelogram lights, M=64, k=5 x1 unbiased "
                         "+ spatial visibility reuse, camera looking into the box (99.9 % geometry)"),
}


DATA = {"nightclub_128pt": "prebuilt cornell-nightclub geometry, 128 point lights",
        "cornell_parallelogram": "prebuilt CornellBox-Mirror-Rotated geometry, 1 parallelogram light",
        "cornell_1024": "prebuilt Cornell box geometry, 32x32 regularLightGrid ceiling lights",
        "cornell_4096": "prebuilt Cornell box geometry, 64x64 regularLightGrid ceiling lights"}


def spatial_px_per_launch(tile, passes, r):
    """Average pixels a spatial launch computes: pass p covers the owned rect grown by (P-1-p)*r, clipped."""
    tot = 0
    for p in range(passes):
        g = (passes - 1 - p) * r
        x0, y0 = max(0, tile.x0 - g), max(0, tile.y0 - g)
        x1 = min(tile.global_width, tile.x0 + tile.width + g)
        y1 = min(tile.global_height, tile.y0 + tile.height + g)
        tot += (x1 - x0) * (y1 - y0)
    return tot / max(1, passes)


def select_halo(torch, world, local, backend, transport, make, check):
    """The halo transport the run times, chosen once and verified: make(transport) builds the HaloFrames
    (it may raise RestirError: no RCCL, a failed attach), check(hf) counts the words where its tile differs from the
    ghost-zone tile, summed over ranks (every rank sees the same count).  A construction failure on any rank moves
    every rank to the torch transport together; a mismatch over the native transport (first run with two or more GPUs
    on the driver's node) is recorded as native_check and the protocol re-checked over the torch transport, which
    carries the same pack / unpack kernels.  Returns (hf, rec, mismatches): hf is the instance the caller must time --
    rec["transport"] is always hf.transport -- and mismatches != 0 means even the fallback failed (exit 3)."""
    from romis_amd import _abi
    rec = {"transport": transport}
    hf = None
    try:
        hf = make(transport)
    except _abi.RestirError as e:
        rec["native_error"] = str(e)[:200]
    dev = torch.device("cuda", local) if backend == "nccl" else "cpu"
    failed = torch.tensor([1 if hf is None else 0], dtype=torch.int32, device=dev)
    if world > 1:
        torch.distributed.all_reduce(failed, op=torch.distributed.ReduceOp.MAX)
    if int(failed.item()) and transport != "torch":   # every rank falls back together
        transport = "torch"
        hf = make(transport)
    bad = check(hf)
    if bad and transport == "native":
        rec["native_check"] = f"{bad} mismatching values"
        transport = "torch"
        hf = make(transport)
        bad = check(hf)
    rec["transport"] = hf.transport
    return hf, rec, bad


def halo_frames(torch, r, rank, world, local, f, cam, GW, GH, tx, ty, passes, args, transport, check_on, fatal=True,
                layout=None):
    """N > 1 with spatial passes: this rank's tile rendered through the reservoir halo exchange (HaloFrames: interior
    launched while the border reservoirs move, border strips after) must equal, bit for bit, the same tile rendered
    with a ghost zone (restir_render on tile + passes * r) -- exits 3 on any mismatch (check_on).  Then the halo-mode
    frame and the exchange alone are timed.  Temporal reuse is off in the check (one frame from no predecessor).
    Returns (hf, rec): the verified HaloFrames -- the halo-mode main loop (c4 / c5, --mode halo) times this instance,
    so the run never times a transport other than the one it checked -- and the JSON record.  fatal = False (the halo
    is only checked, as with c2's ghost-zone frames at N > 1): a mismatch, or a render error that every rank sees as one,
    is recorded and the run goes on (returns hf None) -- the timed frames do not use the halo."""
    from romis_amd import _abi, distributed, restir
    fc = _abi.Features.from_buffer_copy(f)
    fc.temporal_reuse = 0
    ghost = {}

    def make(tr):
        return distributed.HaloFrames(r, GW, GH, (tx, ty), rank, f, transport=tr, layout=layout)

    def check(hf):
        if not check_on:
            return 0
        if "rgb" not in ghost:
            r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
            ghost_tile = restir.tile_plan(GW, GH, tx, ty, rank, passes * args.r, layout=layout)
            ghost["rgb"], _ = r.render_restir(None, cam, GW, GH, fc, tile=ghost_tile, want_grid=False)
        r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
        f0 = hf.f
        hf.f = fc
        try:
            rgb, _ = hf.render(None, cam, want_rgb=True, want_grid=False)
        except _abi.RestirError as e:   # this rank's frame failed: counted as mismatching, so every rank sees it
            rec_err["render_error"] = str(e)[:200]
            rgb = None
        finally:
            hf.f = f0
        if rgb is None:
            import numpy as np
            rgb = np.full_like(ghost["rgb"], np.nan)
        return distributed.tile_mismatches(rgb, ghost["rgb"])   # summed over ranks: every rank decides alike

    rec_err = {}
    hf, rec, bad = select_halo(torch, world, local, args.dist_backend, transport, make, check)
    rec.update(rec_err)
    rec["check"] = ("bit-exact" if bad == 0 else f"{bad} mismatching values") if check_on else "off"
    if bad:
        if not fatal:   # the run's timed frames are the ghost-zone ones: record the failed check and go on
            rec["timed"] = False
            return None, rec
        if rank == 0:
            print(json.dumps({"error": "halo tile differs from the ghost-zone tile", "halo": rec}), flush=True)
        torch.distributed.barrier()
        sys.exit(3)
    # halo-mode frames, timed like the main loop (max over ranks)
    k = max(5, min(args.steps, 20))
    for _ in range(2):
        hf.render(None, cam, want_rgb=False, want_grid=False)
    barrier_sync(torch, world, r)
    t0 = time.perf_counter()
    for _ in range(k):
        hf.render(None, cam, want_rgb=False, want_grid=False)
    barrier_sync(torch, world, r)
    dt = max_over_ranks(torch, world, time.perf_counter() - t0, local) / k
    bytes_pp = max_over_ranks(torch, world, float(sum(s.bytes for s in hf.send)), local)
    rec.update({"frame_ms": round(dt * 1e3, 4), "value": round(GW * GH * f.num_samples_in_reservoir / dt / 1e6, 3),
                "bytes_per_pass": int(bytes_pp), "passes": passes,
                "exchange_us_per_pass": round(distributed.exchange_probe(hf.send, hf.recv), 2),
                "note": "value/frame_ms: the same frames with the reservoir halo exchanged over the process group "
                        "before each spatial pass instead of a ghost zone; exchange_us_per_pass: the pass's "
                        "segments moved alone (torch p2p, max over ranks), which the pass overlaps with its interior"})
    return hf, rec


def main():
    args = parse()
    rank, world, local, torch = dist_setup(args.gpus, args.dist_backend)
    from romis_amd import _abi, restir, scene

    cf = dict(CONFIGS[args.config])
    for key in ("scene", "M", "passes"):
        if getattr(args, key) is not None:
            cf[key] = getattr(args, key)
    tx, ty = restir.tile_grid(world)
    if "tile" in cf:
        tw, th = args.tile_width or cf["tile"][0], args.tile_height or cf["tile"][1]
        GW, GH, scaling = tx * tw, ty * th, "weak"
    else:
        GW, GH, scaling = cf["image"][0], cf["image"][1], "strong"
    # multi-GPU temporal reuse needs the predecessor's reservoirs around each tile: halo-exchange frames
    # strong-scaling configs (c4 / c5: one image split over the ranks) and temporal ones exchange the reservoir
    # halo before each spatial pass (the library's RCCL transport, overlapped with the pass's interior); weak-
    # scaling c2 recomputes a ghost zone instead (no data-path communication)
    halo = world > 1 and (args.mode == "halo" or (args.mode == "auto" and (cf["temporal"] or scaling == "strong")))
    sc = scene.bench_scene(cf["scene"])
    cam = scene.camera_for(cf["scene"], GW, GH, cf.get("camera"))
    passes = cf["passes"]
    f = _abi.default_features(initial_light_samples=cf["M"], num_samples_in_reservoir=args.N,
                              num_neighbours_to_sample=args.k, spatial_resample_radius=args.r,
                              spatial_resampling_passes=passes, spatial_reuse=1 if passes > 0 else 0,
                              temporal_reuse=cf["temporal"], unbiased_combination=cf["unbiased"],
                              spatial_reuse_visibility_check=cf["vis"])
    ghost = passes * args.r

    r = restir.Renderer(local)
    for kv in args.tune:
        key, val = kv.split("=", 1)
        r.set_tuning(key, int(val))
    r.set_scene(sc)
    # the tile layout: a strong-scaling frame's geometry is not spread evenly (C4 / C5's TOML camera: the box fills the
    # middle of the frame), so its cuts follow a cost grid measured once per camera on rank 0 and broadcast
    layout, layout_rec = None, None
    use_balanced = args.layout == "balanced" or (args.layout == "auto" and scaling == "strong")
    if world > 1 and use_balanced:
        from romis_amd import distributed

        def time_tile(L):   # this rank's frame on its tile of L (ghost-zone frames: the tile's kernels, no exchange)
            gt = restir.tile_plan(GW, GH, tx, ty, rank, ghost, layout=L)
            fc = _abi.Features.from_buffer_copy(f)
            fc.temporal_reuse = 0
            r.render_restir(None, cam, GW, GH, fc, tile=gt, want_rgb=False, want_grid=False)
            r.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                r.render_restir(None, cam, GW, GH, fc, tile=gt, want_rgb=False, want_grid=False)
            r.synchronize()
            return (time.perf_counter() - t0) / 3

        layout, layout_rec = distributed.balanced_layout(
            r, lambda w, h: scene.camera_for(cf["scene"], w, h, cf.get("camera")), GW, GH, (tx, ty),
            time_tile=time_tile, rounds=args.layout_rounds)
    tile = restir.tile_plan(GW, GH, tx, ty, rank, ghost, layout=layout)
    r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
    state = {"grid": None}
    transport = args.halo_transport
    if transport == "auto":
        transport = "native" if args.dist_backend == "nccl" else "torch"
    hf = None
    halo_rec = None
    check_on = world > 1 and passes > 0 and args.halo_check != "off"
    if halo or check_on:
        # one HaloFrames per run, chosen and verified by halo_frames (select_halo); the halo-mode loop times it
        hf_checked, halo_rec = halo_frames(torch, r, rank, world, local, f, cam, GW, GH, tx, ty, passes, args, transport,
                                           check_on, fatal=halo, layout=layout)
        r.set_seed(_abi.RESTIR_DEFAULT_SEED, 0)
        if halo:
            hf = hf_checked
            tile = hf.tile
            halo_rec["timed"] = True   # the main loop's frames are this transport's

    def step():
        if hf is not None:   # RCCL halo exchange of the reservoirs before every spatial pass
            _, g = hf.render(state["grid"] if cf["temporal"] else None, cam, want_rgb=False, want_grid=cf["temporal"])
            state["grid"] = g
        elif cf["temporal"]:   # thread the previous frame's grid (main.cpp:165)
            _, g = r.render_restir(state["grid"], cam, GW, GH, f, tile=tile, want_rgb=False, want_grid=True)
            state["grid"] = g   # the previous handle is released when dropped
        else:
            r.render_restir(None, cam, GW, GH, f, tile=tile, want_rgb=False, want_grid=False)

    # the practical HBM-read ceiling reported beside the roofline, then the GPU clock pre-warm (not a frame, not timed)
    # right before the warm-up frames
    measured = r.measure_read_bandwidth(4 << 30, 10)
    if args.prewarm_gemm_ms > 0:
        gemm_prewarm(torch, local, args.prewarm_gemm_ms)
    for _ in range(args.warmup):
        step()
    # Timed region: the spatial kernel (the roofline's) carries a HIP start / stop event pair recorded inside its
    # own dispatch (hipExtLaunchKernelGGL).  Timing every kernel this way costs ~20 us per frame
    # (profiles/r1), so the per-kernel breakdown comes from a separate run of the same frames.
    r.reset_timings()
    r.set_tuning("timing.mask", -1 if args.time_kernels == "all" else 1 << _abi.K_SPATIAL)
    # a halo pass is several launches averaged per pass below: every launch keeps its events there
    r.set_tuning("timing.every", 1 if halo else max(1, args.timing_every))
    r.enable_timing(True)
    barrier_sync(torch, world, r)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier_sync(torch, world, r)
    t1 = time.perf_counter()
    r.enable_timing(False)
    elapsed = max_over_ranks(torch, world, t1 - t0, local)
    kt = r.timings()
    # per-kernel breakdown: serial frames (no overlap), every launch timed
    r.reset_timings()
    r.set_tuning("timing.mask", -1)
    r.set_tuning("timing.every", 1)
    r.enable_timing(True)
    for _ in range(min(args.steps, 20)):
        step()
    r.synchronize()
    r.enable_timing(False)
    kt_all = r.timings()
    bg_info = r.background_pixels()
    # per-rank GPU kernel time per frame of that run (the balance of the tile layout, measured): gathered to rank 0
    n_kf = max(1, min(args.steps, 20))
    busy_ms = sum(v[0] for v in kt_all.values()) / n_kf
    rank_busy = [busy_ms]
    if world > 1:
        on_gpu = torch.distributed.get_backend() == "nccl"
        bt = torch.tensor([busy_ms], dtype=torch.float64, device=torch.device("cuda", local) if on_gpu else "cpu")
        outs = [torch.zeros_like(bt) for _ in range(world)]
        torch.distributed.all_gather(outs, bt)
        rank_busy = [float(o.item()) for o in outs]
    state["grid"] = None

    ms_per_step = elapsed / args.steps * 1e3
    total = GW * GH * args.N
    value = total / (elapsed / args.steps) / 1e6

    cfg = {"workload": cf["workload"], "config": args.config, "scene": cf["scene"],
           "tile": [tile.width, tile.height] if scaling == "strong" else [GW // tx, GH // ty], "image": [GW, GH],
           "tiles": [tx, ty], "M": cf["M"], "N": args.N, "k": args.k, "r": args.r, "passes": passes,
           "temporal": cf["temporal"], "unbiased": cf["unbiased"], "spatial_visibility": cf["vis"],
           "parallelism": f"screen tiles {tx}x{ty}" + (" cost-balanced" if layout is not None else "") + ", " +
                          (f"RCCL reservoir halo {args.r}px" if halo else f"ghost {ghost}px")}
    if layout_rec is not None:
        # this rank's share and the spread over ranks of the measured per-rank frame times (max over ranks is `value`)
        layout_rec["owned"] = [tile.x0, tile.y0, tile.width, tile.height]
        cfg["layout"] = layout_rec
    if cf.get("camera"):
        cfg["camera"] = camera_record(cf["camera"])

    # roofline of the spatial pass: algorithmic bytes per pixel = read 32 (own G-buffer) + 32 N (own
    # reservoir), write 32 N; neighbour gathers are cache traffic, not counted
    sp_ms, sp_n = kt["spatial"]
    roofline = None
    if sp_n:
        sp_px = tile.width * tile.height if halo else spatial_px_per_launch(tile, passes, args.r)
        bytes_per_launch = int(sp_px * (32 + 32 * args.N + 32 * args.N))
        # a halo pass is 1-5 launches (interior + border strips): average over passes, not launches
        avg_s = sp_ms / (args.steps * passes if halo else sp_n) / 1e3
        achieved = bytes_per_launch / avg_s / 1e9
        traffic, traffic_src = (pmc_traffic(args.traffic_csv), args.traffic_csv) if args.traffic_csv else (None, None)
        if traffic is None:
            traffic, traffic_src = committed_traffic(cfg)
        roofline = {"kernel": "k_spatial", "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": traffic, "traffic_source": traffic_src, "bytes_per_launch": bytes_per_launch,
                    "avg_launch_us": round(avg_s * 1e6, 2),
                    "read_only_frac": round(sp_px * (32 + 32 * args.N) / avg_s / 1e9 / HBM_PEAK_GBS, 4)}
        # the compulsory-byte figure beside the contract's: a pixel of a RIS-flagged background tile is
        # written from the flag without reading anything (32 N B), the rest moves the contract's bytes; the last frame's
        # flag count (restir_background_pixels) -- ghost-zone frames apply the computed region's share to the pass
        if not halo and bg_info is not None and bg_info[1]:
            share = bg_info[0] / bg_info[1]
            comp = sp_px * ((1.0 - share) * (32 + 64 * args.N) + share * 32 * args.N)
            roofline["background_share"] = round(share, 4)
            roofline["compulsory_bytes_per_launch"] = int(comp)
            roofline["frac_compulsory"] = round(comp / avg_s / 1e9 / HBM_PEAK_GBS, 4)
            # the survey's read-only bar (§8d: 64 B/px, <= 41.5 us at 1080p for 0.40)
            roofline["read_only_bar_us"] = round(sp_px * (32 + 32 * args.N) / (0.40 * HBM_PEAK_GBS * 1e9) * 1e6, 2)
        # the practical ceiling next to the spec: a streaming-read kernel over 4 GiB (past the Infinity Cache), run
        # before the warm-up frames
        roofline["measured_read_peak"] = round(measured, 1)
        roofline["frac_of_measured_peak"] = round(achieved / measured, 4)
        if cf.get("geometry") is not None:
            # the TOML camera's C4 / C5 frame (profiles/r5/balance.json: 13.2 % of the pixels hit the box): background
            # tiles are written from the RIS flags without reads, so frac is an algorithmic rate, not bytes moved and
            # not roofline evidence -- the framed configs c4f / c5f measure the pass on geometry
            roofline["geometry_share"] = cf["geometry"]
            roofline["frac_kind"] = "algorithmic rate over a background-dominated frame (not a roofline; see c4f / c5f)"

    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline:
        rows = args.cpu_rows or min(GH, max(8, 1036800 // GW))   # ~1 Mpx of the workload, ~0.3 s on 16 cores
        cpu = cpu_baseline(sc, lambda w, h: scene.camera_for(cf["scene"], w, h, cf.get("camera")), f, rows, GW, GH)
        if args.cpu_stages:
            def feats(c):   # the config's frame at N, k, r of this run
                return _abi.default_features(initial_light_samples=c["M"], num_samples_in_reservoir=args.N,
                                             num_neighbours_to_sample=args.k, spatial_resample_radius=args.r,
                                             spatial_resampling_passes=c["passes"],
                                             spatial_reuse=1 if c["passes"] > 0 else 0, temporal_reuse=c["temporal"],
                                             unbiased_combination=c["unbiased"], spatial_reuse_visibility_check=c["vis"])
            cpu["stages"] = cpu_stages(args.config, scene.bench_scene, scene.camera_for, feats, cpu["cores"])

    kernels = {k: {"us_per_launch": round(v[0] / v[1] * 1e3, 2) if v[1] else None, "launches": int(v[1])}
               for k, v in kt_all.items()}
    # roofline of initial RIS (the frame's largest kernel): SURVEY.md §8(d) prices a candidate at ~160 flop
    # (target pdf incl. sqrt, divisions and powf, the weight and the reservoir update); candidates per launch =
    # the launch's pixels x M.  The fused k_primary_ris also traces the primary rays, which are not counted.
    # Its time comes from the separate all-kernel run above (HIP events on the kernel's own dispatch).
    roofline_ris = None
    rk = "primary_ris" if kt_all.get("primary_ris", (0, 0))[1] else "ris"
    rms, rn = kt_all.get(rk, (0.0, 0))
    if rn:
        cand = tile.width * tile.height * cf["M"]
        avg_s = rms / rn / 1e3
        tf = cand * RIS_FLOP_PER_CANDIDATE / avg_s / 1e12
        roofline_ris = {"kernel": "k_primary_ris" if rk == "primary_ris" else "k_ris", "bound": "valu",
                        "achieved": round(tf, 2), "peak": FP32_VECTOR_PEAK_TFS, "unit": "TFLOP/s",
                        "frac": round(tf / FP32_VECTOR_PEAK_TFS, 4), "flop_per_candidate": RIS_FLOP_PER_CANDIDATE,
                        "candidates_per_launch": cand, "avg_launch_us": round(avg_s * 1e6, 2),
                        "flop_model": "the reference's operations per candidate (SURVEY.md §8d), powf included; the "
                                      "kernel skips powf exactly where a material has ks = 0 (7 of the 8 Cornell "
                                      "materials: c1, c4, c5), so there achieved is an algorithmic rate that can "
                                      "exceed the FP32 peak, not the SIMDs' FLOP rate"}
        valu = committed_valu(args.config, cfg["N"], roofline_ris["kernel"])
        if valu:   # measured issue: VALU wave-instructions per candidate (SQ_INSTS_VALU / (pixels x M / 64))
            roofline_ris.update(valu)
    # visibility reuse (c5): the spatial pass is ray-bound, so its rate is reported as shadow-ray slots per second --
    # (k + 1) N per pixel, an upper bound on the rays cast (a ray is skipped where p-hat = 0 and the whole Z loop
    # where W = 0) -- next to the final pass's one ray per pixel per sub-reservoir
    roofline_rays = None
    sms, sn = kt_all.get("spatial", (0.0, 0))
    fms, fn = kt_all.get("final", (0.0, 0))
    if cf["vis"] and sn and fn:
        px = tile.width * tile.height
        slots = px * (args.k + 1) * args.N
        roofline_rays = {"kernel": "k_spatial (unbiased + visibility)", "bound": "rays",
                         "ray_slots_per_launch": slots, "avg_launch_us": round(sms / sn * 1e3, 2),
                         "grays_per_s": round(slots / (sms / sn * 1e-3) / 1e9, 2),
                         "final_grays_per_s": round(px * args.N / (fms / fn * 1e-3) / 1e9, 2),
                         "note": "ray slots = (k+1) N per pixel, an upper bound on the shadow rays cast; final = 1 per "
                                 "pixel and sub-reservoir (also an upper bound: no ray where the shaded value is 0)"}
    kernels["note"] = "separate run after the timed region, every kernel's dispatch recording HIP events"
    # every rank computed the same mismatch count (select_halo sums it over ranks): all exit alike
    halo_failed = halo_rec is not None and halo_rec.get("check") not in ("bit-exact", "off")
    if rank == 0:
        out = {
            "metric": "Mpixel-reservoirs/s at 1080p, M=32, k=5 spatial; 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "Mpixel-reservoirs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic ({DATA[cf['scene']]}, keyed RNG seed 0x5EED0001)",
            "config": cfg,
            "roofline": roofline,
            "roofline_ris": roofline_ris,
            "roofline_rays": roofline_rays,
            "cpu_baseline": cpu,
            "kernels": kernels,
        }
        if world > 1:
            out["balance"] = {"kernel_ms_per_frame_per_rank": [round(v, 4) for v in rank_busy],
                              "efficiency": round(float(np.mean(rank_busy) / max(rank_busy)), 4) if max(rank_busy) > 0 else None,
                              "note": "GPU kernel time per frame on each rank (HIP events, the per-kernel run): mean / max "
                                      "is the tile layout's balance, halo transfers excluded"}
        if halo_rec is not None:
            out["halo"] = halo_rec
        if halo_failed:   # a non-fatal halo check that failed still fails the run (after the record)
            out["error"] = "halo tile differs from the ghost-zone tile (halo.check)"
        print(json.dumps(out), flush=True)
    r.close()
    if world > 1:
        torch.distributed.destroy_process_group()
    if halo_failed:
        sys.exit(3)


if __name__ == "__main__":
    main()
