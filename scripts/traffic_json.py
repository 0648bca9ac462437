#!/usr/bin/env python3
"""profiles/traffic.json from a scripts/traffic_study.sh run (gpurun_out/<tag>): the spatial kernel's HBM-side bytes
per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE in separate --pmc passes; KiB; FETCH doubled for wide streams on
gfx950, MI355X_MICROARCH.md "HBM") for C2 (the handle pass and the n_t-window pass), C4, C4f and C5f, against the algorithmic bytes (64 B
read + 32 B written per pixel at N = 1).

    python scripts/traffic_json.py r3c_traffic --profile profiles/r3/r3c_traffic
"""
import argparse
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from romis_amd import build  # noqa: E402


def counter(path, name):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Kernel_Name"].startswith("k_spatial") and r["Counter_Name"] == name]
    return sum(vals) / len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--profile", required=True, help="where the raw CSVs are kept (committed)")
    args = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", args.tag)
    dst = os.path.join(ROOT, args.profile)
    os.makedirs(dst, exist_ok=True)
    entries = []
    orders_of = {"c2": [("chunks", 255), ("ntl", 255)], "c4": [("chunks", 255)], "c4f": [("chunks", 255), ("ntl", 255)],
                 "c5f": [("chunks", 255)]}
    for cfgname, orders in orders_of.items():
        cf = bench.CONFIGS[cfgname]
        W, H = cf.get("tile") or cf["image"]
        px = W * H
        times = json.load(open(os.path.join(src, f"{cfgname}_times.json")))["us_per_launch"]
        for order, rows in orders:
            f = os.path.join(src, f"{cfgname}_{order}_FETCH_SIZE", "run_counter_collection.csv")
            w = os.path.join(src, f"{cfgname}_{order}_WRITE_SIZE", "run_counter_collection.csv")
            for p, tag in ((f, "fetch"), (w, "write")):
                shutil.copy(p, os.path.join(dst, f"{cfgname}_{order}_{tag}.csv"))
            fetch = counter(f, "FETCH_SIZE") * 1024 * 2
            write = counter(w, "WRITE_SIZE") * 1024
            alg = px * 96
            cfg = {"config": cfgname, "scene": cf["scene"], "tile": [W, H], "M": cf["M"], "N": 1, "k": 5, "r": 10,
                   "passes": cf["passes"]}
            if cf.get("camera"):
                cfg["camera"] = bench.camera_record(cf["camera"])
            kernels = sorted({r["Kernel_Name"] for r in csv.DictReader(open(f)) if r["Kernel_Name"].startswith("k_spatial")})
            entries.append({
                "config": cfg, "xcd_order": "chunks" if order == "ntl" else order, "variant": order,
                "spatial.xcd_rows": rows, "kernel": ",".join(kernels),
                "traffic_bytes_per_launch": int(fetch + write), "fetch_bytes": int(fetch), "write_bytes": int(write),
                "algorithmic_bytes": alg, "ratio": round((fetch + write) / alg, 3),
                "fetch_B_per_px": round(fetch / px, 1), "write_B_per_px": round(write / px, 1),
                "spatial_us": times[order]["spatial"]})
    c2 = next(e for e in entries if e["config"]["config"] == "c2" and e["variant"] == "chunks")
    rec = {"source_hash": build.source_hash(), "kernel": c2["kernel"], "profile": args.profile,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over scripts/cfg_kbench.py; "
                     "bytes = FETCH_SIZE KiB x 1024 x 2 (gfx950 wide-read correction) + WRITE_SIZE KiB x 1024",
           # the headline (c2, default XCD chunk order) at the top level, as bench.py reads it
           "config": c2["config"], "traffic_bytes_per_launch": c2["traffic_bytes_per_launch"], "entries": entries}
    with open(os.path.join(ROOT, "profiles", "traffic.json"), "w") as fh:
        json.dump(rec, fh, indent=1)
    for e in entries:
        print(e["config"]["config"], e["variant"], e["ratio"], e["fetch_B_per_px"], e["write_B_per_px"], e["spatial_us"])


if __name__ == "__main__":
    main()
