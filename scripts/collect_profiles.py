#!/usr/bin/env python3
"""Copy one gpurun_out/<tag> profiling run (scripts/gpu_profile.sh) into profiles/<round>/<tag>/ and write a
summary: per-kernel average duration (rocprofv3 --kernel-trace --stats) and per-launch HBM traffic from the
separate FETCH_SIZE / WRITE_SIZE --pmc passes, corrected as MI355X_MICROARCH.md "HBM" prescribes
(counters in KiB; FETCH_SIZE reads half the bytes of wide coalesced streams on gfx950, so it is doubled).

    python scripts/collect_profiles.py r1e --round r1
"""
import argparse
import csv
import json
import os
import shutil
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_stats(path):
    out = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            out[row["Name"]] = {"calls": int(row["Calls"]), "avg_us": float(row["AverageNs"]) / 1e3,
                                "pct": float(row["Percentage"])}
    return out


def pmc(path, counter):
    per = {}
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if row["Counter_Name"] != counter:
                continue
            per.setdefault(row["Kernel_Name"], []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--round", default="r1")
    args = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", args.tag)
    dst = os.path.join(ROOT, "profiles", args.round, args.tag)
    os.makedirs(dst, exist_ok=True)
    keep = ["bench.json", "trace/run_kernel_stats.csv", "trace/run_kernel_trace.csv", "pmc_fetch/run_counter_collection.csv",
            "pmc_write/run_counter_collection.csv", "trace_bench.json", "tests.log", "kbench.json",
            "sq/run_counter_collection.csv"]
    for k in keep:
        p = os.path.join(src, k)
        if os.path.exists(p):
            q = os.path.join(dst, k.replace("/", "__"))
            shutil.copy(p, q)
    summary = {"tag": args.tag}
    try:
        summary["git_rev"] = subprocess.check_output(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"]).decode().strip()
    except Exception:
        pass
    ks = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(ks):
        summary["kernel_stats"] = kernel_stats(ks)
    fp = os.path.join(src, "pmc_fetch", "run_counter_collection.csv")
    wp = os.path.join(src, "pmc_write", "run_counter_collection.csv")
    if os.path.exists(fp) and os.path.exists(wp):
        fetch = pmc(fp, "FETCH_SIZE")
        write = pmc(wp, "WRITE_SIZE")
        summary["hbm_per_launch"] = {
            k: {"fetch_kib_raw": round(fetch.get(k, 0.0), 1), "write_kib": round(write.get(k, 0.0), 1),
                "hbm_bytes_corrected": round(fetch.get(k, 0.0) * 1024 * 2 + write.get(k, 0.0) * 1024)}
            for k in sorted(set(fetch) | set(write))}
    sh = os.path.join(src, "source_hash.txt")
    if os.path.exists(sh) and "hbm_per_launch" in summary:
        with open(sh) as fh:
            summary["source_hash"] = fh.read().strip()
        sp = {k: v for k, v in summary["hbm_per_launch"].items() if k.startswith("k_spatial")}
        if len(sp) == 1:
            (kname, t), = sp.items()
            trace_bench = os.path.join(src, "trace_bench.json")
            cfg = None
            if os.path.exists(trace_bench):
                with open(trace_bench) as fh:
                    cfg = json.loads(fh.read().strip().splitlines()[-1]).get("config")
            rec = {"source_hash": summary["source_hash"], "kernel": kname,
                   "traffic_bytes_per_launch": t["hbm_bytes_corrected"], "config": cfg,
                   "profile": os.path.relpath(dst, ROOT),
                   "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; bytes = "
                             "FETCH_SIZE KiB x 1024 x 2 (gfx950 wide-read correction) + WRITE_SIZE KiB x 1024"}
            # the per-config / per-order attribution study (scripts/traffic_json.py) stays, under its own hash
            tpath = os.path.join(ROOT, "profiles", "traffic.json")
            try:
                with open(tpath) as fh:
                    old = json.load(fh)
            except (OSError, ValueError):
                old = {}
            if old.get("entries"):
                rec["attribution"] = {"source_hash": old.get("source_hash"), "profile": old.get("profile"),
                                      "method": old.get("method"), "entries": old["entries"]}
            elif old.get("attribution"):
                rec["attribution"] = old["attribution"]
            with open(tpath, "w") as fh:
                json.dump(rec, fh, indent=1)
    bj = os.path.join(src, "bench.json")
    if os.path.exists(bj):
        with open(bj) as fh:
            summary["bench"] = json.loads(fh.read().strip().splitlines()[-1])
    with open(os.path.join(dst, "summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "bench"}, indent=1))


if __name__ == "__main__":
    main()
