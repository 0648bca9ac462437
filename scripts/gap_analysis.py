#!/usr/bin/env python3
"""Per-frame timeline of bench.py from a rocprofv3 --kernel-trace CSV: kernel durations, the gaps between
consecutive kernels of a frame and between frames, for every frame in dispatch order.

    python scripts/gap_analysis.py <run_kernel_trace.csv> [--warmup W --steps K]

A frame = the kernels from one k_primary_ris* dispatch up to the next.  With --warmup / --steps the frames are
labelled (bench.py renders W warm-up frames, K timed ones, then min(K, 20) all-kernel-timed ones).  Prints one
JSON object: per-frame spans, and averages over the timed frames (kernel sum, in-frame gaps, frame-to-frame gap).
"""
import argparse
import csv
import json
import statistics


def load(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def frames_of(rows):
    frames, cur = [], None
    for s, e, name in rows:
        if name.startswith("k_primary_ris") or name.startswith("k_primary"):
            if cur:
                frames.append(cur)
            cur = []
        if cur is not None and name.startswith("k_"):
            cur.append((s, e, name))
    if cur:
        frames.append(cur)
    return frames


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--steps", type=int, default=None)
    args = ap.parse_args()
    fr = frames_of(load(args.csv))
    out = {"frames": []}
    prev_end = None
    for i, f in enumerate(fr):
        ks = [{"k": n.split("(")[0], "us": round((e - s) / 1e3, 2)} for s, e, n in f]
        gaps = [round((f[j + 1][0] - f[j][1]) / 1e3, 2) for j in range(len(f) - 1)]
        rec = {"i": i, "span_us": round((f[-1][1] - f[0][0]) / 1e3, 2), "kernels": ks, "gaps_us": gaps,
               "from_prev_us": round((f[0][0] - prev_end) / 1e3, 2) if prev_end is not None else None}
        if args.warmup is not None and args.steps is not None:
            rec["phase"] = "warmup" if i < args.warmup else ("timed" if i < args.warmup + args.steps else "kernel_timed")
        out["frames"].append(rec)
        prev_end = f[-1][1]
    if args.warmup is not None and args.steps is not None:
        timed = [r for r in out["frames"] if r.get("phase") == "timed"]
        if timed:
            t0 = fr[args.warmup][0][0]
            t1 = fr[args.warmup + args.steps - 1][-1][1]
            out["timed"] = {
                "frames": len(timed),
                "wall_us_per_frame_first_start_to_last_end": round((t1 - t0) / 1e3 / len(timed), 2),
                "kernel_sum_us": round(statistics.mean(sum(k["us"] for k in r["kernels"]) for r in timed), 2),
                "in_frame_gaps_us": round(statistics.mean(sum(r["gaps_us"]) for r in timed), 2),
                "between_frames_us": round(statistics.mean(r["from_prev_us"] for r in timed[1:]), 2) if len(timed) > 1 else None,
                "span_first3_us": [r["span_us"] for r in timed[:3]],
                "span_last3_us": [r["span_us"] for r in timed[-3:]],
                "per_kernel_mean_us": {},
            }
            names = sorted({k["k"] for r in timed for k in r["kernels"]})
            for n in names:
                v = [k["us"] for r in timed for k in r["kernels"] if k["k"] == n]
                out["timed"]["per_kernel_mean_us"][n] = {"mean": round(statistics.mean(v), 2), "first": v[0], "last": v[-1]}
    print(json.dumps(out, indent=None))


if __name__ == "__main__":
    main()
