#!/usr/bin/env python3
"""Gaps between consecutive dispatches per kernel name in a rocprofv3 kernel trace (scripts/probes/gap_probe2.hip):
median start(k + 1) - end(k) for each pair of consecutive kernels of the same variant.   gap2_analyze.py <trace.csv>"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
by = {}
for p, q in zip(rows, rows[1:]):
    if p["Kernel_Name"] == q["Kernel_Name"]:
        by.setdefault(p["Kernel_Name"].split("(")[0], []).append((int(q["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3)
for k, g in by.items():
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if r["Kernel_Name"].split("(")[0] == k]
    print(f'{{"kernel": "{k}", "gap_us_median": {statistics.median(g):.2f}, "kernel_us_median": {statistics.median(dur):.2f}, "n": {len(g)}}}')
