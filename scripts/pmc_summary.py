#!/usr/bin/env python3
"""Average rocprofv3 counter values per kernel over the pmc*/run_counter_collection.csv files of a tag.
    python scripts/pmc_summary.py gpurun_out/<tag> [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
keys = sys.argv[2:]
d = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "pmc*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if keys and not any(s in k for s in keys):
            continue
        d[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = sorted({k for k, _ in d})
ctrs = sorted({c for _, c in d})
print("counter".ljust(26) + "".join(k[:22].rjust(24) for k in kern))
for c in ctrs:
    print(c.ljust(26) + "".join((f"{sum(d[(k, c)]) / len(d[(k, c)]):.4g}" if (k, c) in d else "-").rjust(24) for k in kern))
