#!/usr/bin/env python3
"""profiles/valu.json from an SQ counter pass over the headline bench (scripts/pmc_passes.sh <tag> "SQ_INSTS_VALU
SQ_WAVES ..."): VALU wave-instructions per launch of the initial-RIS kernel and per candidate (SQ_INSTS_VALU counts
one per wave-level instruction; a wave carries 64 pixels' candidates in lock step, so per candidate =
SQ_INSTS_VALU / (pixels x M / 64)), at the source hash the pass ran on.  bench.py reports it beside roofline_ris.

    python scripts/valu_json.py profiles/r3/s2j
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    d = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(os.path.join(d, "sq_counter_collection.csv"))):
        agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    src = open(os.path.join(d, "source_hash.txt")).read().strip()
    bench = json.load(open(os.path.join(d, "pmc0.json")))
    W, H = bench["config"]["tile"]
    cand = W * H * bench["config"]["M"]
    out = {"source_hash": src, "profile": os.path.relpath(d, ROOT), "config": bench["config"]["config"],
           "N": bench["config"]["N"],
           "counters": "rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES (one pass)",
           "kernels": {}}
    for k, cs in agg.items():
        if not k.startswith("k_"):
            continue
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"sq_insts_valu": mean.get("SQ_INSTS_VALU"), "sq_insts_salu": mean.get("SQ_INSTS_SALU"),
             "sq_waves": mean.get("SQ_WAVES"), "launches": len(cs.get("SQ_INSTS_VALU", []))}
        if "ris" in k:
            e["candidates_per_launch"] = cand
            e["valu_instr_per_candidate"] = round(mean["SQ_INSTS_VALU"] / (cand / 64.0), 1)
        out["kernels"][k] = e
    with open(os.path.join(ROOT, "profiles", "valu.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
