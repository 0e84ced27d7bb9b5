#!/usr/bin/env python3
"""Per-dispatch means of the k_parse_span rows of tools/tlb_pmc.sh's
rocprofv3 outputs (counter_collection.csv per pass, kernel_trace.csv per
mode), skipping each run's first 20 dispatches (the first ~30 ms of a process
run slower).
usage: python tools/tlb_summary.py gpurun_out/tlb"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    res = defaultdict(dict)
    for path in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        mode = os.path.relpath(path, root).split(os.sep)[0].split("_")[0]
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(path)):
            if "k_parse_span" not in row.get("Kernel_Name", ""):
                continue
            per[row["Counter_Name"]][int(row["Dispatch_Id"])] += float(row["Counter_Value"])
        for name, d in per.items():
            ids = sorted(d)[20:] or sorted(d)
            res[mode][name] = round(sum(d[i] for i in ids) / len(ids), 1)
    for path in glob.glob(os.path.join(root, "*_trace", "**", "*kernel_trace.csv"), recursive=True):
        mode = os.path.relpath(path, root).split(os.sep)[0].split("_")[0]
        ds = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open(path))
              if "k_parse_span" in r.get("Kernel_Name", "")]
        ds = ds[20:] or ds
        res[mode]["kernel_ms"] = round(sum(ds) / len(ds) / 1e6, 4) if ds else None
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
