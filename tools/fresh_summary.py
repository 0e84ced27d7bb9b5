#!/usr/bin/env python3
"""tools/fresh_pmc.sh output: the k_parse_span dispatches in launch order,
30 per copy per round (10 warmup + 20 timed, tools/placement_ab.py --fresh),
averaged over each copy's timed dispatches; beside each copy its rate from the
run's own stdout.
usage: python tools/fresh_summary.py gpurun_out/fresh_pmc"""
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
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(path)):
            if "k_parse_span" not in row.get("Kernel_Name", ""):
                continue
            per[int(row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        ids = sorted(per)
        for k in range(len(ids) // 30):
            block = ids[30 * k + 10: 30 * k + 30]  # the timed 20 of copy k % 8, round k // 8
            for name in per[ids[0]]:
                res[f"round{k // 8}_copy{k % 8}"][name] = round(sum(per[i][name] for i in block) / len(block), 1)
    for log in glob.glob(os.path.join(root, "*.log")):
        for line in open(log):
            if line.startswith('{"round"'):
                d = json.loads(line)
                res[f"round{d['round']}_copy{d['copy']}"].setdefault("frac_" + os.path.basename(log)[:-4], d["frac"])
    for k in sorted(res):
        print(k, json.dumps(res[k]))


if __name__ == "__main__":
    main()
