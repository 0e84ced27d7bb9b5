#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/pmc.sh output) into per-launch HBM
bytes for the parse path of each workload.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. On gfx950, FETCH_SIZE counts
exactly half the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md
§HBM), so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
Only nexg:: kernels count; generator kernels (k_gen_*), calibration kernels (k_probe_*,
k_chase*, the stamped k_parse_span<..., true> instance), the
real-traffic batch's one checksum fix-up (k_recompute) and torch setup kernels are skipped.

usage: tools/pmc_summary.py <pmc dir> <out dir>   (writes pmc_summary.json and
       traffic.json into <out dir>)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    src, dst = sys.argv[1], sys.argv[2]
    rows = []
    per_wl = defaultdict(lambda: {"read_bytes": 0.0, "write_bytes": 0.0, "kernels": []})
    for path in sorted(glob.glob(os.path.join(src, "*_*_SIZE", "*counter_collection.csv"))):
        name = os.path.basename(os.path.dirname(path))  # <wl>[.<out>]_<COUNTER>
        counter = "FETCH_SIZE" if name.endswith("_FETCH_SIZE") else "WRITE_SIZE"
        wl = name[: -len(counter) - 1]
        vals = defaultdict(list)
        with open(path) as f:
            for r in csv.DictReader(f):
                kn = r["Kernel_Name"]
                if "nexg::" not in kn or "k_gen_" in kn or "k_probe_" in kn or "k_recompute" in kn or "k_chase" in kn:
                    continue
                if "k_parse_span" in kn and kn.split("(")[0].rstrip().endswith("true>"):
                    continue  # the stamped calibration instance (nexg_probe_span_clock), one launch per object

                vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        for kern, v in vals.items():
            kb = sum(v) / len(v)
            corrected = kb * 1024 * (2 if counter == "FETCH_SIZE" else 1)
            rows.append({"workload": wl, "kernel": kern, "counter": counter, "dispatches": len(v),
                         "raw_kb_per_launch": kb, "bytes_per_launch_corrected": corrected})
            key = "read_bytes" if counter == "FETCH_SIZE" else "write_bytes"
            per_wl[wl][key] += corrected
            if kern not in per_wl[wl]["kernels"]:
                per_wl[wl]["kernels"].append(kern)
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(rows, f, indent=1)
    traffic = {}
    for wl, t in per_wl.items():
        key = wl.replace(".", ":") if "." in wl else f"{wl}:desc"
        traffic[key] = {
            "hbm_bytes_per_launch": int(t["read_bytes"] + t["write_bytes"]),
            "read_bytes": int(t["read_bytes"]), "write_bytes": int(t["write_bytes"]),
            "kernels": t["kernels"],
            "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes ({dst}), "
                      "FETCH_SIZE x2 gfx950 correction (MI355X_MICROARCH.md §HBM)"}
    with open(os.path.join(dst, "traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
