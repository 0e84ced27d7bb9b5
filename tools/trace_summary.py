#!/usr/bin/env python3
"""Per-workload kernel-time summary from `tools/gpu_session.sh prof` output
(rocprofv3 --kernel-trace --stats over bench.py --steps 60 --warmup W): for the
dominant nexg:: kernel of each run, the launch count, the average over all
launches, over the last 60 (bench.py's timed region) and the minimum. The
kernel_stats.csv of each run is copied beside it.

usage: tools/trace_summary.py <gpurun_out dir> <profiles out dir>
"""
import csv
import glob
import json
import os
import shutil
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    out = {}
    for d in sorted(glob.glob(os.path.join(src, "prof_*"))):
        name = os.path.basename(d)[5:]
        traces = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        if not traces:
            continue
        launches = {}
        with open(traces[0]) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                # generators and calibration kernels (the ser run's write-only ceiling
                # k_probe_write, the stream probes, the latency chase) are not the object
                if "nexg::" not in k or any(c in k for c in ("k_gen_", "k_probe_", "k_chase", "k_recompute")):
                    continue
                launches.setdefault(k, []).append((int(r["Start_Timestamp"]),
                                                   int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        if not launches:
            continue
        kern = max(launches, key=lambda k: sum(t for _, t in launches[k]))
        ts = [t for _, t in sorted(launches[kern])]
        last = ts[-60:]
        out[name] = {"kernel": kern, "launches": len(ts),
                     "avg_ms_all": round(sum(ts) / len(ts) / 1e6, 4),
                     "avg_ms_timed_last60": round(sum(last) / len(last) / 1e6, 4),
                     "min_ms": round(min(ts) / 1e6, 4),
                     "note": "rocprofv3 --kernel-trace --stats over bench.py --steps 60; the last 60 "
                             "launches of the kernel are bench.py's timed region"}
        if stats:
            shutil.copy(stats[0], os.path.join(dst, f"{name}_kernel_stats.csv"))
    with open(os.path.join(dst, "kernel_trace_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
