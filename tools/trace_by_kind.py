#!/usr/bin/env python3
"""Median duration (us) of each parse kernel per bench_malformed kind, from a
rocprofv3 kernel trace: the nexg parse launches come in blocks of `per`
(warmup + steps) per kind, in kind order.
usage: trace_by_kind.py run_kernel_trace.csv clean,all 15"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
kinds = sys.argv[2].split(",")
per = int(sys.argv[3])
names = ("k_parse_span", "k_span_deferred", "k_tail_sums", "k_parse_lane80")
sel = sorted((r for r in rows if any(n in r["Kernel_Name"] for n in names)), key=lambda r: int(r["Start_Timestamp"]))
first = [r for r in sel if "k_parse_span" in r["Kernel_Name"] or "k_tail_sums" in r["Kernel_Name"]]
blocks = {}
k = -1
for r in sel:
    if r is first[0] or ("k_parse_span" in r["Kernel_Name"] and first.index(r) % per == 0):
        k += 1
    name = r["Kernel_Name"].split("(")[0].replace("void nexg::", "")
    blocks.setdefault(kinds[min(k, len(kinds) - 1)], {}).setdefault(name, []).append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for kind in kinds:
    d = blocks.get(kind, {})
    tot = sum(statistics.median(v) for v in d.values())
    print(kind, {n: round(statistics.median(v), 1) for n, v in d.items()}, "sum", round(tot, 1))
