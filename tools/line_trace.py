#!/usr/bin/env python3
"""A kernel-trace row for every timed object of one bench.py line, from a
rocprofv3 --kernel-trace run of that same bench command (tools/gpu_session.sh
step `lineprof`).

bench.py times its objects one after the other, each as W + K back-to-back
launches of one kernel (the warmup continues until 0.25 s have passed), so
the trace is a sequence of long runs of one kernel name. The objects' run
order is bench.py main()'s execution order (not the order the line prints
them in). For each object the row gives the kernel, the launches in its run,
the trace's average over the run's last K launches (the timed region), the
line's HIP-event kernel_ms, the algorithmic bytes and both fractions of
8 TB/s: bytes / trace average and the line's own.

usage: tools/line_trace.py <rocprof dir> <bench stdout log> <out json>
"""
import csv
import glob
import json
import sys

PEAK = 8000.0  # GB/s, MI355X HBM3E (MI355X_MICROARCH.md)
#: calibration kernels bench.py runs between objects that are not objects themselves
SKIP = ("k_gen_", "k_chase", "k_recompute")


def expected(line):
    """(object path, kernel-name substring, K, algorithmic bytes, line kernel_ms)
    in bench.py's execution order."""
    rl = line["roofline"]
    top_k = "k_build" if "udp_ping" in line["metric"] or "build" in line["metric"] else "k_parse"
    ex = [("main", top_k, line["steps"], rl["algorithmic_bytes_per_launch"], rl["kernel_ms"])]
    sc = rl.get("stream_ceilings") or {}
    nb = rl["algorithmic_bytes_per_launch"]
    if "read_only_gbs" in sc:
        ex.append(("stream.read_only", "k_probe_stream<false, false>", line["steps"], nb // 16384 * 16384, None))
        ex.append(("stream.read64_write8", "k_probe_stream<true, false>", line["steps"], nb // 16384 * 16384, None))
        if "read64_write8_6cu_gbs" in sc:
            ex.append(("stream.read64_write8_6cu", "k_probe_stream<true, true>", line["steps"], nb // 16384 * 16384,
                       None))
        for k in ("desc_output", "flags_output", "verdict_output", "sparse_output", "grouped_output"):
            if k in sc:
                ex.append((f"stream.{k}", "k_parse", line["steps"], nb, sc[k]["kernel_ms"]))
    for name in ("imix", "malformed", "real_traffic"):
        o = line.get(name)
        if o is None:
            continue
        ex.append((name, "k_parse_span", o["steps"], o["roofline"]["alg_bytes"], o["roofline"]["kernel_ms"]))
        for k, v in (o.get("other_outputs") or {}).items():
            ex.append((f"{name}.{k}", "k_parse_span", o["steps"], o["roofline"]["alg_bytes"], v["kernel_ms"]))
    ser = line.get("ser")
    if ser is not None:
        ex.append(("ser.write_only", "k_probe_write", ser["steps"], None, None))
        ex.append(("ser", "k_build_udp4", ser["steps"], ser["roofline"]["alg_bytes"], ser["roofline"]["kernel_ms"]))
        for k, kern in (("tuples", "k_build_udp4"), ("tcp_ping", "k_build_"), ("icmp_ping", "k_build_"),
                        ("udp6", "k_build_")):
            o = ser.get(k)
            if o is not None:
                ex.append((f"ser.{k}", kern, o["steps"], o["roofline"]["alg_bytes"], o["roofline"]["kernel_ms"]))
    lg = line.get("large")
    if lg is not None:
        ex.append(("large", "k_parse", lg["steps"], lg["roofline"]["alg_bytes"], lg["roofline"]["kernel_ms"]))
    return ex


def runs(trace_csv):
    """Consecutive launches of one nexg:: kernel, in dispatch order."""
    rows = []
    with open(trace_csv) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"]
            if "nexg::" not in k or any(s in k for s in SKIP):
                continue
            # (kernel, LDS size): the occupancy-capped stream (dynamic LDS) is its own run
            key = (k, r.get("LDS_Block_Size", ""))
            rows.append((int(r["Start_Timestamp"]), key, int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    out = []
    for _, key, d in rows:
        if out and out[-1][2] == key:
            out[-1][1].append(d)
        else:
            out.append((key[0], [d], key))
    return out


def bench_line(log):
    with open(log) as f:
        for ln in f:
            if ln.startswith("{") and '"metric"' in ln:
                return json.loads(ln)
    raise SystemExit(f"no bench line in {log}")


def main():
    src, log, dst = sys.argv[1:4]
    trace = glob.glob(f"{src}/**/*kernel_trace.csv", recursive=True)[0]
    line = bench_line(log)
    rs = runs(trace)
    rows, i = {}, 0
    for name, kern, k, nbytes, line_ms in expected(line):
        while i < len(rs) and not (kern in rs[i][0] and len(rs[i][1]) >= k + 1):
            i += 1
        if i == len(rs):
            rows[name] = {"error": f"no run of {kern} with >= {k + 1} launches left"}
            continue
        kn, ds, _ = rs[i]
        i += 1
        last = ds[-k:]
        avg_ms = sum(last) / len(last) / 1e6
        r = {"kernel": kn.split("(")[0], "launches": len(ds), "timed": k, "trace_avg_ms": round(avg_ms, 4),
             "line_kernel_ms": line_ms}
        if nbytes:
            r["bytes"] = nbytes
            r["frac_trace"] = round(nbytes / avg_ms / 1e6 / PEAK, 4)
            if line_ms:
                r["frac_line"] = round(nbytes / line_ms / 1e6 / PEAK, 4)
                r["line_over_trace"] = round(r["frac_line"] / r["frac_trace"], 4)
        rows[name] = r
    with open(dst, "w") as f:
        json.dump(rows, f, indent=1)
    for name, r in rows.items():
        print(f"{name:28s} {r.get('kernel', r.get('error'))[:60]:60s} {r.get('trace_avg_ms')} "
              f"{r.get('line_kernel_ms')} {r.get('frac_trace')} {r.get('frac_line')}")


if __name__ == "__main__":
    main()
