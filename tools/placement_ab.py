#!/usr/bin/env python3
"""Does where a batch sits in device memory move the parse rate? The same
packed batch (real-traffic, App. C mix or IMIX) is copied into several fresh
device allocations, with other allocations made and freed in between (the
churn of bench.py's earlier objects), and each copy is timed with HIP events
(grouped output, the bench's kernel): a spread across copies of one batch is
placement, not code or box.
usage: python tools/placement_ab.py [--workload real|mix|imix] [--copies 6]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="real")
    ap.add_argument("--copies", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--drift", type=int, default=0, help="rounds of original / copy alternated (0: copies mode)")
    ap.add_argument("--fresh", type=int, default=0, help="N copies in N live allocations, each timed twice")
    ap.add_argument("--reserve", type=int, default=0, help="GiB allocated (unused) before anything else")
    args = ap.parse_args()
    import torch
    from nex_amd import abi, workloads
    from nex_amd.engine import Engine, FrameBatch
    eng = Engine(0)
    reserve = torch.empty(args.reserve << 30, dtype=torch.uint8, device="cuda") if args.reserve else None  # noqa: F841
    if args.workload == "imix":
        b = eng.gen_batch(abi.WL_IMIX, 16 << 20)
    else:
        mk = workloads.malformed_mix if args.workload == "mix" else workloads.real_traffic
        m, _ = mk(eng, 1 << 20, seed=abi.DEFAULT_SEED + (0 if args.workload == "mix" else 7))
        b = workloads.tiled(m, 16)
    out = torch.empty(Engine.out_bytes(abi.OUT_GROUPED, b.count), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    res = []
    keep = []

    def time_batch(c):
        for _ in range(10):
            eng.parse(c, out_kind=abi.OUT_GROUPED, out=out, stream=s)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(args.steps):
            eng.parse(c, out_kind=abi.OUT_GROUPED, out=out, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.steps

    if args.fresh:  # N copies kept alive (N distinct allocations), each timed twice
        copies = []
        rows = []
        for k in range(args.fresh):
            data = torch.empty_like(b.data)
            data.copy_(b.data)
            copies.append(FrameBatch(data=data, count=b.count, offsets=b.offsets))
        for r in range(2):
            for k, c in enumerate(copies):
                ms = time_batch(c)
                rows.append({"round": r, "copy": k, "ptr": hex(c.data.data_ptr()), "kernel_ms": round(ms, 4),
                             "frac": round(b.total_bytes / (ms * 1e-3) / 8e12, 4)})
                print(json.dumps(rows[-1]), flush=True)
        print(json.dumps({"workload": args.workload, "bytes": b.total_bytes, "fresh": rows}), flush=True)
        return
    if args.drift:  # the batch as built and one copy, alternated: drift over time vs placement
        data = torch.empty_like(b.data)
        data.copy_(b.data)
        c = FrameBatch(data=data, count=b.count, offsets=b.offsets)
        rows = []
        import time
        t0 = time.time()
        for r in range(args.drift):
            for name, x in (("original", b), ("copy", c)):
                ms = time_batch(x)
                rows.append({"round": r, "batch": name, "t_s": round(time.time() - t0, 2), "kernel_ms": round(ms, 4),
                             "frac": round(b.total_bytes / (ms * 1e-3) / 8e12, 4)})
                print(json.dumps(rows[-1]), flush=True)
        print(json.dumps({"workload": args.workload, "bytes": b.total_bytes, "drift": rows}), flush=True)
        return
    ms = time_batch(b)  # the batch as built, before any copy
    print(json.dumps({"copy": "original", "ptr": hex(b.data.data_ptr()), "offs_ptr": hex(b.offsets.data_ptr()),
                      "kernel_ms": round(ms, 4), "frac": round(b.total_bytes / (ms * 1e-3) / 8e12, 4)}), flush=True)
    for k in range(args.copies):
        data = torch.empty_like(b.data)
        data.copy_(b.data)
        offs = b.offsets.clone() if k % 2 else b.offsets
        c = FrameBatch(data=data, count=b.count, offsets=offs)
        ms = time_batch(c)
        res.append({"copy": k, "ptr": hex(data.data_ptr()), "offs_copied": bool(k % 2), "kernel_ms": round(ms, 4),
                    "frac": round(b.total_bytes / (ms * 1e-3) / 8e12, 4)})
        print(json.dumps(res[-1]), flush=True)
        # churn: a few allocations of other sizes, some kept, before the next copy
        keep.append(torch.empty((k + 1) * (300 << 20), dtype=torch.uint8, device="cuda"))
        del data, c
        if k % 2:
            keep.pop(0)
    ms = time_batch(b)
    print(json.dumps({"copy": "original_again", "kernel_ms": round(ms, 4),
                      "frac": round(b.total_bytes / (ms * 1e-3) / 8e12, 4)}), flush=True)
    print(json.dumps({"workload": args.workload, "bytes": b.total_bytes, "copies": res}), flush=True)


if __name__ == "__main__":
    main()
