#!/usr/bin/env python3
"""Span-kernel phase cycles per library build: for each workload (IMIX, the
App. C mix, real traffic) and each build, a few timed launches and then one
stamped launch (nexg_probe_span_clock), reduced by clocks.span_summary. Shows
which phase of a workgroup a build change moves.
usage: python tools/span_phases_ab.py --libs A.so,B.so [--workloads imix,mix,real]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--workloads", default="imix,mix,real")
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from nex_amd import _lib, abi, clocks, workloads
    from nex_amd.engine import Engine
    libs = args.libs.split(",")
    engines = []
    for path in libs:
        _lib._lib, _lib.LIB_PATH = None, os.path.abspath(path)
        engines.append(Engine(0))
    s = torch.cuda.current_stream()
    for wl in args.workloads.split(","):
        if wl in ("mix", "real"):
            mk = workloads.malformed_mix if wl == "mix" else workloads.real_traffic
            m, _ = mk(engines[0], 1 << 20, seed=abi.DEFAULT_SEED + (0 if wl == "mix" else 7))
            b = workloads.tiled(m, 16)
        else:
            b = engines[0].gen_batch(abi.WL_IMIX, 16 << 20)
        out = torch.empty(Engine.out_bytes(abi.OUT_GROUPED, b.count), dtype=torch.uint8, device="cuda")
        for path, e in zip(libs, engines):
            for _ in range(5):
                e.parse(b, out_kind=abi.OUT_GROUPED, out=out, stream=s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s)
            for _ in range(args.steps):
                e.parse(b, out_kind=abi.OUT_GROUPED, out=out, stream=s)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.steps
            _, st = e.probe_span_clock(b)
            sm = clocks.span_summary(st.cpu().numpy())
            print(json.dumps({"workload": wl, "lib": os.path.basename(path), "kernel_ms": round(ms, 4),
                              "frac": round(b.total_bytes / (ms * 1e-3) / 8e12, 4),
                              "clock_ghz": sm.get("shader_clock_ghz", {}).get("median"),
                              "wg_cycles": sm.get("workgroup_cycles"), "wg_us": sm.get("workgroup_us"),
                              "phase_cycles": sm.get("phase_cycles")}), flush=True)
        del b, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
