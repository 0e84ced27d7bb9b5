#!/usr/bin/env python3
"""In-process A/B of the parse path across library builds: the same 16M-frame
UDP64 (and optionally IMIX) batch and output buffer, each build timed with HIP
events, interleaved A B C A B C. Output-width experiments write different
bytes, so outputs are compared only with --check.
usage: python tools/bench_parse_ab.py --libs A.so,B.so [--workloads udp64,imix,mix,real] [--out sparse]
       [--tables 64,32]   (each build with the u64 and the NEXG_FRAMES_OFFSETS32 offset table)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--workloads", default="udp64")
    ap.add_argument("--out", default="sparse")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--tables", default="64", help="offset-table forms of packed batches: 64, 32 or 64,32")
    args = ap.parse_args()
    import torch
    from nex_amd import _lib, abi
    from nex_amd.engine import Engine
    kinds = {"desc": abi.OUT_DESC, "record": abi.OUT_RECORD, "flags": abi.OUT_FLAGS,
             "verdict": abi.OUT_VERDICT, "sparse": abi.OUT_SPARSE, "grouped": abi.OUT_GROUPED}
    ok = kinds[args.out]
    libs = args.libs.split(",")
    engines = []
    for path in libs:
        _lib._lib, _lib.LIB_PATH = None, os.path.abspath(path)
        engines.append(Engine(0))
    s = torch.cuda.current_stream()
    for wl in args.workloads.split(","):
        if wl in ("mix", "real"):  # bench.py's App. C malformed mix / real-traffic batch (1M distinct, tiled)
            from nex_amd import workloads
            mk = workloads.malformed_mix if wl == "mix" else workloads.real_traffic
            m, _ = mk(engines[0], 1 << 20, seed=abi.DEFAULT_SEED + (0 if wl == "mix" else 7))
            b = workloads.tiled(m, 16)
        else:
            b = engines[0].gen_batch(abi.WL_UDP64 if wl == "udp64" else abi.WL_IMIX, 16 << 20)
        out = torch.empty(Engine.out_bytes(ok, b.count), dtype=torch.uint8, device="cuda")
        forms = {"64": b}
        if "32" in args.tables.split(",") and b.offsets is not None:
            forms["32"] = b.with_offsets32()
        variants = [(f"{l}:{t}" if len(forms) > 1 else l, e, forms[t]) for l, e in zip(libs, engines)
                    for t in args.tables.split(",") if t in forms]
        if args.check:
            ref = None
            for l, e, bb in variants:
                out.zero_()
                e.parse(bb, out_kind=ok, out=out, stream=s)
                torch.cuda.synchronize()
                ref = out.clone() if ref is None else ref
                assert torch.equal(out, ref), f"{l}: output differs"
        times = {l: [] for l, _, _ in variants}
        for rnd in range(args.rounds):
            for l, e, bb in (variants[::-1] if rnd % 2 else variants):  # alternate the order (first-measured bias)
                for _ in range(args.warmup):
                    e.parse(bb, out_kind=ok, out=out, stream=s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(s)
                for _ in range(args.steps):
                    e.parse(bb, out_kind=ok, out=out, stream=s)
                e1.record(s)
                torch.cuda.synchronize()
                times[l].append(round(e0.elapsed_time(e1) / args.steps, 4))
        print(json.dumps({"workload": wl, "out": args.out, "bytes": b.total_bytes,
                          "kernel_ms": times,
                          "frac_best": {l: round(b.total_bytes / (min(t) * 1e-3) / 8e12, 4) for l, t in times.items()}}),
              flush=True)
        del b, out, forms, variants
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
