#!/usr/bin/env python3
"""Per-mutation cost of the SURVEY.md App. C malformed mix: for each mutation
kind, a 1M-frame IMIX batch with every other frame carrying that mutation,
tiled to 16M frames, parsed with the default span kernel to sparse output.
Prints one JSON line per kind (kernel ms, Mpkt/s, fraction of 8 TB/s on the
algorithmic bytes, share of exception slots). The clean IMIX row is the
baseline; the spread says which fallback costs what.

usage: python tools/bench_malformed.py [--steps K] [--warmup W] [--kinds a,b]
       [--libs A.so,B.so]   (A/B: the same batches timed with each build of
                             libnexg.so in one process, interleaved A B A B)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--distinct", type=int, default=1 << 20)
    ap.add_argument("--tiles", type=int, default=16)
    ap.add_argument("--kinds", default="")
    ap.add_argument("--libs", default="")
    ap.add_argument("--share", type=float, default=0.5, help="share of frames mutated (kinds other than clean)")
    ap.add_argument("--unwrap-vlan", action="store_true", help="parse with NEXG_PARSE_VLAN (ParseOption.unwrap_vlan)")
    ap.add_argument("--out", default="sparse", choices=["sparse", "grouped", "verdict", "flags", "desc"],
                    help="output kind (verdict / flags / desc: fixed-size, no exception slots)")
    args = ap.parse_args()
    import torch
    from nex_amd import _lib, abi, workloads
    from nex_amd.engine import Engine
    from nex_amd.frame import ParseOption
    opt = ParseOption(unwrap_vlan=True) if args.unwrap_vlan else ParseOption()
    engines = []
    for path in (args.libs.split(",") if args.libs else [_lib.LIB_PATH]):
        _lib._lib, _lib.LIB_PATH = None, os.path.abspath(path)
        engines.append(Engine(0))
    eng = engines[0]
    stream = torch.cuda.current_stream()
    ok = {"grouped": abi.OUT_GROUPED, "sparse": abi.OUT_SPARSE, "verdict": abi.OUT_VERDICT, "flags": abi.OUT_FLAGS,
          "desc": abi.OUT_DESC}[args.out]
    kinds = args.kinds.split(",") if args.kinds else ["clean"] + list(workloads.MUTATIONS) + ["all"]
    for k in kinds:
        share = 0.0 if k == "clean" else args.share
        sel = workloads.MUTATIONS if k in ("clean", "all") else (k,)
        mix, counts = workloads.malformed_mix(eng, args.distinct, mutate_share=share, kinds=sel)
        b = workloads.tiled(mix, args.tiles)
        out = torch.empty(Engine.out_bytes(ok, b.count), dtype=torch.uint8, device="cuda")
        def timed(e):
            for _ in range(args.warmup):
                e.parse(b, opt, out_kind=ok, out=out, stream=stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(stream)
            for _ in range(args.steps):
                e.parse(b, opt, out_kind=ok, out=out, stream=stream)
            e1.record(stream)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / 1e3 / args.steps
        rounds = 2 if len(engines) > 1 else 1
        times, same = [], []
        ref = None
        if len(engines) > 1:  # an untimed pass of every build first: a fresh batch's first launches run slow
            for e in engines:
                timed(e)
        for rnd in range(rounds):
            # A B, then B A: the build measured first in a round pays for the
            # batch's first launches, so the order alternates
            order = list(range(len(engines)))[:: -1 if rnd % 2 else 1]
            row = [0.0] * len(engines)
            for j in order:
                row[j] = timed(engines[j])
                if len(engines) > 1:  # every build's output equals the first build's, byte for byte
                    if ref is None:
                        ref = out.clone()
                    else:
                        same.append(bool(torch.equal(out, ref)))
            times.append(row)
        s = min(t[0] for t in times)
        if ok in (abi.OUT_SPARSE, abi.OUT_GROUPED):
            codes = out[: b.count].cpu().numpy() if ok == abi.OUT_SPARSE else abi.grouped_codes(out.cpu().numpy(), b.count)
            exc = float((codes == 0).mean())
        else:
            exc = float("nan")
        line = {"kind": k, "frames": b.count, "bytes": b.total_bytes, "kernel_ms": round(s * 1e3, 4),
                "mpkt_s": round(b.count / s / 1e6, 1), "frac": round(b.total_bytes / s / 8e12, 4),
                "exception_share": round(exc, 4), "mutated": counts.get(k, None)}
        if len(engines) > 1:
            line["kernel_ms_by_lib"] = [[round(x * 1e3, 4) for x in t] for t in times]
            line["outputs_equal"] = all(same)
        print(json.dumps(line), flush=True)
        del b, mix, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
