#!/usr/bin/env python3
"""In-process A/B of the serialize path (configs[3]: 16M udp_ping-shape
frames) across library builds: the same parameter batch and output buffer,
each library timed with HIP events, interleaved A B A B; the first library
also gives the reference bytes every other build must reproduce exactly.
usage: python tools/bench_ser_ab.py --libs A.so,B.so [--steps K] [--shape tuples|aos]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", required=True)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--frames", type=int, default=16 << 20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shape", choices=["tuples", "aos", "probe"], default="tuples",
                    help="five tuple arrays (nexg_build_udp4_batch), 16-B records (nexg_build_udp4_tuples) or "
                         "udp_ping's probe batch (a destination per frame)")
    args = ap.parse_args()
    import torch
    from nex_amd import _lib
    from nex_amd.engine import Engine
    libs = args.libs.split(",")
    engines = []
    for path in libs:
        _lib._lib, _lib.LIB_PATH = None, os.path.abspath(path)
        engines.append(Engine(0))
    F = args.frames
    p = engines[0].gen_udp4_params(F)
    out = torch.empty(F * 42, dtype=torch.uint8, device="cuda")
    ref = None
    macs = (b"\x02\0\0\0\0\1", b"\x02\0\0\0\0\2")
    s = torch.cuda.current_stream()

    tup = engines[0].pack_udp4_tuples(*p) if args.shape == "aos" else None

    def step(e):
        if tup is not None:
            e.build_udp4_tuples(tup, src_mac=macs[0], dst_mac=macs[1], ip_flags=2, out=out, stream=s)
        elif args.shape == "probe":
            e.build_udp4(None, p[1], def_src_ip=0xC0A80164, def_src_port=53443, def_dst_port=33435, src_mac=macs[0],
                         dst_mac=macs[1], ip_flags=2, out=out, stream=s)
        else:
            e.build_udp4(p[0], p[1], p[2], p[3], p[4], src_mac=macs[0], dst_mac=macs[1], ip_flags=2, out=out,
                         stream=s)
    for k, e in enumerate(engines):
        out.zero_()
        step(e)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        assert torch.equal(out, ref), f"{libs[k]} builds different bytes"
    times = {l: [] for l in libs}
    for rnd in range(args.rounds):
        pairs = list(zip(libs, engines))
        for l, e in (pairs[::-1] if rnd % 2 else pairs):  # alternate the order (first-measured bias)
            for _ in range(args.warmup):
                step(e)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s)
            for _ in range(args.steps):
                step(e)
            e1.record(s)
            torch.cuda.synchronize()
            times[l].append(e0.elapsed_time(e1) / args.steps)
    for l in libs:
        ms = min(times[l])
        print(json.dumps({"lib": l, "kernel_ms": round(ms, 4), "frac": round(F * 42 / ms / 1e6 / 8000, 4),
                          "all_ms": [round(t, 4) for t in times[l]]}))


if __name__ == "__main__":
    main()
