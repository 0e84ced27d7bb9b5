#!/usr/bin/env python3
"""Builder cost by frame length and payload: udp_ping's IPv4 probe batch and
icmp_ping's IPv4 probe batch at 16M frames with payloads of 0..26 B (frame
lengths 42..68, odd and even), HIP events around 20 launches after 5 warmup
launches. Tells whether an odd frame length or the payload handling costs.
usage: python tools/stride_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None, help="another build of libnexg.so (A/B)")
    ap.add_argument("--payloads", default="0,1,4,5,6,22,25,26")
    args = ap.parse_args()
    import torch
    from nex_amd import _lib, probes
    from nex_amd.engine import Engine
    if args.lib:
        _lib._lib, _lib.LIB_PATH = None, os.path.abspath(args.lib)
    eng = Engine(0)
    n = 16 << 20
    g = torch.Generator(device="cuda").manual_seed(7)
    d4 = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device="cuda", generator=g)
    dst = torch.randint(0, 256, (n, 4), dtype=torch.uint8, device="cuda", generator=g)
    src = probes.source("icmp_ping", "cuda")
    macs = (b"\x02\0\0\0\0\1", b"\x02\0\0\0\0\2")
    out = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    res = {}
    for plen in (int(x) for x in args.payloads.split(",")):
        pay = torch.tensor(list(range(1, plen + 1)), dtype=torch.uint8, device="cuda") if plen else None
        L = 42 + plen
        shapes = {
            "udp4": lambda: eng.build_udp4(None, d4, def_src_ip=0xC0A80164, def_src_port=53443, def_dst_port=33435,
                                           src_mac=macs[0], dst_mac=macs[1], ip_flags=2, payload=pay, out=out),
            "icmp4": lambda: eng.build_icmp_echo(4, src, dst, def_identifier=0x1234, def_sequence=1, payload=pay,
                                                 src_mac=macs[0], dst_mac=macs[1], ip_flags=2, out=out),
        }
        for name, fn in shapes.items():
            for _ in range(5):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            res[f"{name}_{L}B"] = {"kernel_ms": round(ms, 4), "frac_written": round(n * L / (ms * 1e-3) / 8e12, 4)}
            print(name, L, res[f"{name}_{L}B"], flush=True)
    print(json.dumps({"lib": args.lib or "default", **res}), flush=True)


if __name__ == "__main__":
    main()
