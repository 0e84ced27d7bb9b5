#!/usr/bin/env python3
"""The probe template kernel's rate by frame period: tcp_ping's IPv4 probe
batch (66-B frames, no payload, the template kernel) written at out_stride
66..72, 80, 96, 128 (zero gap after each frame), 16M frames, HIP events over
20 launches. Separates the frame period from the payload handling.
usage: python tools/template_stride.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from nex_amd import probes
    from nex_amd.engine import Engine
    eng = Engine(0)
    n = 16 << 20
    g = torch.Generator(device="cuda").manual_seed(7)
    dst = torch.randint(0, 256, (n, 4), dtype=torch.uint8, device="cuda", generator=g)
    src = probes.source("tcp_ping", "cuda")
    out = torch.empty(n * 128, dtype=torch.uint8, device="cuda")
    res = {}
    for P in (66, 67, 68, 69, 70, 72, 80, 96, 128):
        fn = lambda: eng.build_tcp(4, src, dst, def_src_port=53443, def_dst_port=80, flags=0x02, window=64240,
                                   options=probes.TCP_PING_OPTS, src_mac=probes.SRC_MAC, dst_mac=probes.DST_MAC,
                                   ttl=64, ip_flags=2, out_stride=P, out=out)
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
        res[P] = {"kernel_ms": round(ms, 4), "frac_written": round(n * P / (ms * 1e-3) / 8e12, 4)}
        print(P, res[P], flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
