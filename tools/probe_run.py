#!/usr/bin/env python3
"""One probe batch of nex_amd/probes.py (16M frames) built `--launches`
times, nothing else on the device: the program tools/pmc.sh's PMC passes run
for the bench's ser.<shape> objects (traffic key ser_<shape>:desc).
usage: python tools/probe_run.py --shape tcp_ping [--launches 8]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="tcp_ping")
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--frames", type=int, default=16 << 20)
    args = ap.parse_args()
    import torch
    from nex_amd import probes
    from nex_amd.engine import Engine
    eng = Engine(0)
    n = args.frames
    g = torch.Generator(device="cuda").manual_seed(7)
    d = torch.randint(0, 256, (n, probes.dst_bytes(args.shape)), dtype=torch.uint8, device="cuda", generator=g)
    out = torch.empty(n * probes.frame_len(args.shape), dtype=torch.uint8, device="cuda")
    for _ in range(args.launches):
        probes.build(eng, args.shape, d, out=out)
    torch.cuda.synchronize()
    print(f"{args.shape}: {args.launches} launches of {n} frames")


if __name__ == "__main__":
    main()
