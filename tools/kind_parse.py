#!/usr/bin/env python3
"""One mutation kind of the App. C mix (tools/bench_malformed.py's batches:
1M IMIX frames, `--share` of them mutated, tiled to 16M) parsed `--launches`
times to grouped output, nothing else on the device: the program rocprofv3
PMC passes run to compare kinds (tools/sq_kinds.sh).
usage: python tools/kind_parse.py --kind ver_ihl [--launches 8]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="clean")
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--share", type=float, default=0.5)
    ap.add_argument("--old-tiled", action="store_true", help="the round-4 tiled() construction (A/B)")
    args = ap.parse_args()
    import torch
    from nex_amd import abi, workloads
    from nex_amd.engine import Engine
    eng = Engine(0)
    if args.kind == "clean":
        base = eng.gen_batch(abi.WL_IMIX, 1 << 20)
    else:
        kinds = workloads.MUTATIONS if args.kind == "all" else (args.kind,)
        base, _ = workloads.malformed_mix(eng, 1 << 20, mutate_share=args.share, kinds=kinds)
    if args.old_tiled:  # round 4's construction: repeat, then cat with a 16-B pad (two full-size allocations)
        n, span = base.count, int(base.offsets[base.count].item())
        data = base.data[:span].repeat(16)
        offs = torch.cat([base.offsets[:n] + k * span for k in range(16)] +
                         [torch.tensor([16 * span], dtype=torch.int64, device="cuda")])
        pad = torch.zeros(16, dtype=data.dtype, device=data.device)
        from nex_amd.engine import FrameBatch
        b = FrameBatch(data=torch.cat([data, pad])[: 16 * span], count=n * 16, offsets=offs)
        del data
    else:
        b = workloads.tiled(base, 16)
    out = torch.empty(Engine.out_bytes(abi.OUT_GROUPED, b.count), dtype=torch.uint8, device="cuda")
    for _ in range(args.launches):
        eng.parse(b, out_kind=abi.OUT_GROUPED, out=out)
    torch.cuda.synchronize()
    print(f"{args.kind}: {args.launches} launches of {b.count} frames, {b.total_bytes} bytes")


if __name__ == "__main__":
    main()
