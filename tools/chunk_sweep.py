"""Large UDP64 batches: one launch over the whole batch vs the same batch in
launch-sized slices (1 GiB, 256 MiB), per tile order. Is the 0.67 of a 4-GiB
launch (vs 0.73 at 1 GiB) a property of the launch or of the footprint?

  NEXG_TILE_ORDER=linear|xcd python tools/chunk_sweep.py [frames]   (default 64M = 4 GiB;
  the order is read once per process)
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from nex_amd import abi  # noqa: E402
from nex_amd.engine import Engine, FrameBatch  # noqa: E402


def timed(fn, steps=10, warmup=3):
    for _ in range(warmup):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
    from nex_amd import _lib
    _lib.LIB_PATH = os.path.join(ROOT, "nex_amd", "libnexg_knobs.so")  # reads NEXG_TILE_ORDER
    eng = Engine(0)
    b = eng.gen_batch(abi.WL_UDP64, n)
    out = torch.empty(n * 8, dtype=torch.uint8, device="cuda")
    order = os.environ.get("NEXG_TILE_ORDER", "auto")
    for chunk in (n, 16 << 20, 4 << 20):
        views = [FrameBatch(data=b.data[i * 64:(i + chunk) * 64], count=chunk, stride=64)
                 for i in range(0, n, chunk)]
        outs = [out[i * 8:(i + chunk) * 8] for i in range(0, n, chunk)]

        def run():
            for v, o in zip(views, outs):
                eng.parse(v, out=o)
        ms = timed(run)
        print(f"order={order:6s} chunk={chunk:>10d} launches={len(views):3d} ms={ms:8.3f} "
              f"frac={n * 64 / ms / 1e6 / 8000:.3f}", flush=True)


if __name__ == "__main__":
    main()
